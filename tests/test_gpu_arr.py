"""GPU Fr vector ops and division by a vanishing polynomial, through the reference-named C
ABI (<C>_arr_mont_*, <C>_poly_mont_{div,quot}_by_vanishing): bit-exact against the
reference's own C (oracle/_ref) and the oracle restatement."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]


def fr(gpu, curve, seed, n):
    return gpu.gen_fr(curve, seed, n)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [1, 2, 63, 1000, 65537])
def test_elementwise(gpu, oracle, curve, n):
    a, b, c = (fr(gpu, curve, s + n, n) for s in (1, 2, 3))
    a[n // 2] = 0
    kA, kB = fr(gpu, curve, 4, 1)[0], fr(gpu, curve, 5, 1)[0]
    assert np.array_equal(gpu.arr_neg(curve, a), oracle.arr_op(curve, "neg", n, a))
    assert np.array_equal(gpu.arr_add(curve, a, b), oracle.arr_op(curve, "add", n, a, b))
    assert np.array_equal(gpu.arr_sub(curve, a, b), oracle.arr_op(curve, "sub", n, a, b))
    assert np.array_equal(gpu.arr_sqr(curve, a), oracle.arr_op(curve, "sqr", n, a))
    assert np.array_equal(gpu.arr_mul(curve, a, b), oracle.arr_op(curve, "mul", n, a, b))
    assert np.array_equal(gpu.arr_mul_add(curve, a, b, c), oracle.arr_op(curve, "mul_add", n, a, b, c))
    assert np.array_equal(gpu.arr_mul_sub(curve, a, b, c), oracle.arr_op(curve, "mul_sub", n, a, b, c))
    assert np.array_equal(gpu.arr_scale(curve, kA, a), oracle.arr_op(curve, "scale", n, a, kA=kA))
    assert np.array_equal(gpu.arr_lin_comb1(curve, (kA, a), b), oracle.arr_op(curve, "Ax_plus_y", n, a, b, kA=kA))
    assert np.array_equal(gpu.arr_lin_comb2(curve, (kA, a), (kB, b)),
                          oracle.arr_op(curve, "Ax_plus_By", n, a, b, kA=kA, kB=kB))
    assert np.array_equal(gpu.arr_to_std(curve, a), oracle.arr_op(curve, "to_std", n, a))
    assert np.array_equal(gpu.arr_from_std(curve, a), oracle.arr_op(curve, "from_std", n, a))
    assert np.array_equal(gpu.arr_from_std(curve, gpu.arr_to_std(curve, a)), a)
    assert np.array_equal(gpu.arr_dot_prod(curve, a, b), oracle.arr_dot(curve, a, b))
    assert np.array_equal(gpu.arr_powers(curve, kA, kB, n), oracle.arr_powers(curve, kA, kB, n))
    assert np.array_equal(gpu.arr_append(curve, a, b), np.concatenate([a, b]))


@pytest.mark.parametrize("curve", CURVES)
def test_vs_reference_library(gpu, reference, curve):
    """the same entry points called on the reference's own C give the same bytes"""
    n = 4099
    a, b, c = (fr(gpu, curve, s, n) for s in (41, 42, 43))
    kA = fr(gpu, curve, 44, 1)[0]
    lib = gpu.load()
    for name, args in (("mul", (a, b)), ("add", (a, b)), ("sub", (a, b)), ("sqr", (a,)), ("inv", (a,)),
                       ("div", (a, b)), ("neg", (a,)), ("to_std", (a,)), ("from_std", (a,)),
                       ("mul_add", (a, b, c)), ("mul_sub", (a, b, c)), ("scale", (kA, a)),
                       ("Ax_plus_y", (kA, a, b))):
        want = np.zeros_like(a)
        got = np.zeros_like(a)
        reference.arr(curve, "arr_mont_" + name, n, *args, want)
        conv = [x.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) for x in args]
        getattr(lib, f"{curve}_arr_mont_{name}")(n, *conv, got.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        assert np.array_equal(got, want), name


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [1, 31, 32, 33, 1000, 1 << 17])
def test_batch_inversion(gpu, oracle, curve, n):
    a, b = fr(gpu, curve, 50 + n, n), fr(gpu, curve, 60 + n, n)
    inv = gpu.arr_inv(curve, b)
    assert np.array_equal(inv, oracle.arr_op(curve, "inv", n, b))
    assert np.array_equal(gpu.arr_div(curve, a, b), oracle.arr_op(curve, "div", n, a, b))
    one = gpu.arr_mul(curve, inv, b)
    assert gpu.arr_is_one(curve, one)


@pytest.mark.parametrize("curve", CURVES)
def test_batch_inversion_2_24_ragged(gpu, oracle, curve):
    """the prover-size chunking (128 elements per Fermat inversion from 2^24, zk_arr.hip) with a
    ragged last chunk: inv(b) b == 1 everywhere, sampled elements equal the oracle's inverses,
    and a zero in the LAST chunk still zeroes every output"""
    n = (1 << 24) + 4099
    b = fr(gpu, curve, 97, n)
    db, dt = gpu.DeviceBuffer(b), gpu.DeviceBuffer.empty(b.nbytes)
    try:
        gpu.arr_op_device(curve, "inv", n, db, None, d_tgt=dt)
        inv = dt.to_host(b)
        idx = np.r_[0, 1, 127, 128, np.arange(n - 4100, n, 97), n - 1]
        assert np.array_equal(inv[idx], oracle.arr_op(curve, "inv", len(idx), np.ascontiguousarray(b[idx])))
        gpu.arr_op_device(curve, "mul", n, dt, db, d_tgt=dt)
        assert gpu.arr_is_one(curve, dt.to_host(b))
        b[n - 2] = 0
        db.free()
        db = gpu.DeviceBuffer(b)
        gpu.arr_op_device(curve, "inv", n, db, None, d_tgt=dt)
        assert not dt.to_host(b).any()
    finally:
        for d in (db, dt):
            d.free()


@pytest.mark.parametrize("curve", CURVES)
def test_batch_inversion_zero_rule(gpu, curve):
    """reference batch_inv (Fr_mont.c:258-285): one zero input zeroes EVERY output"""
    b = fr(gpu, curve, 71, 5000)
    b[1234] = 0
    assert not gpu.arr_inv(curve, b).any()
    assert not gpu.arr_div(curve, fr(gpu, curve, 72, 5000), b).any()


@pytest.mark.parametrize("curve", CURVES)
def test_predicates_and_inplace(gpu, reference, curve):
    n = 777
    a, b = fr(gpu, curve, 81, n), fr(gpu, curve, 82, n)
    assert gpu.arr_is_valid(curve, a)
    bad = a.copy()
    bad[3] = np.uint64(0xFFFFFFFFFFFFFFFF)
    assert not gpu.arr_is_valid(curve, bad)
    assert gpu.arr_is_zero(curve, np.zeros((n, 4), np.uint64)) and not gpu.arr_is_zero(curve, a)
    assert gpu.arr_is_equal(curve, a, a.copy()) and not gpu.arr_is_equal(curve, a, b)
    assert gpu.arr_is_zero(curve, np.zeros((0, 4), np.uint64))  # empty: vacuously true
    lib, P = gpu.load(), (lambda x: x.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    for name, want_name, extra in (("add_inplace", "add", (b,)), ("sub_inplace", "sub", (b,)),
                                   ("mul_inplace", "mul", (b,)), ("sqr_inplace", "sqr", ()),
                                   ("neg_inplace", "neg", ()), ("inv_inplace", "inv", ()),
                                   ("div_inplace", "div", (b,))):
        t = a.copy()
        getattr(lib, f"{curve}_arr_mont_{name}")(n, P(t), *[P(x) for x in extra])
        want = np.zeros_like(a)
        reference.arr(curve, "arr_mont_" + want_name, n, a, *extra, want)
        assert np.array_equal(t, want), name
    t = a.copy()
    getattr(lib, f"{curve}_arr_mont_sub_inplace_reverse")(n, P(t), P(b))
    want = np.zeros_like(a)
    reference.arr(curve, "arr_mont_sub", n, b, a, want)
    assert np.array_equal(t, want)
    t = np.zeros_like(a)
    getattr(lib, f"{curve}_arr_mont_set_one")(n, P(t))
    assert gpu.arr_is_one(curve, t)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n1,n", [(40, 8), (33, 16), (7, 8), (64, 1), (100, 32), (0, 4), (3 << 14, 1 << 14)])
def test_div_by_vanishing(gpu, oracle, curve, n1, n):
    poly = fr(gpu, curve, 91 + n1, max(n1, 1))[:n1]
    if n1 > 3:
        poly[-2:] = 0
    eta = fr(gpu, curve, 92, 1)[0]
    q, r = gpu.div_by_vanishing(curve, poly, n, eta)
    wq, wr, ok = oracle.div_by_vanishing(curve, poly, n, eta)
    assert np.array_equal(q, wq) and np.array_equal(r, wr)
    assert (gpu.quot_by_vanishing(curve, poly, n, eta) is not None) == ok


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n1,n,zero_top", [(200000, 4096, 100000), (5000, 37, 0), (130, 100, 3), (9000, 64, 4097),
                                           (70000, 65, 0), (20000, 20000, 0), (12288, 1, 12000),
                                           (1500000, 4096, 1200000), (600000, 1024, 600000)])
def test_div_by_vanishing_shapes(gpu, oracle, curve, n1, n, zero_top):
    """chains of every length mod the wavefront (n < 64, n not a multiple of 64, deg - n < n), and
    degrees far below the buffer's top (the top-down degree scan skips whole chunks)"""
    poly = fr(gpu, curve, 97 + n, n1)
    if zero_top:
        poly[-zero_top:] = 0
    eta = fr(gpu, curve, 98, 1)[0]
    q, r = gpu.div_by_vanishing(curve, poly, n, eta)
    wq, wr, ok = oracle.div_by_vanishing(curve, poly, n, eta)
    assert np.array_equal(q, wq) and np.array_equal(r, wr)
    assert (gpu.quot_by_vanishing(curve, poly, n, eta) is not None) == ok


@pytest.mark.parametrize("curve", CURVES)
def test_quot_by_vanishing_exact(gpu, curve):
    """(x^n - eta) g(x) / (x^n - eta) = g, remainder zero -- at PLONK-like size 2^16"""
    n, m = 1 << 16, 1 << 16
    g = fr(gpu, curve, 93, m)
    eta = fr(gpu, curve, 94, 1)[0]
    p = np.zeros((n + m, 4), dtype=np.uint64)
    p[n:] = g
    p[:m] = gpu.arr_sub(curve, p[:m].copy(), gpu.arr_scale(curve, eta, g))
    q = gpu.quot_by_vanishing(curve, p, n, eta)
    assert q is not None and np.array_equal(q, g)


@pytest.mark.parametrize("curve", CURVES)
def test_device_resident_ops_2_22(gpu, curve):
    """device-resident form at a prover-like size: mul then div round-trips exactly"""
    n = 1 << 22
    a, b = fr(gpu, curve, 95, n), fr(gpu, curve, 96, n)
    da, db, dt = gpu.DeviceBuffer(a), gpu.DeviceBuffer(b), gpu.DeviceBuffer.empty(a.nbytes)
    try:
        gpu.arr_op_device(curve, "mul", n, da, db, d_tgt=dt)
        gpu.arr_op_device(curve, "div", n, dt, db, d_tgt=dt)
        assert np.array_equal(dt.to_host(a), a)
    finally:
        for d in (da, db, dt):
            d.free()
