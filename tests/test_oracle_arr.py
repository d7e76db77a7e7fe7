"""CPU: the oracle's restatement of the Fr vector ops and of division by a vanishing
polynomial, pinned bit-for-bit against the reference's own C (oracle/_ref, compiled from
lib/cbits/curves/array/mont/<C>_arr_mont.c and poly/mont/<C>_poly_mont.c)."""
import ctypes

import numpy as np
import pytest

CURVES = ["bn128", "bls12_381"]
FR = {"bn128": 1, "bls12_381": 3}


def fr(oracle, curve, seed, n):
    return oracle.gen_fr(curve, seed, 0, n)


@pytest.mark.parametrize("curve", CURVES)
def test_elementwise_vs_reference(oracle, reference, curve):
    n = 257
    a, b, c = (fr(oracle, curve, s, n) for s in (1, 2, 3))
    a[5] = 0  # zeros in the mix
    b[7] = 0
    kA, kB = fr(oracle, curve, 4, 1)[0], fr(oracle, curve, 5, 1)[0]
    R = lambda name, *args: reference.arr(curve, "arr_mont_" + name, *args)
    cases = {
        "neg": ((a,), "neg"), "add": ((a, b), "add"), "sub": ((a, b), "sub"), "sqr": ((a,), "sqr"),
        "mul": ((a, b), "mul"), "from_std": ((a,), "from_std"), "to_std": ((a,), "to_std"),
    }
    for op, (args, name) in cases.items():
        want = np.zeros_like(a)
        R(name, n, *args, want)
        got = oracle.arr_op(curve, op, n, *args)
        assert np.array_equal(got, want), op
    for op, name in (("mul_add", "mul_add"), ("mul_sub", "mul_sub")):
        want = np.zeros_like(a)
        R(name, n, a, b, c, want)
        assert np.array_equal(oracle.arr_op(curve, op, n, a, b, c), want), op
    want = np.zeros_like(a)
    R("scale", n, kA, a, want)
    assert np.array_equal(oracle.arr_op(curve, "scale", n, a, kA=kA), want)
    R("Ax_plus_y", n, kA, a, b, want)
    assert np.array_equal(oracle.arr_op(curve, "Ax_plus_y", n, a, b, kA=kA), want)
    R("Ax_plus_By", n, kA, kB, a, b, want)
    assert np.array_equal(oracle.arr_op(curve, "Ax_plus_By", n, a, b, kA=kA, kB=kB), want)
    t = b.copy()
    R("sub_inplace_reverse", n, t, a)
    assert np.array_equal(oracle.arr_op(curve, "sub_rev", n, b, a), t)
    d = np.zeros(4, dtype=np.uint64)
    R("dot_prod", n, a, b, d)
    assert np.array_equal(oracle.arr_dot(curve, a, b), d)
    p = np.zeros((100, 4), dtype=np.uint64)
    R("powers", 100, kA, kB, p)
    assert np.array_equal(oracle.arr_powers(curve, kA, kB, 100), p)


@pytest.mark.parametrize("curve", CURVES)
def test_batch_inversion_vs_reference(oracle, reference, curve):
    n = 300
    a, b = fr(oracle, curve, 11, n), fr(oracle, curve, 12, n)
    for x in (b, np.concatenate([b[:10], np.zeros((1, 4), np.uint64), b[11:]])):  # no zero / one zero
        want = np.zeros_like(x)
        reference.arr(curve, "arr_mont_inv", n, x, want)
        assert np.array_equal(oracle.arr_op(curve, "inv", n, x), want)
        reference.arr(curve, "arr_mont_div", n, a, x, want)
        assert np.array_equal(oracle.arr_op(curve, "div", n, a, x), want)
    z = np.zeros_like(b)
    z[10] = 0
    bz = b.copy()
    bz[10] = 0
    assert not oracle.arr_op(curve, "inv", n, bz).any()  # any zero -> every output zero


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n1,n,eta_one", [(40, 8, False), (40, 8, True), (33, 16, False), (7, 8, False),
                                          (64, 1, False), (100, 32, False), (0, 4, False)])
def test_div_by_vanishing_vs_reference(oracle, reference, curve, n1, n, eta_one):
    poly = fr(oracle, curve, 21 + n1, max(n1, 1))[:n1]
    if n1 > 3:
        poly[-2:] = 0  # degree below n1 - 1
    eta = fr(oracle, curve, 22, 1)[0]
    if eta_one:
        eta = oracle.arr_op(curve, "from_std", 1, np.array([[1, 0, 0, 0]], dtype=np.uint64))[0]
    q, r, ok = oracle.div_by_vanishing(curve, poly, n, eta)
    nq, nr = max(0, n1 - n), n
    wq = np.zeros((max(nq, 1), 4), dtype=np.uint64)
    wr = np.zeros((max(nr, 1), 4), dtype=np.uint64)
    src = poly if n1 else np.zeros((1, 4), dtype=np.uint64)
    reference.arr(curve, "poly_mont_div_by_vanishing", n1, src, n, eta, nq, wq, nr, wr)
    assert np.array_equal(q, wq[:nq]) and np.array_equal(r, wr[:nr])
    wq2 = np.zeros((max(nq, 1), 4), dtype=np.uint64)
    ok_ref = reference.arr(curve, "poly_mont_quot_by_vanishing", n1, src, n, eta, nq, wq2, restype=ctypes.c_uint8)
    assert bool(ok_ref) == ok


@pytest.mark.parametrize("curve", CURVES)
def test_exact_multiple_quotient(oracle, reference, curve):
    """(x^n - eta) * g(x) divides exactly: quot_by_vanishing finds g, remainder zero"""
    n, m = 16, 24
    g = fr(oracle, curve, 31, m)
    eta = fr(oracle, curve, 32, 1)[0]
    # p = x^n g - eta g
    p = np.zeros((n + m, 4), dtype=np.uint64)
    p[n:] = g
    p[:m] = oracle.arr_op(curve, "sub", m, p[:m].copy(), oracle.arr_op(curve, "scale", m, g, kA=eta))
    q, r, ok = oracle.div_by_vanishing(curve, p, n, eta)
    assert ok and np.array_equal(q[:m], g) and not r.any()
