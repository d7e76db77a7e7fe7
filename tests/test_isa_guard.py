"""The shipped library's gfx950 code objects contain no device-function calls and no long
branch through the return-address pair (tools/isa_guard.py).  Round 4's first Jacobian group FFT
left xyzz_scl outlined and LLVM's branch relaxation reused s[30:31] inside it: the kernel hung
(profiles/r05a_fft_outlined_scl.txt holds that variant's assembly).  A later edit or compiler that
outlines a point routine again fails here, on the CPU, before any GPU run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_guard  # noqa: E402


def test_shipped_code_objects_have_no_calls():
    assert os.path.exists(isa_guard.LIB), "build the library first (__graft_entry__.build)"
    n, fft, bad = isa_guard.check()
    assert n > 100
    # every group-FFT kernel (forward / inverse, GLV and integer stages, first inverse stage,
    # membership test; both curves) is in the scan
    for k in ("k_fft_fwd_stage_glv", "k_fft_inv_stage_glv", "k_fft_inv_first_glv", "k_fft_fwd_stage",
              "k_fft_inv_stage", "k_subgroup_check", "k_fft_load"):
        assert sum(k in f for f in fft) >= 2 or k == "k_subgroup_check", k
    assert not bad, bad[:10]


def test_checker_flags_the_outlined_variant():
    """negative control: the committed excerpt of the hanging build is flagged"""
    text = open(os.path.join(ROOT, "profiles", "r05a_fft_outlined_scl.txt")).read()
    bad = isa_guard.violations(isa_guard.functions(text))
    reasons = {why.split(":")[0] for _, why in bad}
    assert "long branch built in the return-address pair" in reasons
    assert "s_setpc_b64 through the return-address pair" in reasons
    assert isa_guard.violations({"k": ["s_swappc_b64 s[30:31], s[0:1]"]})
    assert not isa_guard.violations({"k": ["s_getpc_b64 s[90:91]", "s_add_u32 s90, s90, 0x10",
                                           "s_addc_u32 s91, s91, 0", "s_setpc_b64 s[90:91]"]})
    assert isa_guard.violations({"k": ["s_setpc_b64 s[90:91]"]})
