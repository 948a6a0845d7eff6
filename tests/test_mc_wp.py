"""Weighted prediction in motion compensation (FME_MC_WP, fme_set_wp): the PPS UseWP (P slices) /
WPBiPred (B slices) branch of TComPrediction::motionCompensation (TComPrediction.cpp:509-512,
539-542, 612-619), i.e. each list filtered to HM's 14-bit values, then
TComWeightPrediction::addWeightUni / addWeightBi (TComWeightPrediction.cpp:78-245) with
getWpScaling's parameters (247-324), and xCheckIdenticalMotion not collapsing identical bi motion.

Fixtures (tests/golden/mcwp*_*.npz, oracle/gen_golden.py) come from oracle/_ref, which drives the
reference's own filters and TComWeightPrediction; the C oracle's orc_mc_wp restates it at 8 bits
and agrees (the 10-bit fixture is pinned on the reference alone).  Integer planes: bit-exact."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("mcwp") and f.endswith(".npz"))


def _reference(g):
    from oracle import REF_SO, Reference
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    ref = Reference(bit_depth=int(g["bit_depth"][0]))
    for k in range(len(g["ref_y"])):
        ref.set_picture_yuv(k, g["ref_y"][k], g["ref_cb"][k], g["ref_cr"][k])
    return ref


def _run_ref(ref, g, jobs, wp=None):
    dt = g["pred_y"].dtype
    y = np.zeros_like(g["pred_y"], dtype=dt)
    cb = np.zeros_like(g["pred_cb"], dtype=dt)
    cr = np.zeros_like(g["pred_cr"], dtype=dt)
    if wp is not None:
        for l in range(2):
            for r in range(wp.shape[1]):
                ref.set_wp(l, r, wp[l, r])
    ref.mc(jobs, y, cb, cr)
    return y, cb, cr


def test_mcwp_goldens_cover_the_branches():
    from nnfme.abi import MC_WP
    seen = {"uni": 0, "bi": 0, "identical": 0, "unit_weight": 0, "plain": 0, "10bit": 0}
    for case in CASES:
        g = load_golden(case)
        j, wp = g["jobs"], g["wp"]
        w = (j["flags"] & MC_WP) != 0
        bi = (j["flags"] & 3) == 3
        same = bi & (j["ref_id"][:, 0] == j["ref_id"][:, 1]) & (j["mv"][:, 0, 0] == j["mv"][:, 1, 0]) & \
            (j["mv"][:, 0, 1] == j["mv"][:, 1, 1])
        seen["uni"] += int((w & ~bi).sum())
        seen["bi"] += int((w & bi).sum())
        seen["identical"] += int((w & same).sum())
        seen["plain"] += int((~w).sum())
        seen["unit_weight"] += int((wp[..., 0] == (1 << wp[..., 2])).sum())
        seen["10bit"] += int(g["bit_depth"][0] == 10)
    assert min(seen.values()) > 0, seen


@pytest.mark.parametrize("case", CASES)
def test_mcwp_reference_harness_matches_golden(case):
    g = load_golden(case)
    y, cb, cr = _run_ref(_reference(g), g, g["jobs"], g["wp"])
    assert np.array_equal(y, g["pred_y"]) and np.array_equal(cb, g["pred_cb"]) and np.array_equal(cr, g["pred_cr"])


@pytest.mark.parametrize("case", [c for c in CASES if not c.startswith("mcwp10")])
def test_mcwp_oracle_matches_golden(case):
    """orc_mc_wp (the C restatement of getWpScaling + weightBidir / weightUnidir / noWeightUnidir,
    8-bit) against the reference's own TComWeightPrediction run."""
    from oracle import Oracle
    g = load_golden(case)
    pics = {k: (g["ref_y"][k], g["ref_cb"][k], g["ref_cr"][k]) for k in range(len(g["ref_y"]))}
    y = np.zeros_like(g["pred_y"])
    cb = np.zeros_like(g["pred_cb"])
    cr = np.zeros_like(g["pred_cr"])
    Oracle().mc(pics, g["jobs"], y, cb, cr, wp=g["wp"])
    assert np.array_equal(y, g["pred_y"]) and np.array_equal(cb, g["pred_cb"]) and np.array_equal(cr, g["pred_cr"])


@pytest.mark.parametrize("case", CASES)
def test_mcwp_default_weights_equal_plain_prediction(case):
    """With weight 1 << d and offset 0, addWeightUni is the plain uni-pred rounding and addWeightBi
    the plain average (addAvg): the harness's WP path then reproduces the unweighted planes, except
    identical bi motion, which WPBiPred keeps as two (equal) lists - whose average is the same."""
    from nnfme.abi import MC_WP
    g = load_golden(case)
    ref = _reference(g)
    unit = np.array(g["wp"], copy=True)
    unit[..., 0] = 1 << unit[..., 2]
    unit[..., 1] = 0
    a = _run_ref(ref, g, g["jobs"], unit)
    plain = np.array(g["jobs"], copy=True)
    plain["flags"] &= np.uint8(0xFF & ~MC_WP)
    b = _run_ref(ref, g, plain)
    for p, q in zip(a, b):
        assert np.array_equal(p, q)
    # and the fixture's own weights change the weighted PUs
    assert not np.array_equal(g["pred_y"], b[0])


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_mcwp_matches_golden(case):
    from nnfme.runtime import FmeContext
    g = load_golden(case)
    bd = int(g["bit_depth"][0])
    ctx = FmeContext(nn_mode=0, bit_depth=bd)
    for k in range(len(g["ref_y"])):
        ctx.set_picture(k, g["ref_y"][k])
        ctx.set_picture_chroma(k, g["ref_cb"][k], g["ref_cr"][k])
    for l in range(2):
        for r in range(g["wp"].shape[1]):
            ctx.set_wp(l, r, g["wp"][l, r])
    dt = g["pred_y"].dtype
    y = np.zeros_like(g["pred_y"], dtype=dt)
    cb = np.zeros_like(g["pred_cb"], dtype=dt)
    cr = np.zeros_like(g["pred_cr"], dtype=dt)
    ctx.motion_compensate(g["jobs"], y, cb, cr)
    for got, want, comp in ((y, g["pred_y"], "Y"), (cb, g["pred_cb"], "Cb"), (cr, g["pred_cr"], "Cr")):
        bad = got != want
        assert not bad.any(), f"{case} {comp}: {int(bad.sum())} samples differ"
    # the plain jobs of the same call are unaffected by the table; a bad table entry is refused
    from nnfme.runtime import FmeError
    with pytest.raises(FmeError):
        ctx.set_wp(2, 0, g["wp"][0, 0])


def test_unit_weight_branch_identity():
    """k_mc / k_mc10 use one uni-pred formula, ((w (p + 8192) + 2^(s-1)) >> s) + o with s = d + shiftNum,
    where addWeightUni switches to noWeightUnidir ((p + 8192 + 2^(n-1)) >> n) + o when w == 1 << d
    (TComWeightPrediction.cpp:170-238): the two agree for every 14-bit value, denominator and bit depth."""
    p = np.arange(-8192, 16384 + 1, dtype=np.int64)
    for bd in (8, 10):
        n = max(2, 14 - bd)
        for d in range(8):
            s = d + n
            one = ((1 << d) * (p + 8192) + (1 << (s - 1))) >> s
            two = (p + 8192 + (1 << (n - 1))) >> n
            assert np.array_equal(one, two), (bd, d)
