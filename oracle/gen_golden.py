#!/usr/bin/env python3
"""Generate tests/golden/*.npz — TEST INFRASTRUCTURE ONLY (run in the build container).

Expected outputs come from oracle/_ref/libhmref.so: the reference's own TLibCommon sources
(TComInterpolationFilter, TComRdCost, TComPicYuv, TComPrediction scratch planes) compiled
from /root/reference and driven in TEncSearch's order by oracle/ref_harness.cpp.  Every case
is also run through the plain-C oracle (fme_oracle.c); generation aborts on any mismatch.

Each fixture holds inputs and outputs only (data): pictures, lambdas, bi-pred key blocks,
jobs (fme_job records), results (fme_result records) and the configuration.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(ROOT, "hm16.9-nn_fme_amd")]

from oracle import Oracle, Reference  # noqa: E402
from nnfme import synth, weights  # noqa: E402
from nnfme.abi import JOB_BIPRED, JOB_EMI, JOB_LOSSLESS, JOB_NN_IN, TZ_RING, compare_results  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def edge_jobs(rng, width, height, n):
    """Jobs that hit the corners: search-range edges (< 8 EMI pushes), picture borders with MVs
    pointing outside (edge replication), the largest PUs."""
    sizes = [s for s in synth.ALL_PU_SIZES]
    picks = [sizes[i % len(sizes)] for i in range(n)]
    w = np.array([p[0] for p in picks])
    h = np.array([p[1] for p in picks])
    j = synth.make_jobs(rng, width, height, n, 4, [0, 1, 2], [0, 1, 2, 3], sizes=(w, h))
    for i in range(n):
        kind = i % 6
        if kind == 0:      # TZ best on the left/top range edge
            j["mv_x"][i] = j["lt_x"][i]
            j["mv_y"][i] = j["lt_y"][i]
        elif kind == 1:    # right/bottom edge
            j["mv_x"][i] = j["rb_x"][i]
            j["mv_y"][i] = j["rb_y"][i]
        elif kind == 2:    # PU at the top-left corner, MV far outside
            j["x"][i] = 0
            j["y"][i] = 0
            j["mv_x"][i] = max(int(j["lt_x"][i]), -60)
            j["mv_y"][i] = max(int(j["lt_y"][i]), -60)
        elif kind == 3:    # bottom-right corner
            j["x"][i] = (width - j["w"][i]) // 4 * 4
            j["y"][i] = (height - j["h"][i]) // 4 * 4
        elif kind == 4:    # degenerate range: a single column
            j["lt_x"][i] = j["rb_x"][i] = j["mv_x"][i]
        else:              # lossless CU (SAD in FracDIF)
            j["flags"][i] = JOB_EMI | JOB_LOSSLESS
    # the search range must contain the start point (xTZSearch invariant)
    return j


def build_case(name, seed, width, height, n_jobs, hadme, fen, nn_mode, qp, bipred=0.15, n_edge=96, net=None, gop="ldp",
               bit_depth=8):
    """bit_depth 10: the main10 configurations (cfg/encoder_lowdelay_P_main10.cfg:58): 16-bit
    pictures, _ref's TComInterpolationFilter / TComRdCost run with bitDepth 10.  The lambdas are the
    8-bit ones: HM scales the QP by 6 * (bitDepth - 8 - DISTORTION_PRECISION_ADJUSTMENT(bitDepth - 8))
    = 0 in the shipped build (TypeDef.h:140-143, FULL_NBIT 0), so lambda does not change."""
    rng = np.random.default_rng(seed)
    if bit_depth > 8:
        pics = {i: synth.synth_luma_hbd(width, height, i, bit_depth, seed=seed) for i in range(5)}
    else:
        pics = {i: synth.synth_luma(width, height, i, seed=seed) for i in range(5)}
    if gop == "ra":   # random-access GOP-8 lambdas (TEncSlice.cpp:246-325): entries POC 8, 4, 2, 1
        lambdas = np.array([synth.ra_lambda(qp, e) for e in range(4)], dtype=np.float64)
    else:
        lambdas = np.array(synth.LDP_LAMBDA[qp if qp in synth.LDP_LAMBDA else 22], dtype=np.float64)
    a = synth.make_jobs(rng, width, height, n_jobs, 4, [0, 1, 2, 3], [0, 1, 2, 3], bipred_frac=bipred)
    b = edge_jobs(rng, width, height, n_edge)
    jobs = np.concatenate([b[:8], a, b[8:]])
    # recompute the bi-pred keys over the final order
    jobs["key_offset"][(jobs["flags"] & JOB_BIPRED) != 0] = -2
    keys = synth.make_bipred_keys(rng, jobs, pics)
    ref = Reference(use_hadamard=hadme, nn_mode=nn_mode, fast_inter_mode=fen, bit_depth=bit_depth)
    orc = Oracle(use_hadamard=hadme, nn_mode=nn_mode, qp=qp, fast_inter_mode=fen, bit_depth=bit_depth)
    wts = weights.load_weights(qp)
    for eng in (ref, orc):
        for k, v in pics.items():
            eng.set_picture(k, v)
        for lid, lam in enumerate(lambdas):
            eng.set_lambda(lid, float(lam))
        eng.set_keys(keys if keys.size else np.zeros(1, np.int16))
        eng.load_nn(wts)
        if net is not None:
            eng.load_nn_net(weights.case_net(net))
    r_ref = ref.refine(jobs)
    r_orc = orc.refine(jobs)
    bad, first, counts = compare_results(r_ref, r_orc)
    if bad:
        raise SystemExit(f"{name}: oracle disagrees with _ref on {bad} jobs (first {first}): {counts}")
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(
        path,
        pictures=np.stack([pics[i] for i in range(5)]),
        lambdas=lambdas,
        keys=keys,
        jobs=jobs,
        results=r_ref,
        config=np.array([hadme, fen, nn_mode, qp], dtype=np.int32),
        **({"net": np.array(net)} if net is not None else {}),
        **({"bit_depth": np.array([bit_depth], np.int32)} if bit_depth != 8 else {}),
    )
    print(f"{path}: {len(jobs)} jobs, {int((jobs['flags'] & JOB_BIPRED != 0).sum())} bi-pred, "
          f"{int((r_ref['n_emi'] < 8).sum())} with < 8 EMI pushes")


def mc10_pictures(width, height, refs, seed):
    """Reference pictures at bit depth 10: synthetic 10-bit luma, chroma from the 8-bit generator
    with random low bits (every sample value 0..1023 reachable)."""
    rng = np.random.default_rng(seed + 1000)
    pics = {}
    for k in range(refs):
        cb, cr = synth.synth_chroma(width, height, k, seed=seed)
        lo = rng.integers(0, 4, size=(2,) + cb.shape, dtype=np.uint16)
        pics[k] = (synth.synth_luma_hbd(width, height, k, bit_depth=10, seed=seed),
                   (cb.astype(np.uint16) << 2) | lo[0], (cr.astype(np.uint16) << 2) | lo[1])
    return pics


def build_mc10_case(name, seed, width, height, bi_frac, mv_amp, identical_frac, fill=0):
    """Motion compensation at bit depth 10 (cfg *_main10.cfg InternalBitDepth 10): the predicted
    uint16 planes from _ref's TComInterpolationFilter / TComYuv::addAvg at bitDepth 10 (the C
    restatement's orc_mc is 8-bit: these fixtures pin the HIP path on the reference alone)."""
    rng = np.random.default_rng(seed)
    pics = mc10_pictures(width, height, 3, seed)
    jobs = synth.make_mc_partition(rng, width, height, [0, 1, 2], bi_frac=bi_frac, mv_amp=mv_amp,
                                   identical_frac=identical_frac)
    ref = Reference(bit_depth=10)
    for k, (y, cb, cr) in pics.items():
        ref.set_picture_yuv(k, y, cb, cr)
    y = np.full((height, width), fill, np.uint16)
    cb = np.full((height // 2, width // 2), fill, np.uint16)
    cr = cb.copy()
    ref.mc(jobs, y, cb, cr)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(
        path,
        ref_y=np.stack([pics[k][0] for k in range(3)]),
        ref_cb=np.stack([pics[k][1] for k in range(3)]),
        ref_cr=np.stack([pics[k][2] for k in range(3)]),
        jobs=jobs,
        fill=np.array([fill], np.uint16),
        bit_depth=np.array([10], np.int32),
        pred_y=y, pred_cb=cb, pred_cr=cr,
    )
    print(f"{path}: {len(jobs)} PUs, {int(((jobs['flags'] & 3) == 3).sum())} bi-pred, "
          f"luma {int(y.min())}..{int(y.max())}")


def wp_table(rng, refs):
    """Explicit WP parameters [list][ref][Y, Cb, Cr][iWeight, iOffset, uiLog2WeightDenom] as a slice
    header carries them: one luma and one chroma denominator per slice (0..7), weights
    2^denom + delta (delta -24..24, some exactly 2^denom to reach addWeightUni's unit-weight branch),
    offsets -128..127 (8-bit units) with some zero."""
    t = np.zeros((2, refs, 3, 3), np.int32)
    dl, dc = int(rng.integers(0, 8)), int(rng.integers(0, 8))
    for l in range(2):
        for r in range(refs):
            for c in range(3):
                d = dl if c == 0 else dc
                delta = 0 if rng.random() < 0.25 else int(rng.integers(-24, 25))
                off = 0 if rng.random() < 0.3 else int(rng.integers(-128, 128))
                t[l, r, c] = ((1 << d) + delta, off, d)
    return t


def build_mcwp_case(name, seed, width, height, bi_frac, mv_amp, identical_frac, wp_frac, bit_depth=8):
    """Motion compensation with explicit weighted prediction (FME_MC_WP; PPS UseWP / WPBiPred,
    TComPrediction.cpp:509-512, 612-619): the planes from _ref, which filters each list to the 14-bit
    values and runs the reference's own TComWeightPrediction::addWeightUni / addWeightBi
    (TComWeightPrediction.cpp:78-245) with getWpScaling's derivation; a share of the jobs without
    the flag (plain averaging) and identical bi motion kept as two lists under WP.  The C oracle's
    orc_mc_wp agrees at 8 bits (tests/test_mc_wp.py); the 10-bit fixture rests on the reference."""
    from nnfme.abi import MC_WP
    rng = np.random.default_rng(seed)
    if bit_depth > 8:
        pics = mc10_pictures(width, height, 3, seed)
    else:
        pics = {}
        for k in range(3):
            cb, cr = synth.synth_chroma(width, height, k, seed=seed)
            pics[k] = (synth.synth_luma(width, height, k, seed=seed), cb, cr)
    jobs = synth.make_mc_partition(rng, width, height, [0, 1, 2], bi_frac=bi_frac, mv_amp=mv_amp,
                                   identical_frac=identical_frac)
    wpm = rng.random(len(jobs)) < wp_frac
    jobs["flags"] = np.where(wpm, jobs["flags"] | MC_WP, jobs["flags"])
    wp = wp_table(rng, 3)
    ref = Reference(bit_depth=bit_depth)
    for k, (y, cb, cr) in pics.items():
        ref.set_picture_yuv(k, y, cb, cr)
    for l in range(2):
        for r in range(3):
            ref.set_wp(l, r, wp[l, r])
    dt = np.uint16 if bit_depth > 8 else np.uint8
    y = np.zeros((height, width), dt)
    cb = np.zeros((height // 2, width // 2), dt)
    cr = cb.copy()
    ref.mc(jobs, y, cb, cr)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(
        path,
        ref_y=np.stack([pics[k][0] for k in range(3)]),
        ref_cb=np.stack([pics[k][1] for k in range(3)]),
        ref_cr=np.stack([pics[k][2] for k in range(3)]),
        jobs=jobs, wp=wp, bit_depth=np.array([bit_depth], np.int32),
        pred_y=y, pred_cb=cb, pred_cr=cr,
    )
    bi = (jobs["flags"] & 3) == 3
    same = bi & (jobs["ref_id"][:, 0] == jobs["ref_id"][:, 1]) & (jobs["mv"][:, 0, 0] == jobs["mv"][:, 1, 0]) & \
        (jobs["mv"][:, 0, 1] == jobs["mv"][:, 1, 1])
    print(f"{path}: {len(jobs)} PUs, {int(wpm.sum())} weighted, {int((bi & wpm).sum())} weighted bi-pred, "
          f"{int((same & wpm).sum())} weighted identical-motion, denominators {int(wp[0, 0, 0, 2])}/{int(wp[0, 0, 1, 2])}")


MCWP_CASES = [
    # name, seed, W, H, bi fraction, MV amplitude, identical-motion fraction, WP fraction, bit depth
    ("mcwp_p_uni", 61, 160, 104, 0.0, 40, 0.0, 0.9, 8),
    ("mcwp_b_bi", 62, 168, 96, 0.6, 120, 0.2, 0.8, 8),
    ("mcwp10_b_bi", 63, 128, 80, 0.6, 60, 0.2, 0.8, 10),
]


def build_mc_case(name, seed, width, height, bi_frac, mv_amp, identical_frac, keep_frac=1.0, fill=0):
    """Motion compensation (TComPrediction::motionCompensation): reference pictures with 4:2:0
    chroma, one frame partition of decided PUs, the predicted planes from _ref (the oracle must
    agree).  keep_frac < 1 drops PUs: their samples must keep the initial `fill`."""
    from nnfme.abi import MC_JOB_DTYPE  # noqa: F401
    rng = np.random.default_rng(seed)
    pics = {}
    for k in range(3):
        cb, cr = synth.synth_chroma(width, height, k, seed=seed)
        pics[k] = (synth.synth_luma(width, height, k, seed=seed), cb, cr)
    if name == "mc_shapes":   # every HEVC inter PU shape once, each in its own 64x64 cell
        shapes = synth.ALL_PU_SIZES
        jobs = synth.make_mc_partition(rng, 64 * 6, 64 * 4, [0, 1, 2], bi_frac=bi_frac, mv_amp=mv_amp)[:len(shapes)]
        for i, (w, h) in enumerate(shapes):
            jobs[i]["x"], jobs[i]["y"] = 64 * (i % 6) + (64 - w), 64 * (i // 6)
            jobs[i]["cu_x"], jobs[i]["cu_y"] = 64 * (i % 6), 64 * (i // 6)
            jobs[i]["w"], jobs[i]["h"] = w, h
    else:
        jobs = synth.make_mc_partition(rng, width, height, [0, 1, 2], bi_frac=bi_frac, mv_amp=mv_amp,
                                       identical_frac=identical_frac)
    if keep_frac < 1.0:
        jobs = jobs[rng.random(len(jobs)) < keep_frac]
    ref, orc = Reference(), Oracle()
    for k, (y, cb, cr) in pics.items():
        ref.set_picture_yuv(k, y, cb, cr)
    outs = []
    for eng in (ref, orc):
        y = np.full((height, width), fill, np.uint8)
        cb = np.full((height // 2, width // 2), fill, np.uint8)
        cr = cb.copy()
        if eng is ref:
            eng.mc(jobs, y, cb, cr)
        else:
            eng.mc(pics, jobs, y, cb, cr)
        outs.append((y, cb, cr))
    for a, b, comp in zip(outs[0], outs[1], "Y Cb Cr".split()):
        if not np.array_equal(a, b):
            raise SystemExit(f"{name}: oracle disagrees with _ref on {comp} ({int((a != b).sum())} samples)")
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(
        path,
        ref_y=np.stack([pics[k][0] for k in range(3)]),
        ref_cb=np.stack([pics[k][1] for k in range(3)]),
        ref_cr=np.stack([pics[k][2] for k in range(3)]),
        jobs=jobs,
        fill=np.array([fill], np.uint8),
        pred_y=outs[0][0], pred_cb=outs[0][1], pred_cr=outs[0][2],
    )
    nbi = int(((jobs["flags"] & 3) == 3).sum())
    print(f"{path}: {len(jobs)} PUs, {nbi} bi-pred, {len(set(zip(jobs['w'], jobs['h'])))} PU shapes")


def tz_pictures(width, height, seed, bit_depth):
    """The integer-search fixtures' five pictures: 8-bit, or the same field at bit depth 10 (main10)."""
    if bit_depth > 8:
        return {i: synth.synth_luma_hbd(width, height, i, bit_depth=bit_depth, seed=seed) for i in range(5)}
    return {i: synth.synth_luma(width, height, i, seed=seed) for i in range(5)}


def build_tz_case(name, seed, width, height, calls, fen, search_range, bipred, mvp_noise, bit_depth=8):
    """Integer motion estimation (xTZSearch / xPatternSearch) from _ref; the oracle must agree.
    bit_depth 10: 16-bit pictures, the distortions of TComRdCost at bitDepth 10 (SSE (d * d) >> 4 per
    sample, SAD >> 2 per block)."""
    rng = np.random.default_rng(seed)
    pics = tz_pictures(width, height, seed, bit_depth)
    lambdas = np.array(synth.LDP_LAMBDA[22], dtype=np.float64)
    jobs, ext = synth.make_tz_jobs(rng, width, height, calls, 4, [0, 1, 2, 3], [0, 1, 2, 3], bipred_frac=bipred,
                                   search_range=search_range, mvp_noise=mvp_noise)
    keys = synth.make_bipred_keys(rng, jobs, pics)
    ref = Reference(fast_inter_mode=fen, bit_depth=bit_depth)
    orc = Oracle(fast_inter_mode=fen, bit_depth=bit_depth)
    for eng in (ref, orc):
        for k, v in pics.items():
            eng.set_picture(k, v)
        for lid, lam in enumerate(lambdas):
            eng.set_lambda(lid, float(lam))
        eng.set_keys(keys if keys.size else np.zeros(1, np.int16))
    out_r, sad_r = ref.integer_search(jobs, ext)
    out_o, sad_o = orc.integer_search(jobs, ext)
    bad = (out_r["mv_x"] != out_o["mv_x"]) | (out_r["mv_y"] != out_o["mv_y"]) | (sad_r != sad_o)
    if bad.any():
        raise SystemExit(f"{name}: oracle disagrees with _ref on {int(bad.sum())} jobs")
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, pictures=np.stack([pics[i] for i in range(5)]), lambdas=lambdas, keys=keys,
                        jobs=jobs, ext=ext, mv_x=out_r["mv_x"], mv_y=out_r["mv_y"], sad=sad_r,
                        config=np.array([fen, search_range], dtype=np.int32),
                        **({"bit_depth": np.array([bit_depth], np.int32)} if bit_depth != 8 else {}))
    far = np.abs(out_r["mv_x"] * 4 - jobs["mvp_x"]) + np.abs(out_r["mv_y"] * 4 - jobs["mvp_y"])
    print(f"{path}: {len(jobs)} jobs, {int((jobs['flags'] & JOB_BIPRED != 0).sum())} bi-pred, "
          f"{int((ext['flags'] != 0).sum())} with a 2Nx2N start, {int((far > 4 * 20).sum())} ending > 20 px from the predictor")


def build_tz2_case(name, seed, width, height, calls, fen, search_range, bipred, mvp_noise, mode, bit_depth=8):
    """The other FastSearch settings (fme_tz_ext2): FastSearch 0 (FME_TZ_FULL, xPatternSearch for every
    job) or 3 (FME_TZ_ENHANCED, xTZSearch with bExtendedSettings and the neighbour predictors
    m_acMvPredictors) from _ref; the oracle must agree.  The predictors: near the AMVP predictor, some
    equal to it, some zero, some far (the start-point tests' "not obviously previously tested"
    conditions both ways)."""
    from nnfme.abi import TZ_EXT2_DTYPE
    rng = np.random.default_rng(seed)
    pics = tz_pictures(width, height, seed, bit_depth)
    lambdas = np.array(synth.LDP_LAMBDA[22], dtype=np.float64)
    jobs, ext = synth.make_tz_jobs(rng, width, height, calls, 4, [0, 1, 2, 3], [0, 1, 2, 3], bipred_frac=bipred,
                                   search_range=search_range, mvp_noise=mvp_noise)
    keys = synth.make_bipred_keys(rng, jobs, pics)
    n = len(jobs)
    ext2 = np.zeros(n, dtype=TZ_EXT2_DTYPE)
    ext2["base"] = ext
    uni = (jobs["flags"] & JOB_BIPRED) == 0
    ext2["base"]["flags"] = np.where(uni, ext["flags"] | mode, ext["flags"])
    kind = rng.integers(0, 4, (n, 3))
    for c, comp in ((0, "mvp_x"), (1, "mvp_y")):
        base = jobs[comp].astype(np.int64)[:, None]
        near = base + rng.integers(-12, 13, (n, 3))
        far = rng.integers(-4 * 3 * search_range, 4 * 3 * search_range + 1, (n, 3))
        v = np.where(kind == 0, base, np.where(kind == 1, 0, np.where(kind == 2, near, far)))
        ext2["preds"][:, :, c] = np.clip(v, -32768, 32767)
    ref = Reference(fast_inter_mode=fen, bit_depth=bit_depth)
    orc = Oracle(fast_inter_mode=fen, bit_depth=bit_depth)
    for eng in (ref, orc):
        for k, v in pics.items():
            eng.set_picture(k, v)
        for lid, lam in enumerate(lambdas):
            eng.set_lambda(lid, float(lam))
        eng.set_keys(keys if keys.size else np.zeros(1, np.int16))
    out_r, sad_r = ref.integer_search2(jobs, ext2)
    out_o, sad_o = orc.integer_search2(jobs, ext2)
    bad = (out_r["mv_x"] != out_o["mv_x"]) | (out_r["mv_y"] != out_o["mv_y"]) | (sad_r != sad_o)
    if bad.any():
        raise SystemExit(f"{name}: oracle disagrees with _ref on {int(bad.sum())} jobs")
    # against the shipped FastSearch 1 on the same jobs: the setting changes results
    base_r, _ = ref.integer_search(jobs, ext)
    differ = int(((base_r["mv_x"] != out_r["mv_x"]) | (base_r["mv_y"] != out_r["mv_y"])).sum())
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, pictures=np.stack([pics[i] for i in range(5)]), lambdas=lambdas, keys=keys,
                        jobs=jobs, ext=ext2, mv_x=out_r["mv_x"], mv_y=out_r["mv_y"], sad=sad_r,
                        config=np.array([fen, search_range], dtype=np.int32),
                        **({"bit_depth": np.array([bit_depth], np.int32)} if bit_depth != 8 else {}))
    print(f"{path}: {n} jobs, {int((~uni).sum())} bi-pred, mode 0x{mode:x}, {differ} MVs differ from FastSearch 1")


def build_ring_case(name, seed, width, height, calls, fen, search_range, bipred, mvp_noise, net, qp=22):
    """The backups' own NN input path (configs[4]): xTZSearch with the final square + ring, every
    distortion pushed (FME_TZ_RING: mv, sad and the nine NN inputs per job), then the sub-pel path
    with the deeper net on those inputs (FME_JOB_NN_IN; bi-pred jobs reuse the last uni-pred call's
    inputs).  Both stages from _ref; the oracle must agree on every output."""
    rng = np.random.default_rng(seed)
    pics = {i: synth.synth_luma(width, height, i, seed=seed) for i in range(5)}
    lambdas = np.array(synth.LDP_LAMBDA[qp], dtype=np.float64)
    jobs, ext = synth.make_tz_jobs(rng, width, height, calls, 4, [0, 1, 2, 3], [0, 1, 2, 3], bipred_frac=bipred,
                                   search_range=search_range, mvp_noise=mvp_noise)
    ext["flags"] |= TZ_RING
    keys = synth.make_bipred_keys(rng, jobs, pics)
    ref = Reference(use_hadamard=1, nn_mode=2, fast_inter_mode=fen)
    orc = Oracle(use_hadamard=1, nn_mode=2, qp=qp, fast_inter_mode=fen)
    nnet = weights.case_net(net)
    for eng in (ref, orc):
        for k, v in pics.items():
            eng.set_picture(k, v)
        for lid, lam in enumerate(lambdas):
            eng.set_lambda(lid, float(lam))
        eng.set_keys(keys if keys.size else np.zeros(1, np.int16))
        eng.load_nn_net(nnet)
    out_r, sad_r, nn_r = ref.integer_search_ring(jobs, ext)
    out_o, sad_o, nn_o = orc.integer_search_ring(jobs, ext)
    bad = (out_r["mv_x"] != out_o["mv_x"]) | (out_r["mv_y"] != out_o["mv_y"]) | (sad_r != sad_o) | \
        (nn_r != nn_o).any(axis=1)
    if bad.any():
        raise SystemExit(f"{name}: oracle disagrees with _ref's integer search on {int(bad.sum())} jobs")
    uni = (jobs["flags"] & JOB_BIPRED) == 0
    rjobs = out_r.copy()
    rjobs["flags"] = np.where(uni, JOB_NN_IN, rjobs["flags"]).astype(np.uint8)
    for eng in (ref, orc):
        eng.set_nn_inputs(nn_r)
    r_ref = ref.refine(rjobs)
    r_orc = orc.refine(rjobs)
    bad, first, counts = compare_results(r_ref, r_orc)
    if bad:
        raise SystemExit(f"{name}: oracle disagrees with _ref on {bad} refinements (first {first}): {counts}")
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, pictures=np.stack([pics[i] for i in range(5)]), lambdas=lambdas, keys=keys,
                        jobs=jobs, ext=ext, mv_x=out_r["mv_x"], mv_y=out_r["mv_y"], sad=sad_r, nn_in=nn_r,
                        refine_jobs=rjobs, results=r_ref, net=np.array(net),
                        config=np.array([1, fen, 2, qp, search_range], dtype=np.int32))
    moved = ((out_r["mv_x"] != orc.integer_search(jobs, ext)[0]["mv_x"]) & uni).sum()
    print(f"{path}: {len(jobs)} jobs, {int((~uni).sum())} bi-pred, {int(moved)} moved by the square + ring, "
          f"{int((nn_r[uni, :8] == 0).any(axis=1).sum())} with < 8 pushes, classes {len(set(r_ref['nn_class']))}")


RING_CASES = [
    # name, seed, W, H, calls/CTU/ref, FEN, SearchRange, bi-pred share, predictor noise, net
    ("ring_scr3x40_fen1", 41, 160, 96, 40, 1, 64, 0.15, 24, "scr3x40+tzring"),
    ("ring_b4x40_sr8_fen3", 42, 128, 96, 40, 3, 8, 0.1, 60, "blowing4x40+rezero+tzring"),
    # SearchRange 2: the square and the ring mostly clipped by the range (fewer than 8 pushes)
    ("ring_scr3x40_sr2_fen0", 43, 128, 96, 30, 0, 2, 0.1, 24, "scr3x40+tzring"),
]

TZ_CASES = [
    # name, seed, W, H, calls/CTU/ref, FEN, SearchRange, bi-pred share, predictor noise (qpel)
    ("tz_ldp_fen1", 31, 160, 96, 40, 1, 64, 0.15, 24),
    ("tz_far_fen0_sr32", 32, 160, 96, 40, 0, 32, 0.1, 200),
]

TZ2_CASES = [
    # name, seed, W, H, calls/CTU/ref, FEN, SearchRange, bi-pred share, predictor noise (qpel), mode
    ("tz_full_sr8_fen1", 33, 128, 96, 10, 1, 8, 0.1, 24, 0x04),
    ("tz_enhanced_fen1", 34, 160, 96, 30, 1, 64, 0.1, 24, 0x08),
    ("tz_enhanced_far_fen0_sr32", 35, 160, 96, 30, 0, 32, 0.1, 200, 0x08),
]

TZ10_CASES = [
    # bit depth 10 (the main10 configurations): FastSearch 1 / 0 / 3 with SSE and the SAD widths
    # (FEN 0 and the FEN 1 / 3 row subsampling); (TZ_CASES fields, mode or None, bit depth)
    ("tz10_ldp_fen1", 51, 160, 96, 40, 1, 64, 0.15, 24, None, 10),
    ("tz10_far_fen0_sr32", 52, 160, 96, 40, 0, 32, 0.1, 200, None, 10),
    ("tz10_full_sr8_fen3", 53, 128, 96, 10, 3, 8, 0.1, 24, 0x04, 10),
    ("tz10_enhanced_fen1", 54, 160, 96, 30, 1, 64, 0.1, 24, 0x08, 10),
]


def build_tz10_case(name, seed, width, height, calls, fen, search_range, bipred, mvp_noise, mode, bit_depth):
    if mode is None:
        build_tz_case(name, seed, width, height, calls, fen, search_range, bipred, mvp_noise, bit_depth=bit_depth)
    else:
        build_tz2_case(name, seed, width, height, calls, fen, search_range, bipred, mvp_noise, mode,
                       bit_depth=bit_depth)


MC10_CASES = [
    # name, seed, W, H, bi fraction, MV amplitude (quarter-pel), identical-motion fraction, fill
    ("mc10_ldp_uni", 41, 160, 104, 0.0, 40, 0.0, 0),
    ("mc10_ra_bi_clip", 42, 168, 96, 0.5, 200, 0.2, 0),
    ("mc10_bi_near", 43, 128, 80, 0.8, 12, 0.1, 513),
]

MC_CASES = [
    # name, seed, W, H, bi_frac, mv_amp (pel), identical_frac, keep_frac, fill
    ("mc_ldp_uni", 21, 160, 104, 0.0, 40, 0.0, 1.0, 0),
    ("mc_ra_bi_clip", 22, 168, 96, 0.5, 200, 0.2, 1.0, 0),
    ("mc_sparse", 23, 128, 80, 0.3, 16, 0.1, 0.5, 77),
    ("mc_shapes", 24, 384, 256, 0.5, 24, 0.0, 1.0, 9),
]

CASES = [
    # name, seed, W, H, jobs, HADME, FEN, nn_mode, QP
    ("ldp_qp22_hadme_fen1_nn", 11, 160, 96, 1200, 1, 1, 1, 22),
    ("sad_fen0_nnoff", 12, 160, 96, 600, 0, 0, 0, 22),
    ("fen3_qp27_nn", 13, 128, 96, 400, 1, 3, 1, 27),
    ("qp32_nn", 14, 128, 96, 400, 1, 1, 1, 32),
    ("qp37_nn", 15, 128, 96, 400, 1, 1, 1, 37),
    # configs[1] exactly: HADME on, FEN 1, NN_pred off (the standard FracDIF MV)
    ("hadme_fen1_nnoff_qp22", 18, 160, 96, 800, 1, 1, 0, 22),
    # configs[3]'s random-access lambdas (GOP-8 depths 0..3) with its bi-pred share
    ("ra_qp27_nn", 19, 160, 96, 800, 1, 1, 1, 27, 0.205, 96, None, "ra"),
]


# main10 (InternalBitDepth 10, cfg/encoder_lowdelay_P_main10.cfg:58 and the RA / LD main10 cfgs):
# the sub-pel path with 16-bit pictures; every PU shape, edges, lossless jobs, bi-pred keys
MAIN10_CASES = [
    # name, seed, W, H, jobs, HADME, FEN, nn_mode, QP, bi-pred, edge jobs, net, gop, bit depth
    ("main10_ldp_qp22_hadme_fen1_nn", 51, 160, 96, 1200, 1, 1, 1, 22, 0.15, 96, None, "ldp", 10),
    ("main10_sad_fen0_nnoff", 52, 160, 96, 600, 0, 0, 0, 22, 0.15, 96, None, "ldp", 10),
    ("main10_fen3_qp27_nn", 53, 128, 96, 500, 1, 3, 1, 27, 0.15, 96, None, "ldp", 10),
    ("main10_ra_qp37_nn", 54, 128, 96, 500, 1, 1, 1, 37, 0.205, 96, None, "ra", 10),
]


# nn_mode 2: the reference's deeper nets (BASELINE.json configs[4]) and the master net through the
# generic path.  nn4x40 runs with its X3/X4 carry cleared ("+rezero"): the batch engines do not run
# carried hidden layers (fme_load_nn_net rejects carry_hidden); the oracle and _ref cover both.
DEEP_CASES = [
    ("deep_scr3x40_qp22", 16, 160, 96, 900, 1, 1, 2, 22, 0.15, 96, "scr3x40"),
    ("deep_blowing4x40_qp22", 17, 128, 96, 600, 1, 1, 2, 22, 0.15, 96, "blowing4x40+rezero"),
    ("deep_master_qp22", 11, 160, 96, 1200, 1, 1, 2, 22, 0.15, 96, "master"),
]


def main():
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    if only:
        for c in CASES + DEEP_CASES:
            if c[0] in only:
                build_case(*c)
        return 0
    if "--deep-only" in sys.argv:
        for c in DEEP_CASES:
            build_case(*c)
        return 0
    if "--main10-only" in sys.argv:
        for c in MAIN10_CASES:
            build_case(*c)
        return 0
    if "--tz2-only" in sys.argv:
        for c in TZ2_CASES:
            build_tz2_case(*c)
        return 0
    if "--tz10-only" in sys.argv:
        for c in TZ10_CASES:
            build_tz10_case(*c)
        return 0
    if "--mcwp-only" in sys.argv:
        for c in MCWP_CASES:
            build_mcwp_case(*c)
        return 0
    if "--mc10-only" in sys.argv:
        for c in MC10_CASES:
            build_mc10_case(*c)
        return 0
    if "--ring-only" in sys.argv:
        for c in RING_CASES:
            build_ring_case(*c)
        return 0
    for c in RING_CASES:
        build_ring_case(*c)
    for c in DEEP_CASES:
        build_case(*c)
    if "--mc-only" not in sys.argv and "--tz-only" not in sys.argv:
        for c in CASES + MAIN10_CASES:
            build_case(*c)
    if "--tz-only" not in sys.argv:
        for c in MC_CASES:
            build_mc_case(*c)
        for c in MC10_CASES:
            build_mc10_case(*c)
        for c in MCWP_CASES:
            build_mcwp_case(*c)
    for c in TZ_CASES:
        build_tz_case(*c)
    for c in TZ2_CASES:
        build_tz2_case(*c)
    for c in TZ10_CASES:
        build_tz10_case(*c)
    return 0


if __name__ == "__main__":
    sys.exit(main())
