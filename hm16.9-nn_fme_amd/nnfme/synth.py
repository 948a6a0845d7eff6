"""Synthetic inputs for the fractional-ME path (SURVEY.md §8(d) "Synthetic inputs").

* YUV: 8-bit luma = 128 + sum_{i<12} a_i sin(fx_i (x + 0.37 t) + fy_i (y + 0.21 t) + phi_i)
  + N(0, 2), rounded and clipped; a ~ U[10,40], fx, fy ~ U[0.01, 0.2], phi ~ U[0, 2pi];
  numpy.default_rng(seed) with seed 1 (416x240), 2 (1920x1080), 3 (2560x1600).
* Jobs: the PU-size mix measured on the 1080p P-frame, integer MVs
  U[-64,64]^2 clipped into the search range, AMVP predictors U[-256,256]^2 quarter-pel,
  search range = xSetSearchRange(mvp, 64) with TComDataCU::clipMv (TEncSearch.cpp:4602-4624,
  TComDataCU.cpp:2773-2786), lambda per frame from the LDP GOP table below.
"""
import numpy as np

from .abi import JOB_BIPRED, JOB_DTYPE, JOB_EMI

SEEDS = {(416, 240): 1, (1920, 1080): 2, (2560, 1600): 3}

# PU size (W, H) -> share of FracDIF calls on the 1080p LDP QP22 P-frame.
PU_MIX = [
    ((8, 4), 0.300), ((4, 8), 0.300), ((8, 8), 0.150), ((8, 16), 0.075), ((16, 8), 0.075),
    ((16, 16), 0.037), ((32, 16), 0.018), ((16, 32), 0.018), ((32, 32), 0.009),
    ((64, 32), 0.0045), ((32, 64), 0.0045), ((64, 64), 0.0022),
    # AMP shapes, ~0.6 % together
    ((4, 16), 0.00075), ((12, 16), 0.00075), ((16, 4), 0.00075), ((16, 12), 0.00075),
    ((8, 32), 0.00075), ((24, 32), 0.00075), ((32, 8), 0.00075), ((32, 24), 0.00075),
]
ALL_PU_SIZES = [s for s, _ in PU_MIX] + [(64, 16), (64, 48), (16, 64), (48, 64)]

# lambda per POC % 4 for lowdelay_P (cfg Frame1-4).
LDP_LAMBDA = {
    22: (7.340, 20.196, 14.797, 20.196),
    27: (23.30, 88.78, 66.55, 88.78),
    32: (73.98, 360.16, 273.43, 360.16),
    37: (234.9, 1193.1, 947.0, 1193.1),
}

SEARCH_RANGE = 64      # cfg SearchRange
MAX_CU = 64


def synth_luma(width, height, t, seed=None):
    """One synthetic 8-bit luma frame (uint8[height, width]) at time index t."""
    if seed is None:
        seed = SEEDS.get((width, height), 7)
    rng = np.random.default_rng(seed)
    a = rng.uniform(10, 40, 12)
    fx = rng.uniform(0.01, 0.2, 12)
    fy = rng.uniform(0.01, 0.2, 12)
    phi = rng.uniform(0, 2 * np.pi, 12)
    noise = np.random.default_rng(seed * 1000 + t + 1).normal(0, 2, (height, width))
    x = np.arange(width, dtype=np.float64)[None, :]
    y = np.arange(height, dtype=np.float64)[:, None]
    acc = np.full((height, width), 128.0)
    for i in range(12):
        acc += a[i] * np.sin(fx[i] * (x + 0.37 * t) + fy[i] * (y + 0.21 * t) + phi[i])
    acc += noise
    return np.clip(np.rint(acc), 0, 255).astype(np.uint8)


def synth_luma_hbd(width, height, t, bit_depth=10, seed=None):
    """The same synthetic frame at a higher bit depth (uint16[height, width], main10): the 8-bit
    frame's field at (bit_depth - 8) more bits of precision plus its own noise, clipped to the range."""
    if seed is None:
        seed = SEEDS.get((width, height), 7)
    rng = np.random.default_rng(seed)
    a = rng.uniform(10, 40, 12)
    fx = rng.uniform(0.01, 0.2, 12)
    fy = rng.uniform(0.01, 0.2, 12)
    phi = rng.uniform(0, 2 * np.pi, 12)
    noise = np.random.default_rng(seed * 1000 + t + 1).normal(0, 2, (height, width))
    x = np.arange(width, dtype=np.float64)[None, :]
    y = np.arange(height, dtype=np.float64)[:, None]
    acc = np.full((height, width), 128.0)
    for i in range(12):
        acc += a[i] * np.sin(fx[i] * (x + 0.37 * t) + fy[i] * (y + 0.21 * t) + phi[i])
    acc += noise
    scale = float(1 << (bit_depth - 8))
    return np.clip(np.rint(acc * scale), 0, (1 << bit_depth) - 1).astype(np.uint16)


def _clip_mv_qpel(v, pos, pic, size_max=MAX_CU):
    """TComDataCU::clipMv on quarter-pel values, with the PU position standing in for the
    CU position (TComDataCU.cpp:2778-2785)."""
    vmax = (pic + 8 - pos - 1) << 2
    vmin = (-size_max - 8 - pos + 1) << 2
    return np.minimum(vmax, np.maximum(vmin, v))


def _div4_round(v):
    """TComMv::divideByPowerOf2(2) with ME_ENABLE_ROUNDING_OF_MVS (TComMv.h:122-130)."""
    return (v + 2) >> 2


def sample_sizes(rng, n, mix=PU_MIX):
    sizes = np.array([s for s, _ in mix], dtype=np.int32)
    p = np.array([q for _, q in mix], dtype=np.float64)
    p /= p.sum()
    idx = rng.choice(len(mix), size=n, p=p)
    return sizes[idx, 0], sizes[idx, 1]


def make_jobs(rng, width, height, n, org_id, ref_ids, lambda_ids, sizes=None, bipred_frac=0.0,
              bits_in_max=6):
    """n synthetic jobs for one frame.

    ref_ids / lambda_ids: per-job choice lists (a ref picture slot and the lambda slot of the
    frame).  bipred_frac: share of bi-pred jobs (no EMI, key block from make_bipred_keys).
    Returns a JOB_DTYPE array; bi-pred rows have key_offset = -2 (to be assigned).
    """
    jobs = np.zeros(n, dtype=JOB_DTYPE)
    if sizes is None:
        w, h = sample_sizes(rng, n)
    else:
        w, h = sizes
        w = np.broadcast_to(np.asarray(w, dtype=np.int32), (n,)).copy()
        h = np.broadcast_to(np.asarray(h, dtype=np.int32), (n,)).copy()
    x = (rng.integers(0, (width - w) // 4 + 1)) * 4
    y = (rng.integers(0, (height - h) // 4 + 1)) * 4
    mvp_x = rng.integers(-256, 257, n)
    mvp_y = rng.integers(-256, 257, n)
    # xSetSearchRange(mvp, SearchRange): clip(pred) -/+ SR<<2, clip, round >> 2.
    cpx = _clip_mv_qpel(mvp_x, x, width)
    cpy = _clip_mv_qpel(mvp_y, y, height)
    lt_x = _div4_round(_clip_mv_qpel(cpx - (SEARCH_RANGE << 2), x, width))
    rb_x = _div4_round(_clip_mv_qpel(cpx + (SEARCH_RANGE << 2), x, width))
    lt_y = _div4_round(_clip_mv_qpel(cpy - (SEARCH_RANGE << 2), y, height))
    rb_y = _div4_round(_clip_mv_qpel(cpy + (SEARCH_RANGE << 2), y, height))
    mv_x = np.clip(rng.integers(-64, 65, n), lt_x, rb_x)
    mv_y = np.clip(rng.integers(-64, 65, n), lt_y, rb_y)
    jobs["x"], jobs["y"], jobs["w"], jobs["h"] = x, y, w, h
    jobs["org_id"] = org_id
    jobs["ref_id"] = rng.choice(np.asarray(ref_ids), size=n)
    jobs["lambda_id"] = rng.choice(np.asarray(lambda_ids), size=n)
    jobs["mv_x"], jobs["mv_y"] = mv_x, mv_y
    jobs["mvp_x"], jobs["mvp_y"] = mvp_x, mvp_y
    jobs["lt_x"], jobs["lt_y"], jobs["rb_x"], jobs["rb_y"] = lt_x, lt_y, rb_x, rb_y
    jobs["bits_in"] = rng.integers(1, bits_in_max + 1, n)
    jobs["flags"] = JOB_EMI
    jobs["key_offset"] = -1
    if bipred_frac > 0:
        bi = rng.random(n) < bipred_frac
        jobs["flags"][bi] = JOB_BIPRED
        jobs["key_offset"][bi] = -2
    return jobs


def cu_size_for(w, h):
    """Smallest square CU (8..64) that holds a PU of w x h (HEVC partition shapes)."""
    s = max(w, h)
    return 8 if s <= 8 else (16 if s <= 16 else (32 if s <= 32 else 64))


def motion_field(rng, ctus_x, ctus_y, amp=12.0):
    """Smooth per-CTU motion (full-pel per frame of distance): two low-frequency waves."""
    fx = rng.uniform(0.1, 0.5, 2)
    fy = rng.uniform(0.1, 0.5, 2)
    ph = rng.uniform(0, 2 * np.pi, 4)
    cx = np.arange(ctus_x)[None, :]
    cy = np.arange(ctus_y)[:, None]
    vx = amp * np.sin(fx[0] * cx + fy[0] * cy + ph[0]) + 0.5 * amp * np.sin(fx[1] * cx - fy[1] * cy + ph[1])
    vy = 0.6 * amp * np.sin(fx[0] * cy - fy[0] * cx + ph[2]) + 0.3 * amp * np.sin(fx[1] * cy + ph[3])
    return vx, vy


def make_ctu_jobs(rng, width, height, calls_per_ctu, org_id, ref_ids, lambda_ids, mix=PU_MIX,
                  bipred_frac=0.0, bits_in_max=6):
    """Jobs in HM's order: CTUs in raster order, every PU of a CTU inside it on the CU /
    partition grid (TEncCu quadtree, TComDataCU::getPartIndexAndSize), for every reference
    picture.  Integer MVs follow a smooth per-CTU motion field scaled by the reference distance
    plus a local deviation, the AMVP predictor is near the true motion; the search range and
    the TZ start obey the same clipping rules as make_jobs().  Realistic cache locality: the
    windows of one CTU's jobs overlap, as in the encoder."""
    ctus_x, ctus_y = (width + MAX_CU - 1) // MAX_CU, (height + MAX_CU - 1) // MAX_CU
    vx, vy = motion_field(rng, ctus_x, ctus_y)
    ref_ids = np.asarray(ref_ids)
    nref = len(ref_ids)
    per = calls_per_ctu * nref
    n = ctus_x * ctus_y * per
    w, h = sample_sizes(rng, n, mix)
    ctu = np.repeat(np.arange(ctus_x * ctus_y), per)
    cux = (ctu % ctus_x) * MAX_CU
    cuy = (ctu // ctus_x) * MAX_CU
    cs = np.where(np.maximum(w, h) <= 8, 8, np.where(np.maximum(w, h) <= 16, 16, np.where(np.maximum(w, h) <= 32, 32, 64)))
    # CU position inside the CTU (aligned to its size), PU at either end of the CU
    ncu = MAX_CU // cs
    x = cux + rng.integers(0, ncu) * cs + rng.integers(0, 2, n) * (cs - w)
    y = cuy + rng.integers(0, ncu) * cs + rng.integers(0, 2, n) * (cs - h)
    x = np.minimum(x, (width - w) // 4 * 4)
    y = np.minimum(y, (height - h) // 4 * 4)
    ref_k = np.tile(np.arange(nref), n // nref)          # every PU against each reference
    dist = ref_k + 1
    tx = np.rint(vx.reshape(-1)[ctu] * dist).astype(np.int64) + rng.integers(-4, 5, n)
    ty = np.rint(vy.reshape(-1)[ctu] * dist).astype(np.int64) + rng.integers(-4, 5, n)
    mvp_x = 4 * tx + rng.integers(-16, 17, n)
    mvp_y = 4 * ty + rng.integers(-16, 17, n)
    cpx = _clip_mv_qpel(mvp_x, x, width)
    cpy = _clip_mv_qpel(mvp_y, y, height)
    lt_x = _div4_round(_clip_mv_qpel(cpx - (SEARCH_RANGE << 2), x, width))
    rb_x = _div4_round(_clip_mv_qpel(cpx + (SEARCH_RANGE << 2), x, width))
    lt_y = _div4_round(_clip_mv_qpel(cpy - (SEARCH_RANGE << 2), y, height))
    rb_y = _div4_round(_clip_mv_qpel(cpy + (SEARCH_RANGE << 2), y, height))
    jobs = np.zeros(n, dtype=JOB_DTYPE)
    jobs["x"], jobs["y"], jobs["w"], jobs["h"] = x, y, w, h
    jobs["org_id"] = org_id
    jobs["ref_id"] = ref_ids[ref_k]
    jobs["lambda_id"] = rng.choice(np.asarray(lambda_ids), size=n)
    jobs["mv_x"] = np.clip(tx, lt_x, rb_x)
    jobs["mv_y"] = np.clip(ty, lt_y, rb_y)
    jobs["mvp_x"], jobs["mvp_y"] = mvp_x, mvp_y
    jobs["lt_x"], jobs["lt_y"], jobs["rb_x"], jobs["rb_y"] = lt_x, lt_y, rb_x, rb_y
    jobs["bits_in"] = rng.integers(1, bits_in_max + 1, n)
    jobs["flags"] = JOB_EMI
    jobs["key_offset"] = -1
    if bipred_frac > 0:
        bi = rng.random(n) < bipred_frac
        jobs["flags"][bi] = JOB_BIPRED
        jobs["key_offset"][bi] = -2
    return jobs


def make_bipred_keys(rng, jobs, pictures):
    """Key blocks 2*org - pred_other (TComYuv::removeHighFreq, TComYuv.cpp:411-455, no clip)
    for rows with key_offset == -2; pred_other is an integer-displaced block of another
    picture.  Assigns key_offset and returns the int16 key buffer."""
    sel = np.flatnonzero(jobs["key_offset"] == -2)
    sizes = jobs["w"][sel].astype(np.int64) * jobs["h"][sel].astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    keys = np.zeros(int(offs[-1]), dtype=np.int16)
    ids = sorted(pictures)
    for k, i in enumerate(sel):
        j = jobs[i]
        w, h, x, y = int(j["w"]), int(j["h"]), int(j["x"]), int(j["y"])
        org = pictures[int(j["org_id"])].astype(np.int16)
        oth = pictures[ids[int(rng.integers(0, len(ids)))]]
        dx, dy = int(rng.integers(-8, 9)), int(rng.integers(-8, 9))
        H, W = oth.shape
        rows = np.clip(np.arange(y + dy, y + dy + h), 0, H - 1)
        cols = np.clip(np.arange(x + dx, x + dx + w), 0, W - 1)
        pred = oth[rows][:, cols].astype(np.int16)
        key = 2 * org[y:y + h, x:x + w] - pred
        keys[offs[k]:offs[k + 1]] = key.reshape(-1)
        jobs["key_offset"][i] = offs[k]
    return keys


def lambdas_for_frame(qp, poc):
    return LDP_LAMBDA[qp if qp in LDP_LAMBDA else 22][poc % 4]


# randomaccess_main GOP (cfg/encoder_randomaccess_main.cfg Frame1..8): (POC, QPoffset, QPFactor)
RA_GOP = ((8, 1, 0.442), (4, 2, 0.3536), (2, 3, 0.3536), (1, 4, 0.68), (3, 4, 0.68), (6, 3, 0.3536),
          (5, 4, 0.68), (7, 4, 0.68))


def ra_depth(poc, gop=8):
    """TEncSlice.cpp:165-199: depth of a POC in a GOP (0 for the GOP's key POC; the loop also
    counts the level at which the POC is found)."""
    poc %= gop
    if poc == 0:
        return 0
    depth, step, i = 0, gop, gop >> 1
    while i >= 1:
        found = any(j == poc for j in range(i, gop, step))
        step >>= 1
        depth += 1
        if found:
            break
        i >>= 1
    return depth


def ra_lambda(qp, gop_entry):
    """Lambda of a random-access B slice (TEncSlice.cpp:246-325 with HadamardME on: no 0.95):
    QPFactor * 2^((QP + QPoffset - 12) / 3), times Clip3(2, 4, (QP + QPoffset - 12) / 6) below the
    GOP's top layer."""
    poc, off, factor = RA_GOP[gop_entry % 8]
    qp_temp = float(qp + off - 12)
    lam = factor * 2.0 ** (qp_temp / 3.0)
    if ra_depth(poc) > 0:
        lam *= min(4.0, max(2.0, qp_temp / 6.0))
    return lam


def jobs_per_frame(width, height, refs=4, calls_per_ctu=423):
    ctus = ((width + 63) // 64) * ((height + 63) // 64)
    return ctus * calls_per_ctu * refs


# ---- motion compensation inputs ---------------------------------
def synth_chroma(width, height, t, seed=None):
    """4:2:0 chroma planes (Cb, Cr) of a synthetic frame: the luma generator at half size with
    its own draws (SURVEY.md §8(d) uses flat 128 chroma; textured planes exercise the 4-tap
    filter)."""
    base = SEEDS.get((width, height), 7) if seed is None else seed
    return (synth_luma(width // 2, height // 2, t, seed=base * 31 + 11),
            synth_luma(width // 2, height // 2, t, seed=base * 37 + 13))


# PU partitions of a CU of size s: PartSize (TComDataCU::getPartIndexAndSize) -> PU rectangles
def _cu_parts(rng, s, amp):
    modes = ["2Nx2N", "2NxN", "Nx2N"]
    if s == 8:
        modes = ["2Nx2N", "2NxN", "Nx2N"]          # 8x4 / 4x8 (inter NxN is off)
    elif amp:
        modes += ["2NxnU", "2NxnD", "nLx2N", "nRx2N"]
    m = modes[rng.integers(len(modes))]
    q, h = s // 4, s // 2
    return {
        "2Nx2N": [(0, 0, s, s)],
        "2NxN": [(0, 0, s, h), (0, h, s, h)],
        "Nx2N": [(0, 0, h, s), (h, 0, h, s)],
        "2NxnU": [(0, 0, s, q), (0, q, s, s - q)],
        "2NxnD": [(0, 0, s, s - q), (0, s - q, s, q)],
        "nLx2N": [(0, 0, q, s), (q, 0, s - q, s)],
        "nRx2N": [(0, 0, s - q, s), (s - q, 0, q, s)],
    }[m]


def make_mc_partition(rng, width, height, ref_ids, bi_frac=0.0, mv_amp=64, p_split=(0.35, 0.55, 0.6), amp=True,
                      identical_frac=0.0):
    """One frame's decided inter PUs for motion compensation: every CTU split into CUs by a random
    quad-tree (forced where a CU crosses the picture border, as TEncCu does), each CU into PUs by
    a random PartSize, each PU with quarter-pel MVs U[-4 mv_amp, 4 mv_amp] on 1 or 2 lists.
    Returns an MC_JOB_DTYPE array that tiles the picture (width, height multiples of 8)."""
    from .abi import MC_JOB_DTYPE, MC_L0, MC_L1
    out = []

    def cu(x, y, s, depth):
        if x >= width or y >= height:
            return
        inside = x + s <= width and y + s <= height
        if s > 8 and (not inside or rng.random() < p_split[min(depth, 2)]):
            for dy in (0, s // 2):
                for dx in (0, s // 2):
                    cu(x + dx, y + dy, s // 2, depth + 1)
            return
        for (px, py, pw, ph) in _cu_parts(rng, s, amp):
            out.append((x + px, y + py, pw, ph, x, y))

    for cy in range(0, height, MAX_CU):
        for cx in range(0, width, MAX_CU):
            cu(cx, cy, MAX_CU, 0)
    n = len(out)
    jobs = np.zeros(n, dtype=MC_JOB_DTYPE)
    a = np.array(out, dtype=np.int64)
    jobs["x"], jobs["y"], jobs["w"], jobs["h"], jobs["cu_x"], jobs["cu_y"] = a.T
    bi = rng.random(n) < bi_frac
    one = rng.integers(0, 2, n)   # uni-pred: list 0 or 1
    jobs["flags"] = np.where(bi, MC_L0 | MC_L1, np.where(one == 0, MC_L0, MC_L1))
    ids = np.asarray(ref_ids, dtype=np.int64)
    jobs["ref_id"] = ids[rng.integers(0, len(ids), (n, 2))]
    jobs["mv"] = rng.integers(-4 * mv_amp, 4 * mv_amp + 1, (n, 2, 2))
    same = bi & (rng.random(n) < identical_frac)   # xCheckIdenticalMotion cases
    jobs["ref_id"][same, 1] = jobs["ref_id"][same, 0]
    jobs["mv"][same, 1] = jobs["mv"][same, 0]
    return jobs


def make_bipred_keys_fast(rng, jobs, pictures):
    """Vectorised make_bipred_keys (same key definition, 2*org - pred_other with an integer-
    displaced other-picture block, edge-clamped), grouped by PU shape: for the ~270 K bi-pred jobs
    of a 2560x1600 random-access frame."""
    sel = np.flatnonzero(jobs["key_offset"] == -2)
    sizes = jobs["w"][sel].astype(np.int64) * jobs["h"][sel].astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    keys = np.zeros(int(offs[-1]), dtype=np.int16)
    ids = sorted(pictures)
    stack = np.stack([pictures[i] for i in ids]).astype(np.int16)
    other = rng.integers(0, len(ids), len(sel))
    dx = rng.integers(-8, 9, len(sel))
    dy = rng.integers(-8, 9, len(sel))
    Hp, Wp = stack.shape[1:]
    shapes = set(zip(jobs["w"][sel].tolist(), jobs["h"][sel].tolist()))
    for (w, h) in shapes:
        m = np.flatnonzero((jobs["w"][sel] == w) & (jobs["h"][sel] == h))
        x = jobs["x"][sel[m]].astype(np.int64)
        y = jobs["y"][sel[m]].astype(np.int64)
        org_ids = np.searchsorted(ids, jobs["org_id"][sel[m]])
        ry = y[:, None] + np.arange(h)[None, :]
        rx = x[:, None] + np.arange(w)[None, :]
        org = stack[org_ids[:, None, None], ry[:, :, None], rx[:, None, :]]
        py = np.clip(ry + dy[m][:, None], 0, Hp - 1)
        px = np.clip(rx + dx[m][:, None], 0, Wp - 1)
        pred = stack[other[m][:, None, None], py[:, :, None], px[:, None, :]]
        blk = (2 * org - pred).reshape(len(m), -1)
        idx = offs[m][:, None] + np.arange(w * h)[None, :]
        keys[idx] = blk
        jobs["key_offset"][sel[m]] = offs[m]
    return keys


# ---- integer motion estimation inputs -----------------------------------
def _clip_cu_qpel(v, cu, pic):
    """TComDataCU::clipMv with the CU origin (TComDataCU.cpp:2778-2785), quarter-pel."""
    return np.minimum((pic + 8 - cu - 1) << 2, np.maximum((-MAX_CU - 8 - cu + 1) << 2, v))


def make_tz_jobs(rng, width, height, calls_per_ctu, org_id, ref_ids, lambda_ids, mix=PU_MIX, bipred_frac=0.0,
                 pred2n_frac=0.5, search_range=SEARCH_RANGE, bipred_range=4, amp=12.0, mvp_noise=24):
    """Jobs for the integer search in HM's CTU order: PUs on the CU grid with their CU origin
    (clipMv), the AMVP predictor near a smooth motion field, the search range from
    xSetSearchRange(mvp, SearchRange) (bi-pred: xSetSearchRange(current MV, BipredSearchRange)),
    and for a share of non-2Nx2N PUs the 2Nx2N integer MV as an extra start candidate.
    Returns (fme_job array with FME_JOB_EMI / FME_JOB_BIPRED flags, fme_tz_ext array)."""
    from .abi import TZ_EXT_DTYPE, TZ_PRED2NX2N
    ctus_x, ctus_y = (width + MAX_CU - 1) // MAX_CU, (height + MAX_CU - 1) // MAX_CU
    vx, vy = motion_field(rng, ctus_x, ctus_y, amp)
    ref_ids = np.asarray(ref_ids)
    nref = len(ref_ids)
    per = calls_per_ctu * nref
    n = ctus_x * ctus_y * per
    w, h = sample_sizes(rng, n, mix)
    ctu = np.repeat(np.arange(ctus_x * ctus_y), per)
    cs = np.where(np.maximum(w, h) <= 8, 8, np.where(np.maximum(w, h) <= 16, 16, np.where(np.maximum(w, h) <= 32, 32, 64)))
    ncu = MAX_CU // cs
    cu_x = (ctu % ctus_x) * MAX_CU + rng.integers(0, ncu) * cs
    cu_y = (ctu // ctus_x) * MAX_CU + rng.integers(0, ncu) * cs
    cu_x = np.minimum(cu_x, (width - cs) // 8 * 8)
    cu_y = np.minimum(cu_y, (height - cs) // 8 * 8)
    x = np.minimum(cu_x + rng.integers(0, 2, n) * (cs - w), (width - w) // 4 * 4)
    y = np.minimum(cu_y + rng.integers(0, 2, n) * (cs - h), (height - h) // 4 * 4)
    ref_k = np.tile(np.arange(nref), n // nref)
    dist = ref_k + 1
    mvp_x = 4 * np.rint(vx.reshape(-1)[ctu] * dist).astype(np.int64) + rng.integers(-mvp_noise, mvp_noise + 1, n)
    mvp_y = 4 * np.rint(vy.reshape(-1)[ctu] * dist).astype(np.int64) + rng.integers(-mvp_noise, mvp_noise + 1, n)
    bi = rng.random(n) < bipred_frac
    # bi-pred: the range is centred on the current MV of the list (rcMv), near the predictor
    cen_x = np.where(bi, mvp_x + 4 * rng.integers(-3, 4, n), mvp_x)
    cen_y = np.where(bi, mvp_y + 4 * rng.integers(-3, 4, n), mvp_y)
    rng_pel = np.where(bi, bipred_range, search_range)
    cx = _clip_cu_qpel(cen_x, cu_x, width)
    cy = _clip_cu_qpel(cen_y, cu_y, height)
    jobs = np.zeros(n, dtype=JOB_DTYPE)
    jobs["x"], jobs["y"], jobs["w"], jobs["h"] = x, y, w, h
    jobs["org_id"] = org_id
    jobs["ref_id"] = ref_ids[ref_k]
    jobs["lambda_id"] = rng.choice(np.asarray(lambda_ids), size=n)
    jobs["mvp_x"], jobs["mvp_y"] = mvp_x, mvp_y
    jobs["lt_x"] = _div4_round(_clip_cu_qpel(cx - (rng_pel << 2), cu_x, width))
    jobs["rb_x"] = _div4_round(_clip_cu_qpel(cx + (rng_pel << 2), cu_x, width))
    jobs["lt_y"] = _div4_round(_clip_cu_qpel(cy - (rng_pel << 2), cu_y, height))
    jobs["rb_y"] = _div4_round(_clip_cu_qpel(cy + (rng_pel << 2), cu_y, height))
    jobs["bits_in"] = rng.integers(1, 7, n)
    jobs["flags"] = np.where(bi, JOB_BIPRED, JOB_EMI)
    jobs["key_offset"] = np.where(bi, -2, -1)
    ext = np.zeros(n, dtype=TZ_EXT_DTYPE)
    ext["cu_x"], ext["cu_y"] = cu_x, cu_y
    ext["search_range"] = search_range
    p2 = (~bi) & ((w != cs) | (h != cs)) & (rng.random(n) < pred2n_frac)
    ext["flags"] = np.where(p2, TZ_PRED2NX2N, 0)
    ext["pred2n_x"] = np.where(p2, np.rint(vx.reshape(-1)[ctu] * dist).astype(np.int64) + rng.integers(-6, 7, n), 0)
    ext["pred2n_y"] = np.where(p2, np.rint(vy.reshape(-1)[ctu] * dist).astype(np.int64) + rng.integers(-6, 7, n), 0)
    return jobs, ext


# ---- predInterSearch producer inputs -----------------------------------------
def _cu_partitions(x0, y0, s):
    """(part_size, [(x, y, w, h) per PU]) of one CU in TEncCu::xCompressCU's order (TEncCu.cpp:
    2Nx2N, 2NxN, Nx2N, then the AMP shapes for CUs above 8x8)."""
    from .abi import PART_2Nx2N, PART_2NxN, PART_2NxnD, PART_2NxnU, PART_Nx2N, PART_nLx2N, PART_nRx2N
    h, q = s // 2, s // 4
    parts = [(PART_2Nx2N, [(x0, y0, s, s)]),
             (PART_2NxN, [(x0, y0, s, h), (x0, y0 + h, s, h)]),
             (PART_Nx2N, [(x0, y0, h, s), (x0 + h, y0, h, s)])]
    if s > 8:
        parts += [(PART_2NxnU, [(x0, y0, s, q), (x0, y0 + q, s, s - q)]),
                  (PART_2NxnD, [(x0, y0, s, s - q), (x0, y0 + s - q, s, q)]),
                  (PART_nLx2N, [(x0, y0, q, s), (x0 + q, y0, s - q, s)]),
                  (PART_nRx2N, [(x0, y0, s - q, s), (x0 + s - q, y0, q, s)])]
    return parts


def make_pu_requests(rng, width, height, org_id, ref_ids, lambda_id, max_depth=3, amp=12.0, cand_noise=24,
                     one_cand_frac=0.1, lossless_frac=0.0, search_range=SEARCH_RANGE):
    """fme_pu_req stream of a P frame in encoder call order: CTUs in raster order, each CU quadtree
    depth-first (64 -> 8), per CU every partition's PUs (PU0 then PU1).  AMVP candidates per
    reference index k lie near a smooth motion field scaled by the POC distance k + 1 (the second
    one sometimes equal to the first or zero, as fillMvpCand pads); one_cand_frac of the lists
    hold a single candidate."""
    from .abi import MAX_REFS, PU_LOSSLESS, PU_REQ_DTYPE
    ctus_x, ctus_y = (width + MAX_CU - 1) // MAX_CU, (height + MAX_CU - 1) // MAX_CU
    vx, vy = motion_field(rng, ctus_x, ctus_y, amp)
    rows = []

    def cu(x0, y0, s, d, ctu):
        if x0 >= width or y0 >= height:
            return
        if x0 + s > width or y0 + s > height:   # boundary CUs are split
            if s > 8:
                for cy in (y0, y0 + s // 2):
                    for cx in (x0, x0 + s // 2):
                        cu(cx, cy, s // 2, d + 1, ctu)
            return
        for ps, pus in _cu_partitions(x0, y0, s):
            for (x, y, w, h) in pus:
                rows.append((x, y, w, h, x0, y0, ps, d, ctu))
        if d < max_depth and s > 8:
            for cy in (y0, y0 + s // 2):
                for cx in (x0, x0 + s // 2):
                    cu(cx, cy, s // 2, d + 1, ctu)

    for t in range(ctus_x * ctus_y):
        cu((t % ctus_x) * MAX_CU, (t // ctus_x) * MAX_CU, MAX_CU, 0, t)
    a = np.array(rows, dtype=np.int64).reshape(-1, 9)
    n = len(a)
    nref = len(ref_ids)
    reqs = np.zeros(n, dtype=PU_REQ_DTYPE)
    reqs["x"], reqs["y"], reqs["w"], reqs["h"] = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
    reqs["cu_x"], reqs["cu_y"], reqs["part_size"], reqs["depth"] = a[:, 4], a[:, 5], a[:, 6], a[:, 7]
    reqs["org_id"] = org_id
    reqs["num_refs"] = nref
    reqs["ref_id"][:, :nref] = np.asarray(ref_ids)
    reqs["lambda_id"] = lambda_id
    reqs["search_range"] = search_range
    reqs["flags"] = np.where(rng.random(n) < lossless_frac, PU_LOSSLESS, 0)
    ctu = a[:, 8]
    for k in range(nref):
        bx = 4 * np.rint(vx.reshape(-1)[ctu] * (k + 1)).astype(np.int64)
        by = 4 * np.rint(vy.reshape(-1)[ctu] * (k + 1)).astype(np.int64)
        c0x = bx + rng.integers(-cand_noise, cand_noise + 1, n)
        c0y = by + rng.integers(-cand_noise, cand_noise + 1, n)
        kind = rng.integers(0, 4, n)   # second candidate: 0/1 near the field, 2 equal, 3 zero
        c1x = np.where(kind < 2, bx + rng.integers(-cand_noise, cand_noise + 1, n), np.where(kind == 2, c0x, 0))
        c1y = np.where(kind < 2, by + rng.integers(-cand_noise, cand_noise + 1, n), np.where(kind == 2, c0y, 0))
        reqs["cand"][:, k, 0, 0], reqs["cand"][:, k, 0, 1] = c0x, c0y
        reqs["cand"][:, k, 1, 0], reqs["cand"][:, k, 1, 1] = c1x, c1y
        reqs["n_cand"][:, k] = np.where(rng.random(n) < one_cand_frac, 1, 2)
    assert nref <= MAX_REFS
    return reqs


def make_pu_requests_b(rng, width, height, org_id, l0, l1, lambda_id, max_depth=3, amp=12.0, cand_noise=24,
                       one_cand_frac=0.1, lossless_frac=0.0, search_range=SEARCH_RANGE, bipred_range=4,
                       fast_me_gen_b=True, clip_bipred=False, mvd_l1_zero=False):
    """fme_pu_req_b stream of a B frame in encoder call order (as make_pu_requests).  l0 / l1: lists
    of (picture slot, signed POC distance) per reference index; an L1 slot that is also in L0 gets
    l1_to_l0 = its L0 index (getList1IdxToList0Idx).  Candidates of a reference lie near the
    motion field scaled by its POC distance."""
    from .abi import MAX_REFS, PU_CLIP_BIPRED, PU_FAST_ME_GEN_B, PU_LOSSLESS, PU_MVD_L1_ZERO, PU_REQ_B_DTYPE
    p = make_pu_requests(rng, width, height, org_id, [0], lambda_id, max_depth=max_depth, amp=amp,
                         search_range=search_range)
    n = len(p)
    ctus_x = (width + MAX_CU - 1) // MAX_CU
    vx, vy = motion_field(rng, ctus_x, (height + MAX_CU - 1) // MAX_CU, amp)
    reqs = np.zeros(n, dtype=PU_REQ_B_DTYPE)
    for f in ("x", "y", "w", "h", "cu_x", "cu_y", "part_size", "depth", "org_id", "lambda_id", "search_range"):
        reqs[f] = p[f]
    # part index within the CU and the CU width (the stream lists a CU's PUs consecutively)
    key = np.stack([p["cu_x"], p["cu_y"], p["depth"], p["part_size"]], 1).astype(np.int64)
    same = np.r_[False, (key[1:] == key[:-1]).all(1)]
    idx = np.zeros(n, np.int64)
    for i in range(1, n):
        idx[i] = idx[i - 1] + 1 if same[i] else 0
    reqs["part_idx"] = idx
    reqs["cu_w"] = MAX_CU >> p["depth"].astype(np.int64)
    reqs["bipred_range"] = bipred_range
    flags = np.where(rng.random(n) < lossless_frac, PU_LOSSLESS, 0)
    if fast_me_gen_b:
        flags |= PU_FAST_ME_GEN_B
    if clip_bipred:
        flags |= PU_CLIP_BIPRED
    if mvd_l1_zero:   # a slice-level switch: every request of the frame
        flags |= PU_MVD_L1_ZERO
    reqs["flags"] = flags
    reqs["num_refs"] = [len(l0), len(l1)]
    reqs["l1_to_l0"] = -1
    slots0 = [s for s, _ in l0]
    for k, (s, _) in enumerate(l1):
        if s in slots0:
            reqs["l1_to_l0"][:, k] = slots0.index(s)
    ctu = (p["cu_y"].astype(np.int64) // MAX_CU) * ctus_x + p["cu_x"].astype(np.int64) // MAX_CU
    for l, lst in enumerate((l0, l1)):
        assert len(lst) <= MAX_REFS
        for k, (slot, d) in enumerate(lst):
            reqs["ref_id"][:, l, k] = slot
            bx = 4 * np.rint(vx.reshape(-1)[ctu] * d).astype(np.int64)
            by = 4 * np.rint(vy.reshape(-1)[ctu] * d).astype(np.int64)
            c0x = bx + rng.integers(-cand_noise, cand_noise + 1, n)
            c0y = by + rng.integers(-cand_noise, cand_noise + 1, n)
            kind = rng.integers(0, 4, n)
            c1x = np.where(kind < 2, bx + rng.integers(-cand_noise, cand_noise + 1, n), np.where(kind == 2, c0x, 0))
            c1y = np.where(kind < 2, by + rng.integers(-cand_noise, cand_noise + 1, n), np.where(kind == 2, c0y, 0))
            reqs["cand"][:, l, k, 0, 0], reqs["cand"][:, l, k, 0, 1] = c0x, c0y
            reqs["cand"][:, l, k, 1, 0], reqs["cand"][:, l, k, 1, 1] = c1x, c1y
            reqs["n_cand"][:, l, k] = np.where(rng.random(n) < one_cand_frac, 1, 2)
    return reqs


# TComInterpolationFilter.cpp:57-63 luma taps by quarter-pel fraction
LUMA_TAPS = np.array([[0, 0, 0, 64, 0, 0, 0, 0], [-1, 4, -10, 58, 17, -5, 1, 0],
                      [-1, 4, -11, 40, 40, -11, 4, -1], [0, 1, -5, 17, 58, -10, 4, -1]], dtype=np.int64)


def make_bipred_key_reqs(rng, jobs, org_id, ref_ids, mv_span=40, clip=False):
    """fme_bikey_req per bi-pred job (key_offset == -2): the other list's reference (one of
    ref_ids) and quarter-pel MV (U[-mv_span, mv_span]^2), CU origin = the PU's CTU; assigns
    key_offset (cumulative w*h) in the jobs.  Returns (requests, key count)."""
    from .abi import BIKEY_REQ_DTYPE, PU_CLIP_BIPRED
    sel = np.flatnonzero(jobs["key_offset"] == -2)
    sizes = jobs["w"][sel].astype(np.int64) * jobs["h"][sel].astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    reqs = np.zeros(len(sel), dtype=BIKEY_REQ_DTYPE)
    for f in ("x", "y", "w", "h"):
        reqs[f] = jobs[f][sel]
    reqs["org_id"] = org_id
    reqs["ref_id"] = rng.choice(np.asarray(ref_ids), size=len(sel))
    reqs["cu_x"] = jobs["x"][sel].astype(np.int64) & ~(MAX_CU - 1)
    reqs["cu_y"] = jobs["y"][sel].astype(np.int64) & ~(MAX_CU - 1)
    reqs["mv_x"] = rng.integers(-mv_span, mv_span + 1, len(sel))
    reqs["mv_y"] = rng.integers(-mv_span, mv_span + 1, len(sel))
    reqs["key_offset"] = offs[:-1]
    reqs["flags"] = PU_CLIP_BIPRED if clip else 0
    jobs["key_offset"][sel] = offs[:-1]
    return reqs, int(offs[-1])


def bipred_keys(reqs, pictures, key_count):
    """What fme_build_bipred_keys computes, vectorised per PU shape: the uni-pred luma prediction
    of the other list (clipMv, xPredInterBlk's copy / 1-D / 2-D paths with HM's rounding) and
    key = 2 * org - pred (removeHighFreq).  pictures: {slot: uint8 [H, W]}."""
    keys = np.zeros(key_count, dtype=np.int16)
    ids = sorted(pictures)
    stack = np.stack([pictures[i] for i in ids]).astype(np.int64)
    Hp, Wp = stack.shape[1:]
    shapes = set(zip(reqs["w"].tolist(), reqs["h"].tolist()))
    for (w, h) in shapes:
        m = np.flatnonzero((reqs["w"] == w) & (reqs["h"] == h))
        q = reqs[m]
        x, y = q["x"].astype(np.int64), q["y"].astype(np.int64)
        cux, cuy = q["cu_x"].astype(np.int64), q["cu_y"].astype(np.int64)
        mvx = np.minimum((Wp + 8 - cux - 1) << 2, np.maximum((-MAX_CU - 8 - cux + 1) * 4, q["mv_x"].astype(np.int64)))
        mvy = np.minimum((Hp + 8 - cuy - 1) << 2, np.maximum((-MAX_CU - 8 - cuy + 1) * 4, q["mv_y"].astype(np.int64)))
        fx, fy = mvx & 3, mvy & 3
        rows = np.clip(y[:, None] + (mvy >> 2)[:, None] + np.arange(-3, h + 4)[None, :], 0, Hp - 1)
        cols = np.clip(x[:, None] + (mvx >> 2)[:, None] + np.arange(-3, w + 4)[None, :], 0, Wp - 1)
        ref = np.searchsorted(ids, q["ref_id"])
        win = stack[ref[:, None, None], rows[:, :, None], cols[:, None, :]]          # (n, h+7, w+7)
        ch, cv = LUMA_TAPS[fx], LUMA_TAPS[fy]
        hs = sum(ch[:, k, None, None] * win[:, :, k:k + w] for k in range(8))        # (n, h+7, w)
        a = np.clip((hs[:, 3:3 + h, :] + 32) >> 6, 0, 255)                           # fy == 0
        vs = sum(cv[:, k, None, None] * win[:, k:k + h, 3:3 + w] for k in range(8))  # fx == 0
        b = np.clip((vs + 32) >> 6, 0, 255)
        t = hs - 8192                                                                 # 2-D
        cs = sum(cv[:, k, None, None] * t[:, k:k + h, :] for k in range(8))
        c = np.clip((cs + 2048 + (8192 << 6)) >> 12, 0, 255)
        pred = np.where((fy == 0)[:, None, None], a, np.where((fx == 0)[:, None, None], b, c))
        org = stack[np.searchsorted(ids, q["org_id"])[:, None, None], (y[:, None] + np.arange(h))[:, :, None],
                    (x[:, None] + np.arange(w))[:, None, :]]
        key = 2 * org - pred
        clip = (q["flags"] & 0x04) != 0
        key = np.where(clip[:, None, None], np.clip(key, 0, 255), key)
        idx = q["key_offset"].astype(np.int64)[:, None] + np.arange(w * h)[None, :]
        keys[idx] = key.reshape(len(m), -1)
    return keys


def pu_requests_to_jobs(reqs, width, height):
    """The xMotionEstimation jobs of single-reference, single-candidate requests whose
    m_integerMv2Nx2N reads see the initial (0, 0): mvp = cand[0][0], xSetSearchRange(mvp, range)
    (TEncSearch.cpp:4602-4624), bits_in = xGetBlkBits + m_auiMVPIdxCost[0][2]."""
    from .abi import PART_2Nx2N, PART_NxN, PU_LOSSLESS, TZ_EXT_DTYPE, TZ_PRED2NX2N
    from .abi import JOB_LOSSLESS
    n = len(reqs)
    jobs = np.zeros(n, dtype=JOB_DTYPE)
    ext = np.zeros(n, dtype=TZ_EXT_DTYPE)
    for f in ("x", "y", "w", "h", "org_id"):
        jobs[f] = reqs[f]
    jobs["ref_id"] = reqs["ref_id"][:, 0]
    mx, my = reqs["cand"][:, 0, 0, 0].astype(np.int64), reqs["cand"][:, 0, 0, 1].astype(np.int64)
    jobs["mvp_x"], jobs["mvp_y"] = mx, my
    rng_pel = np.where(reqs["search_range"] == 0, 64, reqs["search_range"]).astype(np.int64)
    cux, cuy = reqs["cu_x"].astype(np.int64), reqs["cu_y"].astype(np.int64)
    cx, cy = _clip_cu_qpel(mx, cux, width), _clip_cu_qpel(my, cuy, height)
    jobs["lt_x"] = _div4_round(_clip_cu_qpel(cx - (rng_pel << 2), cux, width))
    jobs["rb_x"] = _div4_round(_clip_cu_qpel(cx + (rng_pel << 2), cux, width))
    jobs["lt_y"] = _div4_round(_clip_cu_qpel(cy - (rng_pel << 2), cuy, height))
    jobs["rb_y"] = _div4_round(_clip_cu_qpel(cy + (rng_pel << 2), cuy, height))
    jobs["flags"] = JOB_EMI | np.where(reqs["flags"] & PU_LOSSLESS, JOB_LOSSLESS, 0)
    jobs["lambda_id"] = reqs["lambda_id"]
    jobs["bits_in"] = np.where(np.isin(reqs["part_size"], (PART_2Nx2N, PART_NxN)), 1, 3) + 1
    jobs["key_offset"] = -1
    ext["cu_x"], ext["cu_y"] = reqs["cu_x"], reqs["cu_y"]
    ext["search_range"] = rng_pel
    reads = ~((reqs["part_size"] == PART_2Nx2N) & (reqs["depth"] == 0))
    ext["flags"] = np.where(reads, TZ_PRED2NX2N, 0)
    return jobs, ext
