#!/usr/bin/env python3
"""Benchmark: sub-pel PU refinements/s on 1920x1080 lowdelay_P QP22, NN_pred on
(BASELINE.json metric; configs[2] at QP22; other configs with --workload).

A step is one frame batch: every (PU, reference picture) sub-pel job of one synthetic 1080p
P-frame (510 CTUs x 423 calls x 4 references = 862,920 jobs, SURVEY.md §8(d) mix) through
EMI step -> FracDIF -> NN_pred -> xMotionEstimation tail.  `value` times the steps with their
inputs already resident in HBM (the task's measurement contract): per step the frame's pictures and
lambdas are bound, configs[3]'s bi-pred keys are built on the device, and the batch refines the
frame's jobs into a device result buffer.  With N ranks (torchrun, one GPU each) rank r replays
frames r, r+N, ... (weak scaling); each reconstruction is uploaded by one rank and sent (RCCL
point-to-point) to the ranks whose frames reference it, and the NN carried state is chained across
ranks at the end of the timed region (all_gather of 12 words per frame + a device re-run of each
frame's carried-state prefix).  `pcie_inclusive` reports SURVEY.md §8(d)'s wider timing of the same
steps: per step the jobs (32 B each), the frame's original and one reconstructed reference go over
PCIe from pinned host memory and the 16-byte fme_mv_result per job comes back
(nnfme.pipeline.FrameReplay: two steps in flight on separate copy / compute streams); the parity
leg checks that pass's first timed step against oracle/_ref.

Prints one JSON line (rank 0).  `cpu_baseline` times oracle/_ref (the reference's own
TLibCommon primitives driven in TEncSearch order, compiled -O2 like the reference build) on
one host core (HM is single-threaded) over a bounded sample of the same job mix;
`cpu_baseline_all_cores` runs one job stream per host core.  Both run
before the GPU is initialised.

`roofline` is for the main search phase (k_search_lane: the lane-per-unit EMI + FracDIF kernel
of every PU shape, one persistent launch per batch), timed by HIP events recorded on the batch
stream around it: the
path is integer-VALU bound, so `bound` is "valu" with the reference's integer ops (§8(d)) per
second over the VALU peak; the HBM roof of the same phase is the `hbm` entry.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))

from nnfme import synth  # noqa: E402
from nnfme.abi import JOB_BIPRED, JOB_DTYPE, JOB_NN_IN, MV_RESULT_DTYPE, RESULT_DTYPE, TZ_RING  # noqa: E402

W, H, QP = 1920, 1080, 22
METRIC = "sub-pel PU refinements/sec @ 1080p lowdelay_P QP22; bit-exact MV/SATD vs HM"
# BASELINE.json configs as bench workloads (default: the headline, configs[2] at QP22).
#   name: W, H, QP, nn (nn_mode), net (nn_mode 2), engine (0 exact, 1 MFMA), calls (per CTU per
#   reference), refs, bipred (share of bi-pred key jobs), gop ("ldp" / "ra" lambdas), frames (per
#   batch: small frames are batched so a launch fills the chip), desc
WORKLOADS = {
    "c3_qp22": dict(W=1920, H=1080, QP=22, nn=1, calls=423, bipred=0.0, gop="ldp", frames=1,
                    desc="1920x1080 lowdelay_P QP22, NN_pred 2-layer on, 4 refs, 862920 PU jobs per frame "
                         "(configs[2] at QP22)"),
    "c3_qp27": dict(W=1920, H=1080, QP=27, nn=1, calls=423, bipred=0.0, gop="ldp", frames=1,
                    desc="1920x1080 lowdelay_P QP27, NN_pred on, 4 refs (configs[2] at QP27)"),
    "c3_qp32": dict(W=1920, H=1080, QP=32, nn=1, calls=423, bipred=0.0, gop="ldp", frames=1,
                    desc="1920x1080 lowdelay_P QP32, NN_pred on, 4 refs (configs[2] at QP32)"),
    "c3_qp22_main10": dict(W=1920, H=1080, QP=22, nn=1, calls=423, bipred=0.0, gop="ldp", frames=1, bit_depth=10,
                           desc="1920x1080 lowdelay_P main10 (InternalBitDepth 10, cfg/encoder_lowdelay_P_main10.cfg:58) "
                                "QP22, NN_pred on, 4 refs (configs[2] at 10 bit: 16-bit samples, the pixel-per-lane "
                                "kernel k_search_px)"),
    "c3_qp37": dict(W=1920, H=1080, QP=37, nn=1, calls=423, bipred=0.0, gop="ldp", frames=1,
                    desc="1920x1080 lowdelay_P QP37, NN_pred on, 4 refs (configs[2] at QP37)"),
    "c1": dict(W=416, H=240, QP=22, nn=1, calls=331, bipred=0.0, gop="ldp", frames=8,
               desc="416x240 lowdelay_P QP22, NN_pred on, 4 refs (configs[0]: the CPU plumbing baseline's "
                    "workload; 8 frames per batch on the GPU)"),
    "c2": dict(W=416, H=240, QP=22, nn=0, calls=331, bipred=0.0, gop="ldp", frames=8,
               desc="416x240 lowdelay_P QP22, interpolation + SATD only (NN_pred off), 4 refs, 331 calls/CTU/ref, "
                    "8 frames per batch (configs[1])"),
    "c4": dict(W=2560, H=1600, QP=27, nn=1, calls=333, bipred=0.205, gop="ra", frames=1,
               desc="2560x1600 random-access QP27 B-frames, NN_pred on, 2+2 refs, ~1331 calls/CTU, 20.5 % bi-pred "
                    "with 2*org - pred keys built per frame on the device inside the timed step, RA GOP-8 "
                    "lambdas (configs[3])"),
    "c5": dict(W=1920, H=1080, QP=22, nn=2, net="scr3x40+tzring", engine=1, calls=423, bipred=0.0, gop="ldp",
               frames=1, inputs="ring",
               desc="1920x1080 lowdelay_P QP22 with the 3-hidden-layer NN_pred (Backups/4 SCR 9-40-40-40-49, "
                    "double) as a batched MFMA GEMM (v_mfma_f64_16x16x4) (configs[4]) on Backups/4's own input path: "
                    "every xTZSearchHelp distortion pushed, the final square + distance-2 ring (which may move the "
                    "integer MV), C = the least push before the square (fme_integer_search_ring -> FME_JOB_NN_IN "
                    "jobs, 36 B of NN inputs per job uploaded with the job)"),
    "c5_exact": dict(W=1920, H=1080, QP=22, nn=2, net="scr3x40+tzring", engine=0, calls=423, bipred=0.0,
                     gop="ldp", frames=1, inputs="ring",
                     desc="configs[4] net through the exact (scalar, reference-order) engine on Backups/4's own input "
                          "path"),
    "c5_b4x40": dict(W=1920, H=1080, QP=22, nn=2, net="blowing4x40+rezero+tzring", engine=1, calls=423,
                     bipred=0.0, gop="ldp", frames=1, inputs="ring", deviation=(
                         "Backups/15:4955-4962 clears only IN/X1/X2/OUT/array_e per call, so its X3/X4 carry "
                         "across calls; this workload re-zeroes them per job (the batch engines need "
                         "job-independent hidden layers), which is NOT the reference's behaviour"),
                     desc="DEVIATION: 1920x1080 QP22 with the 4x40 blowing net (Backups/15, float) with its X3/X4 "
                          "carry re-zeroed per job, as a batched MFMA GEMM (v_mfma_f32_16x16x4) on Backups/15's own "
                          "input path (the same integer-search tail as Backups/4)"),
}
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
# int32 VALU lane-ops/s: 256 CUs x 4 SIMDs x 32 lanes/clk (a wave64 op issues over 2 clk) x
# 2.4 GHz = 78.6 T (MI355X_MICROARCH.md; = the 157.3 TFLOP/s f32 vector peak / 2)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12


def algorithmic_bytes(jobs, bps=1):
    """W*H (org) + (W+8)(H+8) (reference footprint) samples of bps bytes (2 at
    main10) + 48 (descriptor + result)."""
    w = jobs["w"].astype(np.int64)
    h = jobs["h"].astype(np.int64)
    return int((bps * (w * h + (w + 8) * (h + 8)) + 48).sum())


def main_kernel_mask(ctx, jobs):
    """Jobs the main search launch serves (fme_search_kernel_of_shape == 0)."""
    m = np.zeros(len(jobs), bool)
    shapes = set(zip(jobs["w"].tolist(), jobs["h"].tolist()))
    for w, h in shapes:
        if ctx.search_kernel_of_shape(w, h) == 0:
            m |= (jobs["w"] == w) & (jobs["h"] == h)
    return m


def algorithmic_ops(jobs):
    """SURVEY.md §8(d) integer-op count: 8-tap outputs x16, copies x2, 18 SATDs, 144 cost."""
    w = jobs["w"].astype(np.int64)
    h = jobs["h"].astype(np.int64)
    taps = (w + 1) * (h + 8) + w * (h + 1) + (w + 1) * (h + 1) + 2 * w * (h + 8) + 8 * w * h
    copies = (w + 1) * (h + 8) + w * h + (w + 1) * h
    t8 = ((w % 8) == 0) & ((h % 8) == 0)
    satd = np.where(t8, 575 * (w * h) // 64, 129 * (w * h) // 16)
    return int((16 * taps + 2 * copies + 18 * satd + 144).sum())


def make_frame_jobs(seed, kind="ctu", calls=423, bipred=0.0):
    """One frame's jobs.  "ctu": HM order (CTU raster, PUs on the CU grid, coherent motion);
    "uniform": every PU at a uniformly random frame position (no cache locality, stress)."""
    rng = np.random.default_rng(seed)
    # refs: picture ids 0..3, org: id 4; lambda slot 0 = the frame's value (set per step)
    if kind == "uniform":
        return synth.make_jobs(rng, W, H, synth.jobs_per_frame(W, H, calls_per_ctu=calls), 4, [0, 1, 2, 3], [0],
                               bipred_frac=bipred)
    return synth.make_ctu_jobs(rng, W, H, calls, 4, [0, 1, 2, 3], [0], bipred_frac=bipred)


_CPU = {}   # set before forking the all-cores workers


def _cpu_reference():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Reference
    from nnfme import weights
    ref = Reference(use_hadamard=1, nn_mode=_CPU.get("nn", 1), fast_inter_mode=1, bit_depth=_CPU.get("bd", 8))
    for k, v in _CPU["pics"].items():
        ref.set_picture(k, v)
    ref.set_lambda(0, synth.LDP_LAMBDA[QP][1])
    ref.load_nn(weights.load_weights(QP))
    if _CPU.get("keys") is not None:
        ref.set_keys(_CPU["keys"])
    return ref


def ring_inputs_cpu(jobs, ext, pics, m):
    """The backups' input path for the CPU baseline: the oracle's integer search with the square +
    ring (orc_integer_search_ring) on the first m jobs -> (refine jobs with FME_JOB_NN_IN, rows)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    from nnfme.abi import JOB_BIPRED, JOB_NN_IN
    orc = Oracle(fast_inter_mode=1)
    for k, v in pics.items():
        orc.set_picture(k, v)
    orc.set_lambda(0, synth.LDP_LAMBDA[QP][1])
    out, _, rows = orc.integer_search_ring(jobs[:m], ext[:m])
    out["flags"] = np.where((out["flags"] & JOB_BIPRED) == 0, JOB_NN_IN, out["flags"]).astype(np.uint8)
    return out, rows


def cpu_baseline_ring(jobs, rows, net_name, pics, seconds):
    """oracle/_ref's sub-pel path with the deeper net on the backups' inputs (FME_JOB_NN_IN rows), one
    core, whole passes over the sample until `seconds` have elapsed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Reference
    from nnfme import weights
    ref = Reference(use_hadamard=1, nn_mode=2, fast_inter_mode=1)
    for k, v in pics.items():
        ref.set_picture(k, v)
    ref.set_lambda(0, synth.LDP_LAMBDA[QP][1])
    ref.load_nn_net(weights.case_net(net_name))
    ref.set_nn_inputs(rows)
    ref.refine(jobs[:1000])
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ref.refine(jobs)
        done += len(jobs)
    return done / (time.perf_counter() - t0), time.perf_counter() - t0, done


def cpu_baseline(jobs, pics, seconds):
    """oracle/_ref on one core: whole passes over the frame's jobs (in HM order) until
    `seconds` have elapsed (the last pass partial, in 20k-job chunks)."""
    _CPU["pics"] = pics
    ref = _cpu_reference()
    ref.refine(jobs[:2000])   # warm caches
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        i = done % len(jobs)
        chunk = jobs[i:i + 20000]
        ref.refine(chunk)
        done += len(chunk)
    dt = time.perf_counter() - t0
    return done / dt, dt, done


def _cpu_worker(args):
    lo, hi, reps = args
    ref = _cpu_reference()
    jobs = _CPU["jobs"][lo:hi]
    ref.refine(jobs[:500])
    t0 = time.perf_counter()
    for _ in range(reps):
        ref.refine(jobs)
    return len(jobs) * reps, time.perf_counter() - t0


def cpu_baseline_all_cores(jobs, pics, rate1, seconds, cores):
    """One job stream per core (fork workers, each its own slice of the frame, repeated so each
    runs about `seconds`); value = all jobs / wall time of the slowest worker."""
    _CPU["pics"], _CPU["jobs"] = pics, jobs
    per = len(jobs) // cores
    reps = max(1, int(round(seconds * rate1 / max(per, 1))))
    tasks = [(i * per, (i + 1) * per, reps) for i in range(cores)]
    with mp.get_context("fork").Pool(cores) as pool:
        out = pool.map(_cpu_worker, tasks)
    total = sum(o[0] for o in out)
    wall = max(o[1] for o in out)
    return total / wall, wall, total


def parity_leg(rep, wl, net, step, state, seconds, max_jobs=0):
    """The exact job stream of one timed step against oracle/_ref (the reference's TLibCommon driven
    in TEncSearch order, TEncSearch.cpp:4529-4597) after the timed region: the step's jobs with its
    picture binding (FrameReplay._bind: originals, the four reconstructions, lambdas by POC) and the
    NN state the GPU had before the step (fme_nn_get_state), every xMotionEstimation output of the
    16-byte record (rcMv, ruiBits, ruiCost, NN class) compared, in job order, one host core, until
    `seconds` have passed (whole 20k-job chunks; the whole step when it fits)."""
    from nnfme import weights
    from nnfme.pipeline import ORG0, REFS
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Reference
    nn = wl["nn"]
    ref = Reference(use_hadamard=1, nn_mode=nn, fast_inter_mode=1, bit_depth=wl.get("bit_depth", 8))
    if nn == 1:
        ref.load_nn(weights.load_weights(wl["QP"]))
    elif nn == 2:
        ref.load_nn_net(net)
    F, P = rep.F, rep.P
    f0 = rep.first_frame(step)
    pool = rep.pool.numpy()
    for j in range(F):
        ref.set_picture(ORG0 + j, pool[(f0 + j) % P])
        ref.set_lambda(j, rep.lambda_of(f0 + j))
    for slot in range(F + REFS - 1):
        ref.set_picture(slot, pool[(f0 - REFS + slot) % P])
    keys_s = None
    if rep.kreqs is not None:
        # the step's removeHighFreq keys, built on the device inside the timed step
        # (fme_build_bipred_keys_device), restated on the host from the same bound pictures
        # (synth.bipred_keys, pinned to orc_bi_key / _ref's ref_bi_key by tests/test_pred_inter_b.py)
        from nnfme import synth
        tk = time.perf_counter()
        pics = {ORG0 + j: pool[(f0 + j) % P] for j in range(F)}
        pics.update({slot: pool[(f0 - REFS + slot) % P] for slot in range(F + REFS - 1)})
        ref.set_keys(synth.bipred_keys(rep.kreqs, pics, rep.key_count * F))
        keys_s = round(time.perf_counter() - tk, 2)
    ref.nn_set_state(state)
    jobs, gpu = rep.jobs, rep.results(step)
    n = len(jobs) if max_jobs <= 0 else min(max_jobs, len(jobs))
    fields = ("mv_x", "mv_y", "bits", "cost") + (("nn_class",) if nn else ())
    bad = {f: 0 for f in fields}
    mism = 0
    first = detail = None
    done, t0 = 0, time.perf_counter()
    while done < n and time.perf_counter() - t0 < seconds:
        e = min(done + 20000, n)
        if rep.rows is not None:   # row i of a refine call belongs to its job i
            ref.set_nn_inputs(rep.rows[done:e])
        r = ref.refine(jobs[done:e])
        g = gpu[done:e]
        m = np.zeros(e - done, bool)
        for f in fields:
            d = g[f] != r[f]
            bad[f] += int(d.sum())
            m |= d
        if first is None and m.any():
            i0 = int(np.flatnonzero(m)[0])
            first = done + i0
            detail = {"gpu": {f: int(g[f][i0]) for f in fields}, "ref": {f: int(r[f][i0]) for f in fields}}
        mism += int(m.sum())
        done = e
    out = {"jobs_checked": done, "mismatches": mism, "step": step, "of_step_jobs": len(jobs),
           "fields": list(fields), "per_field": bad, "first_mismatch": first,
           **({"first_mismatch_detail": detail} if detail else {}),
           "reference": "oracle/_ref (the reference's TLibCommon -O2, TEncSearch order restated; NN "
                        "restated scalar) with the step's pictures, lambdas and carried NN state",
           "seconds": round(time.perf_counter() - t0, 2)}
    if keys_s is not None:
        out["keys"] = f"{len(rep.kreqs)} bi-pred key blocks rebuilt on the host ({keys_s} s, synth.bipred_keys)"
    if nn == 2 and wl.get("engine"):
        out["note"] = ("MFMA engine: FMA-chain rounding, not bit-exact by construction (DESIGN.md §3); "
                       "a mismatch is a near-tie class")
        out["agreement"] = 1.0 - mism / max(done, 1)
        out["tolerance"] = ">= 0.995 of jobs equal (tests/test_deep_nn.py)"
    return out


def max_over_ranks(elapsed, dev, world, backend):
    """The slowest rank's time (torch.distributed all-reduce MAX)."""
    if world == 1:
        return elapsed
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if backend == "gloo":
        t = t.cpu()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_path_check(ctx, rep, wl, step, state, net, bd, m=2000):
    """A fresh context on the same device with the step's bindings (host pictures, lambdas) and
    state, refining the step's first m jobs through the host path: which of the replay and the
    reference it agrees with."""
    from nnfme.abi import MV_FIELDS
    from nnfme.pipeline import ORG0, REFS
    from nnfme.runtime import FmeContext
    c2 = FmeContext(device=ctx.device, use_hadamard=1, nn_mode=wl["nn"], qp=wl["QP"], fast_inter_mode=1,
                    max_jobs=m, net=net, nn_engine=wl.get("engine", 0), bit_depth=bd)
    pool = rep.pool.numpy()
    f0 = rep.first_frame(step)
    for j in range(rep.F):
        c2.set_picture(ORG0 + j, pool[(f0 + j) % rep.P])
        c2.set_lambda(j, rep.lambda_of(f0 + j))
    for slot in range(rep.F + REFS - 1):
        c2.set_picture(slot, pool[(f0 - REFS + slot) % rep.P])
    c2.nn_set_state(state)
    b = c2.refine_mv(rep.jobs[:m])
    g = rep.results(step)[:m]
    c2.close()
    return {"jobs": m, "host_vs_replay": {f: int((b[f] != g[f]).sum()) for f in MV_FIELDS},
            "job0": {"job": [int(v) for v in rep.jobs[0].tolist()], "replay": [int(v) for v in g[0].tolist()],
                     "host": [int(v) for v in b[0].tolist()]},
            "lambda": rep.lambda_of(f0), "first_frame": f0}


def mc_algorithmic_bytes(jobs):
    """Motion compensation, per PU and list: the luma 8-tap footprint (w+7)(h+7) and the two
    chroma 4-tap footprints (w/2+3)(h/2+3); per PU: the predicted samples (1.5 w h, written) and
    the 24-byte job."""
    w = jobs["w"].astype(np.int64)
    h = jobs["h"].astype(np.int64)
    lists = np.where((jobs["flags"] & 3) == 3, 2, 1)
    same = ((jobs["flags"] & 3) == 3) & (jobs["ref_id"][:, 0] == jobs["ref_id"][:, 1]) & \
        (jobs["mv"][:, 0, 0] == jobs["mv"][:, 1, 0]) & (jobs["mv"][:, 0, 1] == jobs["mv"][:, 1, 1])
    lists = np.where(same, 1, lists)
    ref = (w + 7) * (h + 7) + 2 * (w // 2 + 3) * (h // 2 + 3)
    return int((lists * ref + (3 * w * h) // 2 + 24).sum())


def drop_in_leg(dev, calls=300):
    """The TEncSearch-shaped single-PU entry points, one call per PU as a live encoder in drop-in
    mode would make them, timed from C++ (tests/cpp/test_hm_adapter.cpp --time-single through
    fme_hm::FracSearch): xPatternSearchFracDIF (fme_frac_dif_single: key and window staged in
    pinned, device-mapped host memory, one launch, one synchronisation) and NN_pred
    (fme_nn_pred_single); median wall microseconds per call.  Latency-bound by construction; the
    batch path is the throughput path."""
    import subprocess
    exe = os.path.join(ROOT, "hm16.9-nn_fme_amd", "host", "test_hm_adapter")
    if not os.path.exists(exe):
        return {"error": f"{exe} not built"}
    p = subprocess.run([exe, "--time-single", str(calls)], capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        return {"error": (p.stdout + p.stderr)[-400:]}
    out = json.loads(p.stdout.strip().splitlines()[-1])
    out["note"] = ("median wall time per synchronous call from C++ (fme_hm::FracSearch), caller's copies of "
                   "the key and the window into the staging block included")
    return out


def mc_leg(dev, stream, reps):
    """Motion compensation of one 1080p frame's decided PUs (TComPrediction::motionCompensation:
    luma 8-tap + 4:2:0 chroma 4-tap), device-resident jobs / pictures / planes; HIP events around
    each launch.  Two partitions: lowdelay_P (uni-pred, 4 refs) and a random-access-like one
    (50 % bi-pred)."""
    import torch
    from nnfme.runtime import FmeContext
    ctx = FmeContext(device=dev.index, nn_mode=0)
    for k, t in zip(range(4), (7, 6, 5, 4)):
        cb, cr = synth.synth_chroma(W, H, t)
        ctx.set_picture_yuv(k, synth.synth_luma(W, H, t), cb, cr)
    dy = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    dcb = torch.zeros((H // 2, W // 2), dtype=torch.uint8, device=dev)
    dcr = torch.zeros_like(dcb)
    out = {}
    for name, bi in (("ldp_uni", 0.0), ("ra_bi50", 0.5)):
        jobs = synth.make_mc_partition(np.random.default_rng(5), W, H, [0, 1, 2, 3], bi_frac=bi, mv_amp=64)
        dj = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)

        def run():
            ctx.motion_compensate_device(dj.data_ptr(), len(jobs), dy.data_ptr(), W, dcb.data_ptr(), dcr.data_ptr(),
                                         W // 2, W, H, stream.cuda_stream)
        for _ in range(3):
            run()
        ctx.set_profiling(True)
        ms = []
        for _ in range(reps):
            run()
            ms.append(ctx.mc_last_ms())
        ctx.set_profiling(False)
        t = float(np.mean(ms))
        nbytes = mc_algorithmic_bytes(jobs)
        gbs = nbytes / (t / 1e3) / 1e9
        out[name] = {"pus": int(len(jobs)), "bi_pred": int(((jobs["flags"] & 3) == 3).sum()),
                     "kernel_ms": t, "pu_per_s": len(jobs) / (t / 1e3),
                     "luma_mpix_per_s": W * H / (t / 1e3) / 1e6,
                     "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": nbytes,
                                  "kernel": "fme::k_mc"}}
    ctx.close()
    return out


def leg_pictures(n, bd):
    """The legs' synthetic 1080p pictures: 8-bit, or the same fields at bit depth 10 (main10)."""
    ts = (7, 6, 5, 4, 0, 3)[:n]
    return {k: (synth.synth_luma(W, H, t) if bd == 8 else synth.synth_luma_hbd(W, H, t, bit_depth=bd))
            for k, t in zip(range(n), ts)}


def tz_cpu_rate(jobs, ext, keys, pics, seconds, bd=8):
    """oracle/_ref integer search (the reference's TComRdCost distortion, xTZSearch restated) on one
    host core over a bounded prefix of the frame's jobs (HM order)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Reference
    ref = Reference(fast_inter_mode=1, bit_depth=bd)
    for k, v in pics.items():
        ref.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[QP]):
        ref.set_lambda(lid, lam)
    if keys is not None and keys.size:
        ref.set_keys(keys)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds and done < len(jobs):
        ref.integer_search(jobs[done:done + 5000], ext[done:done + 5000])
        done += min(5000, len(jobs) - done)
    return done / (time.perf_counter() - t0), done


def tz_roofline(jobs, ext, pics, kernel_ms, sample=20000, bd=8):
    """Work of the frame's integer searches, from the oracle's counters on the first `sample` jobs
    (HM order): points tested per search and distortion samples per point.  Each sample is three
    reference integer ops (SSE: difference, square, accumulate; SAD: difference, absolute value,
    accumulate).  The searches are bound by the latency of their dependent window loads (one per
    tested point), not by ALU or HBM: the fractions say how far from either roof they sit."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    orc = Oracle(nn_mode=0, fast_inter_mode=1, bit_depth=bd)
    for k, v in pics.items():
        orc.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[QP]):
        orc.set_lambda(lid, lam)
    m = min(sample, len(jobs))
    orc.tz_counters(reset=True)
    orc.integer_search(jobs[:m], ext[:m])
    points, samples = orc.tz_counters(reset=True)
    n = len(jobs)
    ops = 3.0 * samples / m * n
    achieved = ops / (kernel_ms * 1e-3) / 1e12
    return {"bound": "latency (dependent window loads)", "achieved": achieved, "peak": VALU_PEAK_TOPS,
            "unit": "Tops/s (int32 VALU lane-ops)", "frac": achieved / VALU_PEAK_TOPS,
            "points_per_search": points / m, "samples_per_point": samples / points,
            "reference_ops_per_frame": ops, "sample": f"oracle counters over the first {m} searches"}


def tz_leg(dev, stream, reps, cpu_seconds, bd=8):
    """Integer motion estimation (xTZSearch / bi-pred xPatternSearch) of one 1080p frame's jobs:
    510 CTUs x 423 calls x 4 refs in HM order, HBM-resident jobs, HIP events around the launches."""
    import torch
    from nnfme.runtime import FmeContext
    rng = np.random.default_rng(2024)
    pics = leg_pictures(5, bd)
    jobs, ext = synth.make_tz_jobs(rng, W, H, 423, 4, [0, 1, 2, 3], [0, 1, 2, 3])
    out = {"workload": f"{W}x{H} lowdelay_P QP{QP}: {len(jobs)} integer searches (xTZSearch from the AMVP "
                       f"predictor, 2Nx2N starts for half the non-2Nx2N PUs, SearchRange 64)"
                       + (f", bit depth {bd}" if bd != 8 else "")}
    if cpu_seconds > 0:
        rate, done = tz_cpu_rate(jobs, ext, None, pics, cpu_seconds, bd)
        out["cpu_baseline"] = {"value": rate, "unit": "PU/s", "cores": 1, "kind": "reference",
                               "sample": f"first {done} jobs of the frame on one host core (oracle/_ref)"}
    ctx = FmeContext(device=dev.index, nn_mode=0, fast_inter_mode=1, max_jobs=len(jobs), bit_depth=bd)
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[QP]):
        ctx.set_lambda(lid, lam)
    src = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    dj = src.clone()
    de = torch.from_numpy(np.ascontiguousarray(ext).view(np.uint8).copy()).to(dev)
    ds = torch.zeros(len(jobs), dtype=torch.int32, device=dev)

    def run():
        ctx.integer_search_device(dj.data_ptr(), de.data_ptr(), ds.data_ptr(), len(jobs), stream.cuda_stream)
    run()
    ctx.set_profiling(True)
    ms = []
    for _ in range(reps):
        dj.copy_(src)
        run()
        ms.append(ctx.integer_search_last_ms())
    ctx.set_profiling(False)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / reps
    t = float(np.median(ms))
    out.update({"kernel_ms": t, "pu_per_s_kernels": len(jobs) / (t / 1e3), "ms_per_frame": wall * 1e3,
                "pu_per_s": len(jobs) / wall, "kernels": "fme::k_tz_staged<4,8>, <8,4>, <8,8>: a workgroup per (kernel, reference, CTU) group with "
                             "its search area in LDS, one wave per PU, three concurrent launches (+ classify, scatter, "
                             "k_tz_pair_count / _scan / _scatter)" if bd == 8 else
                             "fme::k_tz_wave<4,8,-1,10>, <8,4,-1,10>, <8,8,-1,10>: one wave per PU on uint16 planes "
                             "(exact shifted SSE), three concurrent launches (+ classify, scatter)"})
    out["roofline"] = tz_roofline(jobs, ext, pics, t, bd=bd)
    if "cpu_baseline" in out:
        out["speedup_vs_cpu_1core"] = out["pu_per_s"] / out["cpu_baseline"]["value"]
    ctx.close()
    return out


def pred_inter_leg(dev, reps, cpu_seconds, bd=8):
    """predInterSearch's P-slice PU / reference loop over one 1080p P frame:
    every PU of a full 64 -> 8 CU quadtree with AMP in xCompressCU order, 4 references, the AMVP
    candidate lists of nnfme.synth.make_pu_requests, NN on (fme_pred_inter_p, host request arrays).
    Wall time per frame; the oracle's sequential loop (orc_pred_inter_p) on one host core over a
    bounded prefix of the same stream is the CPU baseline."""
    from nnfme import weights
    from nnfme.runtime import FmeContext
    rng = np.random.default_rng(2)
    pics = leg_pictures(6, bd)
    pic5 = pics.pop(5)
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0, 1, 2, 3], lambda_id=0, max_depth=3)
    nj = int(reqs["num_refs"].astype(np.int64).sum())
    out = {"workload": f"{W}x{H} P frame QP{QP}: {len(reqs)} PU requests = {nj} xMotionEstimation jobs (full 64->8 "
                       f"quadtree with AMP, 4 refs, AMVP template choice, xCheckBestMVP, reference choice, NN on)"
                       + (f", bit depth {bd}" if bd != 8 else "")}
    if cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle import Oracle
        orc = Oracle(nn_mode=1, qp=QP, fast_inter_mode=1, bit_depth=bd)
        orc.load_nn(weights.load_weights(QP))
        for k, v in pics.items():
            orc.set_picture(k, v)
        for lid, lam in enumerate(synth.LDP_LAMBDA[QP]):
            orc.set_lambda(lid, lam)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < cpu_seconds and done < len(reqs):
            orc.pred_inter_p(reqs[done:done + 1000])
            done += min(1000, len(reqs) - done)
        rate = done / (time.perf_counter() - t0)
        out["cpu_baseline"] = {"value": rate, "unit": "PU requests/s", "cores": 1, "kind": "port",
                               "sample": f"first {done} requests of the frame, sequential (oracle/fme_oracle.c)"}
    ctx = FmeContext(device=dev.index, nn_mode=1, qp=QP, fast_inter_mode=1, max_jobs=nj, bit_depth=bd)
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[QP]):
        ctx.set_lambda(lid, lam)
    ctx.pred_inter_p(reqs)
    ts = []
    for _ in range(reps):
        ctx.pred_inter_reset()
        t0 = time.perf_counter()
        ctx.pred_inter_p(reqs)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    out["phases_ms"] = {k: round(v, 3) for k, v in ctx.pred_inter_phases().items()}
    out.update({"ms_per_frame": t * 1e3, "requests_per_s": len(reqs) / t, "jobs_per_s": nj / t,
                "note": "bounded by the reference's m_integerMv2Nx2N chain: the bottom CTU row (56 rows) has no "
                        "depth-0 CU, so its 30 CTUs form one sequential chain of ~2,200 levels of 2Nx2N searches, "
                        "one k_tz_level launch each (DESIGN.md section 4)"})
    if "cpu_baseline" in out:
        out["speedup_vs_cpu_1core"] = out["requests_per_s"] / out["cpu_baseline"]["value"]
    # the B-slice producer on the same frame: L0 = {t-1, t-2}, L1 = {t+1, t+2} (fme_pred_inter_b)
    pics[5] = pic5
    ctx.set_picture(5, pics[5])
    reqs_b = synth.make_pu_requests_b(np.random.default_rng(3), W, H, org_id=4, l0=[(0, 1), (1, 2)],
                                      l1=[(5, -1), (2, -2)], lambda_id=0, max_depth=3)
    b = {"workload": f"{W}x{H} B frame: {len(reqs_b)} PU requests, 2 + 2 references, uni-pred over both lists, "
                     f"one bi-pred iteration (FEN 1) on device-built removeHighFreq keys, NN on"}
    if cpu_seconds > 0:
        orc.set_picture(5, pics[5])
        orc.pred_inter_reset()
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < cpu_seconds and done < len(reqs_b):
            e = min(done + 1000, len(reqs_b))
            while e < len(reqs_b) and reqs_b["part_idx"][e] != 0:   # a CU's PUs stay in one call
                e += 1
            orc.pred_inter_b(reqs_b[done:e])
            done = e
        b["cpu_baseline"] = {"value": done / (time.perf_counter() - t0), "unit": "PU requests/s", "cores": 1,
                             "kind": "port", "sample": f"first {done} requests, sequential (orc_pred_inter_b)"}
    ctx.pred_inter_b(reqs_b[:2000])
    ts = []
    for _ in range(reps):
        ctx.pred_inter_reset()
        t0 = time.perf_counter()
        res_b = ctx.pred_inter_b(reqs_b)
        ts.append(time.perf_counter() - t0)
    tb = float(np.median(ts))
    b["phases_ms"] = {k: round(v, 3) for k, v in ctx.pred_inter_phases().items()}
    b.update({"ms_per_frame": tb * 1e3, "requests_per_s": len(reqs_b) / tb,
              "inter_dir_counts": {"L0": int((res_b["inter_dir"] == 1).sum()), "L1": int((res_b["inter_dir"] == 2).sum()),
                                   "bi": int((res_b["inter_dir"] == 3).sum())}})
    if "cpu_baseline" in b:
        b["speedup_vs_cpu_1core"] = b["requests_per_s"] / b["cpu_baseline"]["value"]
    out["b_slice"] = b
    ctx.close()
    return out


def read_pmc_traffic(workload):
    """HBM bytes per main search launch from the committed rocprofv3 PMC summary of this workload
    (profiles/pmc_traffic.json, regenerated by tools/gpu_profile.sh from the current tree)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if workload != "c3_qp22" or not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        return d.get("bytes_per_launch"), d.get("source")
    except Exception:
        return None, None


def write_timeline(path, rep, k0, k1, elapsed_s):
    """The PCIe pass's timeline (FrameReplay timeline=True): per step, ms from the timed region's
    start to the start / end of its H2D uploads (copy stream), its batch (compute stream) and its
    results download (copy stream), then the per-step spans and the overlap of copies with batches."""
    rows = rep.timeline_rows(k0, k1)
    with open(path, "w") as f:
        f.write("# FrameReplay PCIe pass, HIP timing events on the copy and compute streams (ms from the first "
                "timed issue); wall %.3f ms for %d steps\n" % (elapsed_s * 1e3, k1 - k0))
        f.write("# step    up0      up1  | b0       b1   |  d0       d1   | up_ms  batch_ms  down_ms  batch_gap_ms\n")
        prev_b1 = None
        for r in rows:
            gap = (r["b0"] - prev_b1) if prev_b1 is not None else 0.0
            f.write("%5d %8.3f %8.3f | %8.3f %8.3f | %8.3f %8.3f | %6.3f %8.3f %8.3f %8.3f\n" % (
                r["step"], r["up0"], r["up1"], r["b0"], r["b1"], r["d0"], r["d1"], r["up1"] - r["up0"],
                r["b1"] - r["b0"], r["d1"] - r["d0"], gap))
            prev_b1 = r["b1"]
        span = rows[-1]["d1"] - rows[0]["up0"]
        busy = sum(r["b1"] - r["b0"] for r in rows)
        f.write("# first upload start -> last download end %.3f ms; batches busy %.3f ms (%.1f %%); "
                "mean batch %.3f ms, mean upload %.3f ms, mean download %.3f ms\n" % (
                    span, busy, 100 * busy / span, busy / len(rows),
                    sum(r["up1"] - r["up0"] for r in rows) / len(rows),
                    sum(r["d1"] - r["d0"] for r in rows) / len(rows)))


def frame_lambda(wl, f):
    """Lambda of frame f: lowdelay_P by POC % 4 (cfg Frame1-4), random access by GOP-8 entry."""
    if wl["gop"] == "ra":
        return synth.ra_lambda(wl["QP"], f % 8)
    return synth.LDP_LAMBDA[wl["QP"]][(f + 1) % 4]


def nn_tail_roofline(wl, tm, n):
    """configs[4]: the NN tail of nn_mode 2 as a batched GEMM (FLOPs of the hidden and output
    layers per job) over its measured time, against the dense MFMA peak of its dtype."""
    from nnfme import weights
    net = weights.case_net(wl["net"])
    fan = 17 if net.embedding else 9
    flops = 0
    for wdt in net.widths:
        flops += 2 * fan * wdt
        fan = wdt
    flops += 2 * fan * 49
    t = tm["nn_tail"] / 1e3
    achieved = n * flops / t / 1e12
    f64 = net.precision == weights.F64
    # dense matrix peaks: f32 157.3 TF (MI355X_MICROARCH.md); f64 78.6 TF (AMD MI355X spec sheet)
    peak = 78.6 if f64 else 157.3
    return {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
            "kernel": "fme::k_nn_deep_tail<%s, %d, %s, %s>" % ("double" if f64 else "float", len(net.widths),
                                                              "emb" if net.embedding else "noemb",
                                                              "mfma" if wl.get("engine") else "exact"),
            "flops_per_job": flops, "kernel_ms": tm["nn_tail"],
            "dtype": "f64" if f64 else "f32"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-mc", action="store_true", help="skip the motion-compensation leg")
    ap.add_argument("--no-tz", action="store_true", help="skip the integer-search leg")
    ap.add_argument("--no-pi", action="store_true", help="skip the predInterSearch producer leg")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3_qp22",
                    help="BASELINE.json config to run (default: the headline, configs[2] at QP22)")
    ap.add_argument("--jobs", choices=("ctu", "uniform"), default="ctu",
                    help="job stream: HM CTU order (default) or uniformly scattered PUs (stress)")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="cores for cpu_baseline_all_cores (0: all available, at most 16; -1: skip)")
    ap.add_argument("--dist-backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--parity-seconds", type=float, default=30.0,
                    help="bound of the after-run check of one timed step against oracle/_ref (0: skip)")
    ap.add_argument("--download-engine", choices=("kernel", "blit", "sdma"), default="sdma",
                    help="results download: a copy engine (hipMemcpyDeviceToDeviceNoCU into the pinned rows, the "
                         "default: no CUs), the library's few-workgroup copy kernel (fme_download_device) or "
                         "hipMemcpyAsync (a ROCclr blit kernel of hundreds of workgroups beside the search)")
    ap.add_argument("--download-wgs", type=int, default=8, help="workgroups of the download kernel")
    ap.add_argument("--copy-streams", type=int, choices=(1, 2), default=1,
                    help="1: uploads and downloads in series on one copy stream (default); 2: downloads on their "
                         "own stream (round 5's layout)")
    ap.add_argument("--slots", type=int, default=3, help="job / result buffer ring depth of the replay")
    ap.add_argument("--max-ahead", type=int, default=4,
                    help="steps the host may queue ahead of the device (0: unbounded)")
    ap.add_argument("--timeline", default=None,
                    help="write the PCIe pass's per-step copy / batch timeline (HIP timing events) to this file")
    ap.add_argument("--no-warm-engines", action="store_true",
                    help="skip the SDMA engine warm-up before the pipeline (fme_warm_copy_engines; A/B)")
    ap.add_argument("--lazy-events", action="store_true",
                    help="let torch create each step's events at their first record inside the timed region")
    ap.add_argument("--no-packed", action="store_true",
                    help="upload 32-byte fme_job rows instead of 16-byte fme_job_packed rows")
    ap.add_argument("--no-pcie", action="store_true",
                    help="profiling runs: skip the PCIe-inclusive pass (its copies would overlap the kernels); "
                         "`value` is then the HBM-resident rate and says so")
    ap.add_argument("--search-reserve", type=int, default=0,
                    help="resident search workgroups left free for the download kernel (fme_set_search_reserve)")
    ap.add_argument("--download", choices=("deferred", "immediate"), default=None,
                    help="results download of step k: once step k+1's search runs (deferred) or right after "
                         "step k (immediate); default: the workload's measured choice (DESIGN.md section 5)")
    args = ap.parse_args()
    crash = None
    if os.environ.get("FME_CRASH_TRACE"):   # diagnostic: native stack of a fault (tools/probes/crash_trace.c)
        import ctypes
        import faulthandler
        faulthandler.enable()
        crash = ctypes.CDLL(os.path.join(ROOT, "tools", "probes", "libcrash_trace.so"))

    global W, H, QP, METRIC
    wl = WORKLOADS[args.workload]
    W, H, QP = wl["W"], wl["H"], wl["QP"]
    NN, CALLS, BIPRED, WDESC, FPS = wl["nn"], wl["calls"], wl["bipred"], wl["desc"], wl["frames"]
    BD = wl.get("bit_depth", 8)

    def picture(t):   # one synthetic luma plane (uint16 main10 samples at bit depth 10)
        return synth.synth_luma(W, H, t) if BD == 8 else synth.synth_luma_hbd(W, H, t, bit_depth=BD)
    if args.workload != "c3_qp22":
        METRIC = f"sub-pel PU refinements/sec @ {args.workload}: {WDESC.split(',')[0]}; bit-exact MV/SATD vs HM"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # ---- inputs (untimed): one frame's jobs in HM order -----------------------------------------
    RING = wl.get("inputs") == "ring"
    if RING:   # configs[4] on the backups' input path: the frame's integer searches come first
        jobs, tz_ext = synth.make_tz_jobs(np.random.default_rng(1000), W, H, CALLS, 4, [0, 1, 2, 3], [0])
        tz_ext["flags"] |= TZ_RING
    else:
        jobs = make_frame_jobs(1000, args.jobs, CALLS, BIPRED)
    n1 = len(jobs)
    keys = key_reqs = None
    if BIPRED > 0:   # bi-pred keys (removeHighFreq of the other list's prediction), resident with the jobs
        kpics = {k: synth.synth_luma(W, H, t) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
        key_reqs, key_count = synth.make_bipred_key_reqs(np.random.default_rng(77), jobs, 4, [0, 1, 2, 3])
        keys = synth.bipred_keys(key_reqs, kpics, key_count)   # the CPU baseline's copy (same values)

    # ---- CPU baselines first, before anything touches the GPU (fork-safe) -------------------
    cpu = {}
    _CPU["nn"], _CPU["keys"], _CPU["bd"] = min(NN, 1), keys, BD
    if rank == 0 and world == 1 and not args.no_cpu_baseline and RING:
        pics = {k: synth.synth_luma(W, H, t) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
        rjobs, rrows = ring_inputs_cpu(jobs, tz_ext, pics, 20000)
        rate, dt, done = cpu_baseline_ring(rjobs, rrows, wl["net"], pics, args.cpu_seconds)
        cpu["cpu_baseline"] = {
            "value": rate, "unit": "PU/s", "cores": 1, "kind": "reference",
            "sample": f"{done} jobs ({done // len(rjobs)} passes over the first {len(rjobs)} jobs of the frame, HM "
                      f"order) on one host core, {dt:.1f} s; oracle/_ref = the reference's TLibCommon -O2 in "
                      f"TEncSearch order with the backup's net restated scalar (double / float, its loop order) on "
                      f"the backup's NN inputs (their integer searches by the oracle, untimed)",
        }
    elif rank == 0 and world == 1 and not args.no_cpu_baseline:
        pics = {k: picture(t) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
        rate, dt, done = cpu_baseline(jobs, pics, args.cpu_seconds)
        cpu["cpu_baseline"] = {
            "value": rate, "unit": "PU/s", "cores": 1, "kind": "reference",
            "sample": f"{done} jobs ({done / n1:.2f} passes over one {args.workload} frame's jobs, "
                      f"HM order) on one host core, {dt:.1f} s; oracle/_ref = the reference's "
                      f"TLibCommon (interpolation, RdCost) -O2 driven in TEncSearch order, NN "
                      f"restated scalar" + (" (the 2-layer master net: the deeper nets' backups do not "
                                            "build)" if NN == 2 else ""),
        }
        avail = len(os.sched_getaffinity(0))
        cores = min(16, avail) if args.cpu_cores == 0 else args.cpu_cores
        if cores > 1:
            rate_all, wall, total = cpu_baseline_all_cores(jobs, pics, rate, args.cpu_seconds * 0.75, cores)
            cpu["cpu_baseline_all_cores"] = {
                "value": rate_all, "unit": "PU/s", "cores": cores, "kind": "reference",
                "sample": f"{total} jobs, one stream per core over 1/{cores} slices of the frame, "
                          f"{wall:.1f} s wall",
            }

    import torch
    import torch.distributed as dist
    from nnfme import weights
    from nnfme.pipeline import FrameReplay
    from nnfme.runtime import FmeContext

    ndev = torch.cuda.device_count()
    dev_index = local % max(ndev, 1)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_index)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(args.dist_backend)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)

    net = weights.case_net(wl["net"]) if NN == 2 else None
    ctx = FmeContext(device=dev_index, use_hadamard=1, nn_mode=NN, qp=QP, fast_inter_mode=1,
                     max_jobs=n1 * FPS, net=net, nn_engine=wl.get("engine", 0), bit_depth=BD)

    nn_rows = None
    if RING:   # untimed: the frame's integer searches on the GPU, with the backups' square + ring
        for k, t in zip(range(5), (7, 6, 5, 4, 0)):
            ctx.set_picture(k, synth.synth_luma(W, H, t))
        ctx.set_lambda(0, frame_lambda(wl, 0))
        jobs, _, nn_rows = ctx.integer_search_ring(jobs, tz_ext)
        jobs["flags"] = np.where((jobs["flags"] & JOB_BIPRED) == 0, JOB_NN_IN, jobs["flags"]).astype(np.uint8)

    # synthetic frame pool (the trace's originals / reconstructions): frame g -> pool[g % 8]
    pool = np.stack([picture(t) for t in range(8)])
    steps_total = args.warmup + args.steps
    defer = (args.download or wl.get("download", "deferred")) == "deferred"
    if args.no_pcie and world > 1:
        # the sharded resident pass re-runs each step's carried-state prefix, whose length the PCIe
        # pass measures (FrameReplay.finish)
        raise SystemExit("--no-pcie needs one rank (the NN-state fix-up length comes from the PCIe pass)")
    # bi-pred keys (configs[3]): every step builds its frame's removeHighFreq keys on the device from
    # that frame's pictures (fme_build_bipred_keys_device, k_bi_key) inside the timed step
    rep = FrameReplay(ctx, jobs, pool, lambda f: frame_lambda(wl, f), steps_total, frames_per_step=FPS,
                      world=world, rank=rank, device=dev, defer_download=defer,
                      key_reqs=key_reqs, key_count=len(keys) if keys is not None else 0, nn_rows=nn_rows,
                      download_engine=args.download_engine, download_wgs=args.download_wgs,
                      search_reserve=args.search_reserve, packed=not args.no_packed,
                      copy_streams=args.copy_streams, slots=args.slots, max_ahead=args.max_ahead,
                      precreate_events=not args.lazy_events, warm_engines=not args.no_warm_engines,
                      timeline=args.timeline is not None)
    n = rep.n
    rep.prime()

    for s in range(args.warmup):
        rep.issue(s, prefetch=s + 1 < args.warmup)   # the first timed step uploads its own inputs
    rep.drain()
    # the NN_pred state the first timed step starts from (untimed), for the after-run checks
    state0 = ctx.nn_get_state() if world == 1 else None

    # ---- `value`: SURVEY.md §8(d)'s timing, from the first H2D of job descriptors to the last D2H
    # of results.  Per step: H2D of the jobs (16-byte packed rows + one key base per 64 jobs), the
    # frames' originals and one reconstructed reference per frame (RCCL point-to-point to the ranks
    # that reference it when sharded), refine, D2H of the 16-byte fme_mv_result per job; all copies
    # in series on one copy stream beside the batch stream; the NN-state chain fix-up when sharded.
    # The interpreter's garbage collector is off inside the timed loops (a C++ host has none). ----
    import gc
    from nnfme import pipeline as fpipe
    fixed_pcie, value_pcie, elapsed_pcie, snap = 0, None, None, None
    if args.no_pcie:   # (profiling runs) the timed steps' inputs staged into HBM untimed instead
        for s in range(args.warmup, steps_total):
            rep._upload(s)
        rep.s_copy.synchronize()
    else:
        if world > 1:
            dist.barrier()
        gc.collect()
        gc.disable()
        rep.host_ms, rep.host_seg = [], []
        fpipe.SLOW_CALLS.clear()
        torch.cuda.synchronize(dev)
        rep.timeline_start()
        t0 = time.perf_counter()
        for s in range(args.warmup, steps_total):
            rep.issue(s)
        fixed_pcie = rep.finish(first_step=args.warmup)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed_pcie = max_over_ranks(time.perf_counter() - t0, dev, world, args.dist_backend)
        gc.enable()
        rep.check_status(args.warmup)   # no timed step may have been rejected on the device
        if args.timeline:
            write_timeline(args.timeline, rep, args.warmup, steps_total, elapsed_pcie)
        snap = rep.results(args.warmup).copy() if args.parity_seconds > 0 else None
        value_pcie = world * n * args.steps / elapsed_pcie
    host_ms = np.asarray(rep.host_ms, dtype=np.float64)

    parity = None
    if rank == 0 and world == 1 and args.parity_seconds > 0 and not args.no_pcie:
        parity = parity_leg(rep, wl, net, args.warmup, state0, args.parity_seconds)
        mfma = wl["nn"] == 2 and bool(wl.get("engine"))
        if parity.get("mismatches") and not mfma and rep.rows is None:   # localise: the host path, same bindings
            parity["host_path_check"] = host_path_check(ctx, rep, wl, args.warmup, state0, net, BD)
            now = rep.results(args.warmup)
            parity["rows_changed_since_timed_region"] = int((now != snap).sum())

    # ---- `resident`: the same steps with every input already resident in HBM (the pass above
    # uploaded and exchanged each step's pictures, jobs, key requests and NN rows) and the results
    # left there; per step: bind, device-built keys (configs[3]), refine; the NN-state chain fix-up
    # on the device when sharded.  At one rank its timed steps start from the PCIe pass's first NN
    # state, so every step's results must equal the PCIe pass's bit for bit (checked below). ----
    rep.resident_outputs(0, steps_total)
    prefix = rep.last_prefix if world > 1 else 0
    for s in range(args.warmup):
        rep.issue_resident(s)
    if state0 is not None:
        ctx.nn_set_state(state0)   # stream-ordered: applied before the first timed batch
    torch.cuda.synchronize(dev)
    ctx.set_profiling(True)
    ctx.accumulated_timings(reset=True)
    if world > 1:
        dist.barrier()
    gc.collect()
    gc.disable()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.warmup, steps_total):
        rep.issue_resident(s)
    fixed = rep.finish_resident(args.warmup, steps_total, prefix)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev, world, args.dist_backend)
    gc.enable()
    nb, acc = ctx.accumulated_timings(reset=True)
    ctx.set_profiling(False)
    tm = {k: v / max(nb, 1) for k, v in acc.items()}
    value_res = world * n * args.steps / elapsed
    from nnfme.abi import RES_REJECTED
    res_vs_pcie = None
    if not args.no_pcie:
        diff_steps = []
        for s in range(args.warmup, steps_total):
            got = rep.r_out[s].cpu().numpy().view(MV_RESULT_DTYPE)
            if not np.array_equal(got, rep.results(s)):
                diff_steps.append(s)
        res_vs_pcie = {"steps_compared": args.steps, "steps_differing": diff_steps,
                       "equal": not diff_steps, "rank": rank,
                       "how": "every timed step's 16-byte records of the resident pass against the PCIe pass's "
                              "downloaded rows, same NN start state" + (" (after the carried-state fix-up)"
                                                                         if world > 1 else "")}
        if diff_steps:
            raise RuntimeError(f"resident pass differs from the PCIe pass on steps {diff_steps}")
    else:
        last = rep.r_out[steps_total - 1].cpu().numpy().view(MV_RESULT_DTYPE)
        if np.any(last["status"] & RES_REJECTED):
            raise RuntimeError("a resident step's batch was rejected on the device")
    if args.no_pcie:
        value, ms_step, value_kind = value_res, elapsed / args.steps * 1e3, "resident (--no-pcie profiling run)"
    else:
        value, ms_step, value_kind = value_pcie, elapsed_pcie / args.steps * 1e3, "pcie_inclusive (SURVEY.md §8(d))"
    resident = {"value": value_res, "unit": "PU/s", "ms_per_step": elapsed / args.steps * 1e3,
                "timed": "per step, inputs resident in HBM: bind the step's pictures and lambdas, build its bi-pred "
                         "keys on the device (configs[3]), refine the frame's jobs into a device result buffer"
                         + ("; NN-state chain fix-up on the device included" if world > 1 else ""),
                **({"of_resident_pcie": value_pcie / value_res} if value_pcie else {}),
                **({"equals_pcie_pass": res_vs_pcie} if res_vs_pcie else {})}
    d2h = n * MV_RESULT_DTYPE.itemsize
    pcie = None if args.no_pcie else {
        "timed": "from the first H2D of job descriptors to the last D2H of results (SURVEY.md §8(d)): per step H2D "
                 "of the jobs, the frames' originals and one reconstructed reference per frame (when sharded: "
                 "RCCL point-to-point sends to the <= 3 other ranks whose frames reference it), refine, D2H of "
                 "the 16-byte fme_mv_result per job" + ("; NN-state chain fix-up included" if world > 1 else ""),
        "jobs_upload": ("fme_job_packed (16 B per job + 4 B per 64 jobs), unpacked on the device by "
                        "fme_refine_mv_packed_device" if rep.packed else
                        "fme_job (32 B per job)" + (f"; packing refused: {rep.packed_reason}"
                                                    if rep.packed_reason else "")),
        "h2d_bytes_per_step": rep.h2d_bytes_per_step(), "d2h_bytes_per_step": d2h,
        "copies": (f"one copy stream, in series: H2D(k+1) then D2H(k-1) once step k's search runs; ring of "
                   f"{rep.R} job / result slots" if args.copy_streams == 1 else
                   "uploads and downloads on separate copy streams"),
        "download": (f"fme_download_device ({args.download_wgs} workgroups of 256 lanes, non-temporal "
                     f"16-byte stores into the pinned rows)" if args.download_engine == "kernel"
                     else "hipMemcpyAsync DeviceToDeviceNoCU into the pinned rows (copy engine, no CUs)"
                     if args.download_engine == "sdma" else "hipMemcpyAsync (ROCclr blit kernel)"),
        "search_reserve": args.search_reserve,
        "max_ahead": args.max_ahead,
        "copy_engines_warmed": rep.engines_warmed,
        "host_issue_ms": {"median": float(np.median(host_ms)), "max": float(host_ms.max()),
                          "sum": float(host_ms.sum()), "per_step": [round(float(v), 3) for v in host_ms],
                          "slowest_step_parts": dict(zip(rep.host_seg_names, rep.host_seg[int(host_ms.argmax())]))}
        if host_ms.size else None,
        "slow_host_calls": list(fpipe.SLOW_CALLS)[:40],
        "gc": "off inside the timed loops"}
    if world > 1 and pcie:
        pcie["nn_state_fixup_jobs_rank0"] = int(fixed_pcie)

    mc = mc_leg(dev, torch.cuda.current_stream(dev), reps=max(5, args.steps // 2)) \
        if rank == 0 and not args.no_mc and W == 1920 and NN != 2 and BD == 8 else None
    single = drop_in_leg(dev) if rank == 0 and not args.no_mc and W == 1920 and NN == 1 and BD == 8 else None
    pi = None
    if rank == 0 and not args.no_pi and W == 1920 and world == 1 and NN == 1:
        pi = pred_inter_leg(dev, reps=2, cpu_seconds=0.0 if args.no_cpu_baseline else 4.0, bd=BD)
    tz = None
    if rank == 0 and not args.no_tz and W == 1920 and world == 1 and NN == 1:
        tz = tz_leg(dev, torch.cuda.current_stream(dev), reps=max(3, args.steps // 4),
                    cpu_seconds=0.0 if args.no_cpu_baseline else 6.0, bd=BD)

    if rank == 0:
        gj = rep.jobs
        small_jobs = gj[main_kernel_mask(ctx, gj)]
        bytes_small = algorithmic_bytes(small_jobs, 2 if BD > 8 else 1)
        small_s = tm["search_main"] / 1e3
        ops_small = algorithmic_ops(small_jobs)
        valu = ops_small / small_s / 1e12
        gbs = bytes_small / small_s / 1e9
        traffic, traffic_src = read_pmc_traffic(args.workload)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "PU/s",
            "value_kind": value_kind,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "bit_depth": BD,
            "dtype": "int16/int32 (NN f32)" if NN != 2 else
                     "int16/int32 (NN %s)" % ("f64" if net.precision == weights.F64 else "f32"),
            "data": "synthetic (SURVEY.md §8(d) YUV generator + PU-size mix; reference per-QP "
                    "NN weights, no random init)",
            "config": {"workload": WDESC,
                       "workload_id": args.workload,
                       **({"deviation": wl["deviation"]} if "deviation" in wl else {}),
                       **({"nn_net": wl["net"], "nn_inputs": "the backups' own input path (Backups/4:659, "
                           "4343-4359, 4868-4878; Backups/15:1257, 4935-4962, 5440-5445): every xTZSearchHelp "
                           "distortion pushed, final square + distance-2 ring, C = least push before the square, "
                           "U1..U4/V/H = the next 8 pushes, per-call memset; jobs and rows from "
                           "fme_integer_search_ring on the first frame's pictures (untimed), replayed every step "
                           "with their 36-byte input rows uploaded per step"} if NN == 2 else {}),
                       "job_stream": args.jobs,
                       "frames_per_step": FPS,
                       "jobs_per_step_per_gpu": n, "parallelism": f"frame-sharded x{world}",
                       # what torch.distributed actually ran (None: one process, no process group)
                       "dist_backend": dist.get_backend() if dist.is_initialized() else None,
                       "pg_world_size": dist.get_world_size() if dist.is_initialized() else 1,
                       "timed": (pcie or resident)["timed"]},
            "roofline": {
                "bound": "valu",
                "achieved": valu,
                "peak": VALU_PEAK_TOPS,
                "unit": "Tops/s (int32 VALU lane-ops)",
                "frac": valu / VALU_PEAK_TOPS,
                "traffic": traffic,
                "kernel": "main search phase: fme::k_search_lane (EMI + FracDIF, every PU shape, one "
                          "persistent launch per batch)" if BD == 8 else
                          "main search phase at bit depth 10: fme::k_search_lane10 (EMI + FracDIF on int16 samples, "
                          "one lane per 4x8 / 4x4 unit, every PU shape, one persistent launch per batch)",
                "kernel_jobs": int(len(small_jobs)),
                "algorithmic_ops_per_launch": ops_small,
                "algorithmic_bytes_per_launch": bytes_small,
                "kernel_ms": tm["search_main"],
                "profiled_batches": nb,
                "note": "integer-VALU bound (~97 reference int ops per algorithmic byte, SURVEY.md §8(d)); "
                        "achieved counts the reference's arithmetic, not the instructions issued",
                "traffic_source": traffic_src,
                "batch_kernel_ms": tm,
                "hbm": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": gbs / HBM_PEAK_GBS,
                        "traffic_frac_of_algorithmic": (traffic / bytes_small) if traffic else None},
            },
        }
        if NN == 2:
            out["nn_tail_roofline"] = nn_tail_roofline(wl, tm, n)
        out.update(cpu)
        if "cpu_baseline" in cpu:
            out["speedup_vs_cpu_1core"] = value / cpu["cpu_baseline"]["value"]
        if "cpu_baseline_all_cores" in cpu:
            out["speedup_vs_cpu_all_cores"] = value / cpu["cpu_baseline_all_cores"]["value"]
        if pcie:
            out["pcie_inclusive"] = pcie
        out["resident"] = resident
        if parity:
            out["parity"] = parity
        if world > 1:
            out["nn_state_fixup_jobs_rank0"] = int(fixed)
        if mc:
            out["motion_compensation"] = mc
        if single:
            out["drop_in_single_pu"] = single
        if tz:
            out["integer_search"] = tz
        if pi:
            out["pred_inter_search"] = pi
        print(json.dumps(out), flush=True)

    # every HIP resource of the run released here, before interpreter exit (no finaliser of ours
    # runs after the HIP runtime or a profiler's exit handlers)
    rep.close()
    del rep
    ctx.close()
    torch.cuda.synchronize(dev)
    # pinned host blocks go back now, not from a static destructor after the HIP runtime (or a
    # profiler's exit handlers) has gone: the exit-time SIGSEGV in __cxa_finalize under
    # rocprofv3 --memory-copy-trace (round 5's gpurun_out/tlc1.log)
    import gc as _gc
    _gc.collect()
    torch.cuda.empty_cache()
    torch._C._host_emptyCache()
    if world > 1:
        dist.destroy_process_group()
    if crash is not None:
        crash.crash_trace_install()   # ahead of any handler a profiler installed since start-up
    return 0


if __name__ == "__main__":
    sys.exit(main())
