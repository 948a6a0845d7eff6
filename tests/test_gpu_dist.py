"""Frame sharding through the HIP path (nnfme.pipeline.FrameReplay over FmeContext): two ranks
(gloo, both on cuda:0 of the one-GPU box) replay alternate frames from fresh NN states, exchange
the per-frame end states and re-run each frame's carried-state prefix; the merged results must
equal a one-rank sequential replay bit for bit, status bits included.  The frames open with jobs
whose EMI step is clipped to a zero range (no pushes) and a bi-pred job, so every frame after
the first really reads its carry-in."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

W, H, STEPS = 208, 120, 4


def _jobs():
    from nnfme import synth
    rng = np.random.default_rng(5)
    jobs = synth.make_ctu_jobs(rng, W, H, 60, 4, [0, 1, 2, 3], [0])
    for i in range(3):   # zero search range -> no EMI pushes
        jobs["lt_x"][i] = jobs["rb_x"][i] = jobs["mv_x"][i]
        jobs["lt_y"][i] = jobs["rb_y"][i] = jobs["mv_y"][i]
    jobs["flags"][3] = 2   # bi-pred, key = the original (no EMI, reuses the carried state)
    return jobs


def _replay(world, rank, frames_per_step, group=None):
    import torch
    from nnfme import synth
    from nnfme.pipeline import FrameReplay
    from nnfme.runtime import FmeContext
    ctx = FmeContext(device=0, use_hadamard=1, nn_mode=1, qp=22, fast_inter_mode=1)
    pool = np.stack([synth.synth_luma(W, H, t) for t in range(8)])
    lam = lambda f: synth.LDP_LAMBDA[22][(f + 1) % 4]   # noqa: E731
    steps = STEPS * 2 // world
    rep = FrameReplay(ctx, _jobs(), pool, lam, steps, frames_per_step=frames_per_step, world=world, rank=rank,
                      device=torch.device("cuda", 0), group=group)
    rep.prime()
    for k in range(steps):
        rep.issue(k)
    fixed = rep.finish()
    out = {k * world + rank: rep.results(k).copy() for k in range(steps)}
    ctx.close()
    return out, fixed


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, fps, out_dir):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out, fixed = _replay(world, rank, fps)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), fixed=fixed, **{str(k): v for k, v in out.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fps", [1, 3])
def test_two_rank_replay_equals_sequential(tmp_path, fps):
    import torch.multiprocessing as mp
    from nnfme.abi import MV_FIELDS, MV_RESULT_DTYPE
    mp.spawn(_rank_main, args=(2, _free_port(), fps, str(tmp_path)), nprocs=2, join=True)
    want, _ = _replay(1, 0, fps)
    got, fixed = {}, 0
    for r in range(2):
        z = np.load(tmp_path / f"r{r}.npz")
        fixed += int(z["fixed"])
        for k in z.files:
            if k != "fixed":
                got[int(k)] = z[k].view(MV_RESULT_DTYPE)
    assert sorted(got) == sorted(want)
    assert fixed > 0   # the carry-in really mattered
    for b in sorted(want):
        for f in MV_FIELDS:
            assert np.array_equal(got[b][f], want[b][f]), (b, f, np.flatnonzero(got[b][f] != want[b][f])[:5])
