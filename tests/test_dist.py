"""Frame sharding (nnfme.dist) on CPU: the NN carried-state chaining against a sequential run,
and a world_size-2 gloo run of the multi-rank path (picture broadcast ring, per-rank frames,
all_gather of end states, carry-in fix-up, results gathered to rank 0).  The oracle stands in
for the per-rank engine (test infrastructure; the GPU engine has the same host interface)."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))

from nnfme import dist as fdist  # noqa: E402
from nnfme import synth, weights  # noqa: E402
from nnfme.abi import RES_NN_UNINIT, compare_results  # noqa: E402

W, H, NF, REFS = 208, 120, 6, 2


def _frames():
    """NF frames of jobs; frame f uses pictures f (org) and f-1, f-2 (refs) of a ring.
    Every frame starts with jobs whose EMI step is clipped to a zero search range (no pushes)
    and a bi-pred job, so the frame's first NN reads come from the carried state."""
    rng = np.random.default_rng(5)
    frames = []
    for f in range(NF):
        jobs = synth.make_jobs(rng, W, H, 300, 0, [1, 2], [0], bipred_frac=0.0)
        for i in range(3):   # zero search range -> no EMI pushes
            jobs["lt_x"][i] = jobs["rb_x"][i] = jobs["mv_x"][i]
            jobs["lt_y"][i] = jobs["rb_y"][i] = jobs["mv_y"][i]
        jobs["flags"][3] = 2   # bi-pred (no EMI, reuses the previous call's state)
        jobs["key_offset"][3] = -2
        frames.append(jobs)
    return frames


def _pictures():
    return [synth.synth_luma(W, H, t) for t in range(NF + REFS)]


def _engine(pics, f, keys=None):
    from oracle import Oracle
    o = Oracle(use_hadamard=1, nn_mode=1, qp=22, fast_inter_mode=1)
    o.load_nn(weights.load_weights(22))
    o.set_lambda(0, synth.LDP_LAMBDA[22][1])
    _bind(o, pics, f)
    return o


def _bind(o, pics, f):
    o.set_picture(0, pics[f + REFS])       # org of frame f
    o.set_picture(1, pics[f + REFS - 1])   # refs
    o.set_picture(2, pics[f + REFS - 2])


def _keys(frames, pics):
    rng = np.random.default_rng(9)
    out = []
    for f, jobs in enumerate(frames):
        d = {k: pics[f + REFS - (0 if k == 0 else k)] for k in (0, 1, 2)}
        out.append(synth.make_bipred_keys(rng, jobs, d))
    return out


def _sequential(frames, pics, keys):
    o = _engine(pics, 0)
    res = []
    for f, jobs in enumerate(frames):
        _bind(o, pics, f)
        o.set_keys(keys[f])
        res.append(o.refine(jobs))
    return res


def _sharded_frame(pics, frames, keys, f):
    o = _engine(pics, f)
    o.set_keys(keys[f])
    o.nn_reset()
    r = o.refine(frames[f])
    return r, o.nn_get_state()


def test_chain_states_reproduce_sequential_run():
    pics = _pictures()
    frames = _frames()
    keys = _keys(frames, pics)
    want = _sequential(frames, pics, keys)
    per = [_sharded_frame(pics, frames, keys, f) for f in range(NF)]
    carries, _ = fdist.chain_states([s for _, s in per])
    touched = 0
    for f in range(NF):
        r, _ = per[f]
        if f > 0:
            touched += fdist.uninit_prefix(r) > 0
        o = _engine(pics, f)
        o.set_keys(keys[f])
        fixed = fdist.fix_frame_prefix(o, frames[f], r, carries[f])
        n_bad, first, counts = compare_results(fixed, want[f])
        assert n_bad == 0, f"frame {f}: first bad job {first}, {counts}"
        assert np.array_equal(fixed["status"], want[f]["status"]), f"frame {f}: status"
    assert touched >= NF - 1   # every later frame really depended on its carry-in


def test_uninit_prefix_is_last_reader():
    r = np.zeros(6, dtype=[("status", np.uint16)])
    assert fdist.uninit_prefix(r) == 0
    r["status"][[0, 3]] = RES_NN_UNINIT
    assert fdist.uninit_prefix(r) == 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pics = _pictures()
    frames = _frames()
    keys = _keys(frames, pics)
    ring = fdist.PictureRing(W, H, slots=REFS + world + 1, device="cpu", world=world, owner=0)
    mine = fdist.frames_for_rank(NF, world, rank)
    results, states = {}, np.zeros((NF, fdist.STATE_WORDS), np.uint32)
    # publish pictures in encode order: the owner broadcasts, every rank keeps a ring
    for p in range(NF + REFS):
        ring.publish(p, torch.from_numpy(pics[p]) if rank == 0 else None)
        assert np.array_equal(ring.tensor(p).numpy(), pics[p])
        f = p - REFS
        if f >= 0 and f in mine:
            local = [ring.tensor(f + REFS - k).numpy().copy() for k in (2, 1, 0)]
            lp = dict(zip((f, f + 1, f + 2), local))
            view = [lp.get(i) for i in range(NF + REFS)]
            r, st = _sharded_frame(view, frames, keys, f)
            results[f] = r
            states[f] = st
    # exchange end states (12 words per frame), chain, fix prefixes
    t = torch.from_numpy(states.astype(np.int64))
    dist.all_reduce(t)   # each frame's row is non-zero on exactly one rank
    carries, _ = fdist.chain_states(t.numpy().astype(np.uint32))
    for f in mine:
        o = _engine(pics, f)
        o.set_keys(keys[f])
        results[f] = fdist.fix_frame_prefix(o, frames[f], results[f], carries[f])
    gathered = [None] * world
    dist.all_gather_object(gathered, {f: r.tobytes() for f, r in results.items()})
    if rank == 0:
        merged = {}
        for g in gathered:
            merged.update(g)
        np.savez(out_path, **{str(f): np.frombuffer(b, np.uint8) for f, b in merged.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_rank_frame_sharding(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.npz")
    mp.spawn(_rank_main, args=(2, _free_port(), out), nprocs=2, join=True)
    pics = _pictures()
    frames = _frames()
    want = _sequential(frames, pics, _keys(frames, pics))
    got = np.load(out)
    from nnfme.abi import RESULT_DTYPE
    for f in range(NF):
        r = got[str(f)].view(RESULT_DTYPE)
        n_bad, first, counts = compare_results(r, want[f])
        assert n_bad == 0, f"frame {f}: first bad job {first}, {counts}"


# ---- FrameReplay's reconstruction exchange (nnfme.pipeline), CPU rehearsal over gloo ------------
class _Stream:
    def synchronize(self):
        pass


def _exchange_rank(rank, world, port, F, steps, out_path):
    import torch
    import torch.distributed as dist
    from nnfme.pipeline import REFS, FrameReplay
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rep = FrameReplay.__new__(FrameReplay)   # the exchange only: no device, no context
    rep.torch, rep.world, rep.rank, rep.group, rep.F, rep.steps = torch, world, rank, None, F, steps
    frames = steps * world * F
    rep.recon = torch.zeros((frames + REFS, 4, 4), dtype=torch.uint8)
    sends = 0
    for k in range(steps):
        base = k * world * F
        for j in range(F):   # this rank's uploads: frames base + rank F - 1 + j, marked with their number
            h = base + rank * F - 1 + j
            rep.recon[h + REFS].fill_((h + 7) % 251)
            sends += len([d for d in rep.readers(h) if d != rank])
        rep._exchange(k, _Stream())
    have = [int(rep.recon[h + REFS, 0, 0]) for h in range(-REFS, frames)]
    np.save(out_path % rank, np.array(have + [sends], np.int64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,F", [(4, 1), (8, 1), (3, 2)])
def test_frame_replay_exchange_sends_each_reconstruction_to_its_readers(tmp_path, world, F):
    """Every rank ends up holding exactly the reconstructions its frames reference (frames g-1 ..
    g-4 of each of its frames g) - the ones it uploads itself plus what the others sent - and no
    rank sends to more than three others (LDP references the previous four frames)."""
    import torch.multiprocessing as mp
    from nnfme.pipeline import REFS
    steps = 3
    out = str(tmp_path / "have_%d.npy")
    mp.spawn(_exchange_rank, args=(world, _free_port(), F, steps, out), nprocs=world, join=True)
    frames = steps * world * F
    for r in range(world):
        got = np.load(out % r)
        have, sends = got[:-1], int(got[-1])
        mine = [g for g in range(frames) if (g // F) % world == r]
        need = {g - d for g in mine for d in range(1, REFS + 1) if g - d >= -1}
        own = {k * world * F + r * F - 1 + j for k in range(steps) for j in range(F)}
        for h in range(-1, frames):
            v = int(have[h + REFS])
            if h in need or h in own:
                assert v == (h + 7) % 251, (r, h, v)
            else:
                assert v == 0, (r, h, v)   # not sent where nobody reads it
        assert sends <= 3 * steps * F
