"""Frame sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI): the
picture ring and the NN-state chaining (nnfme.pipeline.FrameReplay drives them for the bench).

Sub-pel jobs are independent given (original picture, reference pictures) — SURVEY.md §8(e).
Frames are dealt round-robin to ranks; the only exchange is the rank that owns the pictures
(the trace owner) publishing each new frame to every rank with one broadcast into a device
ring of picture slots.  Ranks keep the last 4 frames (lowdelay_P references) resident, so a
step moves world x 2.07 MB at 1080p, overlapping nothing else on the data path.

NN_pred's carried state (array_e slots, C, PUHeight, PUWidth) crosses frame boundaries in
the reference.  A rank refines each of its frames from a fresh state; jobs that read a slot
no earlier job of the frame wrote carry status FME_RES_NN_UNINIT.  `chain_states` composes the
per-frame end states in encode order (an all_gather of 12 words per frame), and the jobs up
to the last such reader are re-run with the true carry-in (fix_frame_prefix): every later
job reads only state written inside the frame, which the re-run leaves unchanged.  On real
traces the re-run is empty or a few jobs: a frame's first job is a uni-pred 2Nx2N PU whose
EMI step writes all eight slots unless the search range clips it.
"""
import numpy as np

from .abi import RES_NN_UNINIT

STATE_WORDS = 12   # slot[8], C, PUHeight, PUWidth, written-mask


def frames_for_rank(n_frames, world, rank):
    return list(range(rank, n_frames, world))


class PictureRing:
    """Device ring of luma slots; `owner` publishes frame f into slot f % slots on every rank."""

    def __init__(self, width, height, slots, device, world=1, owner=0, group=None):
        import torch
        self.width, self.height, self.slots = width, height, slots
        self.world, self.owner, self.group = world, owner, group
        self.buf = torch.zeros((slots, height, width), dtype=torch.uint8, device=device)
        self.frame_of_slot = [None] * slots

    def slot(self, frame):
        return frame % self.slots

    def publish(self, frame, src=None):
        """Collective when world > 1: every rank calls it with the same frame index; the owner
        passes the frame's luma (device tensor), the others None."""
        import torch.distributed as dist
        s = self.slot(frame)
        dst = self.buf[s]
        if src is not None:
            dst.copy_(src, non_blocking=True)
        if self.world > 1:
            dist.broadcast(dst, src=self.owner, group=self.group)
        self.frame_of_slot[s] = frame

    def tensor(self, frame):
        s = self.slot(frame)
        if self.frame_of_slot[s] != frame:
            raise RuntimeError(f"frame {frame} is not resident (slot {s} holds {self.frame_of_slot[s]})")
        return self.buf[s]

    def bind(self, ctx, pid, frame):
        s = self.slot(frame)
        if self.frame_of_slot[s] != frame:
            raise RuntimeError(f"frame {frame} is not resident (slot {s} holds {self.frame_of_slot[s]})")
        ctx.bind_picture_device(pid, self.buf[s].data_ptr(), self.width, self.width, self.height)


def merge_state(carry, frame_state):
    """NN state after a frame that started from `carry`: slots the frame wrote win."""
    carry = np.asarray(carry, dtype=np.uint32)
    fs = np.asarray(frame_state, dtype=np.uint32)
    out = carry.copy()
    written = int(fs[11])
    for s in range(8):
        if written & (1 << s):
            out[s] = fs[s]
    if written & 0x100:
        out[8:11] = fs[8:11]
    out[11] = int(carry[11]) | written
    return out


def chain_states(frame_states, initial=None):
    """Carry-in state of every frame, given each frame's end state from a fresh start."""
    cur = np.zeros(STATE_WORDS, np.uint32) if initial is None else np.asarray(initial, np.uint32)
    carries = []
    for fs in frame_states:
        carries.append(cur.copy())
        cur = merge_state(cur, fs)
    return carries, cur


def uninit_prefix(results):
    """Length of the shortest prefix holding every job that read the carried state."""
    m = (results["status"] & RES_NN_UNINIT) != 0
    if not m.any():
        return 0
    return int(np.flatnonzero(m)[-1]) + 1


def fix_frame_prefix(engine, jobs, results, carry):
    """Re-run the carried-state prefix of a frame with its true carry-in (engine: anything
    with nn_set_state/refine over host arrays — FmeContext, or the oracle in tests)."""
    k = uninit_prefix(results)
    if k == 0 or not int(np.asarray(carry)[11]):
        return results
    saved = engine.nn_get_state()   # the engine's own state is left as it was
    engine.nn_set_state(carry)
    fixed = engine.refine(jobs[:k])
    engine.nn_set_state(saved)
    out = results.copy()
    out[:k] = fixed
    # status bits are relative to the context, keep the sequential meaning
    return out
