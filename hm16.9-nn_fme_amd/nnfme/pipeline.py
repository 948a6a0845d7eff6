"""Frame replay: the sub-pel path over a stream of frames, as SURVEY.md §8(d) times it.

Per step (one batch of xMotionEstimation jobs = one frame, or a group of F small frames so that
a launch fills the chip):
  * H2D of the batch's job descriptors, of the frames' original pictures and of one
    reconstructed reference picture per frame (trace replay: frame f's references are the
    reconstructions of f-1..f-4; each is uploaded once, by the rank that publishes it, and sent
    over RCCL/xGMI point-to-point to the ranks whose frames reference it - at most three other
    ranks, whatever the world size - when the run is sharded);
  * fme_refine_mv_device (EMI step -> FracDIF -> NN_pred -> cost tail, no host synchronisation);
  * D2H of the 16-byte fme_mv_result per job.
Two steps are in flight: the uploads of step k+1 and the download of step k-1 run on their own
streams while step k computes (events order the double-buffered job / output slots).

Sharding (world > 1): rank r replays batches r, r + world, ... (weak scaling; no collective on
the data path besides the reconstructions' point-to-point sends).  NN_pred's carried state crosses frames in the
reference, so every batch starts from a reset state, each batch's end state is copied on the
device (fme_nn_copy_state_device), and after the run the states are all-gathered (12 words per
batch), chained in encode order (nnfme.dist.chain_states) and the jobs up to each batch's last
carried-state reader are refined again with the true carry-in: the result equals a sequential
run bit for bit (tests/test_gpu_dist.py).  Every picture stays resident in HBM for the run
(288 GB per GPU), so the fix-up moves nothing over PCIe but the prefix's jobs.

Picture slots of a batch of F frames (frames G*F .. G*F+F-1 of batch G): reconstruction of
frame G*F - 4 + s in slot s (s < F + 3), original of frame G*F + j in slot ORG0 + j; frame j's
reference at distance d (the base job's ref_id = d - 1) is slot j + 4 - d, its lambda slot j.
"""
import ctypes
import sys
import time

import numpy as np

from . import dist as fdist
from .abi import JOB_DTYPE, MV_RESULT_DTYPE

_hip = None


def _hip_lib():
    global _hip
    if _hip is None:
        h = ctypes.CDLL("libamdhip64.so.7")   # by SONAME: the runtime torch and libfme_amd.so share
        h.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        h.hipMemcpyAsync.restype = ctypes.c_int
        h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        h.hipEventCreateWithFlags.restype = ctypes.c_int
        h.hipEventDestroy.argtypes = [ctypes.c_void_p]
        h.hipEventDestroy.restype = ctypes.c_int
        h.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        h.hipStreamWaitEvent.restype = ctypes.c_int
        _hip = h
    return _hip


# host calls that blocked for more than 1 ms: (what, bytes, ms) (stall hunting, bench.py reports them)
SLOW_CALLS = []


def _memcpy_async(dst, src, nbytes, kind, stream):
    """hipMemcpyAsync between pinned host and device memory on `stream` (a torch stream): the
    copy engines (SDMA) carry it.  (A torch D2H copy_ runs as a blit kernel on the CUs, which
    then waits for the search kernels' workgroups.)"""
    t0 = time.perf_counter()
    rc = _hip_lib().hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), nbytes, kind, stream.cuda_stream)
    dt = (time.perf_counter() - t0) * 1e3
    if dt > 1.0:
        SLOW_CALLS.append(("hipMemcpyAsync kind %d" % kind, int(nbytes), round(dt, 3)))
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync failed ({rc})")


def _timed(what, f):
    """f() and, if it blocked the host for more than 1 ms, a SLOW_CALLS entry."""
    t0 = time.perf_counter()
    f()
    dt = (time.perf_counter() - t0) * 1e3
    if dt > 1.0:
        SLOW_CALLS.append((what, 0, round(dt, 3)))


class _RawEvent:
    """A hipEvent_t the library records (fme_set_search_event) and a stream waits on: created
    unrecorded, so its only record is the library's."""

    def __init__(self):
        ev = ctypes.c_void_p()
        if _hip_lib().hipEventCreateWithFlags(ctypes.byref(ev), 2) != 0:   # hipEventDisableTiming
            raise RuntimeError("hipEventCreateWithFlags failed")
        self.cuda_event = ev.value

    def wait(self, stream):
        if _hip_lib().hipStreamWaitEvent(stream.cuda_stream, self.cuda_event, 0) != 0:
            raise RuntimeError("hipStreamWaitEvent failed")

    def destroy(self):
        """Explicit release (FrameReplay.close): before interpreter exit, not in a finaliser."""
        if self.cuda_event and _hip is not None:
            _hip.hipEventDestroy(self.cuda_event)
        self.cuda_event = None

    def __del__(self):
        # not at interpreter exit: the HIP runtime may already be torn down (a profiler's exit
        # handlers run first), and the process frees its events anyway
        if sys.is_finalizing() or not self.cuda_event or _hip is None:
            return
        try:
            _hip.hipEventDestroy(self.cuda_event)
        except Exception:
            pass


H2D, D2H = 1, 2
D2D_NOCU = 1024   # hipMemcpyDeviceToDeviceNoCU: the runtime's copy engines instead of a blit kernel


def torch_current_stream(t):
    import torch
    return torch.cuda.current_stream(t.device)


ORG0 = 32      # first original-picture slot
REFS = 4       # lowdelay_P / the workloads' reference count


def group_jobs(base, frames, key_count=0):
    """The job batch of a group of `frames` frames: the base frame's jobs (org_id anything,
    ref_id = reference distance - 1 in 0..3, lambda slot 0) once per frame, slots remapped; frame
    j's bi-pred key blocks follow frame j-1's (key_count elements per frame)."""
    out = []
    for j in range(frames):
        g = np.array(base, dtype=JOB_DTYPE, copy=True)
        g["org_id"] = ORG0 + j
        g["ref_id"] = j + 3 - base["ref_id"].astype(np.int64)
        g["lambda_id"] = j
        bi = g["key_offset"] >= 0
        g["key_offset"][bi] += j * key_count
        out.append(g)
    return np.concatenate(out)


def group_key_reqs(base, frames, key_count):
    """The bi-pred key requests (fme_bikey_req) of a group of frames, remapped like group_jobs:
    frame j's original in slot ORG0 + j, its reference at distance ref_id + 1 in slot
    j + 3 - ref_id, its keys at key_offset + j * key_count."""
    from .abi import BIKEY_REQ_DTYPE
    out = []
    for j in range(frames):
        g = np.array(base, dtype=BIKEY_REQ_DTYPE, copy=True)
        g["org_id"] = ORG0 + j
        g["ref_id"] = j + 3 - base["ref_id"].astype(np.int64)
        g["key_offset"] += j * key_count
        out.append(g)
    return np.concatenate(out)


class FrameReplay:
    def __init__(self, ctx, base_jobs, pool, lambda_of, n_steps, frames_per_step=1, world=1, rank=0, device=None,
                 group=None, defer_download=True, key_reqs=None, key_count=0, nn_rows=None,
                 download_engine="sdma", download_wgs=8, search_reserve=0, packed=True, copy_streams=1, slots=3,
                 max_ahead=4, precreate_events=True, warm_engines=True, timeline=False):
        """ctx: an FmeContext on `device`; base_jobs: one frame's jobs (ref_id = reference
        distance - 1); pool: uint8 [P, H, W] host frames, frame g's pictures are pool[g % P];
        lambda_of(g): frame g's lambda (pool uint16: main10 samples for a bit-depth-10 context,
        the pictures bound with the stride in samples).  key_reqs (fme_bikey_req, ref_id = distance - 1) and
        key_count: the frame's bi-pred key requests; each step uploads them with its jobs and builds
        its frames' removeHighFreq keys on the device from that step's pictures, before its batch
        (fme_build_bipred_keys_device), so the keys are per-frame work inside the timed step.
        nn_rows (uint32 [n][9]): the NN input rows of the frame's FME_JOB_NN_IN jobs (the backups'
        input path); each step uploads them with its jobs and binds them (fme_set_nn_inputs).
        packed: upload the jobs as 16-byte fme_job_packed rows (fme_pack_jobs, unpacked on the device
        by fme_refine_mv_packed_device) instead of 32-byte fme_job rows; a batch outside the packed
        form falls back to fme_job (self.packed_reason says why).
        copy_streams: 1 (default) carries every copy of a step - H2D of step k+1, D2H of step k-1 -
        in series on one copy stream; 2 gives the downloads their own stream (round 5's layout: an
        H2D and a D2H in flight together took 2.57 ms where the two in series take 0.93 ms,
        gpurun_out/d2h.log).  slots: depth of the job / result buffer rings (3: the upload of step
        k+1 never waits for the download of step k-2).  max_ahead: issue(k) first waits for step
        k - max_ahead's batch (0: never): a host left to run ahead blocked inside one
        hipMemcpyAsync for 7-27 ms, until the device had drained nearly every queued step (the
        runtime's copy queue full: profiles/r06_ab.log), which then restarted the pipeline empty.
        download_engine: "sdma" (hipMemcpyDeviceToDeviceNoCU into the pinned rows: a copy engine,
        no CUs), "kernel" (fme_download_device: the library's copy kernel of download_wgs workgroups
        of 256 lanes) or "blit" (hipMemcpyAsync, which this ROCm runs as a blit kernel of hundreds of
        workgroups that take the search kernel's CUs).  search_reserve: resident search workgroups
        left free (fme_set_search_reserve), so the download kernel runs beside the search."""
        import torch
        from .abi import JOB_PACKED_DTYPE
        from .runtime import FmeError, pack_jobs
        self.torch, self.ctx = torch, ctx
        self.world, self.rank, self.group = world, rank, group
        self.F = F = frames_per_step
        self.R = R = int(slots)
        if R < 2:
            raise ValueError("slots >= 2")
        self.lambda_of = lambda_of
        self.steps = n_steps
        P, H, W = pool.shape
        self.P, self.H, self.W = P, H, W
        if pool.dtype not in (np.uint8, np.uint16):
            raise ValueError(f"frame pool dtype {pool.dtype}: uint8 or uint16 (main10) samples")
        self.bps = pool.dtype.itemsize                  # bytes per sample
        pdt = torch.uint8 if self.bps == 1 else torch.int16   # 10-bit samples fit int16
        host = np.ascontiguousarray(pool).view(np.uint8 if self.bps == 1 else np.int16)
        self.pool = torch.from_numpy(host).pin_memory()
        self.key_count = int(key_count)
        self.jobs = group_jobs(base_jobs, F, self.key_count)
        self.n = n = len(self.jobs)
        self.packed, self.packed_reason = bool(packed), None
        if self.packed:
            try:
                pk, kb = pack_jobs(self.jobs)
            except FmeError as e:   # outside the packed form: the 32-byte rows
                self.packed, self.packed_reason = False, str(e)
        if self.packed:
            self.h_jobs = torch.from_numpy(pk.view(np.uint8).copy()).pin_memory()
            self.h_kb = torch.from_numpy(kb.view(np.uint8).copy()).pin_memory()
            self.d_kb = [torch.empty(self.h_kb.numel(), dtype=torch.uint8, device=device) for _ in range(R)]
            assert self.h_jobs.numel() == n * JOB_PACKED_DTYPE.itemsize
        else:
            self.h_jobs = torch.from_numpy(self.jobs.view(np.uint8).copy()).pin_memory()
        self.job_bytes = self.h_jobs.numel() + (self.h_kb.numel() if self.packed else 0)
        self.d_jobs = [torch.empty(self.h_jobs.numel(), dtype=torch.uint8, device=device) for _ in range(R)]
        self.kreqs = None
        if key_reqs is not None and len(key_reqs):
            self.kreqs = group_key_reqs(key_reqs, F, self.key_count)
            self.h_kreqs = torch.from_numpy(self.kreqs.view(np.uint8).copy()).pin_memory()
            self.d_kreqs = [torch.empty(self.h_kreqs.numel(), dtype=torch.uint8, device=device) for _ in range(R)]
        self.rows = None
        if nn_rows is not None:
            self.rows = np.tile(np.ascontiguousarray(nn_rows, dtype=np.uint32).reshape(-1, 9), (F, 1))
            assert len(self.rows) == n
            self.h_rows = torch.from_numpy(self.rows.view(np.uint8).copy()).pin_memory()
            self.d_rows = [torch.empty(self.h_rows.numel(), dtype=torch.uint8, device=device) for _ in range(R)]
        self.d_out = [torch.empty(n * MV_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=device) for _ in range(R)]
        self.h_out = torch.empty((n_steps, n * MV_RESULT_DTYPE.itemsize), dtype=torch.uint8).pin_memory()
        frames = n_steps * world * F
        # every reconstructed picture of the run (frames -4 .. frames - 1) and this rank's originals
        self.recon = torch.empty((frames + REFS, H, W), dtype=pdt, device=device)
        self.org = torch.empty((n_steps * F, H, W), dtype=pdt, device=device)
        self.states = torch.zeros((n_steps, 12), dtype=torch.int32, device=device)
        self.s_comp = torch.cuda.default_stream(device)
        self.s_copy = torch.cuda.Stream(device)   # H2D: jobs, originals, reconstructions (+ D2H: copy_streams 1)
        if copy_streams not in (1, 2):
            raise ValueError("copy_streams 1 or 2")
        self.copy_streams = copy_streams
        self.s_down = self.s_copy if copy_streams == 1 else torch.cuda.Stream(device)
        self.uploaded = -1
        # one event of each kind per step, each recorded once: a stream wait on an event that is
        # recorded again while earlier waits on it are still queued did not always wait for the
        # record it was issued after here (step k's download then read the buffer before step k's
        # batch had written it, or after step k+2's had: tools/parity_debug.py)
        self.ev_in = [torch.cuda.Event() for _ in range(n_steps)]
        self.ev_comp = [torch.cuda.Event() for _ in range(n_steps)]
        self.ev_out = [torch.cuda.Event() for _ in range(n_steps)]
        # recorded by the library right before each batch's search kernel (fme_set_search_event):
        # step k's results are downloaded once step k+1's search runs (see issue())
        self.ev_search = [_RawEvent() for _ in range(n_steps)]
        if precreate_events:
            # torch creates an event's hipEvent_t at its first record: do that for every step's
            # events here, before anything waits on them (a record while no wait on the event is
            # queued), so the timed steps create none
            for e in self.ev_in + self.ev_comp + self.ev_out:
                e.record(self.s_copy)
            self.s_copy.synchronize()
        self.defer_download = defer_download
        if download_engine not in ("kernel", "blit", "sdma"):
            raise ValueError(f"download_engine {download_engine!r}")
        self.download_engine, self.download_wgs = download_engine, int(download_wgs)
        ctx.set_search_reserve(int(search_reserve))   # slots the search leaves to the download kernel
        ctx.set_search_event(None)                # set per step in issue()
        self.pending = None                       # step whose download is not issued yet
        self.fixed_jobs = 0
        self.last_prefix = 0                      # longest carried-state prefix finish() re-ran
        self.r_out = {}
        self.max_ahead = int(max_ahead)
        self.host_ms = []                         # host wall time of each issue() call (stall hunting)
        self.host_seg = []                        # its parts: upload, waits, bind, refine, prefetch, download
        self.host_seg_names = ("upload", "waits", "bind", "refine", "prefetch", "download")
        self.warm_engines = bool(warm_engines)
        self.engines_warmed = None
        # timeline=True (diagnostic): timing events around each step's uploads, batch and download,
        # read back by timeline_rows() (the kernel + copy timeline of the pipeline from the HIP
        # runtime's own clocks)
        self.tl = None
        if timeline:
            self.tl = {kk: [torch.cuda.Event(enable_timing=True) for _ in range(n_steps)]
                       for kk in ("up0", "up1", "b0", "b1", "d0", "d1")}
            self.tl_base = torch.cuda.Event(enable_timing=True)

    def h2d_bytes_per_step(self):
        """Bytes this rank uploads per step: jobs (+ key bases), key requests, NN rows, its frames'
        originals and the reconstructions it publishes (one per frame)."""
        b = self.job_bytes + 2 * self.F * self.H * self.W * self.bps
        if self.kreqs is not None:
            b += self.h_kreqs.numel()
        if self.rows is not None:
            b += self.h_rows.numel()
        return b

    def close(self):
        """Release the replay's HIP resources (events, the library's search-event hook) before the
        interpreter exits: nothing of it is left to a destructor that may run after the HIP runtime
        (or a profiler's exit handlers) has torn down."""
        try:
            self.ctx.set_search_event(None)
        except Exception:
            pass
        for e in self.ev_search:
            e.destroy()
        self.ev_search = []

    def first_frame(self, k):
        """First frame of this rank's step k."""
        return (k * self.world + self.rank) * self.F

    # -- pictures ---------------------------------------------------------------------------
    def _publish(self, g, src_rank):
        """Reconstruction of frame g (before the run: frames -4 .. -2): uploaded by src_rank,
        broadcast to every rank."""
        dst = self.recon[g + REFS]
        if self.rank == src_rank:
            _memcpy_async(dst, self.pool[g % self.P], self.H * self.W * self.bps, H2D, torch_current_stream(dst))
        if self.world > 1:
            import torch.distributed as dist
            if dist.get_backend(self.group) == "gloo":   # CPU rehearsal of the sharded path
                tmp = dst.cpu()
                dist.broadcast(tmp, src=src_rank, group=self.group)
                dst.copy_(tmp, non_blocking=False)
            else:
                dist.broadcast(dst, src=src_rank, group=self.group)

    def rank_of_frame(self, g):
        return (g // self.F) % self.world

    def readers(self, h):
        """Ranks (other than the publisher) whose frames reference reconstruction h: frames h+1 ..
        h+REFS of the run."""
        frames = self.steps * self.world * self.F
        out = []
        for d in range(1, REFS + 1):
            f = h + d
            if 0 <= f < frames:
                r = self.rank_of_frame(f)
                if r not in out:
                    out.append(r)
        return out

    def _exchange(self, k, stream):
        """Step k's reconstructions (frame base + r F - 1 + j, uploaded by rank r) go point-to-point
        to the ranks that reference them (self.readers): every rank runs the same op list, sends of
        its own frames and receives of the frames it needs, in one batch_isend_irecv (one RCCL group
        on the copy stream).  Pictures stay resident for the run, so each is sent once."""
        import torch.distributed as dist
        F, W = self.F, self.world
        base = k * W * F
        gloo = dist.get_backend(self.group) == "gloo"
        ops, fixups = [], []
        for r in range(W):
            for j in range(F):
                h = base + r * F - 1 + j
                dsts = [d for d in self.readers(h) if d != r]
                if self.rank == r:
                    buf = self.recon[h + REFS]
                    if gloo:   # CPU rehearsal: gloo sends host tensors
                        stream.synchronize()
                        buf = buf.cpu()
                    for d in dsts:
                        ops.append(dist.P2POp(dist.isend, buf, d, group=self.group))
                elif self.rank in dsts:
                    buf = self.recon[h + REFS]
                    if gloo:
                        tmp = self.torch.empty_like(buf, device="cpu")
                        fixups.append((buf, tmp))
                        buf = tmp
                    ops.append(dist.P2POp(dist.irecv, buf, r, group=self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        for dst, tmp in fixups:
            dst.copy_(tmp, non_blocking=False)

    def _upload_run(self, dst, d0, g0, count, stream):
        """Planes of frames g0 .. g0+count-1 into dst[d0 ..]: one copy per run of frames that is
        contiguous in the pool (a small-frame batch is a few large copies, not many small ones)."""
        i = 0
        while i < count:
            s = (g0 + i) % self.P
            run = min(count - i, self.P - s)
            _memcpy_async(dst[d0 + i], self.pool[s], run * self.H * self.W * self.bps, H2D, stream)
            i += run

    def _publish_run(self, g0, count, src_rank, stream):
        """Reconstructions of frames g0 .. g0+count-1 that src_rank uploads (one copy per pool
        run); when sharded, _exchange then sends them to their readers."""
        if self.rank == src_rank:
            self._upload_run(self.recon, g0 + REFS, g0, count, stream)

    def prime(self):
        """References of the first frames (recon -4 .. -2), before the run (untimed); every
        host result row is written once by the copy engine, so no timed step is the first DMA
        into fresh pinned pages (on a fresh buffer some hipMemcpyAsync calls blocked the host
        for up to 7 ms each: 2.15 ms per 1080p step against 1.32 once the rows had been used)."""
        if self.warm_engines:   # every SDMA engine's queue created now, not mid-pipeline (fme_warm_copy_engines)
            self.engines_warmed = self.ctx.warm_copy_engines()
        with self.torch.cuda.stream(self.s_copy):
            for g in range(-REFS, -1):
                self._publish(g, 0)
        for k in range(self.steps):
            self._copy_down(k, self.s_down)
        self.s_copy.synchronize()
        self.s_down.synchronize()

    def _refine(self, k, out_ptr, n, stream):
        """Step k's batch (its slot's jobs, first n of them) into out_ptr on `stream`."""
        b = k % self.R
        if self.packed:
            self.ctx.refine_mv_packed_device(self.d_jobs[b].data_ptr(), self.d_kb[b].data_ptr(), out_ptr, n,
                                             stream.cuda_stream)
        else:
            self.ctx.refine_mv_device(self.d_jobs[b].data_ptr(), out_ptr, n, stream.cuda_stream)

    def bind_rows(self, b):
        """Bind slot b's NN input rows for the next batches (no-op without rows)."""
        if self.rows is not None:
            self.ctx.set_nn_inputs(self.d_rows[b].data_ptr(), self.n)

    def _bind(self, k):
        ctx, W, H, F = self.ctx, self.W, self.H, self.F
        self.bind_rows(k % self.R)
        f0 = self.first_frame(k)
        for j in range(F):
            ctx.bind_picture_device(ORG0 + j, self.org[k * F + j].data_ptr(), W, W, H)
            ctx.set_lambda(j, self.lambda_of(f0 + j))
        for s in range(F + REFS - 1):
            ctx.bind_picture_device(s, self.recon[f0 - REFS + s + REFS].data_ptr(), W, W, H)

    # -- one step -----------------------------------------------------------------------------
    # Streams: the batch runs on the device's default stream; every copy runs on one copy stream,
    # in series, as issue(k) queues them: the H2D of step k+1 (jobs, key bases, originals, the
    # published reconstruction; its slot was last read by step k+1-R), then the D2H of step k-1's
    # results, which waits until step k's search kernel runs (the library records ev_search right
    # before each search launch).  In series the two directions take 0.93 ms per 1080p step with
    # 32-byte jobs (H2D 0.68 + D2H 0.25 ms, gpurun_out/d2h.log), less than the batch; in flight
    # together on two streams they took 2.57 ms, which is what bound round 5's pipeline.  The
    # download starting only once the search runs keeps a device-to-host copy's posted PCIe writes
    # off the batch prologue's launches (each held back by the copy's length, ≈ 0.25 ms per step).
    # The "sdma" engine (hipMemcpyDeviceToDeviceNoCU into the pinned rows) moves the download off
    # the CUs: the ROCclr blit kernel shared them with the search (0.92 -> 1.11 ms).  Compute and
    # copy streams stay within the process's four hardware queues (GPU_MAX_HW_QUEUES).
    def _upload(self, k):
        F, R = self.F, self.R
        b = k % R
        f0 = self.first_frame(k)
        cp = self.s_copy
        with self.torch.cuda.stream(cp):
            if k >= R:
                _timed("copy stream wait_event", lambda: cp.wait_event(self.ev_comp[k - R]))   # step k-R is done with the slot
            if self.tl:
                self.tl["up0"][k].record(cp)
            _memcpy_async(self.d_jobs[b], self.h_jobs, self.h_jobs.numel(), H2D, cp)
            if self.packed:
                _memcpy_async(self.d_kb[b], self.h_kb, self.h_kb.numel(), H2D, cp)
            if self.rows is not None:
                _memcpy_async(self.d_rows[b], self.h_rows, self.h_rows.numel(), H2D, cp)
            if self.kreqs is not None:
                _memcpy_async(self.d_kreqs[b], self.h_kreqs, self.h_kreqs.numel(), H2D, cp)
            self._upload_run(self.org, k * F, f0, F, cp)
            base = k * self.world * F
            # recon(first frame of rank r's batch - 1 + j) is uploaded by rank r ...
            self._publish_run(base + self.rank * F - 1, F, self.rank, cp)
            if self.world > 1:   # ... and sent to the ranks whose frames reference it
                self._exchange(k, cp)
            if self.tl:
                self.tl["up1"][k].record(cp)
            _timed("ev_in record", lambda: self.ev_in[k].record(cp))
        self.uploaded = k

    def issue(self, k, prefetch=True):
        """Enqueue step k (and, with prefetch, the upload of step k+1); returns without waiting
        for the device.  self.host_ms / self.host_seg record the host time of each call and of its
        parts (stall hunting: which runtime call blocks)."""
        pc = time.perf_counter
        t = [pc()]
        ctx = self.ctx
        b = k % self.R
        if self.max_ahead > 0 and k >= self.max_ahead:
            self.ev_comp[k - self.max_ahead].synchronize()   # at most max_ahead steps queued
        if self.uploaded < k:
            self._upload(k)
        t.append(pc())
        comp = self.s_comp
        comp.wait_event(self.ev_in[k])
        if k >= self.R:
            comp.wait_event(self.ev_out[k - self.R])       # step k-R's results have left the slot
        t.append(pc())
        self._bind(k)
        if self.kreqs is not None:   # this step's frames' removeHighFreq keys, from this step's pictures
            ctx.build_bipred_keys_device(self.d_kreqs[b].data_ptr(), len(self.kreqs), self.key_count * self.F,
                                         comp.cuda_stream)
        if self.world > 1:
            ctx.nn_reset()                                 # stream-ordered: this batch starts fresh
        if self.defer_download:
            ctx.set_search_event(self.ev_search[k])        # recorded right before this batch's search
        t.append(pc())
        if self.tl:
            self.tl["b0"][k].record(comp)
        self._refine(k, self.d_out[b].data_ptr(), self.n, comp)
        if self.world > 1:
            ctx.nn_copy_state_device(self.states[k].data_ptr(), comp.cuda_stream)
        if self.tl:
            self.tl["b1"][k].record(comp)
        self.ev_comp[k].record(comp)
        t.append(pc())
        if prefetch and k + 1 < self.steps:
            self._upload(k + 1)
        t.append(pc())
        if not self.defer_download:
            self._download(k, self.ev_comp[k])
        else:
            if self.pending is not None:   # step k's search started: k-1 is done (its own batch event otherwise)
                self._download(self.pending, self.ev_search[k] if self.n > 0 else self.ev_comp[self.pending])
            self.pending = k
        t.append(pc())
        self.host_ms.append((t[-1] - t[0]) * 1e3)
        self.host_seg.append([round((t[i + 1] - t[i]) * 1e3, 3) for i in range(len(t) - 1)])

    def _copy_down(self, k, dn):
        b = k % self.R
        if self.download_engine == "kernel":
            self.ctx.download_device(self.d_out[b].data_ptr(), self.h_out[k].data_ptr(), self.h_out.shape[1],
                                     self.download_wgs, dn.cuda_stream)
        elif self.download_engine == "sdma":   # hipMemcpyDeviceToDeviceNoCU: a copy engine, no CUs
            _memcpy_async(self.h_out[k], self.d_out[b], self.h_out.shape[1], D2D_NOCU, dn)
        else:
            _memcpy_async(self.h_out[k], self.d_out[b], self.h_out.shape[1], D2H, dn)

    def _download(self, k, after):
        dn = self.s_down
        if isinstance(after, _RawEvent):
            after.wait(dn)
        else:
            dn.wait_event(after)
        if self.tl:
            self.tl["d0"][k].record(dn)
        self._copy_down(k, dn)
        if self.tl:
            self.tl["d1"][k].record(dn)
        self.ev_out[k].record(dn)

    def drain(self):
        """Issue the last step's download and wait for every stream; the library no longer records
        into this replay's search event afterwards (the context may outlive the replay)."""
        if self.pending is not None:
            self._download(self.pending, self.ev_comp[self.pending])
            self.pending = None
        self.s_copy.synchronize()
        self.s_comp.synchronize()
        self.s_down.synchronize()
        self.ctx.set_search_event(None)

    def check_status(self, first_step=0):
        """Raise if any step's batch was rejected on the device (FME_RES_REJECTED: an invalid job
        or invalid device-built keys); the throughput of a rejected step would count nothing."""
        from .abi import RES_REJECTED
        for k in range(first_step, self.steps):
            if np.any(self.results(k)["status"] & RES_REJECTED):
                raise RuntimeError(f"frame replay: step {k}'s batch was rejected on the device")

    def timeline_start(self):
        """Mark the timeline's zero on the copy and compute streams' device (timeline=True)."""
        if self.tl:
            self.tl_base.record(self.s_comp)

    def timeline_rows(self, k0, k1):
        """Per step k0 .. k1-1: ms from timeline_start() to the start / end of the step's uploads,
        batch and download (after drain())."""
        rows = []
        for k in range(k0, k1):
            r = {"step": k}
            for kk in ("up0", "up1", "b0", "b1", "d0", "d1"):
                r[kk] = round(self.tl_base.elapsed_time(self.tl[kk][k]), 4)
            rows.append(r)
        return rows

    def results(self, k):
        return self.h_out[k].numpy().view(MV_RESULT_DTYPE)

    # -- the HBM-resident run (bench.py's `value`) -------------------------------------------------
    # Steps replayed with every input already in HBM (the pipelined pass uploaded and, when
    # sharded, exchanged them into per-step buffers) and the results left there: one device
    # buffer per step, since a sharded run re-runs each step's carried-state prefix at the end.
    def resident_outputs(self, k0, k1):
        torch = self.torch
        dev = self.d_out[0].device
        self.r_out = {k: torch.empty(self.n * MV_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
                      for k in range(k0, k1)}

    def _resident_batch(self, k, n):
        ctx, comp = self.ctx, self.s_comp
        b = k % self.R
        self._bind(k)
        if self.kreqs is not None:   # this step's keys, built on the device from its pictures
            ctx.build_bipred_keys_device(self.d_kreqs[b].data_ptr(), len(self.kreqs), self.key_count * self.F,
                                         comp.cuda_stream)
        self._refine(k, self.r_out[k].data_ptr(), n, comp)

    def issue_resident(self, k):
        """Step k from HBM-resident inputs into r_out[k] (no copy, no host wait)."""
        ctx, comp = self.ctx, self.s_comp
        ctx.set_search_event(None)
        if self.world > 1:
            ctx.nn_reset()                                 # stream-ordered: this batch starts fresh
        self._resident_batch(k, self.n)
        if self.world > 1:
            ctx.nn_copy_state_device(self.states[k].data_ptr(), comp.cuda_stream)

    def finish_resident(self, k0, k1, prefix):
        """Sharded: all-gather the steps' end states, chain them in encode order and re-run each
        step's carried-state prefix (`prefix` jobs, the same for every step of a replay: see
        finish()) with its true carry-in, on the device.  Returns the number of re-run jobs."""
        if self.world == 1 or prefix <= 0:
            return 0
        import torch.distributed as dist
        torch = self.torch
        self.s_comp.synchronize()
        st = self.states if dist.get_backend(self.group) != "gloo" else self.states.cpu()
        gathered = [torch.zeros_like(st) for _ in range(self.world)]
        dist.all_gather(gathered, st, group=self.group)
        bs = np.zeros((self.steps * self.world, 12), np.uint32)
        for r in range(self.world):
            g = gathered[r].cpu().numpy().view(np.uint32)
            for k in range(self.steps):
                bs[k * self.world + r] = g[k]
        carries, _ = fdist.chain_states(bs)
        fixed = 0
        for k in range(k0, k1):
            carry = carries[k * self.world + self.rank]
            if not int(carry[11]):
                continue
            self.ctx.nn_set_state(carry)
            self._resident_batch(k, prefix)
            fixed += prefix
        return fixed

    # -- end of the run -----------------------------------------------------------------------
    def finish(self, first_step=0):
        """Wait for every step; when sharded, chain the NN states and refine each batch's
        carried-state prefix again (steps >= first_step).  Returns the number of re-run jobs."""
        torch = self.torch
        self.drain()
        if self.world == 1:
            return 0
        import torch.distributed as dist
        st = self.states if dist.get_backend(self.group) != "gloo" else self.states.cpu()
        gathered = [torch.zeros_like(st) for _ in range(self.world)]
        dist.all_gather(gathered, st, group=self.group)
        bs = np.zeros((self.steps * self.world, 12), np.uint32)
        for r in range(self.world):
            g = gathered[r].cpu().numpy().view(np.uint32)
            for k in range(self.steps):
                bs[k * self.world + r] = g[k]
        carries, _ = fdist.chain_states(bs)
        fixed = 0
        ctx, comp = self.ctx, self.s_comp
        for k in range(first_step, self.steps):
            out = self.results(k)
            p = fdist.uninit_prefix(out)
            self.last_prefix = max(self.last_prefix, p)
            carry = carries[k * self.world + self.rank]
            if p == 0 or not int(carry[11]):
                continue
            with torch.cuda.stream(comp):
                self._bind(k)
                if self.kreqs is not None:
                    ctx.build_bipred_keys(self.kreqs, self.key_count * self.F, comp.cuda_stream)
                ctx.nn_set_state(carry)
                out[:p] = ctx.refine_mv(self.jobs[:p], comp.cuda_stream)
            fixed += p
        self.fixed_jobs = fixed
        return fixed
