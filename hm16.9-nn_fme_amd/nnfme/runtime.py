"""ctypes binding of libfme_amd.so (include/fme.h).

This is the product path: every call lands in the HIP kernels of csrc/fme_kernels.hip.  There
is no CPU fallback — a missing or unloadable library raises FmeError at import of the
context, and every failing C call raises FmeError with fme_last_error()'s text.
"""
import ctypes as C
import os
import sys

import numpy as np

from .abi import JOB_DTYPE, MV_RESULT_DTYPE, NN_PARAMS, RESULT_DTYPE
from .weights import load_weights

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("FME_LIB_PATH") or os.path.join(PKG_ROOT, "libfme_amd.so")

ABI_VERSION = 18
TIMING_NAMES = ("classify", "scatter", "search", "nn_tail", "batch", "search_main", "search_aux")

# Every entry point include/fme.h declares (the ABI test checks the .so exports them).
ABI_SYMBOLS = (
    "fme_abi_version", "fme_create", "fme_destroy", "fme_last_error", "fme_set_picture",
    "fme_bind_picture_device", "fme_set_lambda", "fme_set_motion_lambda", "fme_set_keys",
    "fme_load_nn_weights", "fme_nn_reset_state", "fme_nn_get_state", "fme_nn_set_state", "fme_refine", "fme_refine_device",
    "fme_frac_dif_single", "fme_nn_pred_single", "fme_set_profiling", "fme_last_timings",
    "fme_accumulated_timings", "fme_single_last_device_us", "fme_search_kernel_of_shape",
    "fme_set_picture_chroma", "fme_bind_picture_chroma_device", "fme_motion_compensate",
    "fme_motion_compensate_device", "fme_mc_invalid_count", "fme_mc_last_ms",
    "fme_integer_search", "fme_integer_search_device", "fme_integer_search_last_ms",
    "fme_pred_inter_p", "fme_pred_inter_reset", "fme_nn_param_count", "fme_load_nn_net",
    "fme_set_nn_engine", "fme_set_nn_margin_output", "fme_refine_mv", "fme_refine_mv_device",
    "fme_refine_status", "fme_nn_copy_state_device", "fme_template_costs", "fme_pred_inter_b", "fme_build_bipred_keys",
    "fme_set_search_event", "fme_build_bipred_keys_device", "fme_set_nn_logit_output",
    "fme_set_nn_inputs", "fme_integer_search_ring", "fme_integer_search_ring_device",
    "fme_download_device", "fme_pred_inter_phases", "fme_set_search_reserve",
    "fme_pack_jobs", "fme_unpack_jobs", "fme_refine_packed_device", "fme_refine_mv_packed_device",
    "fme_integer_search2", "fme_integer_search2_device", "fme_warm_copy_engines", "fme_set_wp",
)


class FmeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class FmeConfig(C.Structure):
    _fields_ = [("bit_depth", C.c_int32), ("use_hadamard", C.c_int32), ("nn_mode", C.c_int32),
                ("qp", C.c_int32), ("fast_inter_mode", C.c_int32), ("max_jobs", C.c_int32)]


_libs = {}


def load_library(path=None):
    """Load libfme_amd.so (once per path); raise if it has not been built."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise FmeError(-1, f"{path} missing: build it with __graft_entry__.build() or "
                           f"`make -C hm16.9-nn_fme_amd`")
    lib = C.CDLL(path)
    P, I, U32, D = C.c_void_p, C.c_int, C.c_uint32, C.c_double
    sig = {
        "fme_abi_version": (I, []),
        "fme_create": (I, [I, P, P]),
        "fme_destroy": (I, [P]),
        "fme_last_error": (C.c_char_p, []),
        "fme_set_picture": (I, [P, I, P, I, I, I, P]),
        "fme_bind_picture_device": (I, [P, I, P, I, I, I]),
        "fme_set_lambda": (I, [P, I, D]),
        "fme_set_motion_lambda": (I, [P, I, D]),
        "fme_set_keys": (I, [P, P, C.c_size_t, P]),
        "fme_load_nn_weights": (I, [P, P, I]),
        "fme_nn_reset_state": (I, [P]),
        "fme_nn_get_state": (I, [P, P]),
        "fme_nn_set_state": (I, [P, P]),
        "fme_refine": (I, [P, P, P, I, P]),
        "fme_refine_device": (I, [P, P, P, I, P]),
        "fme_frac_dif_single": (I, [P, I, P, I, I, I, P, I, I, I, I, I, D, P, P, P]),
        "fme_nn_pred_single": (I, [P, P, U32, I, I, P, P]),
        "fme_set_profiling": (I, [P, I]),
        "fme_last_timings": (I, [P, P, I]),
        "fme_accumulated_timings": (I, [P, P, I, I]),
        "fme_single_last_device_us": (I, [P, P, I]),
        "fme_search_kernel_of_shape": (I, [I, I]),
        "fme_set_picture_chroma": (I, [P, I, P, P, I, P]),
        "fme_bind_picture_chroma_device": (I, [P, I, P, P, I]),
        "fme_motion_compensate": (I, [P, P, I, P, I, P, P, I, I, I, P]),
        "fme_motion_compensate_device": (I, [P, P, I, P, I, P, P, I, I, I, P]),
        "fme_mc_invalid_count": (I, [P]),
        "fme_set_wp": (I, [P, I, I, P]),
        "fme_mc_last_ms": (I, [P, P]),
        "fme_integer_search": (I, [P, P, P, P, I, P]),
        "fme_integer_search_device": (I, [P, P, P, P, I, P]),
        "fme_integer_search_last_ms": (I, [P, P]),
        "fme_pred_inter_p": (I, [P, P, P, I, P]),
        "fme_pred_inter_reset": (I, [P]),
        "fme_nn_param_count": (I, [P]),
        "fme_load_nn_net": (I, [P, P, P, I]),
        "fme_set_nn_engine": (I, [P, I]),
        "fme_set_nn_margin_output": (I, [P, P, I]),
        "fme_set_nn_logit_output": (I, [P, P, I]),
        "fme_refine_mv": (I, [P, P, P, I, P]),
        "fme_refine_mv_device": (I, [P, P, P, I, P]),
        "fme_refine_status": (I, [P]),
        "fme_nn_copy_state_device": (I, [P, P, P]),
        "fme_set_search_event": (I, [P, P]),
        "fme_template_costs": (I, [P, P, P, I, P]),
        "fme_pred_inter_b": (I, [P, P, P, I, P]),
        "fme_build_bipred_keys": (I, [P, P, I, C.c_size_t, P]),
        "fme_build_bipred_keys_device": (I, [P, P, I, C.c_size_t, P]),
        "fme_set_nn_inputs": (I, [P, P, I]),
        "fme_integer_search_ring": (I, [P, P, P, P, P, I, P]),
        "fme_integer_search_ring_device": (I, [P, P, P, P, P, I, P]),
        "fme_download_device": (I, [P, P, P, C.c_size_t, I, P]),
        "fme_pred_inter_phases": (I, [P, P, I]),
        "fme_set_search_reserve": (I, [P, I]),
        "fme_warm_copy_engines": (I, [P, P]),
        "fme_pack_jobs": (I, [P, I, P, P]),
        "fme_unpack_jobs": (I, [P, P, I, P]),
        "fme_refine_packed_device": (I, [P, P, P, P, I, P]),
        "fme_refine_mv_packed_device": (I, [P, P, P, P, I, P]),
        "fme_integer_search2": (I, [P, P, P, P, I, P]),
        "fme_integer_search2_device": (I, [P, P, P, P, I, P]),
    }
    # an explicitly named library is an A/B variant (tools/ab_bench.py): possibly an older ABI
    strict = os.path.abspath(path) == os.path.abspath(LIB_PATH)
    for name, (res, args) in sig.items():
        f = getattr(lib, name, None)
        if f is None:   # tests/test_abi.py checks that the library exports every fme.h entry point
            continue
        f.restype = res
        f.argtypes = args
    abi = lib.fme_abi_version()
    if strict and abi != ABI_VERSION:
        raise FmeError(-1, "ABI version mismatch")
    if abi != ABI_VERSION:   # an A/B variant: say so, and FmeContext refuses what it cannot honour
        import warnings
        warnings.warn(f"{path}: ABI {abi}, this binding is ABI {ABI_VERSION}")
    lib.fme_abi = abi
    _libs[path] = lib
    return lib


def _check(lib, rc):
    if rc != 0:
        raise FmeError(rc, lib.fme_last_error().decode(errors="replace"))


def _ptr(a):
    return C.c_void_p(a.ctypes.data)


class FmeContext:
    """One device context: pictures, lambdas, keys, NN weights and the carried NN state."""

    def __init__(self, device=0, use_hadamard=1, nn_mode=1, qp=22, fast_inter_mode=1, max_jobs=0,
                 load_nn=True, lib_path=None, net=None, nn_engine=0, bit_depth=8):
        """bit_depth 10 (the main10 configurations): pictures are uint16 sample planes; every entry
        point runs at 10 bits (the refinement batches on k_search_lane10, integer search, template
        costs, bi-pred keys, the producers, motion compensation)."""
        self.lib = load_library(lib_path)
        self.bit_depth = int(bit_depth)
        self.cfg = FmeConfig(self.bit_depth, use_hadamard, nn_mode, qp, fast_inter_mode, max_jobs)
        h = C.c_void_p()
        _check(self.lib, self.lib.fme_create(device, C.byref(self.cfg), C.byref(h)))
        self.h = h
        self.device = device
        if nn_mode == 1 and load_nn:
            self.load_nn(load_weights(qp))
        if nn_mode == 2 and net is not None:
            self.load_nn_net(net)
        if nn_engine:
            self.set_nn_engine(nn_engine)

    def close(self):
        if getattr(self, "h", None):
            self.lib.fme_destroy(self.h)
            self.h = None

    def __del__(self):
        # not at interpreter exit: the HIP runtime (and a profiler's hooks) may be torn down by
        # then; callers close() explicitly (bench.py does, in a finally block)
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    # -- state --------------------------------------------------------------------------
    def set_picture(self, pid, luma, stream=None):
        luma = np.ascontiguousarray(luma, dtype=np.uint16 if self.bit_depth > 8 else np.uint8)
        h, w = luma.shape
        _check(self.lib, self.lib.fme_set_picture(self.h, pid, _ptr(luma), w, w, h, stream))

    def bind_picture_device(self, pid, data_ptr, stride, width, height):
        """A caller-owned device plane (8-bit samples, or uint16 at bit depth 10; stride in samples)."""
        _check(self.lib, self.lib.fme_bind_picture_device(self.h, pid, C.c_void_p(data_ptr), stride, width, height))

    def set_picture_chroma(self, pid, cb, cr, stream=None):
        """4:2:0 chroma planes of picture pid: uint8, or uint16 samples in a bit-depth-10 context."""
        dt = np.uint16 if self.bit_depth > 8 else np.uint8
        cb = np.ascontiguousarray(cb, dtype=dt)
        cr = np.ascontiguousarray(cr, dtype=dt)
        assert cb.shape == cr.shape
        _check(self.lib, self.lib.fme_set_picture_chroma(self.h, pid, _ptr(cb), _ptr(cr), cb.shape[1], stream))

    def set_picture_yuv(self, pid, y, cb, cr, stream=None):
        self.set_picture(pid, y, stream)
        self.set_picture_chroma(pid, cb, cr, stream)

    def bind_picture_chroma_device(self, pid, cb_ptr, cr_ptr, stride):
        _check(self.lib, self.lib.fme_bind_picture_chroma_device(self.h, pid, C.c_void_p(cb_ptr), C.c_void_p(cr_ptr),
                                                                 stride))

    # -- integer motion estimation ------------------------------------------------------------
    def integer_search(self, jobs, ext, stream=None):
        """xTZSearch / xPatternSearch per job (fme_integer_search): returns (jobs with mv_x/mv_y
        = the integer MV, ruiSAD per job).  fme_tz_ext2 records (TZ_EXT2_DTYPE: FastSearch 0 / 3 with
        the neighbour predictors) go to fme_integer_search2."""
        from .abi import TZ_EXT_DTYPE, TZ_EXT2_DTYPE
        if np.asarray(ext).dtype.itemsize == TZ_EXT2_DTYPE.itemsize:
            jobs = np.array(jobs, dtype=JOB_DTYPE, copy=True)
            ext = np.ascontiguousarray(ext, dtype=TZ_EXT2_DTYPE)
            sad = np.zeros(len(jobs), np.uint32)
            _check(self.lib, self.lib.fme_integer_search2(self.h, _ptr(jobs), _ptr(ext), _ptr(sad), len(jobs), stream))
            return jobs, sad
        jobs = np.array(jobs, dtype=JOB_DTYPE, copy=True)
        ext = np.ascontiguousarray(ext, dtype=TZ_EXT_DTYPE)
        sad = np.zeros(len(jobs), np.uint32)
        _check(self.lib, self.lib.fme_integer_search(self.h, _ptr(jobs), _ptr(ext), _ptr(sad), len(jobs), stream))
        return jobs, sad

    def integer_search_ring(self, jobs, ext, stream=None):
        """fme_integer_search_ring: FME_TZ_RING jobs run the backups' xTZSearch tail (square + ring,
        every distortion pushed); returns (jobs, sad, nn_in[n][9] = array_e[index_ref..+7], C)."""
        from .abi import TZ_EXT_DTYPE
        jobs = np.array(jobs, dtype=JOB_DTYPE, copy=True)
        ext = np.ascontiguousarray(ext, dtype=TZ_EXT_DTYPE)
        sad = np.zeros(len(jobs), np.uint32)
        nn_in = np.zeros((len(jobs), 9), np.uint32)
        _check(self.lib, self.lib.fme_integer_search_ring(self.h, _ptr(jobs), _ptr(ext), _ptr(sad), _ptr(nn_in),
                                                          len(jobs), stream))
        return jobs, sad, nn_in

    def integer_search_ring_device(self, d_jobs, d_ext, d_sad, d_nn_in, n, stream=None):
        _check(self.lib, self.lib.fme_integer_search_ring_device(self.h, C.c_void_p(d_jobs), C.c_void_p(d_ext),
                                                                 C.c_void_p(d_sad), C.c_void_p(d_nn_in), n, stream))

    def set_nn_inputs(self, d_ptr, capacity=0):
        """Bind the device rows (uint32 [capacity][9]) FME_JOB_NN_IN jobs read their NN inputs from
        (fme_set_nn_inputs); 0 / None unbinds."""
        _check(self.lib, self.lib.fme_set_nn_inputs(self.h, C.c_void_p(d_ptr) if d_ptr else None,
                                                    int(capacity) if d_ptr else 0))

    def integer_search_device(self, d_jobs, d_ext, d_sad, n, stream=None):
        _check(self.lib, self.lib.fme_integer_search_device(self.h, C.c_void_p(d_jobs), C.c_void_p(d_ext),
                                                            C.c_void_p(d_sad), n, stream))

    def integer_search2_device(self, d_jobs, d_ext2, d_sad, n, stream=None):
        """fme_integer_search2_device: device jobs and fme_tz_ext2 records (FastSearch 0 / 3)."""
        _check(self.lib, self.lib.fme_integer_search2_device(self.h, C.c_void_p(d_jobs), C.c_void_p(d_ext2),
                                                             C.c_void_p(d_sad), n, stream))

    def integer_search_last_ms(self):
        ms = C.c_float()
        _check(self.lib, self.lib.fme_integer_search_last_ms(self.h, C.byref(ms)))
        return ms.value

    # -- predInterSearch P-slice PU / reference loop ------------------------
    def pred_inter_p(self, reqs, stream=None):
        """fme_pred_inter_p: one fme_pu_res per fme_pu_req, in request order."""
        from .abi import PU_REQ_DTYPE, PU_RES_DTYPE
        reqs = np.ascontiguousarray(reqs, dtype=PU_REQ_DTYPE)
        res = np.zeros(len(reqs), dtype=PU_RES_DTYPE)
        if len(reqs):
            _check(self.lib, self.lib.fme_pred_inter_p(self.h, _ptr(reqs), _ptr(res), len(reqs), stream))
        return res

    def pred_inter_b(self, reqs, stream=None):
        """fme_pred_inter_b: predInterSearch on a B slice, one fme_pu_res_b per fme_pu_req_b."""
        from .abi import PU_REQ_B_DTYPE, PU_RES_B_DTYPE
        reqs = np.ascontiguousarray(reqs, dtype=PU_REQ_B_DTYPE)
        res = np.zeros(len(reqs), dtype=PU_RES_B_DTYPE)
        if len(reqs):
            _check(self.lib, self.lib.fme_pred_inter_b(self.h, _ptr(reqs), _ptr(res), len(reqs), stream))
        return res

    def build_bipred_keys(self, reqs, key_count, stream=None):
        """fme_build_bipred_keys: removeHighFreq keys of the other list's prediction, on the device,
        into the context's key buffer (key_count elements)."""
        from .abi import BIKEY_REQ_DTYPE
        reqs = np.ascontiguousarray(reqs, dtype=BIKEY_REQ_DTYPE)
        _check(self.lib, self.lib.fme_build_bipred_keys(self.h, _ptr(reqs), len(reqs), int(key_count), stream))

    def build_bipred_keys_device(self, d_reqs, n, key_count, stream=None):
        """fme_build_bipred_keys_device: the same from a device-resident request array, in stream
        order (no host synchronisation; invalid requests make every later batch that reads
        keys rejected, see fme.h)."""
        _check(self.lib, self.lib.fme_build_bipred_keys_device(self.h, C.c_void_p(d_reqs), int(n), int(key_count),
                                                                C.c_void_p(stream) if stream else None))

    def template_costs(self, reqs, stream=None):
        """fme_template_costs: xGetTemplateCost per (request, reference, candidate) -> uint32
        [n, MAX_REFS, 2] (0xFFFFFFFF where there is no candidate)."""
        from .abi import MAX_REFS, PU_REQ_DTYPE
        reqs = np.ascontiguousarray(reqs, dtype=PU_REQ_DTYPE)
        out = np.zeros((len(reqs), MAX_REFS, 2), np.uint32)
        if len(reqs):
            _check(self.lib, self.lib.fme_template_costs(self.h, _ptr(reqs), _ptr(out), len(reqs), stream))
        return out

    def pred_inter_reset(self):
        _check(self.lib, self.lib.fme_pred_inter_reset(self.h))

    # -- motion compensation ----------------------------------------------------------------
    def motion_compensate(self, mc_jobs, y, cb, cr, stream=None):
        """Predict every job into the (host) planes y, cb, cr in place (fme_motion_compensate)."""
        from .abi import MC_JOB_DTYPE
        jobs = np.ascontiguousarray(mc_jobs, dtype=MC_JOB_DTYPE)
        dt = np.uint16 if self.bit_depth > 8 else np.uint8   # main10: uint16 planes
        for a in (y, cb, cr):
            assert a.dtype == dt and a.flags["C_CONTIGUOUS"]
        h, w = y.shape
        _check(self.lib, self.lib.fme_motion_compensate(self.h, _ptr(jobs), len(jobs), _ptr(y), y.shape[1], _ptr(cb),
                                                        _ptr(cr), cb.shape[1], w, h, stream))

    def set_wp(self, lst, ref_id, params):
        """fme_set_wp: weighted-prediction parameters (Y, Cb, Cr) of reference ref_id in list lst;
        params: 3 rows of (weight, offset, log2_denom) or a WP_PARAM_DTYPE[3] array."""
        from .abi import WP_PARAM_DTYPE, wp_params
        arr = wp_params(params)
        _check(self.lib, self.lib.fme_set_wp(self.h, int(lst), int(ref_id), _ptr(arr)))

    def motion_compensate_device(self, d_jobs, n, d_y, y_stride, d_cb, d_cr, c_stride, width, height, stream=None):
        _check(self.lib, self.lib.fme_motion_compensate_device(self.h, C.c_void_p(d_jobs), n, C.c_void_p(d_y), y_stride,
                                                               C.c_void_p(d_cb), C.c_void_p(d_cr), c_stride, width,
                                                               height, stream))

    def mc_invalid_count(self):
        rc = self.lib.fme_mc_invalid_count(self.h)
        if rc < 0:
            _check(self.lib, rc)
        return rc

    def mc_last_ms(self):
        ms = C.c_float()
        _check(self.lib, self.lib.fme_mc_last_ms(self.h, C.byref(ms)))
        return ms.value

    def set_lambda(self, lid, lam):
        _check(self.lib, self.lib.fme_set_lambda(self.h, lid, float(lam)))

    def set_motion_lambda(self, lid, ml):
        _check(self.lib, self.lib.fme_set_motion_lambda(self.h, lid, float(ml)))

    def set_keys(self, keys, stream=None):
        keys = np.ascontiguousarray(keys, dtype=np.int16)
        _check(self.lib, self.lib.fme_set_keys(self.h, _ptr(keys), keys.size, stream))

    def load_nn(self, params):
        p = np.ascontiguousarray(params, dtype=np.float32)
        if p.size != NN_PARAMS:
            raise FmeError(-1, f"{p.size} NN parameters, expected {NN_PARAMS}")
        _check(self.lib, self.lib.fme_load_nn_weights(self.h, _ptr(p), p.size))

    def load_nn_net(self, net):
        """A generic NN_pred net (nnfme.weights.NnNet) for nn_mode 2 (fme_load_nn_net)."""
        # input flags need ABI 10 (FME_NN_IN_SLOT_RESET) / 11 (FME_NN_IN_TZ_RING): an older A/B
        # variant would ignore them and run a different input path without a word
        need = 11 if net.input_flags & 2 else (10 if net.input_flags else 0)
        if getattr(self.lib, "fme_abi", ABI_VERSION) < need:
            raise FmeError(-1, f"net input flags 0x{net.input_flags:x} need ABI {need}, library has "
                               f"{self.lib.fme_abi}")
        d = net.desc_struct()
        p = np.ascontiguousarray(net.params, dtype=np.float64)
        _check(self.lib, self.lib.fme_load_nn_net(self.h, C.byref(d), _ptr(p), p.size))

    def set_nn_engine(self, engine):
        """0: exact (bit-exact to the reference's loops), 1: MFMA GEMM (k-ordered FMA chain)."""
        _check(self.lib, self.lib.fme_set_nn_engine(self.h, int(engine)))

    def set_nn_margin_output(self, d_ptr, capacity=0):
        """Device float[capacity] receiving top-1 minus top-2 of each later batch's NN outputs (0: off);
        a later batch of more than `capacity` jobs is rejected."""
        _check(self.lib, self.lib.fme_set_nn_margin_output(self.h, C.c_void_p(d_ptr) if d_ptr else None,
                                                           int(capacity) if d_ptr else 0))

    def set_nn_logit_output(self, d_ptr, capacity=0):
        """Device array of capacity x 49 values in the net's precision receiving OUT before the
        output activation for each later nn_mode 2 batch (0: off)."""
        _check(self.lib, self.lib.fme_set_nn_logit_output(self.h, C.c_void_p(d_ptr) if d_ptr else None,
                                                          int(capacity) if d_ptr else 0))

    def nn_reset(self):
        _check(self.lib, self.lib.fme_nn_reset_state(self.h))

    def nn_get_state(self):
        out = np.zeros(12, np.uint32)
        _check(self.lib, self.lib.fme_nn_get_state(self.h, _ptr(out)))
        return out

    def nn_set_state(self, state):
        st = np.ascontiguousarray(state, dtype=np.uint32)
        assert st.size == 12
        _check(self.lib, self.lib.fme_nn_set_state(self.h, _ptr(st)))

    # -- work ---------------------------------------------------------------------------
    def refine(self, jobs, stream=None):
        jobs = np.ascontiguousarray(jobs, dtype=JOB_DTYPE)
        res = np.zeros(len(jobs), dtype=RESULT_DTYPE)
        _check(self.lib, self.lib.fme_refine(self.h, _ptr(jobs), _ptr(res), len(jobs), stream))
        return res

    def refine_device(self, jobs_ptr, res_ptr, n, stream=None):
        """Device-resident jobs/results (e.g. torch uint8 tensors' data_ptr()); asynchronous on
        `stream` (no host synchronisation).  A rejected batch shows in refine_status()."""
        _check(self.lib, self.lib.fme_refine_device(self.h, C.c_void_p(jobs_ptr), C.c_void_p(res_ptr), n, stream))

    def refine_mv(self, jobs, stream=None):
        """fme_refine_mv: the 16-byte xMotionEstimation outputs (MV_RESULT_DTYPE) per job."""
        jobs = np.ascontiguousarray(jobs, dtype=JOB_DTYPE)
        out = np.zeros(len(jobs), dtype=MV_RESULT_DTYPE)
        _check(self.lib, self.lib.fme_refine_mv(self.h, _ptr(jobs), _ptr(out), len(jobs), stream))
        return out

    def refine_mv_device(self, jobs_ptr, out_ptr, n, stream=None):
        _check(self.lib, self.lib.fme_refine_mv_device(self.h, C.c_void_p(jobs_ptr), C.c_void_p(out_ptr), n, stream))

    def refine_packed_device(self, pk_ptr, key_base_ptr, res_ptr, n, stream=None):
        """fme_refine_packed_device: device-resident packed jobs (pack_jobs) -> full records."""
        _check(self.lib, self.lib.fme_refine_packed_device(self.h, C.c_void_p(pk_ptr), C.c_void_p(key_base_ptr),
                                                           C.c_void_p(res_ptr), n, stream))

    def refine_mv_packed_device(self, pk_ptr, key_base_ptr, out_ptr, n, stream=None):
        """fme_refine_mv_packed_device: device-resident packed jobs -> 16-byte fme_mv_result rows."""
        _check(self.lib, self.lib.fme_refine_mv_packed_device(self.h, C.c_void_p(pk_ptr), C.c_void_p(key_base_ptr),
                                                              C.c_void_p(out_ptr), n, stream))

    def refine_status(self):
        """Waits for the last batch: the number of jobs that made the device reject it (0: ran)."""
        rc = self.lib.fme_refine_status(self.h)
        if rc < 0:
            _check(self.lib, rc)
        return rc

    def nn_copy_state_device(self, d_ptr, stream=None):
        """Enqueue a copy of the carried NN state (12 words) to device memory at d_ptr."""
        _check(self.lib, self.lib.fme_nn_copy_state_device(self.h, C.c_void_p(d_ptr), stream))

    def download_device(self, d_src_ptr, h_dst_ptr, nbytes, workgroups=0, stream=None):
        """Copy nbytes of device rows into pinned host memory with the library's few-workgroup copy
        kernel (fme_download_device), asynchronous on `stream`."""
        _check(self.lib, self.lib.fme_download_device(self.h, C.c_void_p(d_src_ptr), C.c_void_p(h_dst_ptr),
                                                      nbytes, workgroups, stream))

    PI_PHASES = ("expand", "amvp", "setup", "level_chain", "refine", "decide", "bi_rounds", "total")

    def pred_inter_phases(self):
        """{phase: ms} of the last fme_pred_inter_p / _b call (fme_pred_inter_phases)."""
        out = np.zeros(8, np.float64)
        _check(self.lib, self.lib.fme_pred_inter_phases(self.h, _ptr(out), 8))
        return dict(zip(self.PI_PHASES, out.tolist()))

    def set_search_event(self, event):
        """Record `event` (a torch.cuda.Event or a raw hipEvent_t, None: off) on the batch stream
        right before each later batch's search kernel (fme_set_search_event)."""
        if event is not None and hasattr(event, "cuda_event"):
            event = event.cuda_event
        _check(self.lib, self.lib.fme_set_search_event(self.h, C.c_void_p(event) if event else None))

    def warm_copy_engines(self):
        """One small copy per SDMA engine and direction before a copy pipeline (fme_warm_copy_engines);
        returns the number of engines warmed."""
        n = C.c_int(0)
        _check(self.lib, self.lib.fme_warm_copy_engines(self.h, C.byref(n)))
        return n.value

    def set_search_reserve(self, workgroups):
        """Resident search workgroups left free for a few-workgroup kernel beside it (fme_set_search_reserve)."""
        _check(self.lib, self.lib.fme_set_search_reserve(self.h, int(workgroups)))

    def frac_dif_single(self, key, ref_window, ref_origin, mv_int, mvp, motion_lambda, lossless=False):
        """xPatternSearchFracDIF argument list: key block (int16 HxW), a padded reference
        plane (int16) with the PU origin at ref_origin=(row, col), full-pel mv_int, qpel mvp."""
        key = np.ascontiguousarray(key, dtype=np.int16)
        ref = np.ascontiguousarray(ref_window, dtype=np.int16)
        h, w = key.shape
        r0, c0 = ref_origin
        base = ref.ctypes.data + (r0 * ref.shape[1] + c0) * 2
        half = np.zeros(2, np.int16)
        qtr = np.zeros(2, np.int16)
        cost = np.zeros(1, np.uint32)
        _check(self.lib, self.lib.fme_frac_dif_single(
            self.h, int(lossless), _ptr(key), w, w, h, C.c_void_p(base), ref.shape[1],
            int(mv_int[0]), int(mv_int[1]), int(mvp[0]), int(mvp[1]), float(motion_lambda),
            _ptr(half), _ptr(qtr), _ptr(cost)))
        return (int(half[0]), int(half[1])), (int(qtr[0]), int(qtr[1])), int(cost[0])

    def search_kernel_of_shape(self, w, h):
        """0: the main search kernel serves w x h PUs, 1: an auxiliary one, -1: unsupported."""
        return int(self.lib.fme_search_kernel_of_shape(int(w), int(h)))

    def set_profiling(self, enable=True):
        _check(self.lib, self.lib.fme_set_profiling(self.h, int(enable)))

    def last_timings(self):
        """Device ms of the last profiled batch, keyed by TIMING_NAMES."""
        ms = np.zeros(len(TIMING_NAMES), np.float32)
        _check(self.lib, self.lib.fme_last_timings(self.h, _ptr(ms), ms.size))
        return dict(zip(TIMING_NAMES, ms.tolist()))

    def single_last_device_us(self, phases=False):
        """Device microseconds of the last single-PU call (the server's read of the request to its
        answer); phases=True: also the FracDIF checkpoints (payload in LDS, first stage, half
        distortions, quarter distortions)."""
        us = np.zeros(5, np.float32)
        _check(self.lib, self.lib.fme_single_last_device_us(self.h, _ptr(us), 5))
        return us.tolist() if phases else float(us[0])

    def accumulated_timings(self, reset=True):
        """(batches, {name: summed device ms}) over the profiled batches since the last reset."""
        ms = np.zeros(len(TIMING_NAMES), np.float64)
        n = self.lib.fme_accumulated_timings(self.h, _ptr(ms), ms.size, int(reset))
        if n < 0:
            _check(self.lib, n)
        return n, dict(zip(TIMING_NAMES, ms.tolist()))

    def nn_pred_single(self, e, c, pu_h, pu_w):
        e = np.ascontiguousarray(e, dtype=np.uint32)
        cls = C.c_int()
        out4 = np.zeros(4, np.int16)
        _check(self.lib, self.lib.fme_nn_pred_single(self.h, _ptr(e), int(c), int(pu_h), int(pu_w), C.byref(cls), _ptr(out4)))
        return cls.value, tuple(int(v) for v in out4)


def pack_jobs(jobs, lib=None):
    """fme_pack_jobs: fme_job rows -> (JOB_PACKED_DTYPE rows, int32 key_base per 64 jobs).  Raises
    FmeError (FME_E_UNSUPPORTED) for a batch outside the packed form (include/fme.h)."""
    from .abi import JOB_PACKED_DTYPE, PACK_WAVE
    lib = lib or load_library()
    jobs = np.ascontiguousarray(jobs, dtype=JOB_DTYPE)
    out = np.zeros(len(jobs), dtype=JOB_PACKED_DTYPE)
    base = np.zeros((len(jobs) + PACK_WAVE - 1) // PACK_WAVE, dtype=np.int32)
    _check(lib, lib.fme_pack_jobs(_ptr(jobs), len(jobs), _ptr(out), _ptr(base)))
    return out, base


def unpack_jobs(packed, key_base, lib=None):
    """fme_unpack_jobs: the canonical fme_job rows of packed jobs (what the device unpacks)."""
    from .abi import JOB_PACKED_DTYPE
    lib = lib or load_library()
    packed = np.ascontiguousarray(packed, dtype=JOB_PACKED_DTYPE)
    key_base = np.ascontiguousarray(key_base, dtype=np.int32)
    out = np.zeros(len(packed), dtype=JOB_DTYPE)
    _check(lib, lib.fme_unpack_jobs(_ptr(packed), _ptr(key_base), len(packed), _ptr(out)))
    return out
