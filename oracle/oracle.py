"""ctypes bindings of the CPU oracle (liboracle.so) and the reference harness (_ref/libhmref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product path (hm16.9-nn_fme_amd/).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# FME_ORACLE_SO: the sanitizer build (liboracle_asan.so, tests/test_sanitize.py) instead
ORACLE_SO = os.environ.get("FME_ORACLE_SO") or os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libhmref.so")

_P = C.c_void_p


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class _ConfigStruct(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("bit_depth", "use_hadamard", "nn_mode", "qp",
                                         "fast_inter_mode", "max_jobs")]


def _load(path):
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (run `make -C oracle` / `make -C oracle ref`)")
    return C.CDLL(path)


class Oracle:
    """Plain-C restatement (fme_oracle.c)."""

    def __init__(self, use_hadamard=1, nn_mode=1, qp=22, fast_inter_mode=1, bit_depth=8):
        self.lib = lib = _load(ORACLE_SO)
        self.bit_depth = bit_depth
        lib.orc_ctx_size.restype = C.c_size_t
        lib.orc_eg_bits.restype = C.c_uint32
        lib.orc_eg_bits.argtypes = [C.c_int]
        lib.orc_cost.restype = C.c_uint32
        lib.orc_cost.argtypes = [C.c_double, C.c_uint32]
        lib.orc_satd.restype = C.c_uint32
        lib.orc_satd.argtypes = [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int]
        lib.orc_sad.restype = C.c_uint32
        lib.orc_sad.argtypes = [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int]
        lib.orc_sse.restype = C.c_uint32
        lib.orc_sse.argtypes = [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int]
        lib.orc_pred_block.argtypes = [_P] + [C.c_int] * 6 + [_P]
        lib.orc_nn_forward.restype = C.c_int
        lib.orc_nn_forward.argtypes = [_P, _P, C.c_uint32, C.c_int, C.c_int, _P]
        lib.orc_emi_push_count.restype = C.c_int
        lib.orc_emi_push_count.argtypes = [C.c_int] * 6
        lib.orc_init.argtypes = [_P, _P]
        lib.orc_set_picture.argtypes = [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int]
        lib.orc_set_picture16.argtypes = [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int]
        lib.orc_set_lambda.argtypes = [_P, C.c_int, C.c_double]
        lib.orc_set_motion_lambda.argtypes = [_P, C.c_int, C.c_double]
        lib.orc_set_keys.argtypes = [_P, _P, C.c_size_t]
        lib.orc_load_nn.argtypes = [_P, _P]
        lib.orc_nn_reset.argtypes = [_P]
        lib.orc_nn_get_state.argtypes = [_P, _P]
        lib.orc_nn_set_state.argtypes = [_P, _P]
        lib.orc_refine.restype = C.c_int
        lib.orc_refine.argtypes = [_P, _P, _P, C.c_int]
        lib.orc_integer_search.restype = C.c_int
        lib.orc_integer_search.argtypes = [_P, _P, _P, _P, C.c_int]
        lib.orc_integer_search_ring.restype = C.c_int
        lib.orc_integer_search_ring.argtypes = [_P, _P, _P, _P, _P, C.c_int]
        lib.orc_integer_search2.restype = C.c_int
        lib.orc_integer_search2.argtypes = [_P, _P, _P, _P, C.c_int]
        lib.orc_set_nn_inputs.argtypes = [_P, _P, C.c_int]
        lib.orc_pred_inter_p.restype = C.c_int
        lib.orc_pred_inter_p.argtypes = [_P, _P, _P, C.c_int]
        lib.orc_pred_inter_reset.argtypes = [_P]
        lib.orc_template_cost.restype = C.c_uint32
        lib.orc_template_cost.argtypes = [_P, _P, C.c_int, C.c_int]
        lib.orc_tz_counters.argtypes = [_P, C.c_int]
        lib.orc_pred_inter_b.restype = C.c_int
        lib.orc_pred_inter_b.argtypes = [_P, _P, _P, C.c_int]
        lib.orc_bi_key.argtypes = [_P] + [C.c_int] * 11 + [_P]
        lib.orc_mc.restype = C.c_int
        lib.orc_mc.argtypes = [_P, _P, C.c_int, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int]
        lib.orc_nn_param_count.restype = C.c_int
        lib.orc_nn_param_count.argtypes = [_P]
        lib.orc_load_nn_net.restype = C.c_int
        lib.orc_load_nn_net.argtypes = [_P, _P, _P, C.c_int]
        lib.orc_nn_net_forward.restype = C.c_int
        lib.orc_nn_net_forward.argtypes = [_P, _P, C.c_uint32, C.c_int, C.c_int, _P]
        lib.orc_nn_net_forward_pre.restype = C.c_int
        lib.orc_nn_net_forward_pre.argtypes = [_P, _P, C.c_uint32, C.c_int, C.c_int, _P, _P]
        self._buf = C.create_string_buffer(lib.orc_ctx_size())
        self.ctx = C.cast(self._buf, C.c_void_p)
        cfg = _ConfigStruct(bit_depth, use_hadamard, nn_mode, qp, fast_inter_mode, 0)
        lib.orc_init(self.ctx, C.byref(cfg))
        self._keep = {}

    def set_picture(self, pid, luma):
        """8-bit planes (uint8), or 16-bit samples (uint16) of the context's bit depth (main10)."""
        if self.bit_depth > 8:
            luma = np.ascontiguousarray(luma, dtype=np.uint16)
            self._keep[("pic", pid)] = luma
            self.lib.orc_set_picture16(self.ctx, pid, _ptr(luma), luma.shape[1], luma.shape[1], luma.shape[0])
            return
        luma = np.ascontiguousarray(luma, dtype=np.uint8)
        self._keep[("pic", pid)] = luma
        self.lib.orc_set_picture(self.ctx, pid, _ptr(luma), luma.shape[1], luma.shape[1], luma.shape[0])

    def set_lambda(self, lid, lam):
        self.lib.orc_set_lambda(self.ctx, lid, lam)

    def set_keys(self, keys):
        keys = np.ascontiguousarray(keys, dtype=np.int16)
        self._keep["keys"] = keys
        self.lib.orc_set_keys(self.ctx, _ptr(keys), keys.size)

    def load_nn(self, params):
        p = np.ascontiguousarray(params, dtype=np.float32)
        self.lib.orc_load_nn(self.ctx, _ptr(p))

    def nn_reset(self):
        self.lib.orc_nn_reset(self.ctx)

    def load_nn_net(self, net):
        """net: nnfme.weights.NnNet (descriptor + float64 parameters), nn_mode 2."""
        d = net.desc_struct()
        p = np.ascontiguousarray(net.params, dtype=np.float64)
        self._keep["net"] = (d, p)
        rc = self.lib.orc_load_nn_net(self.ctx, C.byref(d), _ptr(p), p.size)
        if rc != 0:
            raise RuntimeError(f"orc_load_nn_net failed: {rc}")

    def nn_net_forward(self, e, c, h, w):
        """One NN_pred() call of the loaded generic net: (class, OUT[49] as float64)."""
        e = np.ascontiguousarray(e, dtype=np.uint32)
        logits = np.zeros(49, np.float64)
        cls = self.lib.orc_nn_net_forward(self.ctx, _ptr(e), int(c), int(h), int(w), _ptr(logits))
        if cls < 0:
            raise RuntimeError(f"orc_nn_net_forward failed: {cls}")
        return cls, logits

    def nn_net_forward_pre(self, e, c, h, w):
        """(class, OUT[49], OUT before the output activation[49]), both as float64."""
        e = np.ascontiguousarray(e, dtype=np.uint32)
        logits = np.zeros(49, np.float64)
        pre = np.zeros(49, np.float64)
        cls = self.lib.orc_nn_net_forward_pre(self.ctx, _ptr(e), int(c), int(h), int(w), _ptr(logits), _ptr(pre))
        if cls < 0:
            raise RuntimeError(f"orc_nn_net_forward_pre failed: {cls}")
        return cls, logits, pre

    def nn_get_state(self):
        out = np.zeros(12, np.uint32)
        self.lib.orc_nn_get_state(self.ctx, _ptr(out))
        return out

    def nn_set_state(self, st):
        st = np.ascontiguousarray(st, dtype=np.uint32)
        self.lib.orc_nn_set_state(self.ctx, _ptr(st))

    def refine(self, jobs):
        from nnfme.abi import RESULT_DTYPE
        jobs = np.ascontiguousarray(jobs)
        res = np.zeros(len(jobs), dtype=RESULT_DTYPE)
        rc = self.lib.orc_refine(self.ctx, _ptr(jobs), _ptr(res), len(jobs))
        if rc != 0:
            raise RuntimeError(f"orc_refine failed: {rc}")
        return res

    def nn_class(self, params, e, c, h, w):
        p = np.ascontiguousarray(params, dtype=np.float32)
        e = np.ascontiguousarray(e, dtype=np.uint32)
        logits = np.zeros(49, dtype=np.float32)
        cls = self.lib.orc_nn_forward(_ptr(p), _ptr(e), int(c), int(h), int(w), _ptr(logits))
        return cls, logits

    def integer_search(self, jobs, ext):
        """orc_integer_search: returns (jobs with mv_x/mv_y = the integer MV, sad); fme_tz_ext2
        records (24 bytes) go to orc_integer_search2."""
        if np.asarray(ext).dtype.itemsize == 24:
            return self.integer_search2(jobs, ext)
        jobs = np.array(jobs, copy=True)
        ext = np.ascontiguousarray(ext)
        sad = np.zeros(len(jobs), np.uint32)
        rc = self.lib.orc_integer_search(self.ctx, _ptr(jobs), _ptr(ext), _ptr(sad), len(jobs))
        if rc != 0:
            raise RuntimeError(f"orc_integer_search failed: {rc}")
        return jobs, sad

    def integer_search2(self, jobs, ext2):
        """orc_integer_search2: fme_tz_ext2 records (FastSearch 0 / 3 flags, neighbour predictors)."""
        jobs = np.array(jobs, copy=True)
        ext2 = np.ascontiguousarray(ext2)
        assert ext2.dtype.itemsize == 24
        sad = np.zeros(len(jobs), np.uint32)
        rc = self.lib.orc_integer_search2(self.ctx, _ptr(jobs), _ptr(ext2), _ptr(sad), len(jobs))
        if rc != 0:
            raise RuntimeError(f"orc_integer_search2 failed: {rc}")
        return jobs, sad

    def integer_search_ring(self, jobs, ext):
        """orc_integer_search_ring: (jobs, sad, nn_in[n][9]); FME_TZ_RING jobs run the backups' tail."""
        jobs = np.array(jobs, copy=True)
        ext = np.ascontiguousarray(ext)
        sad = np.zeros(len(jobs), np.uint32)
        nn_in = np.zeros((len(jobs), 9), np.uint32)
        rc = self.lib.orc_integer_search_ring(self.ctx, _ptr(jobs), _ptr(ext), _ptr(sad), _ptr(nn_in), len(jobs))
        if rc != 0:
            raise RuntimeError(f"orc_integer_search_ring failed: {rc}")
        return jobs, sad, nn_in

    def set_nn_inputs(self, rows):
        """The FME_JOB_NN_IN input rows of the next refine calls ([n][9] uint32; None unbinds)."""
        if rows is None:
            self._keep.pop("nn_in", None)
            self.lib.orc_set_nn_inputs(self.ctx, None, 0)
            return
        rows = np.ascontiguousarray(rows, dtype=np.uint32).reshape(-1, 9)
        self._keep["nn_in"] = rows
        self.lib.orc_set_nn_inputs(self.ctx, _ptr(rows), len(rows))

    def pred_inter_p(self, reqs):
        """orc_pred_inter_p: predInterSearch's P-slice PU / reference loop, one fme_pu_res per request."""
        from nnfme.abi import PU_REQ_DTYPE, PU_RES_DTYPE
        reqs = np.ascontiguousarray(reqs, dtype=PU_REQ_DTYPE)
        res = np.zeros(len(reqs), dtype=PU_RES_DTYPE)
        rc = self.lib.orc_pred_inter_p(self.ctx, _ptr(reqs), _ptr(res), len(reqs))
        if rc != 0:
            raise RuntimeError(f"orc_pred_inter_p failed: {rc}")
        return res

    def pred_inter_reset(self):
        self.lib.orc_pred_inter_reset(self.ctx)

    def tz_counters(self, reset=True):
        """(points tested, distortion samples read) by the integer searches since the last reset."""
        out = np.zeros(2, np.uint64)
        self.lib.orc_tz_counters(_ptr(out), int(bool(reset)))
        return int(out[0]), int(out[1])

    def pred_inter_b(self, reqs):
        """orc_pred_inter_b: predInterSearch on a B slice, one fme_pu_res_b per request."""
        from nnfme.abi import PU_REQ_B_DTYPE, PU_RES_B_DTYPE
        reqs = np.ascontiguousarray(reqs, dtype=PU_REQ_B_DTYPE)
        res = np.zeros(len(reqs), dtype=PU_RES_B_DTYPE)
        rc = self.lib.orc_pred_inter_b(self.ctx, _ptr(reqs), _ptr(res), len(reqs))
        if rc != 0:
            raise RuntimeError(f"orc_pred_inter_b failed: {rc}")
        return res

    def bi_key(self, org_id, ref_id, x, y, w, h, cu_x, cu_y, mvx, mvy, clip=False):
        """orc_bi_key: 2 * org - the other list's uni-pred luma prediction (removeHighFreq)."""
        key = np.zeros((h, w), np.int16)
        self.lib.orc_bi_key(self.ctx, org_id, ref_id, x, y, w, h, cu_x, cu_y, mvx, mvy, int(bool(clip)), _ptr(key))
        return key

    def template_cost(self, req, k, m):
        """orc_template_cost: xGetTemplateCost of candidate m of reference k of one fme_pu_req."""
        from nnfme.abi import PU_REQ_DTYPE
        r = np.ascontiguousarray(np.asarray(req, dtype=PU_REQ_DTYPE).reshape(1))
        return int(self.lib.orc_template_cost(self.ctx, _ptr(r), int(k), int(m)))

    def mc(self, pics, mc_jobs, y, cb, cr, wp=None):
        """orc_mc: pics = {id: (Y, Cb, Cr)} reference pictures; predicts into y/cb/cr in place.
        wp: [2][refs][3][3] (iWeight, iOffset, uiLog2WeightDenom) for the FME_MC_WP jobs (orc_mc_wp)."""
        class Yuv(C.Structure):
            _fields_ = [("y", C.c_void_p), ("cb", C.c_void_p), ("cr", C.c_void_p), ("y_stride", C.c_int),
                        ("c_stride", C.c_int), ("width", C.c_int), ("height", C.c_int)]
        arr = (Yuv * 64)()
        keep = []
        for pid, (py, pcb, pcr) in pics.items():
            py, pcb, pcr = (np.ascontiguousarray(a, dtype=np.uint8) for a in (py, pcb, pcr))
            keep += [py, pcb, pcr]
            arr[pid] = Yuv(py.ctypes.data, pcb.ctypes.data, pcr.ctypes.data, py.shape[1], pcb.shape[1],
                           py.shape[1], py.shape[0])
        jobs = np.ascontiguousarray(mc_jobs)
        h, w = y.shape
        if wp is not None:
            t = np.zeros((2, 64, 3, 3), np.int32)
            t[..., 0] = 1
            wp = np.asarray(wp, dtype=np.int32)
            t[:, :wp.shape[1]] = wp
            self.lib.orc_mc_wp.argtypes = [_P, _P, C.c_int, _P, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int]
            rc = self.lib.orc_mc_wp(C.cast(arr, C.c_void_p), _ptr(jobs), len(jobs), _ptr(t), _ptr(y), y.shape[1],
                                    _ptr(cb), _ptr(cr), cb.shape[1], w, h)
        else:
            rc = self.lib.orc_mc(C.cast(arr, C.c_void_p), _ptr(jobs), len(jobs), _ptr(y), y.shape[1], _ptr(cb), _ptr(cr),
                                 cb.shape[1], w, h)
        if rc != 0:
            raise RuntimeError(f"orc_mc: invalid job {-1 - rc}")

    def pred_block(self, luma, x0, y0, w, h, qx, qy):
        """orc_pred_block on a uint8 plane, or a uint16 plane at the oracle's bit depth."""
        wide = np.asarray(luma).dtype == np.uint16
        luma = np.ascontiguousarray(luma, dtype=np.uint16 if wide else np.uint8)
        out = np.zeros((h, w), dtype=np.int16)
        # build an orc_picture on the fly: {const uint8_t*, int stride, width, height, luma16, bd}
        class Pic(C.Structure):
            _fields_ = [("luma", C.c_void_p), ("stride", C.c_int), ("width", C.c_int), ("height", C.c_int),
                        ("luma16", C.c_void_p), ("bd", C.c_int)]
        if wide:
            p = Pic(None, luma.shape[1], luma.shape[1], luma.shape[0], luma.ctypes.data, self.bit_depth)
        else:
            p = Pic(luma.ctypes.data, luma.shape[1], luma.shape[1], luma.shape[0], None, 8)
        self.lib.orc_pred_block(C.byref(p), x0, y0, w, h, qx, qy, _ptr(out))
        return out


class Reference:
    """The reference's own TLibCommon primitives driven in TEncSearch order (_ref)."""

    def __init__(self, use_hadamard=1, nn_mode=1, fast_inter_mode=1, bit_depth=8):
        self.lib = lib = _load(REF_SO)
        self.bit_depth = bit_depth
        lib.ref_create.restype = C.c_void_p
        lib.ref_create.argtypes = [C.c_int, C.c_int, C.c_int]
        lib.ref_destroy.argtypes = [_P]
        lib.ref_set_picture.argtypes = [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int]
        lib.ref_set_picture16.argtypes = [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int]
        lib.ref_set_bit_depth.argtypes = [_P, C.c_int]
        lib.ref_set_lambda.argtypes = [_P, C.c_int, C.c_double]
        lib.ref_set_keys.argtypes = [_P, _P, C.c_size_t]
        lib.ref_load_nn.argtypes = [_P, _P]
        lib.ref_nn_reset.argtypes = [_P]
        lib.ref_nn_set_state.argtypes = [_P, _P]
        lib.ref_nn_class.restype = C.c_int
        lib.ref_nn_class.argtypes = [_P, _P, C.c_uint32, C.c_int, C.c_int]
        lib.ref_pred_block.restype = C.c_int
        lib.ref_pred_block.argtypes = [_P] + [C.c_int] * 7 + [_P]
        lib.ref_load_nn_net.argtypes = [_P, _P, _P, C.c_int]
        lib.ref_nn_net_class.restype = C.c_int
        lib.ref_nn_net_class.argtypes = [_P, _P, C.c_uint32, C.c_int, C.c_int, _P]
        lib.ref_satd.restype = C.c_uint32
        lib.ref_satd.argtypes = [_P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int]
        lib.ref_refine.restype = C.c_int
        lib.ref_refine.argtypes = [_P, _P, _P, C.c_int]
        lib.ref_set_picture_yuv.restype = C.c_int
        lib.ref_set_picture_yuv.argtypes = [_P, C.c_int, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int]
        lib.ref_set_picture_yuv16.restype = C.c_int
        lib.ref_set_picture_yuv16.argtypes = [_P, C.c_int, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int]
        lib.ref_mc16.restype = C.c_int
        lib.ref_mc16.argtypes = [_P, _P, C.c_int, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int]
        lib.ref_integer_search.restype = C.c_int
        lib.ref_integer_search.argtypes = [_P, _P, _P, _P, C.c_int]
        lib.ref_integer_search_ring.restype = C.c_int
        lib.ref_integer_search_ring.argtypes = [_P, _P, _P, _P, _P, C.c_int]
        lib.ref_integer_search2.restype = C.c_int
        lib.ref_integer_search2.argtypes = [_P, _P, _P, _P, C.c_int]
        lib.ref_set_nn_inputs.argtypes = [_P, _P, C.c_int]
        lib.ref_template_cost.restype = C.c_uint32
        lib.ref_template_cost.argtypes = [_P] + [C.c_int] * 12
        lib.ref_bi_key.restype = C.c_int
        lib.ref_bi_key.argtypes = [_P] + [C.c_int] * 11 + [_P]
        lib.ref_mc.restype = C.c_int
        lib.ref_mc.argtypes = [_P, _P, C.c_int, _P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int]
        lib.ref_set_wp.argtypes = [_P, C.c_int, C.c_int, _P]
        self.h = lib.ref_create(use_hadamard, fast_inter_mode, nn_mode)
        if bit_depth != 8:
            lib.ref_set_bit_depth(self.h, bit_depth)

    def __del__(self):
        try:
            self.lib.ref_destroy(self.h)
        except Exception:
            pass

    def set_picture(self, pid, luma):
        """8-bit planes, or 16-bit samples at the harness's bit depth (main10)."""
        if self.bit_depth > 8:
            luma = np.ascontiguousarray(luma, dtype=np.uint16)
            self.lib.ref_set_picture16(self.h, pid, _ptr(luma), luma.shape[1], luma.shape[1], luma.shape[0])
            return
        luma = np.ascontiguousarray(luma, dtype=np.uint8)
        self.lib.ref_set_picture(self.h, pid, _ptr(luma), luma.shape[1], luma.shape[1], luma.shape[0])

    def set_picture_yuv(self, pid, y, cb, cr):
        """A 4:2:0 reference picture for mc(): uint8 planes, or uint16 planes at bit depth 10."""
        if np.asarray(y).dtype == np.uint16:
            y, cb, cr = (np.ascontiguousarray(a, dtype=np.uint16) for a in (y, cb, cr))
            self.lib.ref_set_picture_yuv16(self.h, pid, _ptr(y), y.shape[1], _ptr(cb), _ptr(cr), cb.shape[1],
                                           y.shape[1], y.shape[0])
            return
        y, cb, cr = (np.ascontiguousarray(a, dtype=np.uint8) for a in (y, cb, cr))
        self.lib.ref_set_picture_yuv(self.h, pid, _ptr(y), y.shape[1], _ptr(cb), _ptr(cr), cb.shape[1], y.shape[1],
                                     y.shape[0])

    def integer_search(self, jobs, ext):
        if np.asarray(ext).dtype.itemsize == 24:   # fme_tz_ext2
            return self.integer_search2(jobs, ext)
        jobs = np.array(jobs, copy=True)
        ext = np.ascontiguousarray(ext)
        sad = np.zeros(len(jobs), np.uint32)
        rc = self.lib.ref_integer_search(self.h, _ptr(jobs), _ptr(ext), _ptr(sad), len(jobs))
        if rc != 0:
            raise RuntimeError(f"ref_integer_search failed: {rc}")
        return jobs, sad

    def integer_search2(self, jobs, ext2):
        jobs = np.array(jobs, copy=True)
        ext2 = np.ascontiguousarray(ext2)
        assert ext2.dtype.itemsize == 24
        sad = np.zeros(len(jobs), np.uint32)
        rc = self.lib.ref_integer_search2(self.h, _ptr(jobs), _ptr(ext2), _ptr(sad), len(jobs))
        if rc != 0:
            raise RuntimeError(f"ref_integer_search2 failed: {rc}")
        return jobs, sad

    def integer_search_ring(self, jobs, ext):
        jobs = np.array(jobs, copy=True)
        ext = np.ascontiguousarray(ext)
        sad = np.zeros(len(jobs), np.uint32)
        nn_in = np.zeros((len(jobs), 9), np.uint32)
        rc = self.lib.ref_integer_search_ring(self.h, _ptr(jobs), _ptr(ext), _ptr(sad), _ptr(nn_in), len(jobs))
        if rc != 0:
            raise RuntimeError(f"ref_integer_search_ring failed: {rc}")
        return jobs, sad, nn_in

    def set_nn_inputs(self, rows):
        if rows is None:
            self.lib.ref_set_nn_inputs(self.h, None, 0)
            return
        rows = np.ascontiguousarray(rows, dtype=np.uint32).reshape(-1, 9)
        self._rows = rows   # the library keeps the pointer: keep the array alive
        self.lib.ref_set_nn_inputs(self.h, _ptr(rows), len(rows))

    def set_wp(self, lst, pid, params):
        """Explicit weighted-prediction parameters of picture pid in list lst for FME_MC_WP jobs:
        3 rows (Y, Cb, Cr) of (iWeight, iOffset, uiLog2WeightDenom)."""
        p = np.ascontiguousarray(np.asarray(params, dtype=np.int32).reshape(9))
        self.lib.ref_set_wp(self.h, int(lst), int(pid), _ptr(p))

    def mc(self, mc_jobs, y, cb, cr):
        """Predictions into the planes y / cb / cr in place (uint8, or uint16 at bit depth 10)."""
        jobs = np.ascontiguousarray(mc_jobs)
        h, w = y.shape
        f = self.lib.ref_mc16 if y.dtype == np.uint16 else self.lib.ref_mc
        rc = f(self.h, _ptr(jobs), len(jobs), _ptr(y), y.shape[1], _ptr(cb), _ptr(cr), cb.shape[1], w, h)
        if rc != 0:
            raise RuntimeError(f"ref_mc: invalid job {-1 - rc}")

    def set_lambda(self, lid, lam):
        self.lib.ref_set_lambda(self.h, lid, lam)

    def template_cost(self, org_id, ref_id, x, y, w, h, cu_x, cu_y, mvx, mvy, bits, lambda_id):
        """xGetTemplateCost over the reference's TComInterpolationFilter / TComRdCost."""
        v = self.lib.ref_template_cost(self.h, org_id, ref_id, x, y, w, h, cu_x, cu_y, mvx, mvy, bits, lambda_id)
        if v == 0xFFFFFFFF:
            raise RuntimeError("ref_template_cost: unset picture or bad slot")
        return v

    def bi_key(self, org_id, ref_id, x, y, w, h, cu_x, cu_y, mvx, mvy, clip=False):
        """The reference's TComYuv::removeHighFreq on the other list's prediction (ref_bi_key)."""
        key = np.zeros((h, w), np.int16)
        if self.lib.ref_bi_key(self.h, org_id, ref_id, x, y, w, h, cu_x, cu_y, mvx, mvy, int(bool(clip)), _ptr(key)):
            raise RuntimeError("ref_bi_key: unset picture or bad slot")
        return key

    def set_keys(self, keys):
        keys = np.ascontiguousarray(keys, dtype=np.int16)
        self.lib.ref_set_keys(self.h, _ptr(keys), keys.size)

    def load_nn(self, params):
        p = np.ascontiguousarray(params, dtype=np.float32)
        self.lib.ref_load_nn(self.h, _ptr(p))

    def nn_reset(self):
        self.lib.ref_nn_reset(self.h)

    def nn_set_state(self, st):
        """NN_pred's carried globals from a 12-word state (fme_nn_get_state's layout)."""
        st = np.ascontiguousarray(st, dtype=np.uint32)
        assert st.size >= 11
        self.lib.ref_nn_set_state(self.h, _ptr(st))

    def load_nn_net(self, net):
        d = net.desc_struct()
        p = np.ascontiguousarray(net.params, dtype=np.float64)
        self.lib.ref_load_nn_net(self.h, C.byref(d), _ptr(p), p.size)

    def nn_net_class(self, e, c, h, w):
        e = np.ascontiguousarray(e, dtype=np.uint32)
        logits = np.zeros(49, np.float64)
        return self.lib.ref_nn_net_class(self.h, _ptr(e), int(c), int(h), int(w), _ptr(logits)), logits

    def nn_class(self, e, c, h, w):
        e = np.ascontiguousarray(e, dtype=np.uint32)
        return self.lib.ref_nn_class(self.h, _ptr(e), int(c), int(h), int(w))

    def pred_block(self, pid, x0, y0, w, h, qx, qy):
        out = np.zeros((h, w), dtype=np.int16)
        if self.lib.ref_pred_block(self.h, pid, x0, y0, w, h, qx, qy, _ptr(out)) != 0:
            raise RuntimeError("ref_pred_block: unset picture or bad size")
        return out

    def satd(self, org, cur, hadamard=True):
        org = np.ascontiguousarray(org, dtype=np.int16)
        cur = np.ascontiguousarray(cur, dtype=np.int16)
        h, w = org.shape
        return self.lib.ref_satd(self.h, _ptr(org), w, _ptr(cur), w, w, h, int(hadamard))

    def refine(self, jobs):
        from nnfme.abi import RESULT_DTYPE
        jobs = np.ascontiguousarray(jobs)
        res = np.zeros(len(jobs), dtype=RESULT_DTYPE)
        rc = self.lib.ref_refine(self.h, _ptr(jobs), _ptr(res), len(jobs))
        if rc != 0:
            raise RuntimeError(f"ref_refine failed: {rc}")
        return res
