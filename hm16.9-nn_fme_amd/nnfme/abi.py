"""numpy mirrors of the C-ABI structs in include/fme.h.

fme_job (32 B) and fme_result (64 B) are plain PODs; these structured dtypes have the same
field offsets so arrays can be handed to the library (or the oracle) as raw pointers.
"""
import numpy as np

JOB_DTYPE = np.dtype(
    [
        ("x", "<u2"), ("y", "<u2"),
        ("w", "u1"), ("h", "u1"),
        ("org_id", "u1"), ("ref_id", "u1"),
        ("mv_x", "<i2"), ("mv_y", "<i2"),
        ("mvp_x", "<i2"), ("mvp_y", "<i2"),
        ("lt_x", "<i2"), ("lt_y", "<i2"), ("rb_x", "<i2"), ("rb_y", "<i2"),
        ("flags", "u1"), ("lambda_id", "u1"), ("bits_in", "<u2"),
        ("key_offset", "<i4"),
    ],
    align=False,
)
assert JOB_DTYPE.itemsize == 32

RESULT_DTYPE = np.dtype(
    [
        ("mv_int_x", "<i2"), ("mv_int_y", "<i2"),
        ("mv_x", "<i2"), ("mv_y", "<i2"),
        ("half_x", "i1"), ("half_y", "i1"), ("qtr_x", "i1"), ("qtr_y", "i1"),
        ("frac_cost", "<u4"), ("cost", "<u4"), ("bits", "<u4"), ("c", "<u4"),
        ("emi", "<u4", (8,)),
        ("n_emi", "u1"), ("nn_class", "u1"), ("status", "<u2"),
    ],
    align=False,
)
assert RESULT_DTYPE.itemsize == 64

# fme_mv_result (16 B): xMotionEstimation's outputs alone (fme_refine_mv*)
# fme_job_packed (16 B): the upload form of fme_job (include/fme.h)
JOB_PACKED_DTYPE = np.dtype([("pu", "<u4"), ("ctl", "<u4"), ("mv_x", "<i2"), ("mv_y", "<i2"),
                             ("mvp_x", "<i2"), ("mvp_y", "<i2")], align=False)
assert JOB_PACKED_DTYPE.itemsize == 16
PACK_WAVE = 64

MV_RESULT_DTYPE = np.dtype(
    [("mv_x", "<i2"), ("mv_y", "<i2"), ("cost", "<u4"), ("bits", "<u4"),
     ("nn_class", "u1"), ("reserved", "u1"), ("status", "<u2")],
    align=False,
)
assert MV_RESULT_DTYPE.itemsize == 16
MV_FIELDS = ("mv_x", "mv_y", "cost", "bits", "nn_class", "status")

# fme_mc_job (24 B): one PU of motion compensation (include/fme.h)
MC_JOB_DTYPE = np.dtype(
    [
        ("x", "<u2"), ("y", "<u2"),
        ("w", "u1"), ("h", "u1"),
        ("flags", "u1"), ("reserved", "u1"),
        ("ref_id", "u1", (2,)),
        ("cu_x", "<u2"), ("cu_y", "<u2"),
        ("mv", "<i2", (2, 2)),
        ("reserved2", "<u2"),
    ],
    align=False,
)
assert MC_JOB_DTYPE.itemsize == 24

# fme_tz_ext (12 B): per-job extension of the integer TZ search (include/fme.h)
TZ_EXT_DTYPE = np.dtype(
    [
        ("cu_x", "<u2"), ("cu_y", "<u2"),
        ("pred2n_x", "<i2"), ("pred2n_y", "<i2"),
        ("flags", "u1"), ("search_range", "u1"), ("reserved", "<u2"),
    ],
    align=False,
)
assert TZ_EXT_DTYPE.itemsize == 12
TZ_PRED2NX2N = 0x01
TZ_RING = 0x02          # the backups' xTZSearch tail (fme_integer_search_ring)
TZ_FULL = 0x04          # FastSearch 0: xPatternSearch over lt..rb (uni-pred too)
TZ_ENHANCED = 0x08      # FastSearch 3: xTZSearch with bExtendedSettings (fme_tz_ext2 predictors)
# fme_tz_ext2 (24 B): fme_tz_ext + m_acMvPredictors[left, above, above-right] (quarter-pel)
TZ_EXT2_DTYPE = np.dtype([("base", TZ_EXT_DTYPE), ("preds", "<i2", (3, 2))], align=False)
assert TZ_EXT2_DTYPE.itemsize == 24

# fme_pu_req (64 B) / fme_pu_res (80 B): predInterSearch's P-slice PU / reference loop (include/fme.h)
MAX_REFS = 4
PU_REQ_DTYPE = np.dtype(
    [
        ("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"),
        ("cu_x", "<u2"), ("cu_y", "<u2"),
        ("part_size", "u1"), ("depth", "u1"), ("org_id", "u1"), ("num_refs", "u1"),
        ("ref_id", "u1", (MAX_REFS,)), ("n_cand", "u1", (MAX_REFS,)),
        ("cand", "<i2", (MAX_REFS, 2, 2)),
        ("lambda_id", "u1"), ("search_range", "u1"), ("flags", "u1"), ("reserved", "u1"),
        ("reserved2", "<u2", (3,)),
    ],
    align=False,
)
assert PU_REQ_DTYPE.itemsize == 64
PU_RES_DTYPE = np.dtype(
    [
        ("mv_x", "<i2"), ("mv_y", "<i2"), ("mvp_x", "<i2"), ("mvp_y", "<i2"),
        ("ref_idx", "u1"), ("mvp_idx", "u1"), ("reserved", "<u2"),
        ("bits", "<u4"), ("cost", "<u4"),
        ("ref_cost", "<u4", (MAX_REFS,)), ("ref_bits", "<u4", (MAX_REFS,)),
        ("ref_mv", "<i2", (MAX_REFS, 2)), ("ref_mvp_idx", "u1", (MAX_REFS,)),
        ("reserved2", "<u4", (2,)),
    ],
    align=False,
)
assert PU_RES_DTYPE.itemsize == 80
PU_LOSSLESS = 0x01
PU_FAST_ME_GEN_B = 0x02
PU_CLIP_BIPRED = 0x04
PU_MVD_L1_ZERO = 0x08
# fme_pu_req_b / fme_pu_res_b (include/fme.h): predInterSearch on a B slice
PU_REQ_B_DTYPE = np.dtype(
    [
        ("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"),
        ("cu_x", "<u2"), ("cu_y", "<u2"),
        ("part_size", "u1"), ("depth", "u1"), ("org_id", "u1"), ("part_idx", "u1"),
        ("cu_w", "u1"), ("lambda_id", "u1"), ("search_range", "u1"), ("bipred_range", "u1"),
        ("flags", "u1"), ("num_refs", "u1", (2,)),
        ("ref_id", "u1", (2, MAX_REFS)), ("n_cand", "u1", (2, MAX_REFS)),
        ("l1_to_l0", "i1", (MAX_REFS,)), ("reserved", "u1", (7,)),
        ("cand", "<i2", (2, MAX_REFS, 2, 2)),
    ],
    align=False,
)
assert PU_REQ_B_DTYPE.itemsize == 112
PU_RES_B_DTYPE = np.dtype(
    [
        ("inter_dir", "u1"), ("ref_idx", "u1", (2,)), ("mvp_idx", "u1", (2,)), ("bi_list", "u1"),
        ("bi_iters", "u1"), ("reserved", "u1"),
        ("mv", "<i2", (2, 2)), ("mvp", "<i2", (2, 2)),
        ("bits", "<u4"), ("cost", "<u4"),
        ("uni_cost", "<u4", (2,)), ("uni_bits", "<u4", (2,)),
        ("bi_cost", "<u4"), ("bi_bits", "<u4"),
        ("ref_cost", "<u4", (2, MAX_REFS)), ("ref_mv", "<i2", (2, MAX_REFS, 2)),
        ("bi_ref_cost", "<u4", (MAX_REFS,)), ("bi_ref_mv", "<i2", (MAX_REFS, 2)),
        ("ref_mvp_idx", "u1", (2, MAX_REFS)),
    ],
    align=False,
)
assert PU_RES_B_DTYPE.itemsize == 160
# fme_bikey_req (include/fme.h)
BIKEY_REQ_DTYPE = np.dtype(
    [
        ("x", "<u2"), ("y", "<u2"), ("w", "u1"), ("h", "u1"), ("org_id", "u1"), ("ref_id", "u1"),
        ("cu_x", "<u2"), ("cu_y", "<u2"), ("mv_x", "<i2"), ("mv_y", "<i2"),
        ("key_offset", "<i4"), ("flags", "<u4"),
    ],
    align=False,
)
assert BIKEY_REQ_DTYPE.itemsize == 24
PART_2Nx2N, PART_2NxN, PART_Nx2N, PART_NxN, PART_2NxnU, PART_2NxnD, PART_nLx2N, PART_nRx2N = range(8)

MC_L0 = 0x01
MC_L1 = 0x02
MC_WP = 0x04   # explicit weighted prediction (fme_set_wp parameters)

# fme_wp_param: WPScalingParam's iWeight, iOffset (8-bit units), uiLog2WeightDenom per component
WP_PARAM_DTYPE = np.dtype([("weight", "<i2"), ("offset", "<i2"), ("log2_denom", "u1"), ("reserved", "u1", (3,))])
assert WP_PARAM_DTYPE.itemsize == 8


def wp_params(params):
    """Three fme_wp_param rows (Y, Cb, Cr) from (weight, offset, log2_denom) triples or a
    WP_PARAM_DTYPE array."""
    a = np.asarray(params)
    if a.dtype == WP_PARAM_DTYPE:
        return np.ascontiguousarray(a.reshape(3))
    out = np.zeros(3, WP_PARAM_DTYPE)
    for k, (w, o, d) in enumerate(np.asarray(params, dtype=np.int64).reshape(3, 3)):
        out[k] = (int(w), int(o), int(d), (0, 0, 0))
    return out

CONFIG_FIELDS = ("bit_depth", "use_hadamard", "nn_mode", "qp", "fast_inter_mode", "max_jobs")

JOB_EMI = 0x01
JOB_BIPRED = 0x02
JOB_LOSSLESS = 0x04
JOB_NN_IN = 0x08        # NN inputs from the bound row (the backups' input path)

RES_NN_STALE = 0x01
RES_NN_UNINIT = 0x02
RES_REJECTED = 0x8000

MAX_PICTURES = 64
MAX_LAMBDAS = 64
NN_PARAMS = 2060

E_INVALID, E_DEVICE, E_NOMEM, E_UNSUPPORTED, E_STATE = -1, -2, -3, -4, -5

# Fields that define parity (everything the reference computes).
PARITY_FIELDS = ("mv_int_x", "mv_int_y", "mv_x", "mv_y", "half_x", "half_y", "qtr_x", "qtr_y",
                 "frac_cost", "cost", "bits", "c", "n_emi", "nn_class")


def compare_results(a, b, fields=PARITY_FIELDS):
    """Return (n_mismatched_jobs, first_bad_index_or_None, per-field mismatch counts)."""
    bad = np.zeros(len(a), dtype=bool)
    counts = {}
    for f in fields:
        m = a[f] != b[f]
        counts[f] = int(m.sum())
        bad |= m
    # emi: only the n_emi pushed values are defined
    n = a["n_emi"].astype(np.int64)
    slot = np.arange(8)[None, :] < n[:, None]
    m = ((a["emi"] != b["emi"]) & slot).any(axis=1)
    counts["emi"] = int(m.sum())
    bad |= m
    idx = np.flatnonzero(bad)
    return int(bad.sum()), (int(idx[0]) if len(idx) else None), counts


# fme_nn_net (40 B): descriptor of a generic NN_pred net (include/fme.h, fme_load_nn_net)
import ctypes as _C


class NnNetStruct(_C.Structure):
    _fields_ = [("precision", _C.c_int32), ("n_hidden", _C.c_int32), ("width", _C.c_int32 * 4),
                ("embedding", _C.c_int32), ("out_act", _C.c_int32), ("carry_hidden", _C.c_uint32),
                ("reserved", _C.c_int32)]


assert _C.sizeof(NnNetStruct) == 40
