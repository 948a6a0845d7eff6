"""The reference's training-data format: one `SSE.csv` record per xMotionEstimation call.

TEncSearch.cpp:4560-4582 (the "EMI: Dataset Extraction" block, shipped commented out and
enabled by the authors to build `DL/SSE_<qp>.csv` through `DL/Extract_data.sh`) appends

    array_e[0], array_e[1], array_e[2], array_e[3], C, array_e[4], ..., array_e[7],
    iRoiHeight, iRoiWidth, OUT_CLASS

per call, where OUT_CLASS = ((cMvHalf.x*0.5 + cMvQter.x*0.25) + 0.75)*4
                          + ((cMvHalf.y*0.5 + cMvQter.y*0.25) + 0.75)*28   (0..48)
is HM's own FracDIF decision (the label), `array_e`/`C` are the NN inputs exactly as NN_pred()
reads them (stale slots included: `array_e` is clear()ed, never zeroed) and the
block size is the current PU's.  NN_training.ipynb reads the file as
`names = cont_vars + cat_vars + ['y']` (top_left .. bottom_right, Height, Width, y) and
normalises the nine distortions with sklearn's StandardScaler (`export_mapper` writes the
mean / std to `mapper_<qp>.csv`).

`records()` rebuilds these records from a batch's `fme_result`s (fme_refine output) and the NN
state carried into the batch (`FmeContext.nn_get_state()` before the call): the stale-slot
resolution is the batch path's last-writer rule restated on the host (a forward fill over
job order), so the records of a GPU run need no second pass over the pictures.
"""
import numpy as np

from .abi import JOB_EMI

CONT_VARS = ("top_left", "top_center", "top_right", "left", "center", "right",
             "bottom_left", "bottom_center", "bottom_right")
CAT_VARS = ("Height", "Width")
RECORD_DTYPE = np.dtype([(n, "<u4") for n in CONT_VARS] + [(n, "<i4") for n in CAT_VARS] + [("y", "<i4")])


def out_class(half_x, half_y, qtr_x, qtr_y):
    """OUT_CLASS of TEncSearch.cpp:4576-4578 (the doubles are exact multiples of 0.25)."""
    hx, hy = np.asarray(half_x, np.int32), np.asarray(half_y, np.int32)
    qx, qy = np.asarray(qtr_x, np.int32), np.asarray(qtr_y, np.int32)
    return (2 * hx + qx + 3) + 7 * (2 * hy + qy + 3)


def nn_inputs(jobs, results, state_in=None):
    """What NN_pred() read for every job of a batch, and the state carried out of it.

    Returns (e uint32[n, 8], c uint32[n], pu_h int32[n], pu_w int32[n], state_out uint32[12]).
    Slot s of job i is emi[s] of the last job j <= i whose EMI step pushed more than s values;
    C / PUHeight / PUWidth are those of the last EMI job <= i; anything no job of the batch wrote
    comes from `state_in` (12 words, fme_nn_get_state layout; zeros = process start)."""
    n = len(jobs)
    st = np.zeros(12, np.uint32) if state_in is None else np.asarray(state_in, np.uint32).reshape(12)
    emi_job = (np.asarray(jobs["flags"]) & JOB_EMI) != 0
    idx = np.arange(n, dtype=np.int64)
    e = np.empty((n, 8), np.uint32)
    written = int(st[11])
    for s in range(8):
        src = np.maximum.accumulate(np.where(emi_job & (results["n_emi"] > s), idx, -1)) if n else idx
        have = src >= 0
        e[:, s] = np.where(have, results["emi"][np.maximum(src, 0), s], st[s])
        if n and have[-1]:
            written |= 1 << s
    src = np.maximum.accumulate(np.where(emi_job, idx, -1)) if n else idx
    have = src >= 0
    sc = np.maximum(src, 0)
    c = np.where(have, results["c"][sc], st[8]).astype(np.uint32)
    pu_h = np.where(have, jobs["h"][sc], st[9]).astype(np.int32)
    pu_w = np.where(have, jobs["w"][sc], st[10]).astype(np.int32)
    if n and have[-1]:
        written |= 0x100
    out = st.copy()
    if n:
        out[:8] = e[-1]
        out[8], out[9], out[10] = c[-1], pu_h[-1], pu_w[-1]
    out[11] = written
    return e, c, pu_h, pu_w, out


def records(jobs, results, state_in=None):
    """The SSE.csv records of one fme_refine batch (RECORD_DTYPE[n]) and the carried-out state."""
    e, c, _, _, out = nn_inputs(jobs, results, state_in)
    r = np.zeros(len(jobs), RECORD_DTYPE)
    for s, name in enumerate(("top_left", "top_center", "top_right", "left")):
        r[name] = e[:, s]
    r["center"] = c
    for s, name in enumerate(("right", "bottom_left", "bottom_center", "bottom_right")):
        r[name] = e[:, 4 + s]
    r["Height"] = jobs["h"]
    r["Width"] = jobs["w"]
    r["y"] = out_class(results["half_x"], results["half_y"], results["qtr_x"], results["qtr_y"])
    return r, out


def write_sse_csv(path, recs, append=True):
    """Append records in the reference's text form (`ofstream << a << ',' << ... << endl`)."""
    cols = [np.asarray(recs[n]).astype(np.int64) for n in RECORD_DTYPE.names]
    lines = [",".join(str(v) for v in row) for row in zip(*(c.tolist() for c in cols))]
    with open(path, "a" if append else "w") as f:
        if lines:
            f.write("\n".join(lines) + "\n")


def read_sse_csv(path):
    """SSE_<qp>.csv -> RECORD_DTYPE[n] (the columns NN_training.ipynb names)."""
    raw = np.loadtxt(path, delimiter=",", dtype=np.int64, ndmin=2)
    if raw.size == 0:
        return np.zeros(0, RECORD_DTYPE)
    if raw.shape[1] != len(RECORD_DTYPE.names):
        raise ValueError(f"{path}: {raw.shape[1]} columns, expected {len(RECORD_DTYPE.names)}")
    r = np.zeros(raw.shape[0], RECORD_DTYPE)
    for k, n in enumerate(RECORD_DTYPE.names):
        r[n] = raw[:, k]
    return r


def mapper(recs):
    """(mean, std) float64[9] of the nine distortions as `export_mapper` exports them: the
    notebook casts them to float32 and scales with sklearn's StandardScaler (population std)."""
    x = np.stack([np.asarray(recs[n]).astype(np.float32).astype(np.float64) for n in CONT_VARS], axis=1)
    return x.mean(axis=0), x.std(axis=0)
