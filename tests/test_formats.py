"""the reference's data formats — the SSE.csv training record
(TEncSearch.cpp:4560-4582), the per-QP weight CSV directories (DL/<name>/<qp>/, edit.sh layout)
and the fastai checkpoints (DL/models/*.h5, torch state dicts).

The record's NN inputs are pinned against the oracle: feeding each record's distortions to the
oracle's NN (with the PU size NN_pred() read) must give the class the oracle's batch produced,
job by job, and the carried state must equal the oracle's."""
import glob
import os

import numpy as np
import pytest

from conftest import golden_cases, load_golden
from nnfme import dataset, weights
from nnfme.abi import JOB_DTYPE
from oracle import Oracle

REF_DL = "/root/reference/DL"


def _oracle(g):
    hadme, fen, nn_mode, qp = (int(v) for v in g["config"])
    o = Oracle(use_hadamard=hadme, nn_mode=1, fast_inter_mode=fen, qp=qp)
    for i, p in enumerate(g["pictures"]):
        o.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        o.set_lambda(i, float(lam))
    o.set_keys(g["keys"] if g["keys"].size else np.zeros(1, np.int16))
    params = weights.load_weights(qp)
    o.load_nn(params)
    return o, params


def test_out_class_matches_reference_formula():
    # TEncSearch.cpp:4576-4578 evaluated in double, for every (half, quarter) pair HM produces
    for hx in (-1, 0, 1):
        for qx in (-1, 0, 1):
            for hy in (-1, 0, 1):
                for qy in (-1, 0, 1):
                    mx = int((((hx * 0.5) + (qx * 0.25)) + 0.75) * 4)
                    my = int((((hy * 0.5) + (qy * 0.25)) + 0.75) * 28)
                    assert dataset.out_class(hx, hy, qx, qy) == mx + my
    assert dataset.out_class(-1, -1, 0, 0) == 1 + 7 and dataset.out_class(0, 0, 0, 0) == 24


@pytest.mark.parametrize("case", [c for c in golden_cases() if c.endswith("_nn")])
def test_records_nn_inputs_match_oracle(case):
    """Two consecutive batches (the second starts from the first's carried state): every job's
    record reproduces the oracle's NN class, and the carried state equals the oracle's."""
    g = load_golden(case)
    o, params = _oracle(g)
    jobs = g["jobs"]
    half = len(jobs) // 2
    state = o.nn_get_state()
    n_checked = 0
    for part in (jobs[:half], jobs[half:]):
        res = o.refine(part)
        e, c, ph, pw, state_out = dataset.nn_inputs(part, res, state)
        recs, st2 = dataset.records(part, res, state)
        assert np.array_equal(state_out, st2)
        assert np.array_equal(state_out, o.nn_get_state())
        for i in range(len(part)):
            cls, _ = o.nn_class(params, e[i], c[i], ph[i], pw[i])
            assert cls == res["nn_class"][i], f"{case} job {i}"
        # the record's columns are those inputs in the reference's order
        assert np.array_equal(recs["center"], c)
        assert np.array_equal(recs["top_left"], e[:, 0]) and np.array_equal(recs["bottom_right"], e[:, 7])
        assert np.array_equal(recs["Height"], part["h"]) and np.array_equal(recs["Width"], part["w"])
        assert np.all((recs["y"] >= 0) & (recs["y"] < 49))
        state = state_out
        n_checked += len(part)
    assert n_checked == len(jobs)


def test_records_stale_slots_come_from_state():
    """A batch with no EMI job reads every slot, C and the PU size from the carried state."""
    jobs = np.zeros(3, JOB_DTYPE)
    jobs["w"], jobs["h"] = 8, 16
    from nnfme.abi import RESULT_DTYPE
    res = np.zeros(3, RESULT_DTYPE)
    st = np.arange(1, 13, dtype=np.uint32)
    e, c, ph, pw, out = dataset.nn_inputs(jobs, res, st)
    assert np.all(e == st[:8]) and np.all(c == 9) and np.all(ph == 10) and np.all(pw == 11)
    assert np.array_equal(out, st)
    # one EMI job with 3 pushes: slots 0..2 and C / PU size switch to it from that job on
    jobs["flags"][1] = 0x01
    res["n_emi"][1] = 3
    res["emi"][1] = np.arange(100, 108)
    res["c"][1] = 77
    e, c, ph, pw, out = dataset.nn_inputs(jobs, res, st)
    assert list(e[0]) == list(st[:8])
    assert list(e[1]) == [100, 101, 102] + list(st[3:8]) and list(e[2]) == list(e[1])
    assert list(c) == [9, 77, 77] and list(ph) == [10, 16, 16] and list(pw) == [11, 8, 8]
    assert out[11] == (st[11] | 0x107)


def test_sse_csv_round_trip_and_text(tmp_path):
    rng = np.random.default_rng(5)
    recs = np.zeros(50, dataset.RECORD_DTYPE)
    for n in dataset.CONT_VARS:
        recs[n] = rng.integers(0, 2**20, 50)
    recs["Height"] = rng.choice([4, 8, 16, 64], 50)
    recs["Width"] = rng.choice([4, 8, 12, 48], 50)
    recs["y"] = rng.integers(0, 49, 50)
    p = tmp_path / "SSE_22.csv"
    dataset.write_sse_csv(p, recs[:20], append=False)
    dataset.write_sse_csv(p, recs[20:])            # appended, like ofstream ios::app
    back = dataset.read_sse_csv(p)
    assert np.array_equal(back, recs)
    first = p.read_text().splitlines()[0].split(",")
    assert len(first) == 12 and first[4] == str(recs["center"][0]) and first[11] == str(recs["y"][0])
    m, s = dataset.mapper(recs)
    x = np.stack([recs[n].astype(np.float64) for n in dataset.CONT_VARS], 1)
    np.testing.assert_allclose(m, x.mean(0), rtol=1e-12)
    np.testing.assert_allclose(s, x.std(0), rtol=1e-12)


@pytest.mark.parametrize("qp", [22, 27, 32, 37])
def test_weight_csv_dir_round_trip(tmp_path, qp):
    p = weights.load_weights(qp)
    d = tmp_path / str(qp)
    weights.write_csv_dir(str(d), p, qp)
    assert np.array_equal(weights.load_csv_dir(str(d), qp), p)
    # edit.sh layout: indented rows, ';' after the last value
    txt = (d / "3.lins0-weight.csv").read_text()
    assert txt.startswith("\t\t\t") and txt.rstrip().endswith(";") and txt.count("\n") == 22


def test_state_dict_round_trip(tmp_path):
    import torch
    p = weights.load_weights(32)
    sd = weights.to_state_dict(p)
    f = tmp_path / "m.h5"
    torch.save(sd, f)
    t = weights.unpack(p)
    assert np.array_equal(weights.load_checkpoint(str(f), t["mean"], t["stdev"]), p)


@pytest.mark.skipif(not os.path.isdir(REF_DL), reason="reference DL/ directory not present")
@pytest.mark.parametrize("qp", [22, 27, 32, 37])
def test_reference_weight_files_load_to_the_shipped_sets(qp):
    """The reference's CSV directory and its trained checkpoint both load to the weight set
    the library ships (weights/nn2_qp<qp>.bin), bit for bit."""
    p = weights.load_weights(qp)
    assert np.array_equal(weights.load_csv_dir(f"{REF_DL}/blowing/{qp}", qp), p)
    h5 = glob.glob(f"{REF_DL}/models/QP{qp}_*.h5")
    assert len(h5) == 1
    t = weights.unpack(p)
    assert np.array_equal(weights.load_checkpoint(h5[0], t["mean"], t["stdev"]), p)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in golden_cases() if c.endswith("_nn")][:2])
def test_gpu_records_equal_oracle_records(case, tmp_path):
    """The SSE.csv records built from fme_refine's GPU results (two batches, state carried by
    the context) are the oracle's, byte for byte in the written file."""
    from nnfme.runtime import FmeContext
    g = load_golden(case)
    hadme, fen, nn_mode, qp = (int(v) for v in g["config"])
    ctx = FmeContext(use_hadamard=hadme, nn_mode=1, qp=qp, fast_inter_mode=fen)
    for i, p in enumerate(g["pictures"]):
        ctx.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        ctx.set_lambda(i, float(lam))
    if g["keys"].size:
        ctx.set_keys(g["keys"])
    o, _ = _oracle(g)
    jobs = g["jobs"]
    half = len(jobs) // 2
    for part in (jobs[:half], jobs[half:]):
        st_gpu, st_orc = ctx.nn_get_state(), o.nn_get_state()
        assert np.array_equal(st_gpu, st_orc)
        rg, _ = dataset.records(part, ctx.refine(part), st_gpu)
        ro, _ = dataset.records(part, o.refine(part), st_orc)
        dataset.write_sse_csv(tmp_path / "gpu.csv", rg)
        dataset.write_sse_csv(tmp_path / "orc.csv", ro)
    assert (tmp_path / "gpu.csv").read_bytes() == (tmp_path / "orc.csv").read_bytes()
