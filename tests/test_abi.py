"""The C-ABI library loads and exports every entry point include/fme.h declares; the numpy
struct mirrors match the header.  No compute calls here (no GPU in this container)."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, gpu_available
from nnfme import abi, runtime


def header_functions():
    txt = open(os.path.join(ROOT, "include", "fme.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fme_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header():
    lib = runtime.load_library()
    names = header_functions()
    assert len(names) == 61
    assert set(names) == set(runtime.ABI_SYMBOLS)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.fme_abi_version() == runtime.ABI_VERSION == 18


def test_struct_layouts():
    assert abi.JOB_DTYPE.itemsize == 32
    assert abi.RESULT_DTYPE.itemsize == 64
    assert abi.JOB_DTYPE.fields["key_offset"][1] == 28
    assert abi.RESULT_DTYPE.fields["frac_cost"][1] == 12
    assert abi.RESULT_DTYPE.fields["emi"][1] == 28
    assert abi.RESULT_DTYPE.fields["status"][1] == 62
    # fme_mc_job: x,y @0, w,h @4, flags @6, ref_id[2] @8, cu_x,cu_y @10, mv[2][2] @14
    assert abi.MC_JOB_DTYPE.itemsize == 24
    assert abi.MC_JOB_DTYPE.fields["ref_id"][1] == 8
    assert abi.MC_JOB_DTYPE.fields["cu_x"][1] == 10
    assert abi.MC_JOB_DTYPE.fields["mv"][1] == 14
    assert abi.MV_RESULT_DTYPE.itemsize == 16
    assert abi.MV_RESULT_DTYPE.fields["cost"][1] == 4
    assert abi.MV_RESULT_DTYPE.fields["status"][1] == 14
    assert abi.TZ_EXT_DTYPE.itemsize == 12
    assert abi.WP_PARAM_DTYPE.itemsize == 8 and abi.WP_PARAM_DTYPE.fields["log2_denom"][1] == 4
    assert abi.TZ_EXT_DTYPE.fields["flags"][1] == 8


def test_mc_struct_matches_header():
    """Compile a probe against include/fme.h: sizeof / offsetof of fme_mc_job."""
    import subprocess
    import tempfile
    src = ('#include <stdio.h>\n#include <stddef.h>\n#include "fme.h"\nint main(void){printf("%zu %zu %zu %zu %zu",'
           'sizeof(fme_mc_job), offsetof(fme_mc_job, ref_id), offsetof(fme_mc_job, cu_x), offsetof(fme_mc_job, mv),'
           'offsetof(fme_mc_job, flags));return 0;}')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        got = [int(v) for v in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    d = abi.MC_JOB_DTYPE.fields
    assert got == [abi.MC_JOB_DTYPE.itemsize, d["ref_id"][1], d["cu_x"][1], d["mv"][1], d["flags"][1]]


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_create_without_device_fails_cleanly():
    with pytest.raises(runtime.FmeError) as e:
        runtime.FmeContext()
    assert e.value.code in (-1, -2)


def test_null_arguments_rejected():
    lib = runtime.load_library()
    assert lib.fme_create(0, None, None) == -1
    assert b"null" in lib.fme_last_error()
    assert lib.fme_refine(None, None, None, 1, None) == -1
    assert lib.fme_refine_mv(None, None, None, 1, None) == -1
    assert lib.fme_refine_mv_device(None, None, None, 1, None) == -1
    assert lib.fme_refine_mv_packed_device(None, None, None, None, 1, None) == -1
    assert lib.fme_refine_packed_device(None, None, None, None, 1, None) == -1
    assert lib.fme_pack_jobs(None, 1, None, None) == -1
    assert lib.fme_refine_status(None) == -1
    assert lib.fme_nn_copy_state_device(None, None, None) == -1
    assert lib.fme_set_search_event(None, None) == -1
    assert lib.fme_destroy(None) == 0


def test_hm_adapter_library_exports():
    """libfme_hm.so (the C++ TEncSearch-shaped adapter) links against libfme_amd.so and
    exports the FracSearch / CtuRowBatcher surface include/fme_hm.hpp declares."""
    import subprocess
    so = os.path.join(os.path.dirname(runtime.LIB_PATH), "libfme_hm.so")
    if not os.path.exists(so):
        pytest.skip("libfme_hm.so not built")
    out = subprocess.run(["nm", "-DC", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    for sym in ("fme_hm::FracSearch::xPatternSearchFracDIF", "fme_hm::FracSearch::NN_pred",
                "fme_hm::FracSearch::setPicture", "fme_hm::CtuRowBatcher::submit",
                "fme_hm::CtuRowBatcher::wait", "fme_hm::CtuRowBatcher::addBiPred",
                "fme_hm::loadWeights", "fme_hm::InterSearchP::run", "fme_hm::InterSearchP::reset",
                "fme_hm::InterSearchB::run", "fme_hm::InterSearchB::reset"):
        assert sym in out, sym
    deps = subprocess.run(["ldd", so], capture_output=True, text=True).stdout
    assert "libfme_amd.so" in deps


# ---- fme_job_packed (ABI 16): host packing, pure host code -----------------------------------
def _frame_jobs(bipred=0.0, W=416, H=240):
    from nnfme import synth
    rng = np.random.default_rng(11)
    jobs = synth.make_ctu_jobs(rng, W, H, 331, 4, [0, 1, 2, 3], [0], bipred_frac=bipred)
    if bipred:
        synth.make_bipred_key_reqs(np.random.default_rng(12), jobs, 4, [0, 1, 2, 3])
    return jobs


def _same_refinement_inputs(u, jobs):
    """What the sub-pel path reads of a job: every field, except that the range words enter only
    through the EMI step's four tests (TEncSearch.cpp:1341-1376) and a negative key offset only as
    'unkeyed'."""
    for f in abi.JOB_DTYPE.names:
        if f in ("lt_x", "lt_y", "rb_x", "rb_y", "key_offset"):
            continue
        assert np.array_equal(u[f], jobs[f]), f
    mx, my = jobs["mv_x"].astype(int), jobs["mv_y"].astype(int)
    assert np.array_equal(my - 1 >= u["lt_y"], my - 1 >= jobs["lt_y"])
    assert np.array_equal(my + 1 <= u["rb_y"], my + 1 <= jobs["rb_y"])
    assert np.array_equal(mx - 1 >= u["lt_x"], mx - 1 >= jobs["lt_x"])
    assert np.array_equal(mx + 1 <= u["rb_x"], mx + 1 <= jobs["rb_x"])
    assert np.array_equal(u["key_offset"], np.where(jobs["key_offset"] >= 0, jobs["key_offset"], -1))


def test_pack_jobs_round_trip():
    assert abi.JOB_PACKED_DTYPE.itemsize == 16
    for bipred in (0.0, 0.3):
        jobs = _frame_jobs(bipred)
        pk, kb = runtime.pack_jobs(jobs)
        assert len(kb) == (len(jobs) + 63) // 64
        _same_refinement_inputs(runtime.unpack_jobs(pk, kb), jobs)
        if bipred:
            assert (kb >= 0).any() and (jobs["key_offset"] >= 0).sum() > 1000


def test_pack_jobs_edges_and_refusals():
    jobs = _frame_jobs()[:300].copy()
    # range edges: every combination of the four EMI tests survives the packing
    jobs["lt_x"] = jobs["mv_x"] - (np.arange(300) & 1)
    jobs["rb_x"] = jobs["mv_x"] + ((np.arange(300) >> 1) & 1)
    jobs["lt_y"] = jobs["mv_y"] - ((np.arange(300) >> 2) & 1) * 7
    jobs["rb_y"] = jobs["mv_y"] + ((np.arange(300) >> 3) & 1) * 64
    jobs["bits_in"] = np.arange(300) % 64
    jobs["lambda_id"] = np.arange(300) % 32
    pk, kb = runtime.pack_jobs(jobs)
    _same_refinement_inputs(runtime.unpack_jobs(pk, kb), jobs)
    lib = runtime.load_library()
    for field, value in (("x", 6), ("w", 6), ("bits_in", 64), ("lambda_id", 32), ("ref_id", 64),
                         ("flags", 16), ("mv_x", 32767)):
        bad = jobs.copy()
        bad[field][5] = value
        with pytest.raises(runtime.FmeError) as e:
            runtime.pack_jobs(bad)
        assert e.value.code == -4 and b"job 5" in lib.fme_last_error()
    # keyed blocks must follow each other within a wave
    bad = jobs.copy()
    bad["key_offset"][3] = 0
    bad["key_offset"][4] = 100   # a 4x? block of w*h != 100 before it
    bad["w"][3], bad["h"][3] = 8, 8
    with pytest.raises(runtime.FmeError):
        runtime.pack_jobs(bad)
    ok = jobs.copy()
    ok["key_offset"][64] = 5000   # a new wave may start anywhere
    ok["key_offset"][65] = 5000 + int(ok["w"][64]) * int(ok["h"][64])
    pk, kb = runtime.pack_jobs(ok)
    assert kb[1] == 5000 and kb[0] == -1
    _same_refinement_inputs(runtime.unpack_jobs(pk, kb), ok)
