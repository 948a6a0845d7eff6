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
    return sorted(set(re.findall(r"\b(fme_[a-z_]+)\s*\(", txt)))


def test_library_exports_header():
    lib = runtime.load_library()
    names = header_functions()
    assert len(names) == 53
    assert set(names) == set(runtime.ABI_SYMBOLS)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.fme_abi_version() == runtime.ABI_VERSION == 15


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
