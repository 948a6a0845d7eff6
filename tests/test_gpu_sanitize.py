"""The C++ adapter's GPU test driver (tests/cpp/test_hm_adapter.cpp) built with host-side
AddressSanitizer + UndefinedBehaviorSanitizer over an instrumented C-ABI runtime
(libfme_amd_asan.so: fme_api.cpp) and adapter (host/fme_hm.cpp, its CtuRowBatcher worker thread):
every batch, single-PU, motion-compensation and predInterSearch path it drives runs with the host
code checked; any report fails.  Device code is not instrumented (GPU ASan is not used here)."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_cpp_hm_adapter_under_asan_ubsan():
    exe = os.path.join(ROOT, "hm16.9-nn_fme_amd", "host", "test_hm_adapter_asan")
    assert os.path.exists(exe), "build it with __graft_entry__.build() (make sanitize)"
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["FME_WEIGHTS_DIR"] = os.path.join(ROOT, "hm16.9-nn_fme_amd", "weights")   # the adapter is linked in
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    out = p.stdout + p.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
    assert "hm adapter ok" in out
