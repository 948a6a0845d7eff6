"""Host-side AddressSanitizer / UndefinedBehaviorSanitizer runs, in this container.

* The CPU oracle's whole test suite (tests/test_oracle.py: every golden vector, the reference
  harness cross-checks, MC, the producers) on oracle/liboracle_asan.so, gcc's libasan preloaded
  into the Python process.
* The C-ABI runtime's host code (fme_api.cpp built with -fsanitize=address,undefined into
  libfme_amd_asan.so): tests/test_abi.py's checks (exports, struct layouts, the error paths that
  run without a device), clang's ASan runtime preloaded.
The GPU half (the C++ adapter's CTU-row batcher thread and every entry point with a device) is
tests/test_gpu_sanitize.py.  Any sanitizer report fails the run (-fno-sanitize-recover /
halt_on_error).
"""
import glob
import os
import subprocess
import sys

import pytest

from conftest import ROOT

ORACLE_ASAN = os.path.join(ROOT, "oracle", "liboracle_asan.so")
FME_ASAN = os.path.join(ROOT, "hm16.9-nn_fme_amd", "libfme_amd_asan.so")


def _make(path, target):
    subprocess.run(["make", "-C", path, "-j8", target], check=True, capture_output=True, timeout=900)


def _run_suite(test_file, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    p = subprocess.run([sys.executable, "-m", "pytest", test_file, "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = p.stdout + p.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
    return out


def test_oracle_suite_under_asan_ubsan():
    if not os.path.exists(ORACLE_ASAN):
        _make(os.path.join(ROOT, "oracle"), "sanitize")
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    out = _run_suite("tests/test_oracle.py", {"LD_PRELOAD": libasan, "FME_ORACLE_SO": ORACLE_ASAN})
    assert " passed" in out


def test_runtime_host_code_under_asan_ubsan():
    if not os.path.exists(FME_ASAN):
        _make(os.path.join(ROOT, "hm16.9-nn_fme_amd"), "libfme_amd_asan.so")
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not rt:
        pytest.skip("clang's ASan runtime is not in this image")
    out = _run_suite("tests/test_abi.py", {"LD_PRELOAD": rt[-1], "FME_LIB_PATH": FME_ASAN})
    assert " passed" in out
