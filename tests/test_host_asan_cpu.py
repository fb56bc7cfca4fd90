"""The sanitizer build (SURVEY §5 build stance): the host side of libhvs -- PIL resample table
builders, workspace sizes, argument validation of the grouped entry points -- compiled with
AddressSanitizer + UBSan (hipcc -Xarch_host; device code is never sanitised) and exercised by
tools/host_check.cpp through `make asan-host`.  No GPU is used."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "humanoid-vision-system_amd")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_host_code_clean_under_asan_ubsan():
    r = subprocess.run(["make", "-C", PKG, "-j4", "asan-host"], capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "host_check: ok (0 failures)" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out
