"""The C-ABI's host code under AddressSanitizer: the ASan build
(gibbssampler_amd.build variant "asan": -Xarch_host -fsanitize=address, device
code unchanged) runs the CPU C-ABI suite -- argument validation, error
channel, size checks, plan-creation rejections -- in a child process with the
clang ASan runtime preloaded; any ASan report fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_capi_host_code_under_asan():
    from gibbssampler_amd.build import asan_runtime, build
    rt = asan_runtime()
    if rt is None:
        pytest.skip("clang ASan runtime not found")
    lib = build(variant="asan", verbose=False)
    pre = os.environ.get("LD_PRELOAD", "")
    env = dict(os.environ, GIBBS_HIP_LIB=lib, LD_PRELOAD=rt + (":" + pre if pre else ""),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "tests/test_capi_cpu.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=800)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " passed" in r.stdout
