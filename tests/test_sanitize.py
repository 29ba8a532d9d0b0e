"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run.

tools/sanitize/ builds the CPU oracle into an instrumented driver together with
libsalp's C ABI compiled with its host half instrumented (hipcc -Xarch_host
-fsanitize=address,undefined); the driver runs every oracle entry point (sizes
1/7/64, 0/2/4 obstacles, masks, randomisation, recording) and the ABI's
argument checks and error paths.  Any finding aborts the run.  The same driver
with --gpu runs the ABI end to end on an MI355X (tools/gpu_sanitize.sh).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/llvm/bin/clang") or shutil.which("make") is None,
                    reason="needs ROCm clang and make")
def test_host_code_is_asan_and_ubsan_clean():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "sanitize"), "run"], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "oracle + ABI host paths ok" in r.stdout
