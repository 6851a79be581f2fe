"""Host C++ runtime under AddressSanitizer+UBSan and ThreadSanitizer (the
reference has no race detection).  Builds csrc/host/selftest with tools/sanitize_host.sh
and runs the concurrent ZMTP / VecEnv / codec / NativePolicy stress test under both."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_host_runtime_clean_under_asan_ubsan_tsan():
    r = subprocess.run([os.path.join(REPO, "tools", "sanitize_host.sh")], capture_output=True, text=True,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count("host selftest OK") == 2
    assert "ThreadSanitizer" not in out and "AddressSanitizer" not in out and "runtime error" not in out
