"""Native runtime self-tests built plain, with ASan+UBSan and with TSan -- host code only:
topology, wire codec, safetensors, the multi-threaded WorkerServer, and the native text /
SD workers (native_worker.cpp: concurrent masters, the compute lock, request
validation, mid-request disconnects, stop) over a host stub of the engine library."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("variant", ["plain", "asan", "tsan"])
def test_runtime_selftest_under_sanitizers(variant, tmp_path):
    env = dict(os.environ, VARIANTS=variant, OUT_DIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize_runtime.sh")], env=env,
                       capture_output=True, text=True, timeout=600)
    sys.stdout.write(r.stdout[-2000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.count(" ok") == 6
