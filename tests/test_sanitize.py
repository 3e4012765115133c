"""CPU: the engine's host logic under sanitizers — `make -C nebula_amd sanitize`
builds window_core.hpp (replay window, exact receive rounds, thread pool) and queue_core.hpp (the
submission queue, on a CPU device running the oracle) with ASan+UBSan and with TSan and runs them;
each test also checks its results against the packet-by-packet receive / the oracle."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan/libtsan")
def test_sanitizer_builds_run_clean():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "nebula_amd"), "sanitize"], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("window_test: ok") == 2 and r.stdout.count("queue_test: ok") == 2, r.stdout
