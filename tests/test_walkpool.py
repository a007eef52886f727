"""The host walk's thread pool (ipfixprobe_amd/csrc/ipxg_walkpool.hpp) under the host sanitizers
(VERDICT r3 item 7): tests/walkpool_check.cpp compiled with g++ against the engine's own header,
once with AddressSanitizer (a job handed a thread index past its run's count writes past a heap
array sized by that count -- the round-3 fault) and once with ThreadSanitizer
(the job hand-off, the completion count and the escaped-exception flag).  CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "walkpool_check.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("san", ["address", "thread"])
def test_walkpool_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / ("walkpool_" + san))
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=" + san, "-pthread", SRC, "-o", exe],
                   check=True, capture_output=True, text=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "walkpool ok" in r.stdout
