"""The native runtime under AddressSanitizer + UndefinedBehaviorSanitizer, on the host.

``tools/build_ext.py --asan-host`` compiles csrc/runtime/stage_runner.cpp (with
csrc/comm/rccl_engine.h) by g++ against stand-in HIP / RCCL / torch headers and runs
csrc/tests/host_asan_test.cpp: two ranks replay pipeline tapes (COPY, GRAPH, SYNC, POST
with receive-early, WAIT, COLL, CALL, profiled timelines) through an in-process fabric
for hundreds of steps while a watchdog thread polls progress(), then exercise the error,
close and abort paths.  The reference has no native runtime to check this way; its C++
pieces are torch's own (SURVEY §5 race/failure detection).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_is_clean_under_asan_and_ubsan():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build_ext.py"), "--asan-host"],
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "0 failures" in out, out[-4000:]
    for marker in ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:"):
        assert marker not in out, out[-4000:]
    # the run moved real traffic: sends matched by receives, collectives, graph replays
    line = [l for l in out.splitlines() if l.startswith("host_asan_test:")][0]
    counts = [int(w) for w in line.replace(",", " ").split() if w.isdigit()]
    assert counts[0] > 300 and counts[2] > 300 and counts[3] > 300
