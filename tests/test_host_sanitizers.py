"""Host-code sanitizer builds: tests/host/sanitize_harness.cpp drives the engine's host
concurrency (the in-process rank group's RankBarrier, the S-LBFGS twin's TaskFifo; host_sync.hpp) and the
minibatch sampler (sampler.cpp) on the CPU, compiled with g++ under ThreadSanitizer and under
AddressSanitizer + UndefinedBehaviorSanitizer. No GPU: the HIP launches are stubbed by host work.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "tests", "host", "sanitize_harness.cpp"),
       os.path.join(ROOT, "lbfgs-ffnn_amd", "csrc", "sampler.cpp")]
INC = os.path.join(ROOT, "lbfgs-ffnn_amd", "csrc")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def build(tmp_path, flags, name):
    exe = str(tmp_path / name)
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", *flags, "-I" + INC, *SRC, "-o", exe, "-pthread"], check=True,
                   capture_output=True, text=True)
    return exe


def run(exe, *args):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=env)


def test_thread_sanitizer(tmp_path):
    exe = build(tmp_path, ["-fsanitize=thread"], "tsan")
    # the build is live: a deliberate race is reported
    canary = run(exe, "canary")
    assert "WARNING: ThreadSanitizer: data race" in canary.stderr
    r = run(exe)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "sanitize harness ok" in r.stdout


def test_address_undefined_sanitizer(tmp_path):
    exe = build(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"], "asan")
    r = run(exe)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "sanitize harness ok" in r.stdout
