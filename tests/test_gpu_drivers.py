"""The C++ boundary: drivers written against include/lbfgs_amd/hip_backend.hpp (the reference's
UnifiedLauncher / UnifiedConfig / CudaMinimizerBase API shape, HipBackend) run on the GPU."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
BUILD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lbfgs-ffnn_amd", "build")


def run(exe, *args, timeout=300):
    r = subprocess.run([os.path.join(BUILD, exe), *map(str, args)], capture_output=True, text=True,
                       timeout=timeout, cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_known_answer_through_loss_grad_callback():
    out = run("known_answer_hip")
    assert "[RESULT] ok" in out, out


def test_unified_launcher_driver():
    out = run("main_hip", 20000, 20)
    assert "[RESULT] ok" in out, out
    assert "Training Results: MSE=" in out and "Test Results: MSE=" in out
    assert os.path.exists("/tmp/HIP_LBFGS_m10_history.csv")
    head = open("/tmp/HIP_LBFGS_m10_history.csv").readline().strip()
    assert head == "Iteration,Loss,GradNorm,TimeMs"
