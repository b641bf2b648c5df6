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
    assert "[RESULT] gd iters=" in out and "[RESULT] sgd epochs=3" in out
    assert os.path.exists("/tmp/HIP_GD_history.csv") and os.path.exists("/tmp/HIP_SGD_history.csv")


def test_driver_reads_idx_files(tmp_path, pkg):
    """main_hip with an MNIST directory: the C++ MNISTLoader mirror (tests/mnist/mnist_loader.hpp) feeds
    UnifiedLauncher<HipBackend>. IDX files written here from the synthetic MNIST-shaped data."""
    import struct

    import numpy as np

    for name, n, seed in [("train", 512, 123), ("t10k", 128, 124)]:
        X, Y = pkg.synth_mnist(n, seed=seed)
        px = np.rint(X * 255.0).astype(np.uint8)
        (tmp_path / f"{name}-images.idx3-ubyte").write_bytes(struct.pack(">IIII", 2051, n, 28, 28) + px.tobytes())
        lab = np.argmax(Y, 1).astype(np.uint8)
        (tmp_path / f"{name}-labels.idx1-ubyte").write_bytes(struct.pack(">II", 2049, n) + lab.tobytes())
    out = run("main_hip", 512, 5, str(tmp_path))
    assert "[RESULT] ok" in out, out
    assert "Train: 512 samples" in out
