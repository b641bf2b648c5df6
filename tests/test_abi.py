"""CPU tests of the C ABI library: it loads, exports every symbol include/lbfgs_amd.h declares, and its
host-side random streams reproduce the reference's libstdc++ draws (checked against the oracle)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lbfgs_amd.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(lbf_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(pkg):
    L = pkg.lib()
    syms = declared_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (lbf_\w+)", out))
    assert set(syms) <= exported, set(syms) - exported
    assert set(pkg._lib.EXPORTS) == set(syms)


def test_library_targets_gfx950(pkg):
    blob = open(pkg.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa" in blob and b"gfx950" in blob


def test_version_and_error_path(pkg):
    L = pkg.lib()
    assert L.lbf_version().decode().startswith("lbfgs_amd")
    # invalid arguments are reported, not aborted (cf. cuda_check abort in the reference)
    rc = L.lbf_synth_mnist(-1, 1, 1, 0, None, None)
    assert rc == 1
    assert "invalid argument" in L.lbf_last_error().decode()


def test_synth_data_matches_oracle(pkg, O):
    X, Y = pkg.synth_mnist(300, 784, 10, 123)
    Xo, Yo = O.synth_mnist(300, 784, 10, 123)
    assert np.array_equal(X, Xo.astype(np.float32))
    assert np.array_equal(Y, Yo.astype(np.float32))
    # pixel values are k/255 like the reference IDX loader (mnist_loader.hpp:57)
    k = np.round(Xo * 255)
    assert np.allclose(Xo, k / 255.0)


@pytest.mark.parametrize("dims,acts", [([784, 128, 10], ["relu", "linear"]),
                                       ([784, 256, 128, 64, 10], ["relu", "relu", "relu", "linear"]),
                                       ([5, 3, 2], ["tanh", "sigmoid"])])
@pytest.mark.parametrize("mode", ["cpu", "cuda"])
def test_init_stream_matches_oracle(pkg, O, dims, acts, mode):
    h = pkg.init_params_host(dims, acts, 123, mode)
    net = O.Net(dims, acts)
    ref = net.init_cpu(123).astype(np.float32) if mode == "cpu" else net.init_cuda(123)
    assert np.array_equal(h, ref)


def test_init_stream_seed123_draws(pkg):
    """seed-123 reference draws for the 784->128 ReLU layer."""
    h = pkg.init_params_host([784, 128, 10], ["relu", "linear"], 123, "cpu")
    ref = np.array([-0.028769634317892048, 0.085652536823551173, 0.056107483088271008], np.float32)
    assert np.array_equal(h[:3], ref)


def test_sample_indices_match_oracle(pkg, O):
    a = pkg.sample_indices(60000, 256, 123, calls=5)
    b = O.sample_indices(60000, 256, 123, calls=5)
    assert np.array_equal(a, b)
    # full-batch and b >= N cases (s_lbfgs.hpp:143-148)
    assert np.array_equal(pkg.sample_indices(10, 10, 1, 1)[0], np.arange(10))
    assert np.array_equal(pkg.sample_indices(10, 12, 1, 1)[0, :10], np.arange(10))


def test_sampler_reuse_matches_oracle(pkg, O):
    """The library draws every minibatch of an epoch from one reusable permutation (swaps undone after each
    draw); many draws in a row, b close to N and b = 1 give the oracle's fresh-iota lists (s_lbfgs.hpp:141-160)."""
    for N, b, seed, calls in [(1000, 999, 7, 40), (1000, 1, 3, 200), (517, 128, 11, 60), (60000, 128, 5, 30)]:
        assert np.array_equal(pkg.sample_indices(N, b, seed, calls=calls), O.sample_indices(N, b, seed, calls=calls))


def test_flop_model():
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    # per-sample flops 784-128-10 -> 409,088 ; 784-128-64-10 -> 454,400
    assert pkg.grad_flops_per_sample([784, 128, 10]) == 409088
    assert pkg.grad_flops_per_sample([784, 128, 64, 10]) == 454400
    assert pkg.grad_flops_per_sample([784, 512, 256, 10]) == 2407424
    assert pkg.grad_flops_per_sample([4096, 2048, 1024, 1]) == 46143488


def test_cpp_header_compiles_with_plain_gxx(tmp_path):
    """include/lbfgs_amd/hip_backend.hpp needs no HIP/Eigen/torch headers (C++17 + the C ABI)."""
    src = tmp_path / "t.cpp"
    src.write_text('#include "lbfgs_amd/hip_backend.hpp"\nint main(){ UnifiedConfig c; (void)c; return 0; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", f"-I{os.path.join(ROOT, 'include')}",
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
