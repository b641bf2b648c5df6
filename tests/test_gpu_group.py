"""The grouped weight-gradient launch (gemm.hip gemm_group, runtime.cpp Mlp::backward_phase).

Small batches (S-LBFGS minibatches, b = 256) run the dW GEMMs of layers 1 and 0 as one launch whose
z-planes hold both problems' split-K grids. Each split still sums its own k range in the same order and
the slabs are reduced as before, so the gradient must be bitwise the one of two separate launches
(LBF_NO_GROUP=1, read when an Mlp is built), and both must match the fp64 oracle.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


CASES = [([784, 512, 256, 10], ["relu", "relu", "linear"], 256),   # config 4's minibatch
         ([784, 512, 256, 10], ["tanh", "sigmoid", "linear"], 128),  # its Hessian batch
         ([784, 256, 128, 64, 10], ["relu", "relu", "relu", "linear"], 512),
         ([100, 96, 72, 10], ["relu", "tanh", "linear"], 64)]


@pytest.mark.parametrize("dims,acts,B", CASES)
def test_grouped_dw_bitwise_separate(ctx, pkg, O, monkeypatch, dims, acts, B):
    Xh, Yh = pkg.synth_mnist(B, dims[0], dims[-1], 7)
    X, Y = dev(Xh), dev(Yh)
    monkeypatch.delenv("LBF_NO_GROUP", raising=False)
    net_g = pkg.Mlp(ctx, dims, acts)
    monkeypatch.setenv("LBF_NO_GROUP", "1")
    net_s = pkg.Mlp(ctx, dims, acts)
    monkeypatch.delenv("LBF_NO_GROUP")
    P = net_g.init_params(123, "cpu")
    lg, gg = net_g.loss_grad(P, X, Y, inv_scale=1.0 / B)
    ls, gs = net_s.loss_grad(P, X, Y, inv_scale=1.0 / B)
    torch.cuda.synchronize()
    assert torch.equal(gg, gs)
    assert lg == ls
    # and the fp64 oracle agrees with both (test_gpu_parity.py's tolerances)
    lo, go = O.Net(dims, acts).loss_grad(P.double().cpu().numpy(), Xh.astype(np.float64), Yh.astype(np.float64))
    gd = gg.double().cpu().numpy()
    assert abs(lg - lo) <= 1e-5 * abs(lo)
    assert np.linalg.norm(gd - go) <= 1e-4 * np.linalg.norm(go)
