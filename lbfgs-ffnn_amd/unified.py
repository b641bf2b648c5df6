"""Host-side mirror of the reference's unified API for the HIP backend.

Same names, argument meaning and defaults as src/unified_optimization.hpp / src/unified_launcher.hpp /
src/iteration_recorder.hpp, so a driver like tests/mnist/main-gpu.cpp reads the same:

    launcher = UnifiedLauncher()                     # UnifiedLauncher<HipBackend>
    launcher.addLayer(784, 128, "relu"); launcher.addLayer(128, 10, "linear"); launcher.buildNetwork()
    launcher.setData(dataset)                        # UnifiedDataset (numpy, [N][In] == In x N col-major)
    cfg = UnifiedConfig(name="MNIST_LBFGS_m10", max_iters=1000, tolerance=1e-3, m_param=10, log_interval=1)
    launcher.train(UnifiedLBFGS(), cfg); launcher.test()

Data parallelism: if torch.distributed is initialised, each rank holds its contiguous shard of the
training rows for full-batch L-BFGS (one RCCL all-reduce of [grad | loss] per evaluation) and all rows
for S-LBFGS (minibatch index lists are sliced across ranks).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from . import engine
from ._lib import LbfError


@dataclass
class UnifiedConfig:
    """src/unified_optimization.hpp:26-48 (+ HIP extensions: line_search, init)."""
    name: str = "Experiment"
    max_iters: int = 100
    tolerance: float = 1e-4
    learning_rate: float = 0.01
    momentum: float = 0.0
    lr_decay: float = 0.0
    lr_decay_rate: int = 1
    batch_size: int = 128
    m_param: int = 10
    L_param: int = 10
    b_H_param: int = 0
    log_interval: int = 10
    reset_params: bool = True
    seed: int = 123
    line_search: str = "wolfe"   # "wolfe" = CPU semantics (parity target), "armijo" = CUDA semantics
    init: str = "cpu"            # "cpu" (network.hpp:45-71) or "cuda" (network.cuh:36-59) init stream
    write_csv: bool = True


@dataclass
class UnifiedDataset:
    """src/unified_optimization.hpp:54-59; arrays are [N][features] (== the reference's column-major)."""
    train_x: np.ndarray = field(default_factory=lambda: np.zeros((0, 0)))
    train_y: np.ndarray = field(default_factory=lambda: np.zeros((0, 0)))
    test_x: np.ndarray = field(default_factory=lambda: np.zeros((0, 0)))
    test_y: np.ndarray = field(default_factory=lambda: np.zeros((0, 0)))


class IterationRecorder:
    """src/iteration_recorder.hpp:13-146 (loss, grad-norm, cumulative ms per iteration)."""

    def __init__(self):
        self.loss, self.grad_norm, self.time_ms = [], [], []

    def init(self, capacity: int):
        self.reset()

    def reset(self):
        self.loss, self.grad_norm, self.time_ms = [], [], []

    def record(self, idx: int, loss: float, grad_norm: float, time_ms: float = 0.0):
        while len(self.loss) <= idx:
            self.loss.append(0.0)
            self.grad_norm.append(0.0)
            self.time_ms.append(0.0)
        self.loss[idx], self.grad_norm[idx], self.time_ms[idx] = loss, grad_norm, time_ms

    def copy_to_host(self):
        return list(self.loss), list(self.grad_norm), list(self.time_ms)

    def size(self) -> int:
        return len(self.loss)


def log_filename(config: UnifiedConfig) -> str:
    return (config.name or "run") + "_history.csv"   # unified_optimization.hpp:61-64


def write_history_csv(filename: str, recorder: IterationRecorder, log_interval: int) -> None:
    """unified_optimization.hpp:66-85 / :446-465: `Iteration,Loss,GradNorm,TimeMs`, strided."""
    if log_interval <= 0 or recorder.size() == 0:
        return
    loss, grad, tms = recorder.copy_to_host()
    with open(filename, "w") as f:
        f.write("Iteration,Loss,GradNorm,TimeMs\n")
        for i in range(0, len(loss), max(1, log_interval)):
            f.write(f"{i},{loss[i]:g},{grad[i]:g},{tms[i]:g}\n")


class _DeviceNet:
    """What NetworkWrapper<HipBackend> wraps: the HIP MLP and its flat parameter tensor."""

    def __init__(self, ctx: engine.Context):
        self.ctx = ctx
        self.layers = []
        self.mlp: Optional[engine.Mlp] = None
        self.params: Optional[torch.Tensor] = None

    def addLayer(self, In: int, Out: int, act):
        if self.layers and self.layers[-1][1] != In:
            raise LbfError(f"layer input {In} does not match previous output {self.layers[-1][1]}")
        self.layers.append((int(In), int(Out), act))

    def bindParams(self, seed: int = 123, mode: str = "cpu"):
        dims = [self.layers[0][0]] + [l[1] for l in self.layers]
        if self.mlp is None:
            self.mlp = engine.Mlp(self.ctx, dims, [l[2] for l in self.layers])
            self.params = self.mlp.new_params()
        self.mlp.init_params(seed, mode, self.params)

    def getParamsSize(self) -> int:
        return self.mlp.nparams if self.mlp else 0


class UnifiedOptimizer:
    def optimize(self, net: _DeviceNet, data: "_DeviceData", config: UnifiedConfig) -> IterationRecorder:
        raise NotImplementedError


class UnifiedLBFGS(UnifiedOptimizer):
    """UnifiedLBFGS<HipBackend> (unified_optimization.hpp:191-214 / 560-592)."""

    def optimize(self, net, data, config):
        hist, info = engine.lbfgs_solve(net.mlp, net.params, data.x, data.y, n_global=data.n_global,
                                        line_search=config.line_search, m=config.m_param if config.m_param > 0 else 10,
                                        max_iters=config.max_iters, tol=config.tolerance)
        rec = IterationRecorder()
        for i in range(len(hist["loss"])):
            rec.record(i, float(hist["loss"][i]), float(hist["grad_norm"][i]), float(hist["time_ms"][i]))
        self.info = info
        self.history = hist
        return rec


class UnifiedSLBFGS(UnifiedOptimizer):
    """UnifiedSLBFGS<HipBackend>: the reference has it CPU-only (static_assert for CUDA,
    unified_optimization.hpp:635-641, 688-696); here it runs on the GPU with the CPU semantics of
    UnifiedSLBFGS_CPU (unified_optimization.hpp:306-408)."""

    def optimize(self, net, data, config):
        b_H = config.b_H_param if config.b_H_param > 0 else config.batch_size // 2   # :325
        hist, info = engine.slbfgs_solve(net.mlp, net.params, data.x_full, data.y_full, max_epochs=config.max_iters,
                                         tol=config.tolerance, M=config.m_param, L=config.L_param,
                                         b=config.batch_size, b_H=b_H, step=config.learning_rate, lam=1e-4,
                                         seed=123)
        rec = IterationRecorder()
        for i in range(len(hist["loss"])):
            rec.record(i, float(hist["loss"][i]), float(hist["grad_norm"][i]), float(hist["time_ms"][i]))
        self.info = info
        self.history = hist
        return rec


class UnifiedGD(UnifiedOptimizer):
    """UnifiedGD<HipBackend> (unified_optimization.hpp:518-554: CudaGD with the config's learning_rate,
    momentum, max_iters, tolerance)."""

    def optimize(self, net, data, config):
        hist, info = engine.gd_solve(net.mlp, net.params, data.x, data.y, n_global=data.n_global,
                                     lr=config.learning_rate, momentum=config.momentum, max_iters=config.max_iters,
                                     tol=config.tolerance)
        rec = IterationRecorder()
        for i in range(len(hist["loss"])):
            rec.record(i, float(hist["loss"][i]), float(hist["grad_norm"][i]), float(hist["time_ms"][i]))
        self.info = info
        self.history = hist
        return rec


class UnifiedSGD(UnifiedOptimizer):
    """UnifiedSGD<HipBackend> (unified_optimization.hpp:595-632: CudaSGD with learning_rate, momentum,
    batch_size, max_iters epochs and setLearningRateDecay(lr_decay, lr_decay_rate); the tolerance is
    not passed, so CudaSGD's default 1e-6 applies). Single rank."""

    def optimize(self, net, data, config):
        hist, info = engine.sgd_solve(net.mlp, net.params, data.x_full, data.y_full, lr=config.learning_rate,
                                      momentum=config.momentum, batch=config.batch_size, max_epochs=config.max_iters,
                                      decay_rate=config.lr_decay, decay_step=config.lr_decay_rate)
        rec = IterationRecorder()
        for i in range(len(hist["loss"])):
            rec.record(i, float(hist["loss"][i]), float(hist["grad_norm"][i]), float(hist["time_ms"][i]))
        self.info = info
        self.history = hist
        return rec


class _DeviceData:
    def __init__(self, dataset: UnifiedDataset, device: str, rank: int, world: int, need_full: bool = True):
        tx = np.ascontiguousarray(dataset.train_x, np.float32)   # fp64 -> fp32 upload (unified_launcher.hpp:105-128)
        ty = np.ascontiguousarray(dataset.train_y, np.float32)
        N = tx.shape[0]
        lo, hi = N * rank // world, N * (rank + 1) // world
        self.n_global = N
        self.x = torch.from_numpy(tx[lo:hi]).to(device)
        self.y = torch.from_numpy(ty[lo:hi]).to(device)
        if world == 1:
            self.x_full, self.y_full = self.x, self.y
        elif need_full:
            self.x_full = torch.from_numpy(tx).to(device)
            self.y_full = torch.from_numpy(ty).to(device)
        self.test_x = torch.from_numpy(np.ascontiguousarray(dataset.test_x, np.float32)).to(device) \
            if dataset.test_x.size else None
        self.test_y = np.asarray(dataset.test_y, np.float64)
        self.train_y_host = np.asarray(dataset.train_y, np.float64)
        torch.cuda.synchronize()


class UnifiedLauncher:
    """UnifiedLauncher<HipBackend> (src/unified_launcher.hpp:83-205)."""

    def __init__(self, device: Optional[int] = None):
        rank, world = 0, 1
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            rank, world = torch.distributed.get_rank(), torch.distributed.get_world_size()
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count())
        self.ctx = engine.Context(device)
        if world > 1:
            uid = [engine.Context.unique_id() if rank == 0 else None]
            torch.distributed.broadcast_object_list(uid, src=0)
            self.ctx.comm_init(world, rank, uid[0])
        self.rank, self.world = rank, world
        self.net_wrapper_ = _DeviceNet(self.ctx)
        self.data_: Optional[_DeviceData] = None
        self.dataset_ = None

    def addLayer(self, In: int, Out: int, act="linear"):
        self.net_wrapper_.addLayer(In, Out, act)

    def buildNetwork(self):
        self.net_wrapper_.bindParams()

    def setData(self, data: UnifiedDataset):
        self.dataset_ = data
        self.data_ = _DeviceData(data, f"cuda:{self.ctx.device}", self.rank, self.world)

    def train(self, optimizer: UnifiedOptimizer, config: UnifiedConfig):
        if self.rank == 0:
            print(f">>> Running HIP Experiment: {config.name}")
        if config.reset_params:
            self.net_wrapper_.bindParams(config.seed, config.init)
        recorder = optimizer.optimize(self.net_wrapper_, self.data_, config)
        if config.write_csv and self.rank == 0:
            write_history_csv(log_filename(config), recorder, config.log_interval)
        self.last_recorder = recorder
        return self.evaluate(self.data_.x_full if self.world == 1 else self.data_.x_full,
                             self.data_.train_y_host, "Training Results")

    def test(self):
        if self.data_ is None or self.data_.test_x is None:
            return None
        return self.evaluate(self.data_.test_x, self.data_.test_y, "Test Results")

    def evaluate(self, x: torch.Tensor, y: np.ndarray, label: str):
        """unified_launcher.hpp:154-199: forward on the device, accuracy + mean MSE on the host."""
        out = self.net_wrapper_.mlp.forward(self.net_wrapper_.params, x).double().cpu().numpy()
        mse = float(((out - y) ** 2).mean()) if out.size else 0.0
        acc = float((out.argmax(1) == y.argmax(1)).mean() * 100.0) if out.size else 0.0
        if self.rank == 0:
            print(f"{label}: MSE={mse:g}, Accuracy={acc:g}%")
        return dict(mse=mse, accuracy=acc)

    def getWrapper(self):
        return self.net_wrapper_
