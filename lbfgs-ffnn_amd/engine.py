"""Object layer over the C ABI: context, MLP, solvers (all compute in liblbfgs_amd_abi3.so).

Mirrors the reference's GPU-side pieces: ``CublasHandle`` -> :class:`Context`,
``CudaNetwork`` -> :class:`Mlp` (src/cuda/network.cuh), ``CudaLBFGS::solve`` -> :func:`lbfgs_solve`
(src/cuda/lbfgs.cuh:39-194, plus the CPU semantics of src/minimizer/lbfgs.hpp:38-100), and the S-LBFGS
of src/minimizer/s_lbfgs.hpp:165-290 -> :func:`slbfgs_solve`.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np
import torch

from ._lib import (ACTS, INIT_CPU, INIT_CUDA, LS_ARMIJO, LS_WOLFE, SLBFGS_DP_REPLICATED, SLBFGS_DP_SLICED, GdParams,
                   LbfError, LbfgsParams, Record, SgdParams, SlbfgsParams, SolveInfo, check, lib, ptr)


class Context:
    """One per GPU: device, stream (torch's current stream), optional RCCL communicator."""

    def __init__(self, device: int = 0, use_torch_stream: bool = True):
        if not torch.cuda.is_available():
            raise LbfError("no HIP device visible: the MI355X engine has no CPU fallback")
        self.device = device
        torch.cuda.set_device(device)
        stream = torch.cuda.current_stream(device).cuda_stream if use_torch_stream else 0
        h = C.c_void_p()
        check(lib().lbf_ctx_create(device, C.c_void_p(stream) if stream else None, C.byref(h)), "lbf_ctx_create")
        self.h = h
        self.rank, self.world = 0, 1

    def sync(self):
        check(lib().lbf_ctx_sync(self.h), "lbf_ctx_sync")

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().lbf_comm_unique_id(buf), "lbf_comm_unique_id")
        return buf.raw

    def comm_init(self, world: int, rank: int, uid: bytes):
        check(lib().lbf_comm_init(self.h, world, rank, uid), "lbf_comm_init")
        self.rank, self.world = rank, world

    @staticmethod
    def comm_init_local(ctxs: Sequence["Context"]):
        """In-process rank group (lbf_comm_init_local): ctxs[r] becomes rank r. The contexts share one device
        and each must then be driven by its own thread with the same call sequence."""
        arr = (C.c_void_p * len(ctxs))(*[c.h.value for c in ctxs])
        check(lib().lbf_comm_init_local(arr, len(ctxs)), "lbf_comm_init_local")
        for r, c in enumerate(ctxs):
            c.rank, c.world = r, len(ctxs)

    def allreduce_(self, t: torch.Tensor):
        check(lib().lbf_allreduce_sum(self.h, ptr(t), t.numel()), "lbf_allreduce_sum")
        return t

    def dot(self, x: torch.Tensor, y: torch.Tensor) -> float:
        out = C.c_double()
        check(lib().lbf_dot(self.h, x.numel(), ptr(x), ptr(y), C.byref(out)), "lbf_dot")
        return out.value

    def nrm2(self, x: torch.Tensor) -> float:
        out = C.c_double()
        check(lib().lbf_nrm2(self.h, x.numel(), ptr(x), C.byref(out)), "lbf_nrm2")
        return out.value

    def axpy_(self, alpha: float, x: torch.Tensor, y: torch.Tensor):
        check(lib().lbf_axpy(self.h, x.numel(), alpha, ptr(x), ptr(y)), "lbf_axpy")
        return y

    def two_loop(self, S: Optional[torch.Tensor], Y: Optional[torch.Tensor], rho: Sequence[float],
                 g: torch.Tensor, mode: int = 0) -> torch.Tensor:
        """Two-loop recursion on an explicit history (logical order, oldest first).
        mode 0: CPU semantics (returns -Hg), 1: S-LBFGS (+Hg), 2: CUDA (-Hg), 3: S-LBFGS through the solver's pair
        updates and direction-only step (rho computed on the device, `rho` ignored)."""
        k = 0 if S is None else int(S.shape[0])
        out = torch.empty_like(g)
        rho_arr = (C.c_double * max(k, 1))(*[float(r) for r in rho]) if k else None
        check(lib().lbf_two_loop(self.h, g.numel(), k, ptr(S) if k else None, ptr(Y) if k else None,
                                 C.cast(rho_arr, C.POINTER(C.c_double)) if k else None, ptr(g), ptr(out), mode),
              "lbf_two_loop")
        return out

    PROF_KINDS = ["gemm_fwd", "gemm_dw", "gemm_dx", "loss", "splitk_reduce", "finalize", "gram_sweep",
                  "hist_coef", "combine_sweep", "ls_axpy", "allreduce"]

    def prof_enable(self, on: bool = True):
        check(lib().lbf_prof_enable(self.h, int(on)), "lbf_prof_enable")

    def prof_select(self, section=None):
        """Time only `section` ("kind[layer]"), or every section when None."""
        sid = -1
        if section is not None:
            kind, layer = section.split("[")
            sid = self.PROF_KINDS.index(kind) * 16 + int(layer.rstrip("]"))
        check(lib().lbf_prof_select(self.h, sid), "lbf_prof_select")

    def prof_sample(self, every: int = 1):
        """Time only every `every`-th launch of the selected sections."""
        check(lib().lbf_prof_sample(self.h, int(every)), "lbf_prof_sample")

    def prof_read_work(self):
        """{section name: work units of the timed launches} (GEMM sections: batch rows)."""
        n = C.c_int(0)
        check(lib().lbf_prof_read_work(self.h, 0, None, None, C.byref(n)), "lbf_prof_read_work")
        cap = n.value
        ids = (C.c_int * max(cap, 1))()
        work = (C.c_double * max(cap, 1))()
        check(lib().lbf_prof_read_work(self.h, cap, ids, work, C.byref(n)), "lbf_prof_read_work")
        out = {}
        for i in range(min(cap, n.value)):
            kind, layer = divmod(ids[i], 16)
            name = self.PROF_KINDS[kind] if kind < len(self.PROF_KINDS) else f"k{kind}"
            out[f"{name}[{layer}]"] = work[i]
        return out

    def prof_read(self):
        """{section name: (total ms, launches)}; section = kind[layer]."""
        n = C.c_int(0)
        check(lib().lbf_prof_read(self.h, 0, None, None, None, C.byref(n)), "lbf_prof_read")
        cap = n.value
        ids = (C.c_int * max(cap, 1))()
        ms = (C.c_double * max(cap, 1))()
        cnt = (C.c_longlong * max(cap, 1))()
        check(lib().lbf_prof_read(self.h, cap, ids, ms, cnt, C.byref(n)), "lbf_prof_read")
        out = {}
        for i in range(min(cap, n.value)):
            kind, layer = divmod(ids[i], 16)
            name = self.PROF_KINDS[kind] if kind < len(self.PROF_KINDS) else f"k{kind}"
            out[f"{name}[{layer}]"] = (ms[i], int(cnt[i]))
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().lbf_ctx_destroy(self.h)
                self.h = None
        except Exception:
            pass


class Mlp:
    """Dense MLP; flat fp32 params in the reference layout [W (Out x In col-major) | b] per layer."""

    def __init__(self, ctx: Context, dims: Sequence[int], acts: Sequence):
        self.ctx = ctx
        self.dims = [int(d) for d in dims]
        self.acts = [ACTS[a] if isinstance(a, str) else int(a) for a in acts]
        assert len(self.dims) == len(self.acts) + 1
        d = (C.c_int * len(self.dims))(*self.dims)
        a = (C.c_int * len(self.acts))(*self.acts)
        h = C.c_void_p()
        check(lib().lbf_mlp_create(ctx.h, len(self.acts), d, a, C.byref(h)), "lbf_mlp_create")
        self.h = h
        self.nparams = int(lib().lbf_mlp_param_count(h))

    def _check_data(self, X: torch.Tensor, Y: Optional[torch.Tensor]):
        """X [rows][In], Y [rows][Out] (the reference's column-major In x N / Out x N)."""
        if X is not None and (X.dim() != 2 or X.shape[1] != self.dims[0]):
            raise LbfError(f"X must be [rows][{self.dims[0]}], got {tuple(X.shape)}")
        if Y is not None and (Y.dim() != 2 or Y.shape[1] != self.dims[-1] or Y.shape[0] != X.shape[0]):
            raise LbfError(f"Y must be [{X.shape[0]}][{self.dims[-1]}], got {tuple(Y.shape)}")

    def new_params(self) -> torch.Tensor:
        return torch.empty(self.nparams, dtype=torch.float32, device=f"cuda:{self.ctx.device}")

    def init_params(self, seed: int = 123, mode: str = "cpu", out: Optional[torch.Tensor] = None):
        out = self.new_params() if out is None else out
        check(lib().lbf_mlp_init_params(self.h, seed, INIT_CPU if mode == "cpu" else INIT_CUDA, ptr(out)),
              "lbf_mlp_init_params")
        return out

    def forward(self, params: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
        out = torch.empty((X.shape[0], self.dims[-1]), dtype=torch.float32, device=X.device)
        self._check_data(X, None)
        check(lib().lbf_mlp_forward(self.h, ptr(params, numel=self.nparams), ptr(X), X.shape[0], ptr(out)),
              "lbf_mlp_forward")
        return out

    def loss_grad(self, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, idx: Optional[torch.Tensor] = None,
                  inv_scale: Optional[float] = None, l2: float = 0.0, grad: Optional[torch.Tensor] = None):
        """LossGradFun (src/cuda/minimizer_base.cuh:15-16): returns (loss, grad)."""
        B = int(idx.numel()) if idx is not None else int(X.shape[0])
        if inv_scale is None:
            inv_scale = 1.0 / max(B, 1)
        grad = self.new_params() if grad is None else grad
        self._check_data(X, Y)
        loss = C.c_double()
        check(lib().lbf_mlp_loss_grad(self.h, ptr(params, numel=self.nparams), ptr(grad, numel=self.nparams), ptr(X),
                                      ptr(Y), ptr(idx, torch.int32), B, inv_scale, l2, C.byref(loss)),
              "lbf_mlp_loss_grad")
        return loss.value, grad

    def batch_grads(self, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, nmb: int,
                    inv_scale: Optional[float] = None, l2: float = 0.0) -> torch.Tensor:
        """Gradients of nmb consecutive minibatches of X / Y (X.shape[0] // nmb rows each, a multiple of 32) at
        one point, in one evaluation (lbf_mlp_batch_grads): returns an (nmb, nparams) tensor."""
        rows = int(X.shape[0])
        if nmb <= 0 or rows % nmb:
            raise LbfError(f"batch_grads: {rows} rows do not split into {nmb} equal minibatches")
        cnt = rows // nmb
        if cnt % 32:
            raise LbfError(f"batch_grads: {cnt} rows per minibatch, need a multiple of 32")
        if inv_scale is None:
            inv_scale = 1.0 / cnt
        self._check_data(X, Y)
        out = torch.empty((nmb, self.nparams), dtype=torch.float32, device=params.device)
        check(lib().lbf_mlp_batch_grads(self.h, ptr(params, numel=self.nparams), ptr(X), ptr(Y), nmb, cnt, inv_scale,
                                        l2, ptr(out), self.nparams), "lbf_mlp_batch_grads")
        return out

    def loss(self, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, idx: Optional[torch.Tensor] = None,
             inv_scale: Optional[float] = None) -> float:
        """Forward + MSE only (lbf_mlp_loss): the f of a line-search trial."""
        B = int(idx.numel()) if idx is not None else int(X.shape[0])
        if inv_scale is None:
            inv_scale = 1.0 / max(B, 1)
        self._check_data(X, Y)
        out = C.c_double()
        check(lib().lbf_mlp_loss(self.h, ptr(params, numel=self.nparams), ptr(X), ptr(Y), ptr(idx, torch.int32), B,
                                 inv_scale, C.byref(out)), "lbf_mlp_loss")
        return out.value

    def hvp(self, params: torch.Tensor, v: torch.Tensor, X: torch.Tensor, Y: torch.Tensor,
            idx: Optional[torch.Tensor] = None, inv_scale: Optional[float] = None, l2: float = 0.0,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Exact H(params) v of the loss_grad batch loss (R-operator, lbf_mlp_hvp)."""
        B = int(idx.numel()) if idx is not None else int(X.shape[0])
        if inv_scale is None:
            inv_scale = 1.0 / max(B, 1)
        out = self.new_params() if out is None else out
        self._check_data(X, Y)
        n = self.nparams
        check(lib().lbf_mlp_hvp(self.h, ptr(params, numel=n), ptr(v, numel=n), ptr(X), ptr(Y), ptr(idx, torch.int32),
                                B, inv_scale, l2, ptr(out, numel=n)), "lbf_mlp_hvp")
        return out

    def fd_hvp(self, params: torch.Tensor, v: torch.Tensor, X: torch.Tensor, Y: torch.Tensor,
               idx: Optional[torch.Tensor] = None, inv_scale: Optional[float] = None, l2: float = 0.0,
               eps: float = 1e-4, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """finite_difference_hvp_batch (s_lbfgs.hpp:88-101), the S-LBFGS curvature pair's y."""
        B = int(idx.numel()) if idx is not None else int(X.shape[0])
        if inv_scale is None:
            inv_scale = 1.0 / max(B, 1)
        out = self.new_params() if out is None else out
        self._check_data(X, Y)
        n = self.nparams
        check(lib().lbf_mlp_fd_hvp(self.h, ptr(params, numel=n), ptr(v, numel=n), ptr(X), ptr(Y),
                                   ptr(idx, torch.int32), B, inv_scale, l2, eps, ptr(out, numel=n)), "lbf_mlp_fd_hvp")
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().lbf_mlp_destroy(self.h)
                self.h = None
        except Exception:
            pass


class History:
    """Host arrays receiving the per-iteration record (IterationRecorder, src/iteration_recorder.hpp)."""

    def __init__(self, cap: int):
        self.cap = max(int(cap), 1)
        self.loss = np.zeros(self.cap)
        self.grad_norm = np.zeros(self.cap)
        self.time_ms = np.zeros(self.cap)
        self.alpha = np.zeros(self.cap)
        self.ls_trials = np.zeros(self.cap, np.int32)
        self.accepted = np.full(self.cap, -1, np.int32)
        self.rec = Record(self.loss.ctypes.data_as(C.POINTER(C.c_double)),
                          self.grad_norm.ctypes.data_as(C.POINTER(C.c_double)),
                          self.time_ms.ctypes.data_as(C.POINTER(C.c_double)),
                          self.alpha.ctypes.data_as(C.POINTER(C.c_double)),
                          self.ls_trials.ctypes.data_as(C.POINTER(C.c_int)),
                          self.accepted.ctypes.data_as(C.POINTER(C.c_int)), self.cap, 0)

    @property
    def size(self) -> int:
        return int(self.rec.size)

    def as_dict(self):
        n = self.size
        return dict(loss=self.loss[:n].copy(), grad_norm=self.grad_norm[:n].copy(), time_ms=self.time_ms[:n].copy(),
                    alpha=self.alpha[:n].copy(), ls_trials=self.ls_trials[:n].copy(),
                    accepted=self.accepted[:n].copy())


def lbfgs_params(line_search: str = "wolfe", **kw) -> LbfgsParams:
    p = LbfgsParams()
    lib().lbf_lbfgs_default_params(C.byref(p), LS_ARMIJO if line_search == "armijo" else LS_WOLFE)
    for k, v in kw.items():
        if v is not None:
            setattr(p, k, v)
    return p


def slbfgs_params(**kw) -> SlbfgsParams:
    p = SlbfgsParams()
    lib().lbf_slbfgs_default_params(C.byref(p))
    if isinstance(kw.get("dp_mode"), str):
        kw["dp_mode"] = {"replicated": SLBFGS_DP_REPLICATED, "sliced": SLBFGS_DP_SLICED}[kw["dp_mode"]]
    for k, v in kw.items():
        if v is not None:
            setattr(p, "reg" if k == "lam" else k, v)
    return p


def lbfgs_solve(net: Mlp, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, n_global: Optional[int] = None,
                line_search: str = "wolfe", **kw):
    """Full-batch L-BFGS; params updated in place. Returns (history dict, SolveInfo)."""
    p = lbfgs_params(line_search, **kw)
    hist = History(p.max_iters)
    info = SolveInfo()
    n_local = int(X.shape[0])
    check(lib().lbf_lbfgs_solve(net.h, C.byref(p), ptr(params), ptr(X), ptr(Y), n_local,
                                int(n_global or n_local), C.byref(hist.rec), C.byref(info)), "lbf_lbfgs_solve")
    return hist.as_dict(), info


class LbfgsRun:
    """Stateful L-BFGS (begin / iterate / end) used by the benchmark."""

    def __init__(self, net: Mlp, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor,
                 n_global: Optional[int] = None, line_search: str = "wolfe", record_cap: int = 100000, **kw):
        self.p = lbfgs_params(line_search, **kw)
        self.hist = History(record_cap)
        self.info = SolveInfo()
        self._keep = (net, params, X, Y)
        h = C.c_void_p()
        check(lib().lbf_lbfgs_begin(net.h, C.byref(self.p), ptr(params), ptr(X), ptr(Y), int(X.shape[0]),
                                    int(n_global or X.shape[0]), C.byref(h)), "lbf_lbfgs_begin")
        self.h = h

    def iterate(self, iters: int):
        check(lib().lbf_lbfgs_iterate(self.h, iters, C.byref(self.hist.rec), C.byref(self.info)),
              "lbf_lbfgs_iterate")
        return self.info

    def close(self):
        if self.h:
            lib().lbf_lbfgs_end(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def slbfgs_solve(net: Mlp, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, pair_trace: int = 0, **kw):
    """S-LBFGS (SVRG + FD-HVP curvature pairs); X/Y hold all N rows on every rank. pair_trace > 0 records up
    to that many curvature-pair candidates (diagnostics, synchronous) into hist["pairs"]: rows of (epoch, t,
    y.s, s.s, y.y, accepted, live pairs, 0)."""
    p = slbfgs_params(**kw)
    trace = None
    if pair_trace > 0:
        trace = np.full((int(pair_trace), 8), np.nan)
        p.pair_trace = trace.ctypes.data_as(C.POINTER(C.c_double))
        p.pair_trace_cap = int(pair_trace)
    hist = History(p.max_epochs)
    info = SolveInfo()
    check(lib().lbf_slbfgs_solve(net.h, C.byref(p), ptr(params), ptr(X), ptr(Y), int(X.shape[0]),
                                 C.byref(hist.rec), C.byref(info)), "lbf_slbfgs_solve")
    out = hist.as_dict()
    if trace is not None:
        out["pairs"] = trace[~np.isnan(trace[:, 0])]
    return out, info


class SlbfgsRun:
    """Stateful S-LBFGS (begin / iterate / end) used by the benchmark: the epochs of one solve across several
    iterate() calls (the breakdown, warmup and timed epochs), bitwise one lbf_slbfgs_solve."""

    def __init__(self, net: Mlp, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, record_cap: int = 100000,
                 pair_trace: int = 0, **kw):
        self.p = slbfgs_params(**kw)
        self.p.max_epochs = max(int(self.p.max_epochs), 1 << 30)
        self.trace = None
        if pair_trace > 0:  # diagnostics: rows as slbfgs_solve's hist["pairs"], and pair0()
            self.trace = np.full((int(pair_trace), 8), np.nan)
            self.p.pair_trace = self.trace.ctypes.data_as(C.POINTER(C.c_double))
            self.p.pair_trace_cap = int(pair_trace)
        self.hist = History(record_cap)
        self.info = SolveInfo()
        self._keep = (net, params, X, Y)
        h = C.c_void_p()
        check(lib().lbf_slbfgs_begin(net.h, C.byref(self.p), ptr(params), ptr(X), ptr(Y), int(X.shape[0]),
                                     C.byref(h)), "lbf_slbfgs_begin")
        self.h = h

    def iterate(self, epochs: int):
        check(lib().lbf_slbfgs_iterate(self.h, epochs, C.byref(self.hist.rec), C.byref(self.info)),
              "lbf_slbfgs_iterate")
        return self.info

    def pairs(self):
        return None if self.trace is None else self.trace[~np.isnan(self.trace[:, 0])]

    def pair0(self):
        """The first traced curvature-pair candidate's (w_t, u, s, y) as device tensors (lbf_slbfgs_pair0)."""
        n = int(self._keep[1].numel())
        out = [torch.empty(n, dtype=torch.float32, device=self._keep[1].device) for _ in range(4)]
        check(lib().lbf_slbfgs_pair0(self.h, *[ptr(t) for t in out]), "lbf_slbfgs_pair0")
        return out

    def pair_io(self, cap: int, record: bool = True, force: Optional[torch.Tensor] = None):
        """Teacher forcing of the curvature pairs (lbf_slbfgs_pair_io; call before iterate). Returns the record
        tensor [cap, 4, ld] ([w_{t+1} | u | g(u + eps s) | g(u - eps s)] per curvature event) or None; `force`
        (same shape, e.g. another run's record) replaces u and the two gradients of each event."""
        n = int(self._keep[1].numel())
        ld = (n + 3) & ~3
        dev = self._keep[1].device
        rec = torch.zeros((int(cap), 4, ld), dtype=torch.float32, device=dev) if record else None
        if force is not None:
            if tuple(force.shape) != (int(cap), 4, ld):
                raise LbfError(f"force: expected shape {(int(cap), 4, ld)}, got {tuple(force.shape)}")
        self._pio = (rec, force)  # kept alive while the solver may write / read them
        check(lib().lbf_slbfgs_pair_io(self.h, int(cap), ptr(rec), ptr(force)), "lbf_slbfgs_pair_io")
        return rec

    def close(self):
        if self.h:
            lib().lbf_slbfgs_end(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gd_solve(net: Mlp, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, n_global: Optional[int] = None,
             **kw):
    """CudaGD::solve (src/cuda/gd.cuh:38-106); params updated in place. kw: lr, momentum, max_iters, tol."""
    p = GdParams()
    lib().lbf_gd_default_params(C.byref(p))
    for k, v in kw.items():
        if v is not None:
            setattr(p, k, v)
    hist = History(max(p.max_iters, 1))
    info = SolveInfo()
    n_local = int(X.shape[0])
    check(lib().lbf_gd_solve(net.h, C.byref(p), ptr(params), ptr(X), ptr(Y), n_local, int(n_global or n_local),
                             C.byref(hist.rec), C.byref(info)), "lbf_gd_solve")
    return hist.as_dict(), info


def sgd_solve(net: Mlp, params: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, record: bool = True, **kw):
    """CudaSGD::solve (src/cuda/sgd.cuh:50-153). kw: lr, momentum, batch, decay_rate, decay_step,
    max_epochs, tol. record=False runs without the recorder (no full-batch evaluations)."""
    p = SgdParams()
    lib().lbf_sgd_default_params(C.byref(p))
    for k, v in kw.items():
        if v is not None:
            setattr(p, k, v)
    hist = History(p.max_epochs + 1)
    info = SolveInfo()
    check(lib().lbf_sgd_solve(net.h, C.byref(p), ptr(params), ptr(X), ptr(Y), int(X.shape[0]),
                              C.byref(hist.rec) if record else None, C.byref(info)), "lbf_sgd_solve")
    return hist.as_dict(), info


def init_params_host(dims: Sequence[int], acts: Sequence, seed: int = 123, mode: str = "cpu") -> np.ndarray:
    """Host-side copy of the init stream (for tests; the device path is Mlp.init_params)."""
    a = [ACTS[x] if isinstance(x, str) else int(x) for x in acts]
    d = (C.c_int * len(dims))(*[int(x) for x in dims])
    ac = (C.c_int * len(a))(*a)
    n = sum((dims[i] + 1) * dims[i + 1] for i in range(len(a)))
    out = np.empty(n, np.float32)
    check(lib().lbf_init_params_host(len(a), d, ac, seed, INIT_CPU if mode == "cpu" else INIT_CUDA,
                                     out.ctypes.data_as(C.c_void_p)), "lbf_init_params_host")
    return out


def synth_mnist(N: int, In: int = 784, classes: int = 10, seed: int = 123):
    """Synthetic MNIST-shaped data; host float32 arrays [N][In], [N][classes]."""
    X = np.empty((N, In), np.float32)
    Y = np.empty((N, classes), np.float32)
    check(lib().lbf_synth_mnist(N, In, classes, seed, X.ctypes.data_as(C.c_void_p), Y.ctypes.data_as(C.c_void_p)),
          "lbf_synth_mnist")
    return X, Y


def synth_regression(ctx: Context, N: int, In: int = 4096, seed_x: int = 123, seed_t: int = 124, row0: int = 0):
    """BASELINE config 5 data on the device: rows [row0, row0+N) of X ~ N(0,1) [.][In] and
    y = tanh(v.x/64) + 0.01 e [.][1]."""
    X = torch.empty((N, In), dtype=torch.float32, device=f"cuda:{ctx.device}")
    Y = torch.empty((N, 1), dtype=torch.float32, device=f"cuda:{ctx.device}")
    check(lib().lbf_synth_regression(ctx.h, row0, N, In, seed_x, seed_t, ptr(X), ptr(Y)), "lbf_synth_regression")
    return X, Y


def load_idx_images(path: str, max_images: int = 0) -> np.ndarray:
    """MNISTLoader::loadImages (tests/mnist/mnist_loader.hpp:21-61): [N][rows*cols] float32 in [0, 1]."""
    n, r, c = C.c_longlong(0), C.c_int(0), C.c_int(0)
    check(lib().lbf_idx_read_images(path.encode(), max_images, None, C.byref(n), C.byref(r), C.byref(c)),
          "lbf_idx_read_images")
    out = np.empty((n.value, r.value * c.value), np.float32)
    check(lib().lbf_idx_read_images(path.encode(), max_images, out.ctypes.data_as(C.c_void_p), C.byref(n),
                                    C.byref(r), C.byref(c)), "lbf_idx_read_images")
    return out


def load_idx_labels(path: str, max_labels: int = 0, classes: int = 10) -> np.ndarray:
    """MNISTLoader::loadLabels (tests/mnist/mnist_loader.hpp:63-100): one-hot [N][classes] float32."""
    n = C.c_longlong(0)
    check(lib().lbf_idx_read_labels(path.encode(), max_labels, classes, None, C.byref(n)), "lbf_idx_read_labels")
    out = np.empty((n.value, classes), np.float32)
    check(lib().lbf_idx_read_labels(path.encode(), max_labels, classes, out.ctypes.data_as(C.c_void_p), C.byref(n)),
          "lbf_idx_read_labels")
    return out


def sample_indices(N: int, b: int, seed: int = 123, calls: int = 1) -> np.ndarray:
    out = np.empty(calls * b, np.int64)
    check(lib().lbf_sample_indices(N, b, seed, calls, out.ctypes.data_as(C.c_void_p)), "lbf_sample_indices")
    return out.reshape(calls, b)


def grad_flops_per_sample(dims: Sequence[int]) -> int:
    """Algorithmic flops of one loss+grad per sample: fwd + dW + dX (layer 0 has no dX)."""
    f = 0
    for l in range(len(dims) - 1):
        io = dims[l] * dims[l + 1]
        f += 2 * io + 2 * io + (2 * io if l > 0 else 0)
    return f
