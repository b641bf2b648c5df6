"""oracle/oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes binding of ``oracle/build/liboracle.so`` (the CPU restatement in ``oracle.hpp``). Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this module;
the product package (``lbfgs-ffnn_amd/``) never does.

Every function mirrors a reference entry point; citations are in ``oracle.hpp``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

ACTS = {"linear": 0, "tanh": 1, "relu": 2, "sigmoid": 3}

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_fp = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lp = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    if os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", _HERE, "ref"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.oracle_param_count.restype = C.c_longlong
        L.oracle_param_count.argtypes = [C.c_int, _ip, _ip]
        L.oracle_init_params_cpu.argtypes = [C.c_int, _ip, _ip, C.c_uint, _dp]
        L.oracle_init_params_cuda.argtypes = [C.c_int, _ip, _ip, C.c_uint, _fp]
        L.oracle_loss_grad.restype = C.c_double
        L.oracle_loss_grad.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_void_p, C.c_longlong, C.c_double,
                                       C.c_void_p]
        L.oracle_fd_hvp.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, _dp, C.c_void_p, C.c_longlong, C.c_double,
                                    C.c_double, _dp]
        L.oracle_fd_hvp_f32.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, _dp, C.c_void_p, C.c_longlong,
                                        C.c_longlong, C.c_double, C.c_double, _dp]
        L.oracle_loss_grad_f32.restype = C.c_double
        L.oracle_loss_grad_f32.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_longlong, _dp]
        L.oracle_loss.restype = C.c_double
        L.oracle_loss.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_longlong, C.c_void_p]
        L.oracle_two_loop.argtypes = [C.c_int, C.c_longlong, C.c_int, _dp, _dp, _dp, _dp, _dp]
        L.oracle_lbfgs_wolfe_mlp.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_longlong, C.c_int, C.c_int,
                                             C.c_double, C.c_int, _dp, C.POINTER(C.c_int), C.POINTER(C.c_long),
                                             C.POINTER(C.c_long), C.POINTER(C.c_double)]
        L.oracle_lbfgs_armijo_mlp.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_longlong, C.c_int, C.c_int,
                                              C.c_double, C.c_int, C.c_double, C.c_double, C.c_int, _dp,
                                              C.POINTER(C.c_int)]
        L.oracle_slbfgs_mlp.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_longlong, C.c_int, C.c_double,
                                        C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, _dp,
                                        C.POINTER(C.c_int), C.c_void_p, C.c_longlong, C.c_void_p, C.c_int,
                                        C.POINTER(C.c_int), C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.oracle_gd_mlp.restype = C.c_int
        L.oracle_gd_mlp.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_longlong, C.c_double, C.c_double, C.c_int,
                                    C.c_double, C.c_int, _dp]
        L.oracle_sgd_mlp.restype = C.c_int
        L.oracle_sgd_mlp.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_longlong, C.c_int, C.c_double, C.c_double,
                                     C.c_double, C.c_int, C.c_int, C.c_double, C.c_int, _dp]
        L.oracle_lbfgs_testfn.restype = C.c_double
        L.oracle_lbfgs_testfn.argtypes = [C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.c_double, C.POINTER(C.c_int)]
        L.oracle_sample_indices.argtypes = [C.c_longlong, C.c_int, C.c_uint, C.c_int, _lp]
        L.oracle_synth_mnist.argtypes = [C.c_longlong, C.c_int, C.c_int, C.c_uint, _dp, _dp]
        L.oracle_ring_trace.argtypes = [C.c_int, C.c_int, _ip, _ip]
        L.oracle_num_threads.restype = C.c_int
        L.oracle_set_threads.argtypes = [C.c_int]
        _lib = L
    return _lib


class Net:
    """Layer spec: dims = [In, h1, ..., Out], acts = per-layer activation names."""

    def __init__(self, dims, acts):
        self.dims = np.ascontiguousarray(dims, dtype=np.int32)
        self.acts = np.ascontiguousarray([ACTS[a] if isinstance(a, str) else int(a) for a in acts], dtype=np.int32)
        self.nl = len(acts)
        assert len(dims) == self.nl + 1

    @property
    def nparams(self) -> int:
        return int(lib().oracle_param_count(self.nl, self.dims, self.acts))

    def init_cpu(self, seed: int = 123) -> np.ndarray:
        out = np.empty(self.nparams, np.float64)
        lib().oracle_init_params_cpu(self.nl, self.dims, self.acts, seed, out)
        return out

    def init_cuda(self, seed: int = 123) -> np.ndarray:
        out = np.empty(self.nparams, np.float32)
        lib().oracle_init_params_cuda(self.nl, self.dims, self.acts, seed, out)
        return out

    def loss_grad(self, P, X, Y, idx=None, lam: float = 0.0):
        P = np.ascontiguousarray(P, np.float64)
        X = np.ascontiguousarray(X, np.float64)
        Y = np.ascontiguousarray(Y, np.float64)
        g = np.empty(self.nparams, np.float64)
        if idx is not None:
            idx = np.ascontiguousarray(idx, np.int64)
            B = len(idx)
            ip = idx.ctypes.data
        else:
            B = X.shape[0]
            ip = None
        l = lib().oracle_loss_grad(self.nl, self.dims, self.acts, P, X, Y, ip, B, lam, g.ctypes.data)
        return l, g

    def fd_hvp(self, P, V, X, Y, idx=None, lam: float = 0.0, eps: float = 1e-4):
        """finite_difference_hvp_batch (s_lbfgs.hpp:88-101), fp64."""
        idx = None if idx is None else np.ascontiguousarray(idx, np.int64)
        B = len(idx) if idx is not None else X.shape[0]
        y = np.empty(self.nparams, np.float64)
        lib().oracle_fd_hvp(self.nl, self.dims, self.acts, np.ascontiguousarray(P, np.float64),
                            np.ascontiguousarray(V, np.float64), np.ascontiguousarray(X, np.float64),
                            np.ascontiguousarray(Y, np.float64), idx.ctypes.data if idx is not None else None, B, lam,
                            eps, y)
        return y

    def fd_hvp_f32(self, P, V, X, Y, idx, lam: float = 0.0, eps: float = 1e-4):
        """finite_difference_hvp_batch in the fp32 instantiation (the oracle's fp32 S-LBFGS pairs)."""
        idx = np.ascontiguousarray(idx, np.int64)
        y = np.empty(self.nparams, np.float64)
        lib().oracle_fd_hvp_f32(self.nl, self.dims, self.acts, np.ascontiguousarray(P, np.float64),
                                np.ascontiguousarray(V, np.float64), np.ascontiguousarray(X, np.float64),
                                np.ascontiguousarray(Y, np.float64), idx.ctypes.data, len(idx), X.shape[0], lam, eps,
                                y)
        return y

    def loss_grad_f32(self, P, X, Y):
        g = np.empty(self.nparams, np.float64)
        l = lib().oracle_loss_grad_f32(self.nl, self.dims, self.acts, np.ascontiguousarray(P, np.float64),
                                       np.ascontiguousarray(X, np.float64), np.ascontiguousarray(Y, np.float64),
                                       X.shape[0], g)
        return l, g

    def loss(self, P, X, Y, want_out=False):
        out = np.empty((X.shape[0], self.dims[-1]), np.float64) if want_out else None
        l = lib().oracle_loss(self.nl, self.dims, self.acts, np.ascontiguousarray(P, np.float64),
                              np.ascontiguousarray(X, np.float64), np.ascontiguousarray(Y, np.float64), X.shape[0],
                              out.ctypes.data if want_out else None)
        return (l, out) if want_out else l

    def lbfgs_wolfe(self, P, X, Y, m=10, max_iters=20, tol=0.0, fp32=False):
        P = np.array(P, np.float64, copy=True)
        rec = np.zeros((max_iters, 6), np.float64)
        it, nf, nb, ms = C.c_int(0), C.c_long(0), C.c_long(0), C.c_double(0)
        lib().oracle_lbfgs_wolfe_mlp(self.nl, self.dims, self.acts, P, np.ascontiguousarray(X, np.float64),
                                     np.ascontiguousarray(Y, np.float64), X.shape[0], m, max_iters, tol, int(fp32),
                                     rec, C.byref(it), C.byref(nf), C.byref(nb), C.byref(ms))
        return P, rec[: it.value], dict(iters=it.value, n_fwd=nf.value, n_bwd=nb.value, ms=ms.value)

    def lbfgs_armijo(self, P, X, Y, m=10, max_iters=20, tol=0.0, max_ls=20, c1=1e-4, rho=0.5, fp32=False):
        P = np.array(P, np.float64, copy=True)
        rec = np.zeros((max_iters, 6), np.float64)
        it = C.c_int(0)
        lib().oracle_lbfgs_armijo_mlp(self.nl, self.dims, self.acts, P, np.ascontiguousarray(X, np.float64),
                                      np.ascontiguousarray(Y, np.float64), X.shape[0], m, max_iters, tol, max_ls, c1,
                                      rho, int(fp32), rec, C.byref(it))
        return P, rec[: it.value]

    def gd(self, P, X, Y, lr=0.01, momentum=0.9, max_iters=20, tol=1e-6, fp32=True):
        """CudaGD (gd.cuh:38-106); returns (params, rec [iters x (loss, ||g||)])."""
        P = np.array(P, np.float64, copy=True)
        rec = np.zeros((max_iters, 2), np.float64)
        n = lib().oracle_gd_mlp(self.nl, self.dims, self.acts, P, np.ascontiguousarray(X, np.float64),
                                np.ascontiguousarray(Y, np.float64), X.shape[0], lr, momentum, max_iters, tol,
                                int(fp32), rec)
        return P, rec[:n]

    def sgd(self, P, X, Y, batch=128, lr=0.01, momentum=0.9, decay_rate=1.0, decay_step=0, max_epochs=3, tol=1e-6,
            fp32=True):
        """CudaSGD (sgd.cuh:50-153); returns (params, rec [(1 + epochs) x (loss, ||g||)])."""
        P = np.array(P, np.float64, copy=True)
        rec = np.zeros((max_epochs + 1, 2), np.float64)
        n = lib().oracle_sgd_mlp(self.nl, self.dims, self.acts, P, np.ascontiguousarray(X, np.float64),
                                 np.ascontiguousarray(Y, np.float64), X.shape[0], batch, lr, momentum, decay_rate,
                                 decay_step, max_epochs, tol, int(fp32), rec)
        return P, rec[:n]

    def slbfgs(self, P, X, Y, epochs=2, tol=0.0, M=10, L=10, b=32, bH=16, step=0.02, lam=1e-4, fp32=False,
               want_idx=False, pair_trace=0, pair0=None, pio_rec=None, pio_force=None):
        """Returns (params, rec, idx) or, with pair_trace > 0, (params, rec, idx, pairs): one row per curvature
        pair candidate (epoch, t, y.s, s.s, y.y, accepted, live pairs, 0), as the device's pair trace.
        pair0: an fp64 array of 4 * nparams receiving the first candidate's iterate w_t (after step t), the
        iterate average u, s = u - u_prev and y (diagnostics; lbf_slbfgs_pair0 on the device).
        pio_rec / pio_force: fp64 arrays [cap, 4, nparams], the curvature events' record [w_{t+1} | u | g+ | g-] and
        the teacher forcing of u, g+, g- (PairIO in oracle.hpp; lbf_slbfgs_pair_io on the device)."""
        P = np.array(P, np.float64, copy=True)
        rec = np.zeros((epochs, 6), np.float64)
        it = C.c_int(0)
        N = X.shape[0]
        cap = 0
        idx = None
        if want_idx:
            m = max(1, N // b)
            cap = epochs * (m * b + (m // max(L, 1) + 1) * bH)
            idx = np.full(cap, -1, np.int64)
        pairs = np.zeros((max(int(pair_trace), 1), 8), np.float64)
        npairs = C.c_int(0)
        cap_io = 0
        for a in (pio_rec, pio_force):
            if a is not None:
                assert a.dtype == np.float64 and a.flags.c_contiguous and a.ndim == 3 and a.shape[1:] == (4, P.size)
                cap_io = a.shape[0] if cap_io == 0 else min(cap_io, a.shape[0])
        lib().oracle_slbfgs_mlp(self.nl, self.dims, self.acts, P, np.ascontiguousarray(X, np.float64),
                                np.ascontiguousarray(Y, np.float64), N, epochs, tol, M, L, b, bH, step, lam, int(fp32),
                                rec, C.byref(it), idx.ctypes.data if want_idx else None, cap,
                                pairs.ctypes.data if pair_trace > 0 else None, int(pair_trace), C.byref(npairs),
                                pair0.ctypes.data if pair0 is not None else None, cap_io,
                                pio_rec.ctypes.data if pio_rec is not None else None,
                                pio_force.ctypes.data if pio_force is not None else None)
        if want_idx:
            idx = idx[idx >= 0]
        if pair_trace > 0:
            return P, rec[: it.value], idx, pairs[: npairs.value]
        return P, rec[: it.value], idx


def torch_loss_grad(dims, acts, P, X, Y, threads=None):
    """The same MLP loss (0.5 * SSE / N) and gradient by torch CPU fp64 autograd on BLAS GEMMs: the pin of the C
    restatement's loss_grad (tests/test_oracle.py, 1e-12), used where the restatement's loops are too slow (cfg 5
    at tens of thousands of rows). P: the reference's flat layout, per layer W (Out x In column-major == [In][Out])
    then b."""
    import torch
    if threads:
        torch.set_num_threads(int(threads))
    t = torch.tensor(np.asarray(P, np.float64), dtype=torch.float64, requires_grad=True)
    a = torch.as_tensor(np.asarray(X, np.float64))
    f = {"relu": torch.relu, "tanh": torch.tanh, "sigmoid": torch.sigmoid, "linear": lambda z: z}
    off = 0
    for li, act in enumerate(acts):
        i, o = int(dims[li]), int(dims[li + 1])
        W = t[off:off + i * o].view(i, o)
        b = t[off + i * o: off + i * o + o]
        off += (i + 1) * o
        a = f[act](a @ W + b)
    L = 0.5 * ((a - torch.as_tensor(np.asarray(Y, np.float64))) ** 2).sum() / a.shape[0]
    L.backward()
    return float(L.detach()), t.grad.numpy().copy()


def two_loop(mode: int, S, Y, rho, g):
    S = np.ascontiguousarray(S, np.float64)
    Y = np.ascontiguousarray(Y, np.float64)
    k, n = S.shape if S.ndim == 2 else (0, len(g))
    out = np.empty(len(g), np.float64)
    if k == 0:
        S = np.zeros((1, len(g)))
        Y = np.zeros((1, len(g)))
    lib().oracle_two_loop(mode, len(g), k, S, Y, np.ascontiguousarray(rho if k else [0.0], np.float64),
                          np.ascontiguousarray(g, np.float64), out)
    return out


def lbfgs_testfn(fid: int, x0, m=16, max_iters=4000, tol=1e-12):
    x = np.array(x0, np.float64, copy=True)
    it = C.c_int(0)
    gn = lib().oracle_lbfgs_testfn(fid, len(x), x, m, max_iters, tol, C.byref(it))
    return x, gn, it.value


def sample_indices(N: int, b: int, seed: int = 123, calls: int = 1) -> np.ndarray:
    out = np.empty(calls * b, np.int64)
    lib().oracle_sample_indices(N, b, seed, calls, out)
    return out.reshape(calls, b)


def synth_mnist(N: int, In: int = 784, classes: int = 10, seed: int = 123):
    X = np.empty((N, In), np.float64)
    Y = np.empty((N, classes), np.float64)
    lib().oracle_synth_mnist(N, In, classes, seed, X, Y)
    return X, Y


def ring_trace(cap: int, npush: int):
    out = np.empty(npush * cap, np.int32)
    heads = np.empty(npush, np.int32)
    lib().oracle_ring_trace(cap, npush, out, heads)
    return heads, out.reshape(npush, cap)


def num_threads() -> int:
    return int(lib().oracle_num_threads())


def set_threads(n: int) -> None:
    """OpenMP threads of the oracle's later calls (omp_set_num_threads)."""
    lib().oracle_set_threads(int(n))


# ---- BASELINE config 5 data (test infrastructure; restates lbfgs-ffnn_amd/csrc/synth.hip) ----------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return x ^ (x >> np.uint64(31))


def synth_normal(seed: int, idx: np.ndarray) -> np.ndarray:
    """Normal number idx of stream `seed` (fp64): Box-Muller on splitmix64 uniform pairs."""
    idx = np.asarray(idx, np.uint64)
    j = idx >> np.uint64(1)
    base = np.uint64(seed) << np.uint64(32)
    with np.errstate(over="ignore"):
        a = _splitmix64(base + np.uint64(2) * j)
        b = _splitmix64(base + np.uint64(2) * j + np.uint64(1))
    u1 = ((a >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * 2.0 ** -53
    u2 = (b >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    r, th = np.sqrt(-2.0 * np.log(u1)), 6.283185307179586 * u2
    return np.where((idx & np.uint64(1)) == 1, r * np.sin(th), r * np.cos(th))


def synth_regression(N: int, In: int = 4096, seed_x: int = 123, seed_t: int = 124):
    """X ~ N(0,1) [N][In] fp32, y = tanh(v.x / 64) + 0.01 e [N][1] fp32 (config 5 recipe)."""
    X = synth_normal(seed_x, np.arange(N * In, dtype=np.uint64)).astype(np.float32).reshape(N, In)
    v = synth_normal(seed_t, np.arange(In, dtype=np.uint64))
    e = synth_normal(seed_t, In + np.arange(N, dtype=np.uint64))
    y = np.tanh((X.astype(np.float64) @ v) / 64.0) + 0.01 * e
    return X, y.astype(np.float32).reshape(N, 1)
