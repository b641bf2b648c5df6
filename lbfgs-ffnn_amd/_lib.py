"""ctypes binding of ``build/liblbfgs_amd_abi3.so`` (C ABI: ``include/lbfgs_amd.h``).

The shared library is the product: every numeric operation below runs in its HIP kernels. There is
no CPU fallback; a missing or unloadable library raises :class:`LbfError` immediately.
torch is imported first so that the HIP runtime torch loaded (SONAME ``libamdhip64.so.7``) is the
one the library binds to, and torch tensors are used purely as device allocations.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
ABI_VERSION = 3  # include/lbfgs_amd.h LBF_ABI_VERSION (also in the library's file name)
LIB_PATH = os.environ.get("LBF_LIB_PATH") or os.path.join(_HERE, "build", f"liblbfgs_amd_abi{ABI_VERSION}.so")
SLBFGS_DP_REPLICATED, SLBFGS_DP_SLICED = 0, 1
LS_WOLFE, LS_ARMIJO = 0, 1
INIT_CPU, INIT_CUDA = 0, 1
ACTS = {"linear": 0, "tanh": 1, "relu": 2, "sigmoid": 3}


class LbfError(RuntimeError):
    pass


class LbfgsParams(C.Structure):
    _fields_ = [("m", C.c_int), ("max_iters", C.c_int), ("tol", C.c_double), ("line_search", C.c_int),
                ("max_line_iters", C.c_int), ("c1", C.c_double), ("c2", C.c_double), ("rho", C.c_double)]


class SlbfgsParams(C.Structure):
    _fields_ = [("max_epochs", C.c_int), ("tol", C.c_double), ("M", C.c_int), ("L", C.c_int), ("b", C.c_int),
                ("b_H", C.c_int), ("step", C.c_double), ("reg", C.c_double), ("seed", C.c_uint),
                ("fd_eps", C.c_double), ("hvp_exact", C.c_int), ("pair_trace", C.POINTER(C.c_double)),
                ("pair_trace_cap", C.c_int), ("dp_mode", C.c_int)]


class GdParams(C.Structure):
    _fields_ = [("lr", C.c_double), ("momentum", C.c_double), ("max_iters", C.c_int), ("tol", C.c_double)]


class SgdParams(C.Structure):
    _fields_ = [("lr", C.c_double), ("momentum", C.c_double), ("batch", C.c_int), ("decay_rate", C.c_double),
                ("decay_step", C.c_int), ("max_epochs", C.c_int), ("tol", C.c_double)]


class Record(C.Structure):
    _fields_ = [("loss", C.POINTER(C.c_double)), ("grad_norm", C.POINTER(C.c_double)),
                ("time_ms", C.POINTER(C.c_double)), ("alpha", C.POINTER(C.c_double)),
                ("ls_trials", C.POINTER(C.c_int)), ("accepted", C.POINTER(C.c_int)), ("cap", C.c_int),
                ("size", C.c_int)]


class SolveInfo(C.Structure):
    _fields_ = [("iterations", C.c_int), ("n_evals", C.c_longlong), ("final_loss", C.c_double),
                ("final_grad_norm", C.c_double), ("n_rows", C.c_longlong), ("n_loss_only", C.c_longlong),
                ("n_grad_after_loss", C.c_longlong)]


_lib = None
_vp, _ip, _dp, _fp = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_float)


def lib():
    """Load the HIP library (raises LbfError if it is missing: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LbfError(f"{os.path.basename(LIB_PATH)} not built ({LIB_PATH}); run `make -C lbfgs-ffnn_amd` or "
                       "__graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    sig = {
        "lbf_last_error": (C.c_char_p, []),
        "lbf_version": (C.c_char_p, []),
        "lbf_abi_version": (C.c_int, []),
        "lbf_ctx_create": (C.c_int, [C.c_int, _vp, C.POINTER(_vp)]),
        "lbf_ctx_destroy": (C.c_int, [_vp]),
        "lbf_ctx_sync": (C.c_int, [_vp]),
        "lbf_ctx_stream": (_vp, [_vp]),
        "lbf_comm_unique_id": (C.c_int, [C.c_char_p]),
        "lbf_comm_init": (C.c_int, [_vp, C.c_int, C.c_int, C.c_char_p]),
        "lbf_comm_init_local": (C.c_int, [C.POINTER(_vp), C.c_int]),
        "lbf_comm_rank": (C.c_int, [_vp, _ip, _ip]),
        "lbf_allreduce_sum": (C.c_int, [_vp, _vp, C.c_size_t]),
        "lbf_mlp_create": (C.c_int, [_vp, C.c_int, _ip, _ip, C.POINTER(_vp)]),
        "lbf_mlp_destroy": (C.c_int, [_vp]),
        "lbf_mlp_param_count": (C.c_longlong, [_vp]),
        "lbf_mlp_init_params": (C.c_int, [_vp, C.c_uint, C.c_int, _vp]),
        "lbf_init_params_host": (C.c_int, [C.c_int, _ip, _ip, C.c_uint, C.c_int, _vp]),
        "lbf_mlp_forward": (C.c_int, [_vp, _vp, _vp, C.c_longlong, _vp]),
        "lbf_mlp_loss_grad": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, C.c_longlong, C.c_double, C.c_double, _dp]),
        "lbf_mlp_batch_grads": (C.c_int, [_vp, _vp, _vp, _vp, C.c_int, C.c_longlong, C.c_double, C.c_double, _vp,
                                          C.c_longlong]),
        "lbf_two_loop": (C.c_int, [_vp, C.c_longlong, C.c_int, _vp, _vp, _dp, _vp, _vp, C.c_int]),
        "lbf_dot": (C.c_int, [_vp, C.c_longlong, _vp, _vp, _dp]),
        "lbf_nrm2": (C.c_int, [_vp, C.c_longlong, _vp, _dp]),
        "lbf_axpy": (C.c_int, [_vp, C.c_longlong, C.c_float, _vp, _vp]),
        "lbf_scal": (C.c_int, [_vp, C.c_longlong, C.c_float, _vp]),
        "lbf_lbfgs_default_params": (None, [C.POINTER(LbfgsParams), C.c_int]),
        "lbf_slbfgs_default_params": (None, [C.POINTER(SlbfgsParams)]),
        "lbf_lbfgs_solve": (C.c_int, [_vp, C.POINTER(LbfgsParams), _vp, _vp, _vp, C.c_longlong, C.c_longlong,
                                      C.POINTER(Record), C.POINTER(SolveInfo)]),
        "lbf_lbfgs_begin": (C.c_int, [_vp, C.POINTER(LbfgsParams), _vp, _vp, _vp, C.c_longlong, C.c_longlong,
                                      C.POINTER(_vp)]),
        "lbf_lbfgs_iterate": (C.c_int, [_vp, C.c_int, C.POINTER(Record), C.POINTER(SolveInfo)]),
        "lbf_lbfgs_end": (C.c_int, [_vp]),
        "lbf_lbfgs_solve_fn": (C.c_int, [_vp, C.POINTER(LbfgsParams), C.c_longlong, _vp, _vp, _vp,
                                         C.POINTER(Record), C.POINTER(SolveInfo)]),
        "lbf_device_alloc": (C.c_int, [_vp, C.c_size_t, C.POINTER(_vp)]),
        "lbf_device_free": (C.c_int, [_vp, _vp]),
        "lbf_memcpy": (C.c_int, [_vp, _vp, _vp, C.c_size_t, C.c_int]),
        "lbf_slbfgs_solve": (C.c_int, [_vp, C.POINTER(SlbfgsParams), _vp, _vp, _vp, C.c_longlong, C.POINTER(Record),
                                       C.POINTER(SolveInfo)]),
        "lbf_slbfgs_begin": (C.c_int, [_vp, C.POINTER(SlbfgsParams), _vp, _vp, _vp, C.c_longlong, C.POINTER(_vp)]),
        "lbf_slbfgs_iterate": (C.c_int, [_vp, C.c_int, C.POINTER(Record), C.POINTER(SolveInfo)]),
        "lbf_slbfgs_end": (C.c_int, [_vp]),
        "lbf_slbfgs_pair0": (C.c_int, [_vp, _vp, _vp, _vp, _vp]),
        "lbf_slbfgs_pair_io": (C.c_int, [_vp, C.c_int, _vp, _vp]),
        "lbf_prof_enable": (C.c_int, [_vp, C.c_int]),
        "lbf_prof_select": (C.c_int, [_vp, C.c_int]),
        "lbf_prof_sample": (C.c_int, [_vp, C.c_int]),
        "lbf_prof_read": (C.c_int, [_vp, C.c_int, _ip, _dp, C.POINTER(C.c_longlong), _ip]),
        "lbf_prof_read_work": (C.c_int, [_vp, C.c_int, _ip, _dp, _ip]),
        "lbf_synth_mnist": (C.c_int, [C.c_longlong, C.c_int, C.c_int, C.c_uint, _vp, _vp]),
        "lbf_sample_indices": (C.c_int, [C.c_longlong, C.c_int, C.c_uint, C.c_int, _vp]),
        "lbf_idx_read_images": (C.c_int, [C.c_char_p, C.c_longlong, _vp, C.POINTER(C.c_longlong), _ip, _ip]),
        "lbf_idx_read_labels": (C.c_int, [C.c_char_p, C.c_longlong, C.c_int, _vp, C.POINTER(C.c_longlong)]),
        "lbf_mlp_hvp": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, C.c_longlong, C.c_double, C.c_double, _vp]),
        "lbf_mlp_loss": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_longlong, C.c_double, _dp]),
        "lbf_mlp_fd_hvp": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, C.c_longlong, C.c_double, C.c_double,
                                     C.c_double, _vp]),
        "lbf_gd_default_params": (None, [C.POINTER(GdParams)]),
        "lbf_sgd_default_params": (None, [C.POINTER(SgdParams)]),
        "lbf_gd_solve": (C.c_int, [_vp, C.POINTER(GdParams), _vp, _vp, _vp, C.c_longlong, C.c_longlong,
                                   C.POINTER(Record), C.POINTER(SolveInfo)]),
        "lbf_sgd_solve": (C.c_int, [_vp, C.POINTER(SgdParams), _vp, _vp, _vp, C.c_longlong, C.POINTER(Record),
                                    C.POINTER(SolveInfo)]),
        "lbf_synth_regression": (C.c_int, [_vp, C.c_longlong, C.c_longlong, C.c_int, C.c_uint, C.c_uint, _vp, _vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.lbf_abi_version() != ABI_VERSION:
        raise LbfError(f"{LIB_PATH} implements ABI {L.lbf_abi_version()}, this binding needs {ABI_VERSION}: rebuild it")
    _lib = L
    return L


EXPORTS = ("lbf_last_error lbf_version lbf_abi_version lbf_ctx_create lbf_ctx_destroy lbf_ctx_sync lbf_ctx_stream "
           "lbf_comm_unique_id lbf_comm_init lbf_comm_init_local lbf_comm_rank lbf_allreduce_sum lbf_mlp_create lbf_mlp_destroy "
           "lbf_mlp_param_count lbf_mlp_init_params lbf_init_params_host lbf_mlp_forward lbf_mlp_loss_grad lbf_mlp_batch_grads lbf_two_loop lbf_dot "
           "lbf_nrm2 lbf_axpy lbf_scal lbf_lbfgs_default_params lbf_slbfgs_default_params lbf_lbfgs_solve "
           "lbf_lbfgs_begin lbf_lbfgs_iterate lbf_lbfgs_end lbf_lbfgs_solve_fn lbf_device_alloc lbf_device_free lbf_memcpy lbf_slbfgs_solve lbf_slbfgs_begin lbf_slbfgs_iterate lbf_slbfgs_end lbf_slbfgs_pair0 lbf_slbfgs_pair_io lbf_prof_enable lbf_prof_select lbf_prof_sample lbf_prof_read lbf_prof_read_work lbf_synth_mnist "
           "lbf_sample_indices lbf_synth_regression lbf_gd_default_params lbf_sgd_default_params lbf_gd_solve "
           "lbf_sgd_solve lbf_idx_read_images lbf_idx_read_labels lbf_mlp_hvp lbf_mlp_fd_hvp lbf_mlp_loss").split()


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().lbf_last_error().decode(errors="replace")
        raise LbfError(f"{what} failed (status {rc}): {msg}")


def ptr(t: Optional[torch.Tensor], dtype: torch.dtype = torch.float32, numel: Optional[int] = None):
    """Device pointer of a contiguous tensor of `dtype` (and exactly `numel` elements when given): the
    kernels read raw memory, so an int64 index list or a float64 matrix would be silently misread."""
    if t is None:
        return None
    if not t.is_cuda:
        raise LbfError("expected a device (cuda/hip) tensor")
    if not t.is_contiguous():
        raise LbfError("expected a contiguous tensor")
    if t.dtype != dtype:
        raise LbfError(f"expected a {dtype} tensor, got {t.dtype}")
    if numel is not None and t.numel() != numel:
        raise LbfError(f"expected {numel} elements, got {t.numel()}")
    return C.c_void_p(t.data_ptr())
