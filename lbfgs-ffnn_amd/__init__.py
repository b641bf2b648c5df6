"""lbfgs-ffnn_amd — MI355X-native L-BFGS / S-LBFGS engine for dense FFNNs.

Compute lives in ``build/liblbfgs_amd_abi3.so`` (hand-written HIP kernels for gfx950 behind the C ABI
``include/lbfgs_amd.h``). This package is the host-side mirror of the reference's unified API.
The directory name contains a hyphen, so load it with :func:`load` from the repo root helpers
(``tests/conftest.py``, ``bench.py``, ``__graft_entry__.py``) under the module name ``lbfgs_ffnn_amd``.
"""
from ._lib import LIB_PATH, LbfError, lib  # noqa: F401
from .engine import (Context, History, LbfgsRun, Mlp, SlbfgsRun, gd_solve, grad_flops_per_sample, init_params_host,  # noqa: F401
                     lbfgs_solve, load_idx_images, load_idx_labels, sample_indices, sgd_solve, slbfgs_solve,
                     synth_mnist, synth_regression)
from .unified import (IterationRecorder, UnifiedConfig, UnifiedDataset, UnifiedGD, UnifiedLauncher,  # noqa: F401
                      UnifiedLBFGS, UnifiedSGD, UnifiedSLBFGS, write_history_csv)
