/* include/lbfgs_amd.h — C ABI of the MI355X-native L-BFGS / S-LBFGS engine (liblbfgs_amd_abi3.so).
 *
 * Plain pointers and sizes only (no torch / HIP types in the signatures; a stream is passed as void*).
 * Every entry point names the reference interface it replaces (paths relative to SignorB/lbfgs-FFNN).
 * Conventions:
 *   - return value: LBF_OK (0) or an error code; lbf_last_error() gives the message (thread-local).
 *   - d_* arguments are device pointers (hipMalloc'd or torch tensors' data_ptr), h_* are host pointers.
 *   - calls are asynchronous on the context stream unless they return a host value.
 *   - parameter layout is the reference's flat vector: per layer [W (Out x In, column-major) | b (Out)]
 *     (src/network.hpp:45-71, src/cuda/network.cuh:36-59); data X is In x N column-major and Y is
 *     Out x N column-major, i.e. one sample per contiguous row of In (resp. Out) floats.
 *   - one context per GPU, one host thread per context (the reference is single-threaded too,
 *     src/cuda/common.cuh).
 */
#ifndef LBFGS_AMD_H
#define LBFGS_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBF_OK 0
#define LBF_ERR_INVALID 1 /* bad argument (reference: early return in lbfgs.cuh:45-48)          */
#define LBF_ERR_HIP 2     /* HIP runtime error (reference: cuda_check abort, common.cuh:18-23)  */
#define LBF_ERR_COMM 3    /* RCCL error                                                         */
#define LBF_ERR_STATE 4   /* call out of order                                                  */

/* Activation ids == the reference's ActivationType (src/cuda/kernels.cuh:53-58). */
#define LBF_ACT_LINEAR 0
#define LBF_ACT_TANH 1
#define LBF_ACT_RELU 2
#define LBF_ACT_SIGMOID 3

/* Line-search / two-loop policies.
 * WOLFE  = CPU semantics: src/minimizer/lbfgs.hpp:38-139 + full_batch_minimizer.hpp:126-157.
 * ARMIJO = CUDA semantics: src/cuda/lbfgs.cuh:39-261. */
#define LBF_LS_WOLFE 0
#define LBF_LS_ARMIJO 1

/* Parameter-initialisation streams (both libstdc++ mt19937, seed = UnifiedConfig::seed):
 * CPU  = normal_distribution<double> over all params (src/network.hpp:45-71);
 * CUDA = normal_distribution<float> over weights, zero biases (src/cuda/network.cuh:36-59). */
#define LBF_INIT_CPU 0
#define LBF_INIT_CUDA 1

typedef struct lbf_ctx lbf_ctx;
typedef struct lbf_mlp lbf_mlp;
typedef struct lbf_lbfgs lbf_lbfgs;

/* ABI revision of this header. The library's file name and SONAME carry it (liblbfgs_amd_abi3.so), so a
 * binary linked against another revision fails to load instead of handing this library structs of a
 * different size: ABI 1 had no lbf_abi_version() to check, and lbf_solve_info / lbf_slbfgs_params have
 * grown since. Within one revision structs never change. A caller that loads the library by path (dlopen,
 * ctypes) checks lbf_abi_version() == LBF_ABI_VERSION before passing any struct.
 * 2: lbf_solve_info.n_grad_after_loss; lbf_comm_init_local (in-process rank group).
 * 3: lbf_slbfgs_params.dp_mode; the revision in the library name. */
#define LBF_ABI_VERSION 3

const char *lbf_last_error(void);
const char *lbf_version(void);
int lbf_abi_version(void);

/* ---- context: device, stream, workspace, optional communicator --------------------------------
 * Replaces CublasHandle (src/cuda/cublas_handle.cuh:22-39) + the implicit legacy stream. */
int lbf_ctx_create(int device, void *stream /* hipStream_t or NULL = own stream */, lbf_ctx **out);
int lbf_ctx_destroy(lbf_ctx *ctx);
int lbf_ctx_sync(lbf_ctx *ctx);
void *lbf_ctx_stream(lbf_ctx *ctx);

/* ---- data-parallel communicator (RCCL over xGMI). New in this engine: the reference has no
 * collective. One all-reduce of [grad | loss] per loss+grad evaluation. */
int lbf_comm_unique_id(char out[128]);
int lbf_comm_init(lbf_ctx *ctx, int nranks, int rank, const char id[128]);
/* In-process rank group: ctxs[r] becomes rank r of an nranks-rank group whose all-reduce sums every rank's
 * buffer on the device in rank order (HIP events + a host barrier; no RCCL). All contexts must live on one
 * device and each rank must then be driven by its own host thread, calling the same sequence of
 * evaluations as the others (exactly as one process per GPU would). RCCL refuses two ranks on one GPU,
 * so this is how the multi-rank path (shard offsets, n_global scaling, minibatch slices, replicated
 * line-search decisions over summed data) runs on a single GPU; the product route is lbf_comm_init.
 * ABI 2. */
int lbf_comm_init_local(lbf_ctx **ctxs, int nranks);
int lbf_comm_rank(lbf_ctx *ctx, int *rank, int *nranks);
int lbf_allreduce_sum(lbf_ctx *ctx, float *d_buf, size_t count);

/* ---- dense MLP --------------------------------------------------------------------------------
 * Replaces CudaNetwork (src/cuda/network.cuh:21-158) / CudaDenseLayer (src/cuda/layer.cuh). */
int lbf_mlp_create(lbf_ctx *ctx, int nlayers, const int *dims /* nlayers+1 */, const int *acts /* nlayers */,
                   lbf_mlp **out);
int lbf_mlp_destroy(lbf_mlp *net);
long long lbf_mlp_param_count(const lbf_mlp *net);
/* bindParams(seed) (network.cuh:36-59 / network.hpp:45-71): host libstdc++ RNG, upload to d_params. */
int lbf_mlp_init_params(lbf_mlp *net, unsigned seed, int init_mode, float *d_params);
/* Host-only form of the same draws (h_out holds lbf count of params); no device needed. */
int lbf_init_params_host(int nlayers, const int *dims, const int *acts, unsigned seed, int init_mode, float *h_out);
/* forward_only (network.cuh:79-88): d_out is batch x Out row-major (== Out x batch column-major). */
int lbf_mlp_forward(lbf_mlp *net, const float *d_params, const float *d_X, long long batch, float *d_out);
/* compute_loss_and_grad (network.cuh:97-119) == the LossGradFun of minimizer_base.cuh:15-16:
 *   loss = 0.5*||net(X)-Y||^2 * inv_scale + 0.5*l2*||w||^2,  grad = dloss/dw (written to d_grad).
 * inv_scale is 1/batch in the reference; under data parallelism pass 1/global_batch and the
 * context's communicator sums the shards. d_idx (nullable) gathers rows of X/Y (S-LBFGS minibatches,
 * unified_optimization.hpp:361-364). h_loss receives the loss (synchronises). */
int lbf_mlp_loss_grad(lbf_mlp *net, const float *d_params, float *d_grad, const float *d_X, const float *d_Y,
                      const int *d_idx, long long batch, double inv_scale, double l2, double *h_loss);

/* ---- two-loop recursion (src/minimizer/lbfgs.hpp:106-139 / s_lbfgs.hpp:106-136 /
 * lbfgs.cuh:206-261) on an explicit history given in logical order (oldest first):
 * d_S, d_Y are k x n row-major, h_rho[k]. mode: 0 = CPU (returns -Hg), 1 = S-LBFGS (returns +Hg,
 * gamma guarded and clamped), 2 = CUDA (returns -Hg, gamma guarded), 3 = S-LBFGS as the S-LBFGS solver computes
 * it: each pair offered through the solver's pair update (kept when |y.s| > 1e-10, rho = 1 / y.s on the device,
 * h_rho ignored; s_lbfgs.hpp:245-256), then one direction-only step (the coefficients from the pairs' map K;
 * k <= 16, n % 4 == 0). */
/* Exact Hessian-vector product of the batch loss of lbf_mlp_loss_grad (same inv_scale / l2 / d_idx
 * meaning): d_hv = H(params) d_v, computed with Pearlmutter's R-operator on the device (one forward
 * and backward R-pass; no finite differences). With a communicator the shards' products are summed.
 * Replaces, as an option, the finite-difference HVP of s_lbfgs.hpp:88-101. */
int lbf_mlp_hvp(lbf_mlp *net, const float *d_params, const float *d_v, const float *d_X, const float *d_Y,
                const int *d_idx, long long batch, double inv_scale, double l2, float *d_hv);
/* Per-minibatch gradients at one point (extension; the reference evaluates them one step at a time:
 * SLBFGS::stochastic_solve's batch_g(w) of every inner step, s_lbfgs.hpp:218-230, at the epoch's fixed anchor
 * w): rows [t cnt, (t+1) cnt) of d_X / d_Y are minibatch t, t < nmb; its gradient of
 * 0.5 inv_scale ||net - Y||^2 + 0.5 l2 ||w||^2 is written to d_grads + t ld (ld >= param count). One
 * evaluation over nmb cnt rows whose dW GEMMs split K at the minibatch boundaries. cnt % 32 == 0.
 * Single rank only (a communicator's ranks would each hold partial sums). */
int lbf_mlp_batch_grads(lbf_mlp *net, const float *d_params, const float *d_X, const float *d_Y, int nmb,
                        long long cnt, double inv_scale, double l2, float *d_grads, long long ld);
/* Loss only (CudaNetwork::forward_only, network.cuh:79-88, + the MSE of network.cuh:105; the CPU f closure of
 * unified_optimization.hpp:101-108): forward pass and 0.5 * inv_scale * ||out - Y||^2 (summed over ranks with a
 * communicator), bitwise the loss lbf_mlp_loss_grad reports for the same point. */
int lbf_mlp_loss(lbf_mlp *net, const float *d_params, const float *d_X, const float *d_Y, const int *d_idx,
                 long long batch, double inv_scale, double *h_loss);
/* finite_difference_hvp_batch (src/minimizer/s_lbfgs.hpp:88-101): y = (g(w + eps v) - g(w - eps v)) / (2 eps)
 * of the batch loss (inv_scale, + l2 w), computed exactly as the S-LBFGS solver's curvature pair does
 * (two fused batch evaluations; the fp32 difference times the once-rounded 1/(2 eps)). */
int lbf_mlp_fd_hvp(lbf_mlp *net, const float *d_params, const float *d_v, const float *d_X, const float *d_Y,
                   const int *d_idx, long long batch, double inv_scale, double l2, double eps, float *d_y);
int lbf_two_loop(lbf_ctx *ctx, long long n, int k, const float *d_S, const float *d_Y, const double *h_rho,
                 const float *d_g, float *d_dir, int mode);

/* ---- BLAS-1 with device-side deterministic fp64 reductions (replace kernels.cuh:14-50). */
int lbf_dot(lbf_ctx *ctx, long long n, const float *d_x, const float *d_y, double *h_out);
int lbf_nrm2(lbf_ctx *ctx, long long n, const float *d_x, double *h_out);
int lbf_axpy(lbf_ctx *ctx, long long n, float alpha, const float *d_x, float *d_y);
int lbf_scal(lbf_ctx *ctx, long long n, float alpha, float *d_x);

/* ---- solvers --------------------------------------------------------------------------------- */
typedef struct lbf_lbfgs_params {
  int m;              /* history size (UnifiedConfig::m_param; LBFGS::setHistorySize lbfgs.hpp:29) */
  int max_iters;      /* setMaxIterations                                                         */
  double tol;         /* setTolerance: stop when ||g|| < tol                                      */
  int line_search;    /* LBF_LS_WOLFE | LBF_LS_ARMIJO                                             */
  int max_line_iters; /* 50 (full_batch_minimizer.hpp:116) | 20 (minimizer_base.cuh:63)           */
  double c1, c2, rho; /* 1e-4, 0.9, 0.5 (full_batch_minimizer.hpp:113-115; minimizer_base.cuh:64)  */
} lbf_lbfgs_params;

typedef struct lbf_slbfgs_params {
  int max_epochs;     /* UnifiedConfig::max_iters (outer iterations)                  */
  double tol;         /* full-gradient norm tolerance (s_lbfgs.hpp:208)              */
  int M, L, b, b_H;   /* m_param, L_param, batch_size, b_H_param (unified_optimization.hpp:325) */
  double step;        /* learning_rate                                                */
  double lambda;      /* L2, 1e-4 in the reference (unified_optimization.hpp:334)    */
  unsigned seed;      /* kDefaultSeed = 123 (src/seed.hpp:4; s_lbfgs.hpp:183)        */
  double fd_eps;      /* finite-difference HVP epsilon, 1e-4 (s_lbfgs.hpp:90)        */
  int hvp_exact;      /* 0: the reference's central-difference HVP (s_lbfgs.hpp:88-101); 1: the
                         exact R-operator product (lbf_mlp_hvp), SURVEY §8(f) rank 4          */
  /* ABI 2, diagnostics (NULL / 0: off): one row of LBF_PAIR_TRACE_COLS doubles per curvature-pair
   * candidate (s_lbfgs.hpp:245-256): epoch, inner step t, y.s, s.s, y.y, accepted (|y.s| > 1e-10), live
   * pairs after it, 0. Reading each row back synchronises the stream: not for timed runs. */
  double *pair_trace;
  int pair_trace_cap;
  /* ABI 3, data parallelism (a communicator on the context): LBF_SLBFGS_DP_REPLICATED (default) runs the
   * whole minibatch chain on every rank with no collective (identical inputs, identical bits) and shards
   * only the full-batch gradient at each epoch's anchor (s_lbfgs.hpp:206, 274-284), one all-reduce per
   * epoch; LBF_SLBFGS_DP_SLICED evaluates this rank's 1/p slice of every minibatch and Hessian batch, one
   * all-reduce per inner step. Ignored without a communicator. */
  int dp_mode;
} lbf_slbfgs_params;
#define LBF_PAIR_TRACE_COLS 8
#define LBF_SLBFGS_DP_REPLICATED 0
#define LBF_SLBFGS_DP_SLICED 1

/* Gradient descent with momentum == cuda_mlp::CudaGD (src/cuda/gd.cuh:38-106; setters :22-25). */
typedef struct lbf_gd_params {
  double lr;          /* setLearningRate, 0.01                                               */
  double momentum;    /* setMomentum, 0.9 (0: plain x -= lr g)                               */
  int max_iters;      /* setMaxIterations, 200 (minimizer_base.cuh:62)                       */
  double tol;         /* setTolerance: stop when ||g|| < tol, 1e-6 (minimizer_base.cuh:63)   */
} lbf_gd_params;

/* Minibatch SGD with momentum and step decay == cuda_mlp::CudaSGD (src/cuda/sgd.cuh:50-153).
 * Contiguous, unshuffled batches as in the reference; single rank. */
typedef struct lbf_sgd_params {
  double lr, momentum; /* 0.01, 0.9                                                         */
  int batch;           /* setBatchSize                                                      */
  double decay_rate;   /* setLearningRateDecay(rate, step): lr *= rate every step epochs (1.0) */
  int decay_step;      /* 0: no decay                                                       */
  int max_epochs;      /* setMaxIterations (epochs), 200                                    */
  double tol;          /* relative epoch-loss improvement stop when > 0, 1e-6               */
} lbf_sgd_params;

/* Per-iteration history == IterationRecorder (src/iteration_recorder.hpp:13-146) plus extras.
 * Host arrays of capacity cap; any pointer may be NULL. */
typedef struct lbf_record {
  double *loss, *grad_norm, *time_ms, *alpha;
  int *ls_trials, *accepted;
  int cap, size;
} lbf_record;

typedef struct lbf_solve_info {
  int iterations;
  long long n_evals;  /* fused loss+grad evaluations executed by this solve */
  double final_loss, final_grad_norm;
  long long n_rows;   /* batch rows those evaluations covered on this rank (0 for callback objectives) */
  long long n_loss_only; /* line-search trials evaluated forward + loss only (rejected by Armijo) */
  /* ABI 2: backward passes run on the forward state of a loss-only trial (it passed Armijo). Each is
   * counted in n_evals too, so forward passes = n_evals - n_grad_after_loss + n_loss_only and
   * backward passes = n_evals. */
  long long n_grad_after_loss;
} lbf_solve_info;

void lbf_lbfgs_default_params(lbf_lbfgs_params *p, int line_search);
void lbf_slbfgs_default_params(lbf_slbfgs_params *p);

/* Full-batch L-BFGS (CudaLBFGS::solve lbfgs.cuh:39-194 / LBFGS::solve lbfgs.hpp:38-100): params are
 * updated in place. n_local rows of X/Y live on this rank; n_global = sum over ranks (the loss and
 * gradient are means over n_global, matching the single-process reference). */
int lbf_lbfgs_solve(lbf_mlp *net, const lbf_lbfgs_params *prm, float *d_params, const float *d_X,
                    const float *d_Y, long long n_local, long long n_global, lbf_record *rec,
                    lbf_solve_info *info);

/* Stateful form for benchmarking: begin evaluates the start point; iterate runs up to iters more
 * iterations (returns early on convergence); end releases the history. */
int lbf_lbfgs_begin(lbf_mlp *net, const lbf_lbfgs_params *prm, float *d_params, const float *d_X,
                    const float *d_Y, long long n_local, long long n_global, lbf_lbfgs **out);
int lbf_lbfgs_iterate(lbf_lbfgs *s, int iters, lbf_record *rec, lbf_solve_info *info);
int lbf_lbfgs_end(lbf_lbfgs *s);

/* L-BFGS on an arbitrary objective given as a callback with the reference's LossGradFun contract
 * (src/cuda/minimizer_base.cuh:15-16: loss returned, gradient written to device memory), i.e. the
 * CudaMinimizerBase::solve(n, params, ..., loss_grad) entry point (minimizer_base.cuh:54-59). The
 * history, two-loop and line-search state stay on the device; the callback is invoked once per trial. */
typedef double (*lbf_loss_grad_fn)(void *user, const float *d_params, float *d_grad);
int lbf_lbfgs_solve_fn(lbf_ctx *ctx, const lbf_lbfgs_params *prm, long long n, float *d_params,
                       lbf_loss_grad_fn fn, void *user, lbf_record *rec, lbf_solve_info *info);

/* S-LBFGS (SLBFGS::stochastic_solve s_lbfgs.hpp:165-290 via UnifiedSLBFGS_CPU,
 * unified_optimization.hpp:306-408). X/Y hold all N rows on every rank; minibatches are sampled on
 * the host with the reference's libstdc++ stream and sliced across ranks. */
/* CudaGD::solve / CudaSGD::solve (the reference's CudaMinimizerBase::solve, minimizer_base.cuh:54-59) on
 * the MLP. GD: full batch over the n_local rows of this rank (n_global = sum over ranks, as for
 * lbf_lbfgs_solve). rec: one record per iteration (GD) / the initial full-batch record then one per
 * epoch (SGD, only when rec is non-NULL, like the reference's recorder_ branch). */
void lbf_gd_default_params(lbf_gd_params *p);
void lbf_sgd_default_params(lbf_sgd_params *p);
int lbf_gd_solve(lbf_mlp *net, const lbf_gd_params *prm, float *d_params, const float *d_X, const float *d_Y,
                 long long n_local, long long n_global, lbf_record *rec, lbf_solve_info *info);
int lbf_sgd_solve(lbf_mlp *net, const lbf_sgd_params *prm, float *d_params, const float *d_X, const float *d_Y,
                  long long N, lbf_record *rec, lbf_solve_info *info);

int lbf_slbfgs_solve(lbf_mlp *net, const lbf_slbfgs_params *prm, float *d_params, const float *d_X,
                     const float *d_Y, long long N, lbf_record *rec, lbf_solve_info *info);
/* Stateful S-LBFGS (benchmarking, and callers that check progress between epochs): begin copies nothing
 * yet; iterate runs up to `epochs` more epochs (returns early on convergence) with d_params updated after
 * each call; end releases the solver. One begin + iterate(max_epochs) is lbf_slbfgs_solve. */
typedef struct lbf_slbfgs lbf_slbfgs;
int lbf_slbfgs_begin(lbf_mlp *net, const lbf_slbfgs_params *prm, float *d_params, const float *d_X,
                     const float *d_Y, long long N, lbf_slbfgs **out);
int lbf_slbfgs_iterate(lbf_slbfgs *s, int epochs, lbf_record *rec, lbf_solve_info *info);
int lbf_slbfgs_end(lbf_slbfgs *s);
/* Diagnostics (pair_trace on): the first traced curvature-pair candidate's iterate w_t after inner step t,
 * the iterate average u, s = u - u_prev and the y stored for it (s_lbfgs.hpp:236-256), n floats each into
 * device buffers (any may be NULL). LBF_ERR_INVALID until a candidate has been traced. */
int lbf_slbfgs_pair0(lbf_slbfgs *s, float *d_wt, float *d_u, float *d_s, float *d_y);
/* Diagnostics, teacher forcing of the curvature pairs (set before the first iterate; a new function, so no struct
 * of ABI 3 changes). A curvature event is every inner step t > 0 with t % L == 0 (s_lbfgs.hpp:236-261), the
 * first, which only pushes u, included; with ld = (n + 3) & ~3, event e (counted over epochs, e < cap):
 *   d_rec   (nullable) receives [w_{t+1} | u | g(u + eps s) | g(u - eps s)] at d_rec + 4 e ld (ld floats each;
 *           the two gradients of the batch loss + lambda w, zero at the first event; with hvp_exact the second
 *           is zero and the first is H(u) s);
 *   d_force (nullable, same layout, e.g. another run's d_rec) replaces u before s = u - u_prev and the two
 *           gradients before y = (g+ - g-) / (2 eps) is stored, so the ring receives the other run's pairs
 *           while the iterates w_t stay this run's own. Two routes forced with one run's record then compare
 *           non-chaotically: the gradients at the same points, and the iterates under the same history. */
int lbf_slbfgs_pair_io(lbf_slbfgs *s, int cap, float *d_rec, const float *d_force);

/* ---- profiling: HIP-event timing of every kernel class on the context stream (benchmark use).
 * Section id = kind*16 + layer; kinds: 0 fwd GEMM, 1 dW GEMM, 2 dX GEMM, 3 loss, 4 split-K reduce,
 * 5 finalize, 6 Gram sweep, 7 coefficients, 8 combine sweep, 9 line-search axpy, 10 all-reduce.
 * (The reference times whole iterations only: lbfgs.cuh:80-87, 176-182.) */
int lbf_prof_enable(lbf_ctx *ctx, int on);
/* Restrict timing to one section id (-1: all). Two events per launch of that section only, so the
 * timed region of a benchmark is not serialised by event packets around every kernel. */
int lbf_prof_select(lbf_ctx *ctx, int section_id);
/* Time only every `every`-th launch of the selected sections (1 = all): live timing inside a timed
 * region at 1/every of the event cost (an event record idles the GPU for ~5 us). */
int lbf_prof_sample(lbf_ctx *ctx, int every);
int lbf_prof_read(lbf_ctx *ctx, int cap, int *ids, double *ms, long long *counts, int *n_out);
/* ABI 2: the work units of the timed launches per section, same order as lbf_prof_read (GEMM sections: the
 * batch rows of every timed launch, so a sampled section's flops are 2 * In * Out * work). */
int lbf_prof_read_work(lbf_ctx *ctx, int cap, int *ids, double *work, int *n_out);

/* ---- device memory, so C/C++ consumers need no HIP headers (the reference's DeviceBuffer,
 * src/cuda/device_buffer.cuh:7-96). kind: 0 host->device, 1 device->host, 2 device->device;
 * lbf_memcpy is ordered on the context stream and returns when the copy is complete. */
int lbf_device_alloc(lbf_ctx *ctx, size_t bytes, void **out);
int lbf_device_free(lbf_ctx *ctx, void *p);
int lbf_memcpy(lbf_ctx *ctx, void *dst, const void *src, size_t bytes, int kind);

/* ---- host helpers (not on the timed path) ------------------------------------------------------
 * Synthetic MNIST-shaped data (SURVEY.md §8(d) recipe), row-major [N][In] / [N][classes]. */
int lbf_synth_mnist(long long N, int In, int classes, unsigned seed, float *h_X, float *h_Y);
/* Partial Fisher-Yates minibatch draws from one mt19937(seed) (s_lbfgs.hpp:141-160). */
int lbf_sample_indices(long long N, int b, unsigned seed, int calls, long long *h_out);
/* IDX datasets (MNIST / Fashion-MNIST files) == the reference's MNISTLoader (tests/mnist/mnist_loader.hpp:
 * 8-100): images (magic 2051) scaled by 1/255 into row-major [N][rows*cols] fp32, labels (magic 2049)
 * one-hot into [N][classes] (labels >= classes stay all-zero); max_* > 0 caps the count. Call with a
 * NULL output first to read the header (count, rows, cols), then with a buffer of that size. */
int lbf_idx_read_images(const char *path, long long max_images, float *h_out, long long *count, int *rows,
                        int *cols);
int lbf_idx_read_labels(const char *path, long long max_labels, int classes, float *h_onehot, long long *count);
/* BASELINE config 5's synthetic regression data, generated on the device (no reference counterpart:
 * the reference reads MNIST files): X ~ N(0,1) [N][In], y = tanh(v.x / 64) + 0.01 e [N][1]; stream
 * defined in lbfgs-ffnn_amd/csrc/synth.hip, restated in oracle/oracle.py. Writes rows [row0, row0+N)
 * of the stream (a data-parallel shard). Synchronises. */
int lbf_synth_regression(lbf_ctx *ctx, long long row0, long long N, int In, unsigned seed_x, unsigned seed_t,
                         float *d_X, float *d_Y);

#ifdef __cplusplus
}
#endif

#endif /* LBFGS_AMD_H */
