// extern "C" surface of liblbfgs_amd_abi3.so (declared in include/lbfgs_amd.h). Every call converts
// internal exceptions into a status code + thread-local message (the reference aborts instead:
// src/cuda/common.cuh:18-23, cublas_handle.cuh:14-19).
#include "../../include/lbfgs_amd.h"
#include "host_rng.hpp"
#include "runtime.hpp"
#include "solvers.hpp"

#include <rccl/rccl.h>

#include <cstring>
#include <memory>
#include <string>

using namespace lbf;

struct lbf_ctx {
  Ctx c;
  DevBuf<double> scal;
  DevBuf<float> gscratch;
};
struct lbf_mlp {
  lbf_ctx *ctx;
  std::unique_ptr<Mlp> net;
};
struct lbf_lbfgs {
  std::unique_ptr<Objective> obj;
  std::unique_ptr<LbfgsSolver> s;
};

namespace {
thread_local std::string g_err;

template <class F> int guard(F &&f) {
  try {
    f();
    return LBF_OK;
  } catch (const Error &e) {
    g_err = e.what();
    return e.code;
  } catch (const std::exception &e) {
    g_err = e.what();
    return LBF_ERR_INVALID;
  } catch (...) {
    g_err = "unknown error";
    return LBF_ERR_INVALID;
  }
}

void check_comm(ncclResult_t r, const char *what) {
  if (r != ncclSuccess) throw Error(LBF_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}
} // namespace

extern "C" {

const char *lbf_last_error(void) { return g_err.c_str(); }
const char *lbf_version(void) { return "lbfgs_amd 0.4 (gfx950, abi 3)"; }
int lbf_abi_version(void) { return LBF_ABI_VERSION; }

int lbf_ctx_create(int device, void *stream, lbf_ctx **out) {
  return guard([&] {
    LBF_REQUIRE(out, "out");
    auto *c = new lbf_ctx();
    c->c.device = device;
    try {
      c->c.set_device();
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->c.cus = cus;
      if (stream) {
        c->c.stream = static_cast<hipStream_t>(stream);
      } else {
        // blocking: ordered with the legacy stream torch uses; the highest priority, so that a solver's
        // critical chain is dispatched ahead of its own off-path work (the S-LBFGS twin, lowest priority)
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest < least)
          LBF_HIP(hipStreamCreateWithPriority(&c->c.stream, hipStreamDefault, greatest));
        else
          LBF_HIP(hipStreamCreateWithFlags(&c->c.stream, hipStreamDefault));
        c->c.own_stream = true;
      }
      c->scal.resize(SC_N);
      LBF_HIP(hipMemset(c->scal.get(), 0, SC_N * sizeof(double)));
    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}

int lbf_ctx_destroy(lbf_ctx *ctx) {
  return guard([&] { delete ctx; });
}

int lbf_ctx_sync(lbf_ctx *ctx) {
  return guard([&] {
    LBF_REQUIRE(ctx, "ctx");
    LBF_HIP(hipStreamSynchronize(ctx->c.stream));
  });
}

void *lbf_ctx_stream(lbf_ctx *ctx) { return ctx ? static_cast<void *>(ctx->c.stream) : nullptr; }

int lbf_comm_unique_id(char out[128]) {
  return guard([&] {
    ncclUniqueId id;
    check_comm(ncclGetUniqueId(&id), "ncclGetUniqueId");
    static_assert(sizeof(id) <= 128, "unique id size");
    std::memset(out, 0, 128);
    std::memcpy(out, &id, sizeof(id));
  });
}

int lbf_comm_init(lbf_ctx *ctx, int nranks, int rank, const char id[128]) {
  return guard([&] {
    LBF_REQUIRE(ctx && nranks >= 1 && rank >= 0 && rank < nranks, "comm args");
    LBF_REQUIRE(id, "unique id");
    ctx->c.set_device();
    ctx->c.comm.reset();
    // a 1-rank communicator is created too: it routes evaluations through the data-parallel path
    // (local reduce -> ncclAllReduce -> tail), the single-GPU test of that path
    ctx->c.comm = make_rccl_comm(nranks, rank, id);
    ctx->c.rank = rank;
    ctx->c.nranks = nranks;
  });
}

int lbf_comm_init_local(lbf_ctx **ctxs, int nranks) {
  return guard([&] {
    LBF_REQUIRE(ctxs && nranks >= 1 && nranks <= kMaxLocalRanks, "comm_init_local: 1..16 contexts");
    for (int r = 0; r < nranks; ++r) {
      LBF_REQUIRE(ctxs[r], "comm_init_local: null context");
      LBF_REQUIRE(ctxs[r]->c.device == ctxs[0]->c.device, "comm_init_local: every context on one device");
      for (int q = 0; q < r; ++q) LBF_REQUIRE(ctxs[q] != ctxs[r], "comm_init_local: a context twice");
    }
    auto group = make_local_group(nranks, ctxs[0]->c.device);
    for (int r = 0; r < nranks; ++r) {
      ctxs[r]->c.comm = std::move(group[size_t(r)]);
      ctxs[r]->c.rank = r;
      ctxs[r]->c.nranks = nranks;
    }
  });
}

int lbf_comm_rank(lbf_ctx *ctx, int *rank, int *nranks) {
  return guard([&] {
    LBF_REQUIRE(ctx, "ctx");
    if (rank) *rank = ctx->c.rank;
    if (nranks) *nranks = ctx->c.nranks;
  });
}

int lbf_allreduce_sum(lbf_ctx *ctx, float *d_buf, size_t count) {
  return guard([&] {
    LBF_REQUIRE(ctx, "ctx");
    ctx->c.set_device();
    ctx->c.allreduce(d_buf, count);
  });
}

int lbf_mlp_create(lbf_ctx *ctx, int nlayers, const int *dims, const int *acts, lbf_mlp **out) {
  return guard([&] {
    LBF_REQUIRE(ctx && dims && acts && out, "null argument");
    ctx->c.set_device();
    auto *m = new lbf_mlp();
    m->ctx = ctx;
    try {
      m->net.reset(new Mlp(&ctx->c, nlayers, dims, acts));
    } catch (...) {
      delete m;
      throw;
    }
    *out = m;
  });
}

int lbf_mlp_destroy(lbf_mlp *net) {
  return guard([&] { delete net; });
}

long long lbf_mlp_param_count(const lbf_mlp *net) { return net ? (long long)net->net->nparams() : -1; }

int lbf_mlp_init_params(lbf_mlp *net, unsigned seed, int init_mode, float *d_params) {
  return guard([&] {
    LBF_REQUIRE(net && d_params, "null argument");
    LBF_REQUIRE(init_mode == LBF_INIT_CPU || init_mode == LBF_INIT_CUDA, "init_mode");
    std::vector<float> h;
    init_params_host(net->net->layers(), seed, init_mode, h);
    net->ctx->c.set_device();
    LBF_HIP(hipMemcpyAsync(d_params, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice,
                           net->ctx->c.stream));
    LBF_HIP(hipStreamSynchronize(net->ctx->c.stream));
  });
}

int lbf_init_params_host(int nlayers, const int *dims, const int *acts, unsigned seed, int init_mode, float *h_out) {
  return guard([&] {
    LBF_REQUIRE(dims && acts && h_out && nlayers >= 1, "bad argument");
    LBF_REQUIRE(init_mode == LBF_INIT_CPU || init_mode == LBF_INIT_CUDA, "init_mode");
    std::vector<Layer> layers;
    size_t off = 0;
    for (int l = 0; l < nlayers; ++l) {
      Layer L;
      L.in = dims[l];
      L.out = dims[l + 1];
      L.act = acts[l];
      L.off = off;
      off += size_t(L.in + 1) * L.out;
      layers.push_back(L);
    }
    std::vector<float> h;
    init_params_host(layers, seed, init_mode, h);
    std::copy(h.begin(), h.end(), h_out);
  });
}

int lbf_mlp_forward(lbf_mlp *net, const float *d_params, const float *d_X, long long batch, float *d_out) {
  return guard([&] {
    LBF_REQUIRE(net && d_params && d_X && d_out && batch >= 0, "bad argument");
    net->ctx->c.set_device();
    const float *o = net->net->forward(d_params, d_X, nullptr, batch);
    const int Out = net->net->layers().back().out;
    LBF_HIP(hipMemcpyAsync(d_out, o, size_t(batch) * Out * sizeof(float), hipMemcpyDeviceToDevice,
                           net->ctx->c.stream));
  });
}

int lbf_mlp_loss_grad(lbf_mlp *net, const float *d_params, float *d_grad, const float *d_X, const float *d_Y,
                      const int *d_idx, long long batch, double inv_scale, double l2, double *h_loss) {
  return guard([&] {
    LBF_REQUIRE(net && d_params && d_grad && d_X && d_Y && batch >= 0, "bad argument");
    lbf_ctx *c = net->ctx;
    c->c.set_device();
    const size_t n = net->net->nparams();
    c->gscratch.ensure(n + 4);
    net->net->loss_grad(d_params, c->gscratch.get(), d_X, d_Y, d_idx, batch, inv_scale, l2, nullptr, c->scal.get());
    LBF_HIP(hipMemcpyAsync(d_grad, c->gscratch.get(), n * sizeof(float), hipMemcpyDeviceToDevice, c->c.stream));
    if (h_loss) {
      double tmp[SC_N];
      LBF_HIP(hipMemcpyAsync(tmp, c->scal.get(), SC_N * sizeof(double), hipMemcpyDeviceToHost, c->c.stream));
      LBF_HIP(hipStreamSynchronize(c->c.stream));
      *h_loss = tmp[SC_LOSS];
    }
  });
}

int lbf_mlp_batch_grads(lbf_mlp *net, const float *d_params, const float *d_X, const float *d_Y, int nmb,
                        long long cnt, double inv_scale, double l2, float *d_grads, long long ld) {
  return guard([&] {
    LBF_REQUIRE(net && d_params && d_X && d_Y && d_grads && nmb > 0 && cnt > 0, "bad argument");
    lbf_ctx *c = net->ctx;
    LBF_REQUIRE(!c->c.dp(), "lbf_mlp_batch_grads: single rank only");
    c->c.set_device();
    net->net->batch_grads(d_params, d_X, d_Y, nmb, cnt, inv_scale, l2, d_grads, ld, false);
    LBF_HIP(hipStreamSynchronize(c->c.stream));
  });
}

int lbf_mlp_loss(lbf_mlp *net, const float *d_params, const float *d_X, const float *d_Y, const int *d_idx,
                 long long batch, double inv_scale, double *h_loss) {
  return guard([&] {
    LBF_REQUIRE(net && d_params && d_X && d_Y && h_loss && batch > 0, "bad argument");
    lbf_ctx *c = net->ctx;
    c->c.set_device();
    net->net->loss_only(d_params, d_X, d_Y, d_idx, batch, inv_scale, c->scal.get());
    double tmp[SC_N];
    LBF_HIP(hipMemcpyAsync(tmp, c->scal.get(), SC_N * sizeof(double), hipMemcpyDeviceToHost, c->c.stream));
    LBF_HIP(hipStreamSynchronize(c->c.stream));
    *h_loss = tmp[SC_LOSS];
  });
}

int lbf_mlp_hvp(lbf_mlp *net, const float *d_params, const float *d_v, const float *d_X, const float *d_Y,
                const int *d_idx, long long batch, double inv_scale, double l2, float *d_hv) {
  return guard([&] {
    LBF_REQUIRE(net && d_params && d_v && d_hv && batch >= 0 && (batch == 0 || (d_X && d_Y)), "bad argument");
    net->ctx->c.set_device();
    net->net->hvp(d_params, d_v, d_X, d_Y, d_idx, batch, inv_scale, l2, d_hv);
    LBF_HIP(hipStreamSynchronize(net->ctx->c.stream));
  });
}

int lbf_mlp_fd_hvp(lbf_mlp *net, const float *d_params, const float *d_v, const float *d_X, const float *d_Y,
                   const int *d_idx, long long batch, double inv_scale, double l2, double eps, float *d_y) {
  return guard([&] {
    LBF_REQUIRE(net && d_params && d_v && d_y && batch >= 0 && (batch == 0 || (d_X && d_Y)) && eps > 0.0,
                "bad argument");
    lbf_ctx *c = net->ctx;
    c->c.set_device();
    const size_t n = net->net->nparams(), ld = (n + 3) / 4 * 4, lg = (n + 2 + 3) / 4 * 4;
    DevBuf<float> w(2 * ld), g(2 * lg);
    fd_hvp_grads(net->net.get(), d_params, d_v, d_X, d_Y, d_idx, batch, inv_scale, l2, eps, w.get(), w.get() + ld,
                 g.get(), g.get() + lg, c->scal.get());
    diff_scale(c->c.stream, (long long)n, g.get(), g.get() + lg, float(1.0 / (2.0 * eps)), d_y);
    LBF_HIP(hipStreamSynchronize(c->c.stream));
  });
}

int lbf_two_loop(lbf_ctx *ctx, long long n, int k, const float *d_S, const float *d_Y, const double *h_rho,
                 const float *d_g, float *d_dir, int mode) {
  return guard([&] {
    LBF_REQUIRE(ctx && d_g && d_dir && n > 0 && k >= 0 && k <= 128, "bad argument");
    LBF_REQUIRE(k == 0 || (d_S && d_Y && h_rho), "history pointers");
    LBF_REQUIRE(mode >= 0 && mode <= 3, "mode");
    ctx->c.set_device();
    hipStream_t s = ctx->c.stream;
    const int policy = mode == 0 ? POL_CPU : (mode == 1 || mode == 3 ? POL_SLBFGS : POL_CUDA);
    const double dsign = mode == 1 || mode == 3 ? 1.0 : -1.0;
    History h(&ctx->c, k, n);
    DevBuf<float> zero{size_t(n)};
    LBF_HIP(hipMemsetAsync(zero.get(), 0, size_t(n) * sizeof(float), s));
    if (mode == 3) { // the S-LBFGS solver's own route (SlbfgsSolver::epoch_steps)
      LBF_REQUIRE(k <= DIR_MAXM && n % 4 == 0 && dir_supported(k, n) &&
                      (reinterpret_cast<uintptr_t>(d_g) & 15u) == 0 && (k == 0 || ((reinterpret_cast<uintptr_t>(d_S) |
                      reinterpret_cast<uintptr_t>(d_Y)) & 15u) == 0),
                  "mode 3: k <= 16, n % 4 == 0, 16-B aligned vectors");
      for (int i = 0; i < k; ++i) { // pair updates: |y.s| > 1e-10, rho = 1 / y.s and the map K on the device
        GramArgs ga;
        ga.policy = policy;
        ga.has_pair = 1;
        ga.sa = d_S + size_t(i) * n;
        ga.sb = zero.get();
        ga.ya = d_Y + size_t(i) * n;
        ga.yb = zero.get();
        h.update(ga, 0, 1, dsign);
      }
      DevBuf<float> v{size_t(n)};
      GramArgs gg; // a direction-only step: dir_cols_combine, x_out = 0 + 1 * (+H g)
      gg.policy = policy;
      gg.has_g = 1;
      gg.ga = d_g;
      gg.g_out = v.get();
      LBF_REQUIRE(h.update_combine(gg, 1, dsign, zero.get(), d_dir, nullptr, 1.0),
                  "mode 3: the direction-only step did not take the coefficient-map route");
      ctx->c.host.ensure(1);
      LBF_HIP(hipMemcpyAsync(ctx->c.host.get(), h.view().scal + SC_KERR, sizeof(double), hipMemcpyDeviceToHost, s));
      LBF_HIP(hipStreamSynchronize(s));
      LBF_REQUIRE(ctx->c.host[0] == 0.0, "mode 3: the coefficient map K is out of step with the ring");
      return;
    }
    for (int i = 0; i < k; ++i) {
      GramArgs ga;
      ga.policy = policy;
      ga.has_pair = 1;
      ga.sa = d_S + size_t(i) * n;
      ga.sb = zero.get();
      ga.ya = d_Y + size_t(i) * n;
      ga.yb = zero.get();
      h.update(ga, -1, 1, dsign); // -1: push unconditionally
    }
    if (k > 0)
      LBF_HIP(hipMemcpyAsync(h.view().rho, h_rho, size_t(k) * sizeof(double), hipMemcpyHostToDevice, s));
    GramArgs gg;
    gg.policy = policy;
    gg.has_g = 1;
    gg.ga = d_g;
    h.update(gg, 2, 1, dsign); // 2: direction without the solver's descent fallback
    h.combine(d_g, d_dir, nullptr, nullptr, nullptr, false, 0.0);
    LBF_HIP(hipStreamSynchronize(s));
  });
}

int lbf_dot(lbf_ctx *ctx, long long n, const float *d_x, const float *d_y, double *h_out) {
  return guard([&] {
    LBF_REQUIRE(ctx && d_x && d_y && h_out && n >= 0, "bad argument");
    ctx->c.set_device();
    hipStream_t s = ctx->c.stream;
    const int nw = dots_partials_wg(n);
    ctx->c.part.ensure(size_t(nw));
    ctx->c.red.ensure(1);
    ctx->c.host.ensure(1);
    dot_partials(s, n, d_x, d_y, ctx->c.part.get());
    reduce_rows(s, ctx->c.part.get(), nw, 1, ctx->c.red.get());
    LBF_HIP(hipMemcpyAsync(ctx->c.host.get(), ctx->c.red.get(), sizeof(double), hipMemcpyDeviceToHost, s));
    LBF_HIP(hipStreamSynchronize(s));
    *h_out = ctx->c.host[0];
  });
}

int lbf_nrm2(lbf_ctx *ctx, long long n, const float *d_x, double *h_out) {
  double d = 0;
  int r = lbf_dot(ctx, n, d_x, d_x, &d);
  if (r == LBF_OK && h_out) *h_out = std::sqrt(d);
  return r;
}

int lbf_axpy(lbf_ctx *ctx, long long n, float alpha, const float *d_x, float *d_y) {
  return guard([&] {
    LBF_REQUIRE(ctx && d_x && d_y && n >= 0, "bad argument");
    ctx->c.set_device();
    axpy(ctx->c.stream, n, alpha, d_x, d_y);
  });
}

int lbf_scal(lbf_ctx *ctx, long long n, float alpha, float *d_x) {
  return guard([&] {
    LBF_REQUIRE(ctx && d_x && n >= 0, "bad argument");
    ctx->c.set_device();
    scal(ctx->c.stream, n, alpha, d_x);
  });
}

void lbf_lbfgs_default_params(lbf_lbfgs_params *p, int line_search) {
  if (!p) return;
  p->line_search = line_search;
  if (line_search == LBF_LS_ARMIJO) { // minimizer_base.cuh:63-64, lbfgs.cuh:118 (m_ = 16)
    p->m = 16;
    p->max_iters = 200;
    p->tol = 1e-6;
    p->max_line_iters = 20;
    p->c1 = 1e-4;
    p->c2 = 0.9;
    p->rho = 0.5;
  } else { // full_batch_minimizer.hpp:107-116, lbfgs.hpp:142 (m = 16)
    p->m = 16;
    p->max_iters = 1000;
    p->tol = 1e-10;
    p->max_line_iters = 50;
    p->c1 = 1e-4;
    p->c2 = 0.9;
    p->rho = 0.5;
  }
}

void lbf_gd_default_params(lbf_gd_params *p) { // gd.cuh:103-104, minimizer_base.cuh:62-63
  if (!p) return;
  p->lr = 0.01;
  p->momentum = 0.9;
  p->max_iters = 200;
  p->tol = 1e-6;
}

void lbf_sgd_default_params(lbf_sgd_params *p) { // sgd.cuh:156-161, minimizer_base.cuh:62-63
  if (!p) return;
  p->lr = 0.01;
  p->momentum = 0.9;
  p->batch = 64;
  p->decay_rate = 1.0;
  p->decay_step = 0;
  p->max_epochs = 200;
  p->tol = 1e-6;
}

int lbf_gd_solve(lbf_mlp *net, const lbf_gd_params *prm, float *d_params, const float *d_X, const float *d_Y,
                 long long n_local, long long n_global, lbf_record *rec, lbf_solve_info *info) {
  return guard([&] {
    LBF_REQUIRE(net && prm, "null argument");
    run_gd(net->net.get(), *prm, d_params, d_X, d_Y, n_local, n_global, rec, info);
  });
}

int lbf_sgd_solve(lbf_mlp *net, const lbf_sgd_params *prm, float *d_params, const float *d_X, const float *d_Y,
                  long long N, lbf_record *rec, lbf_solve_info *info) {
  return guard([&] {
    LBF_REQUIRE(net && prm, "null argument");
    run_sgd(net->net.get(), *prm, d_params, d_X, d_Y, N, rec, info);
  });
}

void lbf_slbfgs_default_params(lbf_slbfgs_params *p) {
  if (!p) return;
  p->max_epochs = 1000; // stochastic_minimizer.hpp:44-47
  p->tol = 1e-4;
  p->M = 10;
  p->L = 10;
  p->b = 128;
  p->b_H = 64;
  p->step = 0.01;
  p->lambda = 1e-4;
  p->seed = 123;
  p->fd_eps = 1e-4;
  p->hvp_exact = 0;
  p->pair_trace = nullptr;
  p->pair_trace_cap = 0;
  p->dp_mode = LBF_SLBFGS_DP_REPLICATED;
}

int lbf_lbfgs_begin(lbf_mlp *net, const lbf_lbfgs_params *prm, float *d_params, const float *d_X,
                    const float *d_Y, long long n_local, long long n_global, lbf_lbfgs **out) {
  return guard([&] {
    LBF_REQUIRE(net && prm && out, "null argument");
    LBF_REQUIRE(prm->m >= 0 && prm->m <= 128, "m in [0, 128]");
    net->ctx->c.set_device();
    // a data-parallel rank with an empty shard (n_local == 0) has no data pointers
    LBF_REQUIRE(d_params && (n_local == 0 || (d_X && d_Y)), "null pointer");
    LBF_REQUIRE(n_local >= 0 && n_global > 0, "batch sizes");
    auto *s = new lbf_lbfgs();
    try {
      s->obj.reset(new MlpObjective(net->net.get(), d_X, d_Y, n_local, n_global));
      s->s.reset(new LbfgsSolver(s->obj.get(), *prm, d_params));
    } catch (...) {
      delete s;
      throw;
    }
    *out = s;
  });
}

int lbf_lbfgs_iterate(lbf_lbfgs *s, int iters, lbf_record *rec, lbf_solve_info *info) {
  return guard([&] {
    LBF_REQUIRE(s && iters >= 0, "bad argument");
    s->s->iterate(iters, rec);
    s->s->info(info);
  });
}

int lbf_lbfgs_end(lbf_lbfgs *s) {
  return guard([&] { delete s; });
}

int lbf_lbfgs_solve(lbf_mlp *net, const lbf_lbfgs_params *prm, float *d_params, const float *d_X,
                    const float *d_Y, long long n_local, long long n_global, lbf_record *rec,
                    lbf_solve_info *info) {
  // CudaMinimizerBase::solve contract (minimizer_base.cuh:54-59): n <= 0 or params == nullptr is a
  // no-op with iterations() == 0 (lbfgs.cuh:45-48).
  if (!net || !d_params || net->net->nparams() == 0) {
    if (info) std::memset(info, 0, sizeof(*info));
    return LBF_OK;
  }
  lbf_lbfgs *s = nullptr;
  int r = lbf_lbfgs_begin(net, prm, d_params, d_X, d_Y, n_local, n_global, &s);
  if (r != LBF_OK) return r;
  r = lbf_lbfgs_iterate(s, prm->max_iters, rec, info);
  lbf_lbfgs_end(s);
  return r;
}

int lbf_lbfgs_solve_fn(lbf_ctx *ctx, const lbf_lbfgs_params *prm, long long n, float *d_params,
                       lbf_loss_grad_fn fn, void *user, lbf_record *rec, lbf_solve_info *info) {
  if (!d_params || n <= 0) { // lbfgs.cuh:45-48
    if (info) std::memset(info, 0, sizeof(*info));
    return LBF_OK;
  }
  return guard([&] {
    LBF_REQUIRE(ctx && prm && fn, "null argument");
    LBF_REQUIRE(prm->m >= 0 && prm->m <= 128, "m in [0, 128]");
    ctx->c.set_device();
    CallbackObjective obj(&ctx->c, n, fn, user);
    LbfgsSolver s(&obj, *prm, d_params);
    s.iterate(prm->max_iters, rec);
    s.info(info);
  });
}

int lbf_device_alloc(lbf_ctx *ctx, size_t bytes, void **out) {
  return guard([&] {
    LBF_REQUIRE(ctx && out, "null argument");
    ctx->c.set_device();
    *out = nullptr;
    if (bytes) LBF_HIP(hipMalloc(out, bytes));
  });
}

int lbf_device_free(lbf_ctx *ctx, void *p) {
  return guard([&] {
    LBF_REQUIRE(ctx, "ctx");
    ctx->c.set_device();
    if (p) LBF_HIP(hipFree(p));
  });
}

int lbf_memcpy(lbf_ctx *ctx, void *dst, const void *src, size_t bytes, int kind) {
  return guard([&] {
    LBF_REQUIRE(ctx && (bytes == 0 || (dst && src)) && kind >= 0 && kind <= 2, "bad argument");
    ctx->c.set_device();
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
    if (bytes) LBF_HIP(hipMemcpyAsync(dst, src, bytes, k, ctx->c.stream));
    LBF_HIP(hipStreamSynchronize(ctx->c.stream));
  });
}

int lbf_slbfgs_solve(lbf_mlp *net, const lbf_slbfgs_params *prm, float *d_params, const float *d_X,
                     const float *d_Y, long long N, lbf_record *rec, lbf_solve_info *info) {
  return guard([&] {
    LBF_REQUIRE(net && prm, "null argument");
    net->ctx->c.set_device();
    SlbfgsSolver s(net->net.get(), *prm, d_params, d_X, d_Y, N);
    s.run(rec);
    s.info(info);
  });
}

struct lbf_slbfgs {
  std::unique_ptr<SlbfgsSolver> s;
};

int lbf_slbfgs_begin(lbf_mlp *net, const lbf_slbfgs_params *prm, float *d_params, const float *d_X,
                     const float *d_Y, long long N, lbf_slbfgs **out) {
  return guard([&] {
    LBF_REQUIRE(net && prm && out, "null argument");
    net->ctx->c.set_device();
    auto *h = new lbf_slbfgs();
    try {
      h->s.reset(new SlbfgsSolver(net->net.get(), *prm, d_params, d_X, d_Y, N));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int lbf_slbfgs_iterate(lbf_slbfgs *s, int epochs, lbf_record *rec, lbf_solve_info *info) {
  return guard([&] {
    LBF_REQUIRE(s && epochs >= 0, "bad argument");
    s->s->iterate(epochs, rec);
    s->s->info(info);
  });
}

int lbf_slbfgs_pair0(lbf_slbfgs *s, float *d_wt, float *d_u, float *d_s, float *d_y) {
  return guard([&] {
    LBF_REQUIRE(s, "null argument");
    LBF_REQUIRE(s->s->pair0(d_wt, d_u, d_s, d_y), "no curvature-pair candidate traced (pair_trace off, or none yet)");
  });
}

int lbf_slbfgs_pair_io(lbf_slbfgs *s, int cap, float *d_rec, const float *d_force) {
  return guard([&] {
    LBF_REQUIRE(s && cap >= 0, "bad argument");
    s->s->pair_io(cap, d_rec, d_force);
  });
}

int lbf_slbfgs_end(lbf_slbfgs *s) {
  return guard([&] { delete s; });
}

int lbf_prof_enable(lbf_ctx *ctx, int on) {
  return guard([&] {
    LBF_REQUIRE(ctx, "ctx");
    ctx->c.prof.resolve();
    ctx->c.prof.on = on != 0;
    if (on) {
      ctx->c.prof.ms.clear();
      ctx->c.prof.cnt.clear();
      ctx->c.prof.work.clear();
    }
  });
}

int lbf_prof_select(lbf_ctx *ctx, int section_id) {
  return guard([&] {
    LBF_REQUIRE(ctx, "ctx");
    ctx->c.prof.only = section_id < 0 ? -1 : section_id;
  });
}

int lbf_prof_sample(lbf_ctx *ctx, int every) {
  return guard([&] {
    LBF_REQUIRE(ctx && every >= 1, "ctx / every >= 1");
    ctx->c.prof.every = every;
    ctx->c.prof.seen = 0;
  });
}

int lbf_prof_read(lbf_ctx *ctx, int cap, int *ids, double *ms, long long *counts, int *n_out) {
  return guard([&] {
    LBF_REQUIRE(ctx && n_out, "null argument");
    ctx->c.set_device();
    ctx->c.prof.resolve();
    int k = 0;
    for (size_t i = 0; i < ctx->c.prof.cnt.size(); ++i) {
      if (ctx->c.prof.cnt[i] == 0) continue;
      if (k < cap) {
        if (ids) ids[k] = int(i);
        if (ms) ms[k] = ctx->c.prof.ms[i];
        if (counts) counts[k] = ctx->c.prof.cnt[i];
      }
      ++k;
    }
    *n_out = k;
  });
}

int lbf_prof_read_work(lbf_ctx *ctx, int cap, int *ids, double *work, int *n_out) {
  return guard([&] {
    LBF_REQUIRE(ctx && n_out, "null argument");
    ctx->c.set_device();
    ctx->c.prof.resolve();
    int k = 0;
    for (size_t i = 0; i < ctx->c.prof.cnt.size(); ++i) {
      if (ctx->c.prof.cnt[i] == 0) continue;
      if (k < cap) {
        if (ids) ids[k] = int(i);
        if (work) work[k] = i < ctx->c.prof.work.size() ? ctx->c.prof.work[i] : 0.0;
      }
      ++k;
    }
    *n_out = k;
  });
}

int lbf_synth_mnist(long long N, int In, int classes, unsigned seed, float *h_X, float *h_Y) {
  return guard([&] {
    LBF_REQUIRE(N >= 0 && In > 0 && classes > 0 && h_X && h_Y, "bad argument");
    synth_mnist_host(N, In, classes, seed, h_X, h_Y);
  });
}

int lbf_synth_regression(lbf_ctx *ctx, long long row0, long long N, int In, unsigned seed_x, unsigned seed_t,
                         float *d_X, float *d_Y) {
  return guard([&] {
    LBF_REQUIRE(ctx && row0 >= 0 && N >= 0 && In > 0 && d_X && d_Y, "bad argument");
    ctx->c.set_device();
    synth_regression(ctx->c.stream, row0, N, In, seed_x, seed_t, d_X, d_Y);
    LBF_HIP(hipStreamSynchronize(ctx->c.stream));
  });
}

int lbf_idx_read_images(const char *path, long long max_images, float *h_out, long long *count, int *rows,
                        int *cols) {
  return guard([&] { idx_read_images(path, max_images, h_out, count, rows, cols); });
}

int lbf_idx_read_labels(const char *path, long long max_labels, int classes, float *h_onehot, long long *count) {
  return guard([&] { idx_read_labels(path, max_labels, classes, h_onehot, count); });
}

int lbf_sample_indices(long long N, int b, unsigned seed, int calls, long long *h_out) {
  return guard([&] {
    LBF_REQUIRE(N >= 0 && b >= 0 && calls >= 0 && h_out, "bad argument");
    std::mt19937 rng(seed);
    MinibatchSampler smp{size_t(N)}; // one permutation for every call, like the solver's
    std::vector<int> v;
    for (int c = 0; c < calls; ++c) {
      v.clear();
      smp.draw(size_t(b), rng, v);
      for (size_t i = 0; i < v.size(); ++i) h_out[size_t(c) * b + i] = (long long)v[i];
    }
  });
}

} // extern "C"
