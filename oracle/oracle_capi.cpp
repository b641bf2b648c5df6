// oracle/oracle_capi.cpp — TEST INFRASTRUCTURE ONLY. extern "C" surface over oracle.hpp for ctypes
// (tests/, __graft_entry__.smoke(), bench.py cpu_baseline). See oracle.hpp for the reference citations.
#include "oracle.hpp"

#include <chrono>
#include <cstdio>

using namespace oracle;

namespace {

template <class T> std::vector<T> to_vec(const double *p, size_t n) {
  std::vector<T> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = T(p[i]);
  return v;
}
template <class T> void from_vec(const std::vector<T> &v, double *p) {
  for (size_t i = 0; i < v.size(); ++i) p[i] = double(v[i]);
}

void write_rec(const std::vector<IterRecord> &rec, double *out, int cap) {
  if (!out) return;
  for (int i = 0; i < int(rec.size()) && i < cap; ++i) {
    out[i * 6 + 0] = rec[i].loss;
    out[i * 6 + 1] = rec[i].gnorm;
    out[i * 6 + 2] = rec[i].alpha;
    out[i * 6 + 3] = rec[i].accepted;
    out[i * 6 + 4] = rec[i].ls_trials;
    out[i * 6 + 5] = rec[i].time_ms;
  }
}

// Analytic test problems restated from the reference's known-answer tests (tests/main.cpp).
// id 0: Rosenbrock (main.cpp:71-156), 1: Ackley (:158-258), 2: Rastrigin (:15-69).
double tf_f(int id, const std::vector<double> &v) {
  const int n = int(v.size());
  if (id == 0) {
    double val = 0;
    for (int i = 0; i < n - 1; ++i) {
      double t1 = v[i + 1] - v[i] * v[i], t2 = 1.0 - v[i];
      val += 100.0 * t1 * t1 + t2 * t2;
    }
    return val;
  }
  if (id == 1) {
    double s1 = 0, s2 = 0;
    for (int i = 0; i < n; ++i) {
      s1 += v[i] * v[i];
      s2 += std::cos(2.0 * M_PI * v[i]);
    }
    return -20.0 * std::exp(-0.2 * std::sqrt(s1 / n)) - std::exp(s2 / n) + 20.0 + std::exp(1.0);
  }
  double val = 0, A = 10.0;
  for (int i = 0; i < n; ++i) val += v[i] * v[i] - A * std::cos(2.0 * M_PI * v[i]);
  return A * n + val;
}
std::vector<double> tf_g(int id, const std::vector<double> &v) {
  const int n = int(v.size());
  std::vector<double> g(n, 0.0);
  if (id == 0) {
    if (n > 1) g[0] = -2.0 * (1.0 - v[0]) - 400.0 * v[0] * (v[1] - v[0] * v[0]);
    else g[0] = -2.0 * (1.0 - v[0]);
    for (int i = 1; i < n - 1; ++i)
      g[i] = -2.0 * (1.0 - v[i]) - 400.0 * v[i] * (v[i + 1] - v[i] * v[i]) + 200.0 * (v[i] - v[i - 1] * v[i - 1]);
    if (n > 1) g[n - 1] = 200.0 * (v[n - 1] - v[n - 2] * v[n - 2]);
    return g;
  }
  if (id == 1) {
    double s1 = 0, s2 = 0;
    for (int i = 0; i < n; ++i) {
      s1 += v[i] * v[i];
      s2 += std::cos(2.0 * M_PI * v[i]);
    }
    double ec = std::exp(s2 / n), es = std::exp(-0.2 * std::sqrt(s1 / n));
    for (int i = 0; i < n; ++i) {
      double gs = v[i] / (n * std::sqrt(s1 / n));
      g[i] = 4.0 * es * gs + (2.0 * M_PI / n) * ec * std::sin(2.0 * M_PI * v[i]);
    }
    return g;
  }
  for (int i = 0; i < n; ++i) g[i] = 2.0 * v[i] + 2.0 * M_PI * 10.0 * std::sin(2.0 * M_PI * v[i]);
  return g;
}

template <class T>
int run_wolfe_mlp(const Net &net, double *params, const double *X, const double *Y, int64_t N, int m, int max_iters,
                  double tol, double *rec_out, int *iters, long *nf, long *nb, double *elapsed_ms) {
  std::vector<T> Xt = to_vec<T>(X, size_t(N) * net.dims[0]);
  std::vector<T> Yt = to_vec<T>(Y, size_t(N) * net.dims.back());
  MLPObjective<T> obj{&net, Xt.data(), Yt.data(), N, {}, 0, 0};
  auto f = [&](const Vec<T> &w) { return obj.f(w); };
  auto g = [&](const Vec<T> &w) { return obj.grad(w); };
  LbfgsParams<T> prm;
  prm.m = m;
  prm.max_iters = max_iters;
  prm.tol = tol;
  std::vector<IterRecord> rec;
  auto t0 = std::chrono::steady_clock::now();
  Vec<T> x = lbfgs_wolfe<T>(to_vec<T>(params, net.nparams), f, g, prm, &rec, iters);
  auto t1 = std::chrono::steady_clock::now();
  if (elapsed_ms) *elapsed_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  from_vec(x, params);
  write_rec(rec, rec_out, max_iters);
  if (nf) *nf = obj.n_fwd;
  if (nb) *nb = obj.n_bwd;
  return 0;
}

template <class T>
int run_armijo_mlp(const Net &net, double *params, const double *X, const double *Y, int64_t N, int m, int max_iters,
                   double tol, int max_ls, double c1, double rho, double *rec_out, int *iters) {
  std::vector<T> Xt = to_vec<T>(X, size_t(N) * net.dims[0]);
  std::vector<T> Yt = to_vec<T>(Y, size_t(N) * net.dims.back());
  MLPObjective<T> obj{&net, Xt.data(), Yt.data(), N, {}, 0, 0};
  auto lg = [&](const Vec<T> &w, Vec<T> &g) { return obj.loss_grad_batch(w, nullptr, N, 0.0, g.data()); };
  ArmijoParams<T> prm;
  prm.m = m;
  prm.max_iters = max_iters;
  prm.tol = tol;
  prm.max_line_iters = max_ls;
  prm.c1 = c1;
  prm.rho = rho;
  std::vector<IterRecord> rec;
  Vec<T> x = lbfgs_armijo<T>(to_vec<T>(params, net.nparams), lg, prm, &rec, iters);
  from_vec(x, params);
  write_rec(rec, rec_out, max_iters);
  return 0;
}

template <class T>
int run_slbfgs_mlp(const Net &net, double *params, const double *X, const double *Y, int64_t N, int epochs,
                   double tol, int M, int L, int b, int bH, double step, double lambda, double *rec_out, int *iters,
                   int64_t *idx_out, int64_t idx_cap, double *pair_out, int pair_cap, int *npairs,
                   double *pair0_us, const PairIO *pio) {
  std::vector<T> Xt = to_vec<T>(X, size_t(N) * net.dims[0]);
  std::vector<T> Yt = to_vec<T>(Y, size_t(N) * net.dims.back());
  MLPObjective<T> obj{&net, Xt.data(), Yt.data(), N, {}, 0, 0};
  // batch_g / batch_f of UnifiedSLBFGS_CPU (unified_optimization.hpp:343-400).
  auto bg = [&](const Vec<T> &w, const std::vector<size_t> &ind, Vec<T> &g) {
    if (int64_t(ind.size()) == N) {
      obj.loss_grad_batch(w, nullptr, N, lambda, g.data());
    } else {
      std::vector<int64_t> ii(ind.begin(), ind.end());
      obj.loss_grad_batch(w, ii.data(), int64_t(ii.size()), lambda, g.data());
    }
  };
  auto bf = [&](const Vec<T> &w, const std::vector<size_t> &ind) {
    std::vector<int64_t> ii(ind.begin(), ind.end());
    forward<T>(net, w.data(), obj.X, ii.data(), int64_t(ii.size()), obj.ws);
    double l = half_sse<T>(net, obj.Y, ii.data(), int64_t(ii.size()), obj.ws, false);
    l /= double(ii.size());
    l += 0.5 * lambda * double(dot(w, w));
    return T(l);
  };
  SlbfgsParams prm;
  prm.max_iters = epochs;
  prm.tol = tol;
  prm.M = M;
  prm.L = L;
  prm.b = b;
  prm.b_H = bH;
  prm.step = step;
  prm.N = N;
  prm.m = int(N / b) > 0 ? int(N / b) : 1; // unified_optimization.hpp:326-327
  std::vector<IterRecord> rec;
  std::vector<std::vector<size_t>> sampled;
  std::vector<std::array<double, 8>> pairs;
  std::vector<double> us;
  Vec<T> w = slbfgs<T>(to_vec<T>(params, net.nparams), bg, bf, prm, &rec, iters, idx_out ? &sampled : nullptr,
                       pair_out ? &pairs : nullptr, pair0_us ? &us : nullptr, pio);
  if (pair0_us && !us.empty()) std::copy(us.begin(), us.end(), pair0_us);
  if (pair_out) {
    int k = 0;
    for (auto &r : pairs)
      if (k < pair_cap) {
        for (int j = 0; j < 8; ++j) pair_out[size_t(k) * 8 + j] = r[size_t(j)];
        ++k;
      }
    if (npairs) *npairs = k;
  }
  from_vec(w, params);
  write_rec(rec, rec_out, epochs);
  if (idx_out) {
    int64_t k = 0;
    for (auto &v : sampled)
      for (size_t x : v)
        if (k < idx_cap) idx_out[k++] = int64_t(x);
  }
  return 0;
}

} // namespace

extern "C" {

long long oracle_param_count(int nl, const int *dims, const int *acts) { return (long long)Net(dims, acts, nl).nparams; }

void oracle_init_params_cpu(int nl, const int *dims, const int *acts, unsigned seed, double *out) {
  init_params_cpu(Net(dims, acts, nl), seed, out);
}
void oracle_init_params_cuda(int nl, const int *dims, const int *acts, unsigned seed, float *out) {
  init_params_cuda(Net(dims, acts, nl), seed, out);
}

// Loss + gradient on a batch (fp64). idx may be null (first B rows). lambda adds the S-LBFGS L2 term.
double oracle_loss_grad(int nl, const int *dims, const int *acts, const double *P, const double *X, const double *Y,
                        const long long *idx, long long B, double lambda, double *grad) {
  Net net(dims, acts, nl);
  MLPObjective<double> obj{&net, X, Y, B, {}, 0, 0};
  std::vector<double> w(P, P + net.nparams), g(net.nparams);
  double l = obj.loss_grad_batch(w, reinterpret_cast<const int64_t *>(idx), B, lambda, g.data());
  if (grad) std::copy(g.begin(), g.end(), grad);
  return l;
}

// finite_difference_hvp_batch (s_lbfgs.hpp:88-101) in fp64 on the rows idx (B of them), batch_g of
// UnifiedSLBFGS_CPU (1/B scale, + lambda w; unified_optimization.hpp:343-376).
void oracle_fd_hvp(int nl, const int *dims, const int *acts, const double *P, const double *V, const double *X,
                   const double *Y, const long long *idx, long long B, double lambda, double eps, double *y_out) {
  Net net(dims, acts, nl);
  MLPObjective<double> obj{&net, X, Y, B, {}, 0, 0};
  auto bg = [&](const Vec<double> &w, const std::vector<size_t> &ind, Vec<double> &g) {
    std::vector<int64_t> ii(ind.begin(), ind.end());
    obj.loss_grad_batch(w, ii.data(), int64_t(ii.size()), lambda, g.data());
  };
  std::vector<size_t> S(static_cast<size_t>(B));
  for (long long i = 0; i < B; ++i) S[size_t(i)] = idx ? size_t(idx[i]) : size_t(i);
  Vec<double> w(P, P + net.nparams), v(V, V + net.nparams);
  Vec<double> y = finite_difference_hvp_batch<double>(bg, w, v, S, eps);
  std::copy(y.begin(), y.end(), y_out);
}

// finite_difference_hvp_batch in the fp32 instantiation (w +- eps v, the gradients and their difference in
// float, as the oracle's fp32 S-LBFGS computes its pairs); inputs / output fp64 for ctypes convenience.
void oracle_fd_hvp_f32(int nl, const int *dims, const int *acts, const double *P, const double *V, const double *X,
                       const double *Y, const long long *idx, long long B, long long N, double lambda, double eps,
                       double *y_out) {
  Net net(dims, acts, nl);
  std::vector<float> Xf = to_vec<float>(X, size_t(N) * dims[0]), Yf = to_vec<float>(Y, size_t(N) * dims[nl]);
  MLPObjective<float> obj{&net, Xf.data(), Yf.data(), N, {}, 0, 0};
  auto bg = [&](const Vec<float> &w, const std::vector<size_t> &ind, Vec<float> &g) {
    std::vector<int64_t> ii(ind.begin(), ind.end());
    obj.loss_grad_batch(w, ii.data(), int64_t(ii.size()), lambda, g.data());
  };
  std::vector<size_t> S(static_cast<size_t>(B));
  for (long long i = 0; i < B; ++i) S[size_t(i)] = idx ? size_t(idx[i]) : size_t(i);
  Vec<float> w = to_vec<float>(P, net.nparams), v = to_vec<float>(V, net.nparams);
  Vec<float> y = finite_difference_hvp_batch<float>(bg, w, v, S, eps);
  from_vec(y, y_out);
}

// fp32 instantiation of the same (inputs/outputs as double for ctypes convenience).
double oracle_loss_grad_f32(int nl, const int *dims, const int *acts, const double *P, const double *X,
                            const double *Y, long long B, double *grad) {
  Net net(dims, acts, nl);
  std::vector<float> Xf = to_vec<float>(X, size_t(B) * dims[0]), Yf = to_vec<float>(Y, size_t(B) * dims[nl]);
  MLPObjective<float> obj{&net, Xf.data(), Yf.data(), B, {}, 0, 0};
  std::vector<float> w = to_vec<float>(P, net.nparams), g(net.nparams);
  float l = obj.loss_grad_batch(w, nullptr, B, 0.0, g.data());
  if (grad) from_vec(g, grad);
  return double(l);
}

// Forward-only loss f(w) = 0.5*SSE/N and optional network output [N][Out].
double oracle_loss(int nl, const int *dims, const int *acts, const double *P, const double *X, const double *Y,
                   long long N, double *out) {
  Net net(dims, acts, nl);
  Workspace<double> ws;
  forward<double>(net, P, X, nullptr, N, ws);
  if (out) std::copy(ws.A[nl - 1].begin(), ws.A[nl - 1].end(), out);
  return half_sse<double>(net, Y, nullptr, N, ws, false) / double(N);
}

// Two-loop on a history given in LOGICAL order (oldest first). mode 0: CPU (lbfgs.hpp:106-139, returns -Hg),
// 1: S-LBFGS (s_lbfgs.hpp:106-136, returns +Hv), 2: CUDA (lbfgs.cuh:206-261, returns -Hg).
void oracle_two_loop(int mode, long long n, int k, const double *S, const double *Y, const double *rho,
                     const double *g, double *out) {
  std::vector<double> gv(g, g + n);
  std::vector<double> r;
  if (mode == 2) {
    std::vector<Vec<double>> Sh(k > 0 ? k : 1, Vec<double>(n)), Yh(k > 0 ? k : 1, Vec<double>(n));
    std::vector<double> rh(k > 0 ? k : 1, 0.0);
    for (int i = 0; i < k; ++i) {
      std::copy(S + size_t(i) * n, S + size_t(i + 1) * n, Sh[i].begin());
      std::copy(Y + size_t(i) * n, Y + size_t(i + 1) * n, Yh[i].begin());
      rh[i] = rho[i];
    }
    r = two_loop_cuda<double>(gv, Sh, Yh, rh, k % (k > 0 ? k : 1), k);
  } else {
    Ring<Vec<double>> Sr(k > 0 ? k : 1), Yr(k > 0 ? k : 1);
    Ring<double> rr(k > 0 ? k : 1);
    for (int i = 0; i < k; ++i) {
      Sr.push_back(Vec<double>(S + size_t(i) * n, S + size_t(i + 1) * n));
      Yr.push_back(Vec<double>(Y + size_t(i) * n, Y + size_t(i + 1) * n));
      rr.push_back(rho[i]);
    }
    r = (mode == 0) ? two_loop_cpu<double>(gv, Sr, Yr, rr) : two_loop_slbfgs<double>(Sr, Yr, rr, gv);
  }
  std::copy(r.begin(), r.end(), out);
}

// Full-batch L-BFGS on the MLP, CPU semantics. rec: max_iters x 6 doubles
// (loss, ||g||, alpha, pair accepted, line-search trials, time). fp32 != 0 -> float instantiation.
int oracle_lbfgs_wolfe_mlp(int nl, const int *dims, const int *acts, double *params, const double *X,
                           const double *Y, long long N, int m, int max_iters, double tol, int fp32, double *rec,
                           int *iters, long *n_fwd, long *n_bwd, double *elapsed_ms) {
  Net net(dims, acts, nl);
  if (fp32) return run_wolfe_mlp<float>(net, params, X, Y, N, m, max_iters, tol, rec, iters, n_fwd, n_bwd, elapsed_ms);
  return run_wolfe_mlp<double>(net, params, X, Y, N, m, max_iters, tol, rec, iters, n_fwd, n_bwd, elapsed_ms);
}

// Full-batch L-BFGS on the MLP, CUDA semantics (Armijo + interpolation).
int oracle_lbfgs_armijo_mlp(int nl, const int *dims, const int *acts, double *params, const double *X,
                            const double *Y, long long N, int m, int max_iters, double tol, int max_ls, double c1,
                            double rho, int fp32, double *rec, int *iters) {
  Net net(dims, acts, nl);
  if (fp32) return run_armijo_mlp<float>(net, params, X, Y, N, m, max_iters, tol, max_ls, c1, rho, rec, iters);
  return run_armijo_mlp<double>(net, params, X, Y, N, m, max_iters, tol, max_ls, c1, rho, rec, iters);
}

// S-LBFGS on the MLP (CPU semantics, fp64). idx_out (optional) receives every sampled index list in order;
// pio_rec / pio_force (optional, pio_cap events of 4 x nparams doubles): the pair record / teacher forcing (PairIO).
int oracle_slbfgs_mlp(int nl, const int *dims, const int *acts, double *params, const double *X, const double *Y,
                      long long N, int epochs, double tol, int M, int L, int b, int bH, double step, double lambda,
                      int fp32, double *rec, int *iters, long long *idx_out, long long idx_cap, double *pair_out,
                      int pair_cap, int *npairs, double *pair0_us, int pio_cap, double *pio_rec,
                      const double *pio_force) {
  Net net(dims, acts, nl);
  PairIO pio;
  pio.rec = pio_rec;
  pio.force = pio_force;
  pio.cap = pio_cap;
  const PairIO *pp = (pio_rec || pio_force) ? &pio : nullptr;
  if (fp32)
    return run_slbfgs_mlp<float>(net, params, X, Y, N, epochs, tol, M, L, b, bH, step, lambda, rec, iters,
                                 reinterpret_cast<int64_t *>(idx_out), idx_cap, pair_out, pair_cap, npairs, pair0_us,
                                 pp);
  return run_slbfgs_mlp<double>(net, params, X, Y, N, epochs, tol, M, L, b, bH, step, lambda, rec, iters,
                                reinterpret_cast<int64_t *>(idx_out), idx_cap, pair_out, pair_cap, npairs, pair0_us,
                                pp);
}

// GD (gd.cuh:38-106) / SGD (sgd.cuh:50-153) with momentum on the MLP. rec: 2 doubles per record.
int oracle_gd_mlp(int nl, const int *dims, const int *acts, double *params, const double *X, const double *Y,
                  long long N, double lr, double momentum, int max_iters, double tol, int fp32, double *rec) {
  Net net(dims, acts, nl);
  auto run = [&](auto zero) {
    using T = decltype(zero);
    std::vector<T> Xt = to_vec<T>(X, size_t(N) * net.dims[0]);
    std::vector<T> Yt = to_vec<T>(Y, size_t(N) * net.dims.back());
    MLPObjective<T> obj{&net, Xt.data(), Yt.data(), N, {}, 0, 0};
    auto lg = [&](const Vec<T> &w, Vec<T> &g) { return obj.loss_grad_batch(w, nullptr, N, 0.0, g.data()); };
    Vec<T> x = to_vec<T>(params, net.nparams);
    const int done = gd_momentum<T>(x, lg, T(lr), T(momentum), max_iters, T(tol), rec);
    from_vec(x, params);
    return done;
  };
  return fp32 ? run(0.0f) : run(0.0);
}

int oracle_sgd_mlp(int nl, const int *dims, const int *acts, double *params, const double *X, const double *Y,
                   long long N, int batch, double lr, double momentum, double decay_rate, int decay_step,
                   int max_epochs, double tol, int fp32, double *rec) {
  Net net(dims, acts, nl);
  auto run = [&](auto zero) {
    using T = decltype(zero);
    const int In = net.dims[0], Out = net.dims.back();
    std::vector<T> Xt = to_vec<T>(X, size_t(N) * In);
    std::vector<T> Yt = to_vec<T>(Y, size_t(N) * Out);
    MLPObjective<T> full{&net, Xt.data(), Yt.data(), N, {}, 0, 0};
    auto flg = [&](const Vec<T> &w, Vec<T> &g) { return full.loss_grad_batch(w, nullptr, N, 0.0, g.data()); };
    auto blg = [&](const Vec<T> &w, Vec<T> &g, int64_t r0, int64_t bs) {
      MLPObjective<T> part{&net, Xt.data() + size_t(r0) * In, Yt.data() + size_t(r0) * Out, bs, {}, 0, 0};
      return part.loss_grad_batch(w, nullptr, bs, 0.0, g.data());
    };
    Vec<T> x = to_vec<T>(params, net.nparams);
    const int done = sgd_momentum<T>(x, flg, blg, N, batch, T(lr), T(momentum), T(decay_rate), decay_step,
                                     max_epochs, T(tol), rec);
    from_vec(x, params);
    return done;
  };
  return fp32 ? run(0.0f) : run(0.0);
}

// L-BFGS (CPU semantics) on the reference's analytic test problems. Returns final ||g||.
double oracle_lbfgs_testfn(int id, int n, double *x, int m, int max_iters, double tol, int *iters) {
  auto f = [&](const Vec<double> &v) { return tf_f(id, v); };
  auto g = [&](const Vec<double> &v) { return tf_g(id, v); };
  LbfgsParams<double> prm;
  prm.m = m;
  prm.max_iters = max_iters;
  prm.tol = tol;
  Vec<double> r = lbfgs_wolfe<double>(Vec<double>(x, x + n), f, g, prm, nullptr, iters);
  std::copy(r.begin(), r.end(), x);
  return norm(tf_g(id, r));
}

// Successive sample_minibatch_indices draws from ONE mt19937(seed) (s_lbfgs.hpp:141-160).
void oracle_sample_indices(long long N, int b, unsigned seed, int calls, long long *out) {
  std::mt19937 rng(seed);
  for (int c = 0; c < calls; ++c) {
    auto v = sample_minibatch_indices(size_t(N), size_t(b), rng);
    for (size_t i = 0; i < v.size(); ++i) out[size_t(c) * b + i] = (long long)v[i];
  }
}

void oracle_synth_mnist(long long N, int In, int classes, unsigned seed, double *X, double *Y) {
  synth_mnist(N, In, classes, seed, X, Y);
}

// Ring-buffer trace: push 0..npush-1 into Ring<int>(cap); after each push write cap ints
// (logical contents, -1 padded) to out (npush x cap) and the head index to heads.
void oracle_ring_trace(int cap, int npush, int *out, int *heads) {
  Ring<int> r(cap);
  for (int t = 0; t < npush; ++t) {
    r.push_back(t);
    for (int i = 0; i < cap; ++i) out[t * cap + i] = i < int(r.size()) ? r[i] : -1;
    heads[t] = int(r.head());
  }
}

int oracle_num_threads() {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

// OpenMP threads of the following oracle calls (bench.py's CPU baseline at the host's physical core count)
void oracle_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

} // extern "C"
