// oracle/oracle.hpp — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
//
// CPU restatement of SignorB/lbfgs-FFNN's L-BFGS / S-LBFGS hot path, written from the
// reference's behaviour (not copied). Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this code; the product path (lbfgs-ffnn_amd/) never does.
//
// Pinning:
//   * loss/grad restatement  <-> torch-CPU fp64 autograd (tests/test_oracle.py)
//   * RingBuffer restatement <-> the reference's own ring_buffer.hpp compiled into oracle/_ref/
//   * L-BFGS restatement     <-> the reference's known-answer tests (tests/main.cpp:15-258)
//   * init RNG               <-> seed-123 draws recorded in SURVEY.md §8(c)
// Everything is templated on the scalar T so the fp64 (reference) and fp32 instantiations share code.
//
// Reference citations are relative to /root/reference/.
#pragma once

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <numeric>
#include <random>
#include <stdexcept>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace oracle {

// Activation ids follow the reference's ActivationType (src/cuda/kernels.cuh:53-58).
enum Act : int { LINEAR = 0, TANH = 1, RELU = 2, SIGMOID = 3 };

// src/layer.hpp:16-47 (apply / prime, both on the pre-activation Z) and the init scale (:19,:26,:37,:46).
template <class T> inline T act_apply(int a, T x) {
  switch (a) {
  case TANH: return std::tanh(x);
  case RELU: return x > T(0) ? x : T(0);
  case SIGMOID: return T(1) / (T(1) + std::exp(-x));
  default: return x;
  }
}
template <class T> inline T act_prime(int a, T z) {
  switch (a) {
  case TANH: { T t = std::tanh(z); return T(1) - t * t; }
  case RELU: return z > T(0) ? T(1) : T(0);
  case SIGMOID: { T s = T(1) / (T(1) + std::exp(-z)); return s * (T(1) - s); }
  default: return T(1);
  }
}
inline double act_scale(int a) { return a == RELU ? 1.41421356 : 1.0; }

// ---------------------------------------------------------------------------------------------
// RingBuffer — restates src/minimizer/ring_buffer.hpp:15-134 (push_back :43-59, operator[] :67-80).
// Logical index 0 = oldest; pushing when full overwrites the oldest and advances head.
// ---------------------------------------------------------------------------------------------
template <class T> class Ring {
public:
  explicit Ring(size_t cap = 0) : cap_(cap) { data_.resize(cap); }
  void push_back(const T &v) {
    if (cap_ == 0) return;
    if (count_ < cap_) {
      data_[(head_ + count_) % cap_] = v;
      ++count_;
    } else {
      data_[head_] = v;
      head_ = (head_ + 1) % cap_;
    }
  }
  T &operator[](size_t i) { return data_[(head_ + i) % cap_]; }
  const T &operator[](size_t i) const { return data_[(head_ + i) % cap_]; }
  const T &back() const { return (*this)[count_ - 1]; }
  size_t size() const { return count_; }
  bool empty() const { return count_ == 0; }
  void clear() { head_ = 0; count_ = 0; }
  size_t head() const { return head_; }

private:
  std::vector<T> data_;
  size_t cap_ = 0, head_ = 0, count_ = 0;
};

template <class T> using Vec = std::vector<T>;

template <class T> inline T dot(const Vec<T> &a, const Vec<T> &b) {
  // fp64 accumulation regardless of T (the reference's Eigen dot runs in the vector's own type;
  // for T=double this is identical, for T=float it is the better-conditioned choice).
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += double(a[i]) * double(b[i]);
  return T(s);
}
template <class T> inline T norm(const Vec<T> &a) { return std::sqrt(dot(a, a)); }

// ---------------------------------------------------------------------------------------------
// Dense MLP — restates cpu_mlp::Network (src/network.hpp:21-145) and DenseLayer (src/layer.hpp:74-131).
// Storage: flat params, per layer [W (Out x In, column-major) | b (Out)] (network.hpp:45-71).
// W column-major Out x In is, read row-major, P[i][o] with shape [In][Out]; so the layer segment is
// exactly a row-major [(In+1) x Out] block whose last row is the bias.
// Data: X is In x N column-major in the reference (one sample per column) == row-major [N][In].
// ---------------------------------------------------------------------------------------------
struct Net {
  std::vector<int> dims; // nlayers+1
  std::vector<int> acts; // nlayers
  std::vector<size_t> off;
  size_t nparams = 0;
  Net() = default;
  Net(const int *d, const int *a, int nl) {
    dims.assign(d, d + nl + 1);
    acts.assign(a, a + nl);
    off.resize(nl + 1);
    size_t o = 0;
    for (int l = 0; l < nl; ++l) {
      off[l] = o;
      o += size_t(dims[l]) * dims[l + 1] + dims[l + 1];
    }
    off[nl] = o;
    nparams = o;
  }
  int nl() const { return int(acts.size()); }
};

// network.hpp:45-71 — mt19937(seed); per layer a fresh normal_distribution<double>(0, scale*sqrt(1/In))
// drawn over ALL Out*In+Out params in flat order (biases included).
inline void init_params_cpu(const Net &net, unsigned seed, double *out) {
  std::mt19937 gen(seed);
  for (int l = 0; l < net.nl(); ++l) {
    double sd = act_scale(net.acts[l]) * std::sqrt(1.0 / double(net.dims[l]));
    std::normal_distribution<double> dist(0.0, sd);
    size_t cnt = size_t(net.dims[l]) * net.dims[l + 1] + net.dims[l + 1];
    for (size_t i = 0; i < cnt; ++i) out[net.off[l] + i] = dist(gen);
  }
}

// src/cuda/network.cuh:36-59 — normal_distribution<float>(0, scale*sqrt(1/In)) computed in float,
// weights only (Out*In draws), biases zero. scale from kernels.cuh:61-71.
inline void init_params_cuda(const Net &net, unsigned seed, float *out) {
  std::mt19937 gen(seed);
  for (int l = 0; l < net.nl(); ++l) {
    float scale = net.acts[l] == RELU ? 1.41421356f : 1.0f;
    float sd = scale * std::sqrt(1.0f / float(net.dims[l]));
    std::normal_distribution<float> dist(0.0f, sd);
    size_t w = size_t(net.dims[l]) * net.dims[l + 1];
    for (size_t i = 0; i < w; ++i) out[net.off[l] + i] = dist(gen);
    for (int i = 0; i < net.dims[l + 1]; ++i) out[net.off[l] + w + i] = 0.0f;
  }
}

// Fixed chunking for every batch reduction so results do not depend on the OpenMP thread count.
static constexpr int kChunks = 16;

template <class T> struct Workspace {
  std::vector<Vec<T>> Z, A; // per layer, [B][Out]
  std::vector<Vec<T>> D;    // deltas per layer, [B][Out]
  Vec<T> Xg;                // gathered input when an index list is used
};

// Forward on a batch (rows of X selected by idx if non-null). layer.hpp:100-110: Z = W*A + b, A' = act(Z).
template <class T>
void forward(const Net &net, const T *P, const T *X, const int64_t *idx, int64_t B, Workspace<T> &ws) {
  const int nl = net.nl();
  ws.Z.resize(nl);
  ws.A.resize(nl);
  const T *in = X;
  if (idx) {
    const int In = net.dims[0];
    ws.Xg.resize(size_t(B) * In);
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < B; ++b) std::memcpy(&ws.Xg[size_t(b) * In], X + size_t(idx[b]) * In, sizeof(T) * In);
    in = ws.Xg.data();
  }
  for (int l = 0; l < nl; ++l) {
    const int In = net.dims[l], Out = net.dims[l + 1], a = net.acts[l];
    const T *W = P + net.off[l], *bias = W + size_t(In) * Out;
    ws.Z[l].resize(size_t(B) * Out);
    ws.A[l].resize(size_t(B) * Out);
    T *Z = ws.Z[l].data(), *A = ws.A[l].data();
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < B; ++b) {
      T *z = Z + size_t(b) * Out;
      const T *x = in + size_t(b) * In;
      for (int o = 0; o < Out; ++o) z[o] = T(0);
      for (int i = 0; i < In; ++i) {
        const T xi = x[i];
        const T *w = W + size_t(i) * Out;
        for (int o = 0; o < Out; ++o) z[o] += xi * w[o];
      }
      T *aa = A + size_t(b) * Out;
      for (int o = 0; o < Out; ++o) {
        z[o] += bias[o];
        aa[o] = act_apply<T>(a, z[o]);
      }
    }
    in = A;
  }
}

// Backward from D[nl-1] = loss gradient wrt the output (before the output activation derivative).
// layer.hpp:112-128: dZ = delta .* act'(Z); dW += dZ*A^T; db += rowsum(dZ); delta_prev = W^T dZ
// (network.hpp:98-101: no delta for layer 0). Writes the UNNORMALISED gradient into G.
template <class T>
void backward(const Net &net, const T *P, const T *X, int64_t B, Workspace<T> &ws, T *G) {
  const int nl = net.nl();
  ws.D.resize(nl);
  for (int l = nl - 1; l >= 0; --l) {
    const int In = net.dims[l], Out = net.dims[l + 1], a = net.acts[l];
    T *dZ = ws.D[l].data();
    const T *Z = ws.Z[l].data();
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < B * Out; ++e) dZ[e] *= act_prime<T>(a, Z[e]);
    const T *Ain = (l == 0) ? (ws.Xg.empty() ? X : ws.Xg.data()) : ws.A[l - 1].data();
    // dW/db with a fixed number of batch chunks, summed in chunk order (thread-count independent).
    const size_t seg = size_t(In + 1) * Out;
    std::vector<Vec<double>> part(kChunks, Vec<double>(seg, 0.0));
#pragma omp parallel for schedule(static)
    for (int c = 0; c < kChunks; ++c) {
      int64_t b0 = B * c / kChunks, b1 = B * (c + 1) / kChunks;
      double *pw = part[c].data();
      for (int64_t b = b0; b < b1; ++b) {
        const T *ai = Ain + size_t(b) * In;
        const T *dz = dZ + size_t(b) * Out;
        for (int i = 0; i < In; ++i) {
          const double x = ai[i];
          double *row = pw + size_t(i) * Out;
          for (int o = 0; o < Out; ++o) row[o] += x * double(dz[o]);
        }
        double *brow = pw + size_t(In) * Out;
        for (int o = 0; o < Out; ++o) brow[o] += double(dz[o]);
      }
    }
    T *g = G + net.off[l];
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < int64_t(seg); ++e) {
      double s = 0.0;
      for (int c = 0; c < kChunks; ++c) s += part[c][e];
      g[e] = T(s);
    }
    if (l > 0) {
      const T *W = P + net.off[l];
      ws.D[l - 1].resize(size_t(B) * In);
      T *dp = ws.D[l - 1].data();
#pragma omp parallel for schedule(static)
      for (int64_t b = 0; b < B; ++b) {
        const T *dz = dZ + size_t(b) * Out;
        T *d = dp + size_t(b) * In;
        for (int i = 0; i < In; ++i) {
          const T *w = W + size_t(i) * Out;
          T s = T(0);
          for (int o = 0; o < Out; ++o) s += w[o] * dz[o];
          d[i] = s;
        }
      }
    }
  }
}

// 0.5 * sum ||out - y||^2 over the batch (deterministic chunked sum). Optionally leaves diff in D.
template <class T>
double half_sse(const Net &net, const T *Y, const int64_t *idx, int64_t B, Workspace<T> &ws, bool keep_diff) {
  const int nl = net.nl(), Out = net.dims[nl];
  const T *out = ws.A[nl - 1].data();
  if (keep_diff) {
    ws.D.resize(nl);
    ws.D[nl - 1].resize(size_t(B) * Out);
  }
  double part[kChunks];
#pragma omp parallel for schedule(static)
  for (int c = 0; c < kChunks; ++c) {
    int64_t b0 = B * c / kChunks, b1 = B * (c + 1) / kChunks;
    double s = 0.0;
    for (int64_t b = b0; b < b1; ++b) {
      const T *y = Y + size_t(idx ? idx[b] : b) * Out;
      for (int o = 0; o < Out; ++o) {
        T d = out[size_t(b) * Out + o] - y[o];
        if (keep_diff) ws.D[nl - 1][size_t(b) * Out + o] = d;
        s += double(d) * double(d);
      }
    }
    part[c] = s;
  }
  double s = 0.0;
  for (int c = 0; c < kChunks; ++c) s += part[c];
  return 0.5 * s;
}

// ---------------------------------------------------------------------------------------------
// Objective closures — restate run_full_batch_cpu (src/unified_optimization.hpp:87-124) and the
// S-LBFGS batch_g / batch_f (src/unified_optimization.hpp:343-400, lambda = 1e-4 at :334).
// ---------------------------------------------------------------------------------------------
template <class T> struct MLPObjective {
  const Net *net;
  const T *X, *Y;
  int64_t N;
  Workspace<T> ws;
  long n_fwd = 0, n_bwd = 0; // evaluation counters (for the CPU-baseline flop accounting)

  // f(w) = 0.5*||net(X)-Y||^2 / N   (unified_optimization.hpp:101-108)
  T f(const Vec<T> &w) {
    forward<T>(*net, w.data(), X, nullptr, N, ws);
    ++n_fwd;
    double l = half_sse<T>(*net, Y, nullptr, N, ws, false);
    return T(N > 0 ? l / double(N) : l);
  }
  // grad(w) = backprop(out-Y) / N   (unified_optimization.hpp:110-120)
  Vec<T> grad(const Vec<T> &w) {
    Vec<T> g(net->nparams);
    loss_grad_batch(w, nullptr, N, 0.0, g.data());
    return g;
  }
  // Shared worker: loss and gradient on a batch (idx == nullptr -> first B rows / full batch).
  // Returns 0.5*SSE/B + 0.5*lambda*||w||^2; g = backprop/B + lambda*w.
  T loss_grad_batch(const Vec<T> &w, const int64_t *idx, int64_t B, double lambda, T *g) {
    forward<T>(*net, w.data(), X, idx, B, ws);
    double l = half_sse<T>(*net, Y, idx, B, ws, true);
    backward<T>(*net, w.data(), X, B, ws, g);
    ++n_fwd;
    ++n_bwd;
    const T inv = B > 0 ? T(1.0 / double(B)) : T(0);
    for (size_t j = 0; j < net->nparams; ++j) g[j] = g[j] * inv + T(lambda) * w[j];
    double loss = B > 0 ? l / double(B) : l;
    if (lambda != 0.0) loss += 0.5 * lambda * double(dot(w, w));
    return T(loss);
  }
};

// ---------------------------------------------------------------------------------------------
// Two-loop recursions.
// ---------------------------------------------------------------------------------------------
// src/minimizer/lbfgs.hpp:106-139 — returns -H*g; gamma = s_k.y_k / y_k.y_k (no guard); empty -> -g.
template <class T>
Vec<T> two_loop_cpu(const Vec<T> &g, const Ring<Vec<T>> &S, const Ring<Vec<T>> &Y, const Ring<double> &rho) {
  const size_t n = g.size();
  Vec<T> r(n);
  if (S.empty()) {
    for (size_t j = 0; j < n; ++j) r[j] = -g[j];
    return r;
  }
  Vec<T> q = g;
  std::vector<double> alpha(S.size());
  for (int i = int(S.size()) - 1; i >= 0; --i) {
    alpha[i] = rho[i] * double(dot(S[i], q));
    for (size_t j = 0; j < n; ++j) q[j] -= T(alpha[i]) * Y[i][j];
  }
  double gamma = double(dot(S.back(), Y.back())) / double(dot(Y.back(), Y.back()));
  Vec<T> z(n);
  for (size_t j = 0; j < n; ++j) z[j] = T(gamma) * q[j];
  for (size_t i = 0; i < S.size(); ++i) {
    double beta = rho[i] * double(dot(Y[i], z));
    for (size_t j = 0; j < n; ++j) z[j] += S[i][j] * T(alpha[i] - beta);
  }
  for (size_t j = 0; j < n; ++j) r[j] = -z[j];
  return r;
}

// src/minimizer/s_lbfgs.hpp:106-136 — returns +H*v; gamma = 1 if |y.y|<1e-12, clamped to [1e-6, 1e6].
template <class T>
Vec<T> two_loop_slbfgs(const Ring<Vec<T>> &S, const Ring<Vec<T>> &Y, const Ring<double> &rho, const Vec<T> &v) {
  const size_t n = v.size();
  const int M = int(S.size());
  std::vector<double> alpha(M);
  Vec<T> q = v;
  for (int i = M - 1; i >= 0; --i) {
    alpha[i] = rho[i] * double(dot(S[i], q));
    for (size_t j = 0; j < n; ++j) q[j] = q[j] - T(alpha[i]) * Y[i][j];
  }
  double gamma = 1.0;
  if (M > 0) {
    double denom = double(dot(Y.back(), Y.back()));
    gamma = std::abs(denom) < 1e-12 ? 1.0 : double(dot(S.back(), Y.back())) / denom;
    gamma = std::min(std::max(gamma, 1e-6), 1e6);
  }
  Vec<T> r(n);
  for (size_t j = 0; j < n; ++j) r[j] = T(gamma) * q[j];
  for (int i = 0; i < M; ++i) {
    double beta = rho[i] * double(dot(Y[i], r));
    for (size_t j = 0; j < n; ++j) r[j] = r[j] + S[i][j] * T(alpha[i] - beta);
  }
  return r;
}

// src/cuda/lbfgs.cuh:206-261 — returns -H*g over the physical ring; gamma = ys/yy if yy>0 else 1.
template <class T>
Vec<T> two_loop_cuda(const Vec<T> &g, const std::vector<Vec<T>> &Sh, const std::vector<Vec<T>> &Yh,
                     const std::vector<double> &rho, int head, int count) {
  const size_t n = g.size();
  Vec<T> p(n);
  if (count <= 0 || Sh.empty()) {
    for (size_t j = 0; j < n; ++j) p[j] = -g[j];
    return p;
  }
  const int m = int(Sh.size());
  auto phys = [&](int li) {
    int start = (head - count) % m;
    if (start < 0) start += m;
    return (start + li) % m;
  };
  Vec<T> q = g;
  std::vector<double> alpha(count);
  for (int li = count - 1; li >= 0; --li) {
    int i = phys(li);
    alpha[li] = rho[i] * double(dot(Sh[i], q));
    for (size_t j = 0; j < n; ++j) q[j] -= T(alpha[li]) * Yh[i][j];
  }
  int last = phys(count - 1);
  double ys = double(dot(Sh[last], Yh[last])), yy = double(dot(Yh[last], Yh[last]));
  double gamma = yy > 0 ? ys / yy : 1.0;
  Vec<T> z(n);
  for (size_t j = 0; j < n; ++j) z[j] = T(gamma) * q[j];
  for (int li = 0; li < count; ++li) {
    int i = phys(li);
    double b = rho[i] * double(dot(Yh[i], z));
    for (size_t j = 0; j < n; ++j) z[j] += T(alpha[li] - b) * Sh[i][j];
  }
  for (size_t j = 0; j < n; ++j) p[j] = -z[j];
  return p;
}

// ---------------------------------------------------------------------------------------------
// Full-batch L-BFGS, CPU semantics — restates LBFGS::solve (src/minimizer/lbfgs.hpp:38-100) and
// FullBatchMinimizer::line_search (src/minimizer/full_batch_minimizer.hpp:126-157; c1=1e-4, c2=0.9,
// rho=0.5, 50 trials at :113-116). The call pattern (including the redundant f/grad re-evaluations)
// is reproduced literally so the CPU baseline does the reference's work.
// ---------------------------------------------------------------------------------------------
struct IterRecord {
  double loss = 0, gnorm = 0, alpha = 0, time_ms = 0;
  int accepted = 0, ls_trials = 0;
};

template <class T> struct LbfgsParams {
  int m = 16, max_iters = 1000;
  double tol = 1e-10, c1 = 1e-4, c2 = 0.9, rho = 0.5;
  int max_line_iters = 50;
};

template <class T, class F, class G>
Vec<T> lbfgs_wolfe(Vec<T> x, F &&f, G &&Gradient, const LbfgsParams<T> &prm, std::vector<IterRecord> *rec,
                   int *iters_out) {
  Ring<Vec<T>> s_list(prm.m), y_list(prm.m);
  Ring<double> rho_list(prm.m);
  Vec<T> grad = Gradient(x);
  const size_t n = x.size();
  int it = 0;
  for (it = 0; it < prm.max_iters; ++it) {
    if (double(norm(grad)) < prm.tol) break;
    Vec<T> p = two_loop_cpu(grad, s_list, y_list, rho_list);
    double alpha;
    int trials = 0;
    if (it == 0) {
      alpha = std::min(1.0, 1.0 / double(norm(grad)));
    } else {
      // line_search(x, p, f, Gradient)
      double f_old = double(f(x));
      double gfo = double(dot(Gradient(x), p));
      const double inf = std::numeric_limits<double>::infinity();
      double amin = 0.0, amax = inf;
      alpha = 1.0;
      bool done = false;
      for (int i = 0; i < prm.max_line_iters; ++i) {
        ++trials;
        Vec<T> xn(n);
        for (size_t j = 0; j < n; ++j) xn[j] = x[j] + T(alpha) * p[j];
        double fn = double(f(xn));
        if (fn > f_old + prm.c1 * alpha * gfo) {
          amax = alpha;
          alpha = prm.rho * (amin + amax);
          continue;
        }
        double gnp = double(dot(Gradient(xn), p));
        if (gnp < prm.c2 * gfo) {
          amin = alpha;
          alpha = (amax == inf) ? alpha * 2 : prm.rho * (amin + amax);
          continue;
        }
        done = true;
        break;
      }
      (void)done;
    }
    Vec<T> xn(n), s(n);
    for (size_t j = 0; j < n; ++j) xn[j] = x[j] + T(alpha) * p[j];
    for (size_t j = 0; j < n; ++j) s[j] = xn[j] - x[j];
    Vec<T> gn = Gradient(xn);
    Vec<T> y(n);
    for (size_t j = 0; j < n; ++j) y[j] = gn[j] - grad[j];
    x = xn;
    double ys = double(dot(y, s));
    int acc = 0;
    if (ys > 1e-10) {
      s_list.push_back(s);
      y_list.push_back(y);
      rho_list.push_back(1.0 / ys);
      acc = 1;
    }
    grad = gn;
    if (rec) {
      IterRecord r;
      r.loss = double(f(x));
      r.gnorm = double(norm(grad));
      r.alpha = alpha;
      r.accepted = acc;
      r.ls_trials = trials;
      rec->push_back(r);
    }
  }
  if (iters_out) *iters_out = it;
  return x;
}

// ---------------------------------------------------------------------------------------------
// Full-batch L-BFGS, CUDA semantics — restates CudaLBFGS::solve (src/cuda/lbfgs.cuh:39-194):
// Armijo backtracking (c1, rho, max_line_iters; defaults minimizer_base.cuh:63-64) with quadratic
// interpolation accepted in [0.1a, 0.9a]; descent fallback + history reset; reset on LS failure;
// the rejected pair still overwrites slot hist_head (:149-169).
// ---------------------------------------------------------------------------------------------
template <class T> struct ArmijoParams {
  int m = 16, max_iters = 200, max_line_iters = 20;
  double tol = 1e-6, c1 = 1e-4, rho = 0.5;
};

template <class T, class LG>
Vec<T> lbfgs_armijo(Vec<T> x, LG &&loss_grad, const ArmijoParams<T> &prm, std::vector<IterRecord> *rec,
                    int *iters_out) {
  const size_t n = x.size();
  const int m = prm.m;
  std::vector<Vec<T>> Sh(m, Vec<T>(n)), Yh(m, Vec<T>(n));
  std::vector<double> rho_h(m, 0.0);
  int head = 0, count = 0;
  Vec<T> grad(n), gnew(n);
  T loss = loss_grad(x, grad);
  int done = 0;
  for (int it = 0; it < prm.max_iters; ++it) {
    T gnorm = norm(grad);
    if (double(gnorm) < prm.tol) break;
    Vec<T> p = two_loop_cuda(grad, Sh, Yh, rho_h, head, count);
    T gdp = dot(grad, p);
    if (gdp >= T(0)) {
      for (size_t j = 0; j < n; ++j) p[j] = -grad[j];
      gdp = -dot(grad, grad);
      head = 0;
      count = 0;
    }
    T alpha = (it == 0) ? std::min(T(1), T(1) / gnorm) : T(1);
    Vec<T> xb = x;
    T lnew = 0;
    bool ok = false;
    int trials = 0;
    for (int ls = 0; ls < prm.max_line_iters; ++ls) {
      ++trials;
      for (size_t j = 0; j < n; ++j) x[j] = xb[j] + alpha * p[j];
      lnew = loss_grad(x, gnew);
      if (lnew <= loss + T(prm.c1) * alpha * gdp) {
        ok = true;
        break;
      }
      T den = T(2) * (lnew - loss - gdp * alpha);
      bool fb = true;
      if (std::abs(den) > T(1e-20)) {
        T na = -(gdp * alpha * alpha) / den;
        if (na >= T(0.1) * alpha && na <= T(0.9) * alpha) {
          alpha = na;
          fb = false;
        }
      }
      if (fb) alpha *= T(prm.rho);
    }
    if (!ok) {
      head = 0;
      count = 0;
    }
    int acc = 0;
    if (m > 0) {
      const int slot = head;
      for (size_t j = 0; j < n; ++j) {
        Sh[slot][j] = x[j] - xb[j];
        Yh[slot][j] = gnew[j] - grad[j];
      }
      T ys = dot(Yh[slot], Sh[slot]);
      if (ys > T(1e-10)) {
        rho_h[slot] = 1.0 / double(ys);
        head = (head + 1) % m;
        count = std::min(count + 1, m);
        acc = 1;
      }
    }
    grad = gnew;
    loss = lnew;
    if (rec) {
      IterRecord r;
      r.loss = double(loss);
      r.gnorm = double(norm(grad));
      r.alpha = double(alpha);
      r.accepted = acc;
      r.ls_trials = trials;
      rec->push_back(r);
    }
    ++done;
  }
  if (iters_out) *iters_out = done;
  return x;
}

// ---------------------------------------------------------------------------------------------
// S-LBFGS — restates SLBFGS::stochastic_solve (src/minimizer/s_lbfgs.hpp:165-290),
// sample_minibatch_indices (:141-160) and finite_difference_hvp_batch (:88-101).
// ---------------------------------------------------------------------------------------------
inline std::vector<size_t> sample_minibatch_indices(size_t N, size_t b, std::mt19937 &rng) {
  if (N == 0 || b == 0) return {};
  std::vector<size_t> idx(N);
  std::iota(idx.begin(), idx.end(), 0);
  if (b >= N) return idx;
  for (size_t i = 0; i < b; ++i) {
    std::uniform_int_distribution<size_t> dist(i, N - 1);
    size_t j = dist(rng);
    std::swap(idx[i], idx[j]);
  }
  idx.resize(b);
  return idx;
}

// finite_difference_hvp_batch (s_lbfgs.hpp:88-101): y = (g_S(w + eps v) - g_S(w - eps v)) / (2 eps) on the
// Hessian batch S, eps = 1e-4 (:90).
// hook(gp, gm) (diagnostics, PairIO below) may read or replace the two gradients before the difference.
template <class T, class BG, class Hook>
Vec<T> finite_difference_hvp_batch(BG &&batch_g, const Vec<T> &w, const Vec<T> &v, const std::vector<size_t> &S,
                                   double eps, Hook &&hook) {
  const size_t n = w.size();
  Vec<T> wp(n), wm(n), gp(n, T(0)), gm(n, T(0)), y(n);
  for (size_t j = 0; j < n; ++j) {
    wp[j] = w[j] + T(eps) * v[j];
    wm[j] = w[j] - T(eps) * v[j];
  }
  batch_g(wp, S, gp);
  batch_g(wm, S, gm);
  hook(gp, gm);
  for (size_t j = 0; j < n; ++j) y[j] = (gp[j] - gm[j]) / T(2.0 * eps);
  return y;
}
template <class T, class BG>
Vec<T> finite_difference_hvp_batch(BG &&batch_g, const Vec<T> &w, const Vec<T> &v, const std::vector<size_t> &S,
                                   double eps) {
  return finite_difference_hvp_batch<T>(batch_g, w, v, S, eps, [](Vec<T> &, Vec<T> &) {});
}

// Diagnostics (test only; the device's lbf_slbfgs_pair_io): at curvature event e (each t > 0 with t % L == 0, the
// first included) record [w_{t+1} | u | g(u + eps s) | g(u - eps s)] (n doubles each, the gradients zero at the
// first event) into rec + 4 e n, and replace u and the two gradients by force + 4 e n's before use.
struct PairIO {
  double *rec = nullptr;
  const double *force = nullptr;
  int cap = 0;
};

struct SlbfgsParams {
  int max_iters = 1000; // epochs
  double tol = 1e-4;
  int m = 0;            // inner steps per epoch (N / b)
  int M = 10, L = 10, b = 256, b_H = 128;
  double step = 0.01;
  int64_t N = 0;
  unsigned seed = 123; // kDefaultSeed (src/seed.hpp:4), used at s_lbfgs.hpp:183
};

// BG(w, idx, g): batch gradient; BF(w, idx) -> batch loss.
template <class T, class BG, class BF>
Vec<T> slbfgs(Vec<T> weights, BG &&batch_g, BF &&batch_f, const SlbfgsParams &prm, std::vector<IterRecord> *rec,
              int *iters_out, std::vector<std::vector<size_t>> *sampled = nullptr,
              std::vector<std::array<double, 8>> *pairs = nullptr, std::vector<double> *pair0_us = nullptr,
              const PairIO *pio = nullptr) {
  int nev = 0;
  const size_t n = weights.size();
  const int M = prm.M;
  Ring<Vec<T>> u_list(M > 0 ? M + 1 : 0), s_list(M > 0 ? M : 0), y_list(M > 0 ? M : 0);
  Ring<double> rho_list(M > 0 ? M : 0);
  std::mt19937 rng(prm.seed);
  Vec<T> wt = weights;
  Ring<Vec<T>> w_hist(prm.L + 1);
  std::vector<size_t> full(prm.N);
  std::iota(full.begin(), full.end(), 0);
  int it = 0;
  while (it < prm.max_iters) {
    w_hist.clear();
    Vec<T> mu(n, T(0));
    batch_g(weights, full, mu);
    if (double(norm(mu)) < prm.tol) break;
    wt = weights;
    w_hist.push_back(wt);
    for (int t = 0; t < prm.m; ++t) {
      auto mb = sample_minibatch_indices(size_t(prm.N), size_t(prm.b), rng);
      if (sampled) sampled->push_back(mb);
      Vec<T> g1(n, T(0)), g2(n, T(0)), v(n);
      batch_g(wt, mb, g1);
      batch_g(weights, mb, g2);
      for (size_t j = 0; j < n; ++j) v[j] = (g1[j] - g2[j]) + mu[j];
      Vec<T> d = two_loop_slbfgs(s_list, y_list, rho_list, v);
      for (size_t j = 0; j < n; ++j) wt[j] = wt[j] - T(prm.step) * d[j];
      w_hist.push_back(wt);
      if (t > 0 && t % prm.L == 0) {
        Vec<T> u(n, T(0));
        const int nw = int(w_hist.size());
        for (size_t i = 0; i < w_hist.size(); ++i)
          for (size_t j = 0; j < n; ++j) u[j] += w_hist[i][j];
        if (nw > 0)
          for (size_t j = 0; j < n; ++j) u[j] /= T(nw);
        const int ev = nev++;
        double *pr = pio && pio->rec && ev < pio->cap ? pio->rec + size_t(ev) * 4 * n : nullptr;
        const double *pf = pio && pio->force && ev < pio->cap ? pio->force + size_t(ev) * 4 * n : nullptr;
        if (pr) {
          for (size_t j = 0; j < n; ++j) {
            pr[j] = double(wt[j]);
            pr[n + j] = double(u[j]);
            pr[2 * n + j] = pr[3 * n + j] = 0.0;
          }
        }
        if (pf)
          for (size_t j = 0; j < n; ++j) u[j] = T(pf[n + j]);
        if (!u_list.empty()) {
          const Vec<T> &up = u_list.back();
          Vec<T> s(n);
          for (size_t j = 0; j < n; ++j) s[j] = u[j] - up[j];
          auto hb = sample_minibatch_indices(size_t(prm.N), size_t(prm.b_H), rng);
          if (sampled) sampled->push_back(hb);
          Vec<T> y = (pr || pf) ? finite_difference_hvp_batch<T>(batch_g, u, s, hb, 1e-4, [&](Vec<T> &gp, Vec<T> &gm) {
            for (size_t j = 0; j < n; ++j) {
              if (pr) {
                pr[2 * n + j] = double(gp[j]);
                pr[3 * n + j] = double(gm[j]);
              }
              if (pf) {
                gp[j] = T(pf[2 * n + j]);
                gm[j] = T(pf[3 * n + j]);
              }
            }
          })
                                           : finite_difference_hvp_batch<T>(batch_g, u, s, hb, 1e-4);
          if (pair0_us && pair0_us->empty()) { // diagnostics: the first candidate's w_t, u, s, y (fp64 copies)
            pair0_us->assign(wt.begin(), wt.end());
            pair0_us->insert(pair0_us->end(), u.begin(), u.end());
            pair0_us->insert(pair0_us->end(), s.begin(), s.end());
            pair0_us->insert(pair0_us->end(), y.begin(), y.end());
          }
          double ys = double(dot(y, s));
          const bool acc = std::abs(ys) > 1e-10;
          if (acc) {
            s_list.push_back(s);
            y_list.push_back(y);
            rho_list.push_back(1.0 / ys);
          }
          // diagnostics row (the device's lbf_slbfgs_params.pair_trace): epoch, t, y.s, s.s, y.y, accepted, live
          if (pairs)
            pairs->push_back({double(it), double(t), ys, double(dot(s, s)), double(dot(y, y)), acc ? 1.0 : 0.0,
                              double(s_list.size()), 0.0});
        }
        u_list.push_back(u);
      }
    }
    if (w_hist.size() >= 2) {
      std::uniform_int_distribution<size_t> pick(0, w_hist.size() - 2);
      weights = w_hist[pick(rng)];
    } else {
      weights = wt;
    }
    if (rec) {
      IterRecord r;
      r.loss = double(batch_f(weights, full));
      Vec<T> gl(n, T(0));
      batch_g(weights, full, gl);
      r.gnorm = double(norm(gl));
      r.accepted = int(s_list.size());
      rec->push_back(r);
    }
    ++it;
  }
  if (iters_out) *iters_out = it;
  return weights;
}

// ---------------------------------------------------------------------------------------------
// Gradient descent with momentum — restates cuda_mlp::CudaGD::solve (src/cuda/gd.cuh:38-106): a
// full-batch loss/grad, then per iteration: stop if ||g|| < tol (:73), v = m*v - lr*g, x += v (:79-82;
// plain x -= lr*g without momentum, :84-85), re-evaluate and record (loss, ||g||) (:87-97).
// T = float mirrors the reference's fp32 scalars (the axpys are FMAs, like cuBLAS saxpy).
// rec: max_iters x 2 (loss, ||g||). Returns the iterations done.
// ---------------------------------------------------------------------------------------------
template <class T, class LG>
int gd_momentum(Vec<T> &x, LG &&loss_grad, T lr, T momentum, int max_iters, T tol, double *rec) {
  const size_t n = x.size();
  Vec<T> g(n), v(n, T(0));
  loss_grad(x, g);
  int done = 0;
  for (int it = 0; it < max_iters; ++it) {
    if (norm(g) < tol) break;
    if (momentum > T(0)) {
      for (size_t j = 0; j < n; ++j) {
        v[j] = std::fma(-lr, g[j], v[j] * momentum);
        x[j] = x[j] + v[j];
      }
    } else {
      for (size_t j = 0; j < n; ++j) x[j] = std::fma(-lr, g[j], x[j]);
    }
    const T loss = loss_grad(x, g);
    rec[2 * done + 0] = double(loss);
    rec[2 * done + 1] = double(norm(g));
    ++done;
  }
  return done;
}

// ---------------------------------------------------------------------------------------------
// Minibatch SGD with momentum and step decay — restates cuda_mlp::CudaSGD::solve (src/cuda/sgd.cuh:
// 50-153): an initial full-batch record (:93-98); per epoch: lr *= decay_rate every decay_step epochs
// (:101-103), contiguous (unshuffled) batches of `batch` rows (:107-112) each followed by the momentum
// update (:115-124), the epoch loss as the batch-size-weighted sum of batch losses (:126), the
// relative-improvement stop when tol > 0 (:129-135), then a full-batch record (:138-148).
// batch_lg(x, g, row0, rows) evaluates rows [row0, row0 + rows). rec: (max_epochs + 1) x 2.
// ---------------------------------------------------------------------------------------------
template <class T, class LG, class BLG>
int sgd_momentum(Vec<T> &x, LG &&full_lg, BLG &&batch_lg, int64_t N, int batch, T lr, T momentum, T decay_rate,
                 int decay_step, int max_epochs, T tol, double *rec) {
  const size_t n = x.size();
  Vec<T> g(n), v(n, T(0));
  int done = 0;
  {
    const T loss = full_lg(x, g);
    rec[2 * done + 0] = double(loss);
    rec[2 * done + 1] = double(norm(g));
    ++done;
  }
  T cur_lr = lr;
  const int64_t nb = (N + batch - 1) / batch;
  T prev = std::numeric_limits<T>::infinity();
  for (int it = 0; it < max_epochs; ++it) {
    if (decay_step > 0 && it > 0 && it % decay_step == 0) cur_lr *= decay_rate;
    T esum = T(0);
    for (int64_t b = 0; b < nb; ++b) {
      const int64_t r0 = b * batch, bs = std::min<int64_t>(batch, N - r0);
      const T bl = batch_lg(x, g, r0, bs);
      if (momentum > T(0)) {
        for (size_t j = 0; j < n; ++j) {
          v[j] = std::fma(-cur_lr, g[j], v[j] * momentum);
          x[j] = x[j] + v[j];
        }
      } else {
        for (size_t j = 0; j < n; ++j) x[j] = std::fma(-cur_lr, g[j], x[j]);
      }
      esum = esum + bl * T(bs);
    }
    const T avg = esum / T(N);
    if (tol > T(0) && std::isfinite(prev)) {
      const T rel = std::abs(prev - avg) / std::max(T(1), std::abs(prev));
      if (rel < tol) break;
    }
    prev = avg;
    const T loss = full_lg(x, g);
    rec[2 * done + 0] = double(loss);
    rec[2 * done + 1] = double(norm(g));
    ++done;
  }
  return done;
}

// ---------------------------------------------------------------------------------------------
// Synthetic data (SURVEY.md §8(d) cfg 1/2 recipe). Shared by the product generator and the oracle;
// tests/test_oracle.py checks the product generator against this one byte for byte.
//   prototypes P_c ~ U[0,1)^In (mt19937(seed)); for each sample: c ~ U{0..classes-1},
//   x = round(255*clip(0.5*P_c + 0.5*U[0,1), 0, 1)) / 255, Y = one-hot(c).
// Output row-major [N][In] / [N][classes] (== the reference's column-major In x N).
// ---------------------------------------------------------------------------------------------
inline void synth_mnist(int64_t N, int In, int classes, unsigned seed, double *X, double *Y) {
  std::mt19937 gen(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<double> proto(size_t(classes) * In);
  for (auto &v : proto) v = U(gen);
  std::uniform_int_distribution<int> C(0, classes - 1);
  for (int64_t b = 0; b < N; ++b) {
    int c = C(gen);
    for (int k = 0; k < classes; ++k) Y[size_t(b) * classes + k] = (k == c) ? 1.0 : 0.0;
    for (int i = 0; i < In; ++i) {
      double v = 0.5 * proto[size_t(c) * In + i] + 0.5 * U(gen);
      v = std::min(1.0, std::max(0.0, v));
      X[size_t(b) * In + i] = std::round(255.0 * v) / 255.0;
    }
  }
}

} // namespace oracle
