// Solver drivers: full-batch L-BFGS (CPU/Wolfe and CUDA/Armijo semantics) and S-LBFGS.
#pragma once

#include "../../include/lbfgs_amd.h"
#include "runtime.hpp"

#include <chrono>
#include <random>

namespace lbf {

// Full-batch L-BFGS on the MLP. All vectors, the (s, y) ring and its Gram state stay on the device;
// the host only reads a 16-double status block once per line-search trial.
class LbfgsSolver {
public:
  LbfgsSolver(Mlp *net, const lbf_lbfgs_params &prm, float *d_params, const float *X, const float *Y,
              long long n_local, long long n_global);
  // Runs up to `iters` iterations. Returns the number run (fewer on convergence).
  int iterate(int iters, lbf_record *rec);
  void info(lbf_solve_info *out) const;
  bool converged() const { return converged_; }

private:
  void eval(const float *x, float *g, const float *pdir); // fused loss+grad, status -> hs_
  void read_status();
  void writeback();
  int iterate_wolfe(int iters, lbf_record *rec);
  int iterate_armijo(int iters, lbf_record *rec);
  void record(lbf_record *rec, double loss, double gnorm, double alpha, int trials, int accepted);

  Mlp *net_;
  Ctx *ctx_;
  lbf_lbfgs_params prm_;
  float *user_params_;
  const float *X_, *Y_;
  long long nloc_, nglob_;
  long long n_;
  History hist_;
  DevBuf<float> xbuf_[3], gbuf_[3], p_;
  float *x_, *xp_, *xt_, *g_, *gp_, *gt_;
  PinnedBuf<double> hs_;
  double loss_ = 0, gg_ = 0;
  float lossf_ = 0;
  int iter_ = 0;
  bool pending_pair_ = false, pending_reset_ = false, converged_ = false;
  int rec_idx_ = 0;
  std::chrono::steady_clock::time_point t0_;
};

class SlbfgsSolver {
public:
  SlbfgsSolver(Mlp *net, const lbf_slbfgs_params &prm, float *d_params, const float *X, const float *Y,
               long long N);
  int run(lbf_record *rec);
  void info(lbf_solve_info *out) const;

private:
  void eval_batch(const float *w, float *g, const int *d_idx, long long count, const float *pdir);
  Mlp *net_;
  Ctx *ctx_;
  lbf_slbfgs_params prm_;
  float *user_params_;
  const float *X_, *Y_;
  long long N_, n_;
  History hist_;
  DevBuf<float> w_, wt_, mu_, g1_, g2_, v_, r_, u_, up_, s_, wp_, wm_, gp_, gm_, wh_;
  DevBuf<int> idx_;
  PinnedBuf<double> hs_;
  int iters_ = 0;
  double last_loss_ = 0, last_gnorm_ = 0;
};

// libstdc++ partial Fisher-Yates (s_lbfgs.hpp:141-160); shared with the ABI helper.
std::vector<size_t> sample_minibatch(size_t N, size_t b, std::mt19937 &rng);

} // namespace lbf
