// The reference's known-answer problems (tests/main.cpp: Rosenbrock n=4, Ackley n=3) minimised by
// hip_mlp::HipLBFGS through the generic LossGradFun path (CudaMinimizerBase::solve contract,
// minimizer_base.cuh:15-16, 54-59): the objective is evaluated on the host from device buffers and
// the engine keeps the history, two-loop and line search on the device. fp32, so the thresholds are
// the fp32 analogues of the reference's (which are for fp64).
#include "lbfgs_amd/hip_backend.hpp"

#include <cmath>
#include <cstdio>
#include <vector>

using hip_mlp::HipScalar;

static double rosen(const std::vector<double> &v, std::vector<double> &g) {
  const int n = int(v.size());
  double f = 0.0;
  g.assign(n, 0.0);
  for (int i = 0; i < n - 1; ++i) {
    const double t1 = v[i + 1] - v[i] * v[i], t2 = 1.0 - v[i];
    f += 100.0 * t1 * t1 + t2 * t2;
    g[i] += -400.0 * v[i] * t1 - 2.0 * t2;
    g[i + 1] += 200.0 * t1;
  }
  return f;
}

int main() {
  hip_mlp::HipHandle h;
  const int n = 4;
  hip_mlp::DeviceBuffer<HipScalar> x(h, n);
  const std::vector<HipScalar> x0 = {-1.2f, 1.0f, -1.2f, 1.0f};
  int fails = 0;
  for (int ls : {LBF_LS_WOLFE, LBF_LS_ARMIJO}) {
    x.copy_from_host(x0.data(), n);
    auto loss_grad = [&](const HipScalar *p, HipScalar *grad, const HipScalar *, const HipScalar *, int) {
      std::vector<HipScalar> hp(n), hg(n);
      hip_mlp::hip_check(lbf_memcpy(h.get(), hp.data(), p, n * sizeof(HipScalar), 1), "d2h");
      std::vector<double> v(hp.begin(), hp.end()), gd;
      const double f = rosen(v, gd);
      for (int i = 0; i < n; ++i) hg[i] = HipScalar(gd[i]);
      hip_mlp::hip_check(lbf_memcpy(h.get(), grad, hg.data(), n * sizeof(HipScalar), 0), "h2d");
      return HipScalar(f);
    };
    hip_mlp::HipLBFGS opt(h);
    opt.setMemory(16);
    opt.setLineSearch(ls);
    opt.setMaxIterations(4000);
    opt.setTolerance(1e-5f);
    opt.solve(n, x.data(), nullptr, nullptr, 0, loss_grad);
    std::vector<HipScalar> r(n);
    x.copy_to_host(r.data(), n);
    double dist = 0.0;
    for (int i = 0; i < n; ++i) dist += (r[i] - 1.0) * (r[i] - 1.0);
    dist = std::sqrt(dist);
    std::printf("[RESULT] rosenbrock ls=%d iters=%d x=(%g,%g,%g,%g) dist=%.3e\n", ls, opt.iterations(), r[0], r[1],
                r[2], r[3], dist);
    if (!(dist < 1e-3)) ++fails;
  }
  std::printf("[RESULT] %s\n", fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}
