// The speculative first trial's sufficient-decrease (Armijo) test, shared by the fused tail's decision
// (tail.hip tail_fin_body) and the early test in the trial's first backward GEMM (gemm.hip
// gemm_early_exit), so both take the same decision from the same loss bit for bit.
//   Wolfe  (CPU semantics): fn > f_old + c1 alpha g.p rejects, full_batch_minimizer.hpp:138-141;
//   Armijo (CUDA semantics): fp32 lnew <= f_old + c1 alpha g.p accepts, lbfgs.cuh:159-163.
// L.first (Wolfe iteration 0) takes the trial without a search (lbfgs.hpp:49-52).
#pragma once

#include "kernels.hpp"

#include <hip/hip_runtime.h>

namespace lbf {

// fold_dev: the status block's SC_FOLD (Wolfe) / SC_FOLDF (Armijo); gfo: its SC_GTP
__device__ __forceinline__ bool ls_sufficient_decrease(const LsCtlArgs &L, double fn, double fold_dev, double gfo) {
  if (!L.armijo) {
    const double fo = L.host_fold ? L.fold : fold_dev;
    return L.first || !(fn > __dadd_rn(fo, __dmul_rn(__dmul_rn(L.c1, L.alpha), gfo)));
  }
  const float foldf = L.host_fold ? L.foldf : float(fold_dev);
  const float lnew = float(fn), gdp = float(gfo);
  return lnew <= __fadd_rn(foldf, __fmul_rn(__fmul_rn(float(L.c1), L.alphaf), gdp));
}

} // namespace lbf
