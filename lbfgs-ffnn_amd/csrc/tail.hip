// Fused optimizer tail of a speculative L-BFGS iteration (see TailArgs in kernels.hpp).
//
// Replaces, on the fast path (first trial accepted), the sequence reduce_all -> finish -> ls_ctl ->
// gram sweep -> history step by three launches:
//   tail_reduce  (one block per 64-column group): the gradient column from its split-K slabs (or as
//                written), s = x_t - x_prev and y = g_t - g_prev stored into the ring's write slot,
//                and the Gram sweep of (s, y, g_t) against every live history vector -> one row of
//                partial dots per block;
//   tail_cols    (one block per dot column): fixed-order reduction of the rows;
//   tail_fin     (one block): loss and status block, the line-search decision with its host record
//                (ls_ctl's rule), and on acceptance the push + two-loop coefficients (hist_core.hpp).
// The reference's counterpart is one LBFGS::solve iteration after its line search
// (lbfgs.hpp:77-98 / lbfgs.cuh:143-190) with the gradient of MLPObjective / CudaNetwork.
#include "hist_core.hpp"
#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace lbf {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double t_wave_sum(double v) { return wave_sum_f64(v); }

// One 64-column group per block. Wave w owns split stripe w of the slab reduction and history vectors
// v = w + 4j (v < count: S_{L[v]}, else Y_{L[v-count]}; VPW per wave). Every global load of the block
// (history values, slabs, operands) is issued before the first use: one round trip, then LDS.
template <int VPW>
__global__ __launch_bounds__(256) void tail_reduce_kernel(const TailArgs a) {
  const RedAllArgs &ra = a.ra;
  if (ra.abort && *ra.abort) return;
  __shared__ double part[4][RA_COLS];
  __shared__ float lsv[RA_COLS], lyv[RA_COLS], lgv[RA_COLS];
  __shared__ int ist[IST_ORDER + TAIL_MAXM];
  const HistView &h = a.h;
  const int t = threadIdx.x, lane = t & 63, stripe = t >> 6, wave = stripe;
  KT(48);
  KTB(0);
#ifdef LBF_KTRACE
  if (t == 0 && blockIdx.x >= 1024 && blockIdx.x < 2048) lbf_kt_blk[5 * 1024 + blockIdx.x - 1024] = wall_clock64();
#endif
  // the ring header in one round trip (count, free slot, order)
  if (t < IST_ORDER + h.m) ist[t] = h.ist[t];
  __syncthreads();
  KTB(1);
  const int count0 = ist[IST_COUNT];
  const int w = hist_write_slot(ist, h.m, a.policy, 0);
  if (blockIdx.x == 0 && t == 0) h.ist[IST_WSLOT] = w;
  const int nvec = 2 * count0;
  const int cg = blockIdx.x;
  int si = 0;
  while (si + 1 < ra.nseg && ra.seg[si + 1].cg0 <= cg) ++si;
  const RedSeg &S = ra.seg[si];
  const long long col = (long long)(cg - S.cg0) * RA_COLS + lane;
  const bool live = col < S.count;
  const long long e = S.goff + col;
  // ---- history values of this wave's vectors (in flight while the slabs load) ----
  float vv[VPW];
#pragma unroll
  for (int j = 0; j < VPW; ++j) {
    const int v = wave + 4 * j;
    vv[j] = 0.0f;
    if (v < nvec && live) {
      const int slot = ist[IST_ORDER + (v < count0 ? v : v - count0)];
      if (!(a.has_pair && slot == w)) vv[j] = (v < count0 ? h.S : h.Y)[(long long)slot * h.ld + e];
    }
  }
  // ---- operands (wave 0) ----
  float wv = 0.f, xp = 0.f, gp = 0.f, pv = 0.f, gw = 0.f;
  if (wave == 0 && live) {
    wv = ra.w[e];
    if (a.has_pair) {
      xp = a.x_prev[e];
      gp = a.g_prev[e];
    }
    if (ra.p) pv = ra.p[e];
    if (S.splits == 0) gw = ra.G[e];
  }
  KT(49);
  // ---- gradient column: split-K slabs in split order (4 stripes) ----
  double acc = 0.0;
  if (live && S.splits > 0) {
    const float *src = S.slab + col;
    for (int k = stripe; k < S.splits; k += 4 * 16) { // sixteen independent loads in flight
      float x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) x[u] = k + 4 * u < S.splits ? src[(long long)(k + 4 * u) * S.stride] : 0.0f;
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (k + 4 * u < S.splits) acc += double(x[u]);
    }
  }
  KT(50);
  part[stripe][lane] = acc;
  __syncthreads();
  KT(51);
  KTB(2);
  double *row = a.rows + (long long)blockIdx.x * a.nc;
  if (wave == 0) {
    float gv = 0.f, sv = 0.f, yv = 0.f;
    double sf[8] = {0, 0, 0, 0, 0, 0, 0, 0}; // s.s s.y y.y g.s g.y g.g g.p w.w
    if (live) {
      gv = S.splits > 0 ? float(((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]) : gw;
      if (ra.lambda != 0.0) gv = gv + float(ra.lambda) * wv; // finalize_kernel's update
      if (S.splits > 0 || ra.lambda != 0.0) ra.G[e] = gv;
      if (a.has_pair) {
        sv = wv - xp;
        yv = gv - gp;
        h.S[(long long)w * h.ld + e] = sv;
        h.Y[(long long)w * h.ld + e] = yv;
      }
      const double s = sv, y = yv, g = gv;
      sf[0] = s * s;
      sf[1] = s * y;
      sf[2] = y * y;
      sf[3] = g * s;
      sf[4] = g * y;
      sf[5] = g * g;
      sf[6] = g * double(pv);
      sf[7] = double(wv) * double(wv);
    }
    lsv[lane] = sv;
    lyv[lane] = yv;
    lgv[lane] = gv;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const double x = t_wave_sum(sf[q]);
      if (lane == 0) row[6 * h.m + q] = x;
    }
  }
  KT(52);
  __syncthreads();
  KT(53);
  KTB(3);
  // ---- Gram sweep of this column group ----
  const double s = lsv[lane], y = lyv[lane], g = lgv[lane];
#pragma unroll
  for (int j = 0; j < VPW; ++j) {
    const int v = wave + 4 * j;
    if (v < nvec) { // wave-uniform
      const double x = vv[j];
      const double d0 = t_wave_sum(x * s), d1 = t_wave_sum(x * y), d2 = t_wave_sum(x * g);
      if (lane == 0) {
        const int i = v < count0 ? v : v - count0, c = v < count0 ? 0 : 1;
        row[6 * i + c + 0] = d0; // S_i.s | Y_i.s
        row[6 * i + c + 2] = d1; // S_i.y | Y_i.y
        row[6 * i + c + 4] = d2; // S_i.g | Y_i.g
      }
    }
  }
  KT(54);
  KTB(4);
#ifdef LBF_KTRACE
  if (t == 0 && blockIdx.x >= 1024 && blockIdx.x < 2048) lbf_kt_blk[6 * 1024 + blockIdx.x - 1024] = wall_clock64();
#endif
}

// dots[c] = sum over rows in row order (per-thread strided rows, then a fixed tree).
__global__ __launch_bounds__(256) void tail_cols_kernel(const TailArgs a) {
  if (a.ra.abort && *a.ra.abort) return;
  __shared__ double ws[4];
  const int c = blockIdx.x, t = threadIdx.x;
  const int count0 = a.h.ist[IST_COUNT];
  // only the columns in use (live pairs and the self block)
  if (c < 6 * a.h.m && c >= 6 * count0) return;
  double v[8];
  double s = 0.0;
  for (int r0 = t; r0 < a.nb; r0 += 256 * 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + 256 * u;
      v[u] = r < a.nb ? a.rows[(long long)r * a.nc + c] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  s = t_wave_sum(s);
  if ((t & 63) == 0) ws[t >> 6] = s;
  __syncthreads();
  if (t == 0) a.dots[c] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

constexpr int TF_THREADS = 256;

__global__ __launch_bounds__(TF_THREADS) void tail_fin_kernel(const TailArgs a) {
  const RedAllArgs &ra = a.ra;
  if (ra.abort && *ra.abort) return;
  extern __shared__ double dyn[]; // sy [2*m*m] (SY and its transpose) | yy [m*m]
  __shared__ HistSmem sm;
  __shared__ double v[4];
  __shared__ int s_status;
  const HistView &h = a.h;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // ---- status: dots and the SSE (partials on one rank, the all-reduced pair otherwise) ----
  KT(40);
  const double *D = a.dots;
  const int m = h.m;
  {
    double sse = 0.0;
    if (!a.hilo)
      for (int r = t; r < ra.nsse; r += TF_THREADS) sse += ra.sse_part[r];
    sse = t_wave_sum(sse);
    if (lane == 0) v[wave] = sse;
  }
  __syncthreads();
  double *sc = h.scal;
  if (t == 0) {
    const double sse = a.hilo ? (double(a.hilo[0]) + double(a.hilo[1])) : ((v[0] + v[1]) + v[2]) + v[3];
    const double tgg = D[6 * m + 5], tgp = D[6 * m + 6], ww = D[6 * m + 7];
    double loss = 0.5 * sse * ra.inv_scale;
    if (ra.lambda != 0.0) loss += 0.5 * ra.lambda * ww;
    sc[SC_TGG] = tgg;
    sc[SC_TGP] = tgp;
    sc[SC_WW] = ww;
    sc[SC_SSE] = sse;
    sc[SC_LOSS] = loss;
    // ---- the line-search decision (ls_ctl_kernel's rule, vec_kernels.hip) ----
    const LsCtlArgs &L = a.ls;
    const double fn = loss, gfo = sc[SC_GTP];
    bool ok, conv;
    if (!L.armijo) {
      const double fold = L.host_fold ? L.fold : sc[SC_FOLD];
      ok = L.first || (!(fn > __dadd_rn(fold, __dmul_rn(__dmul_rn(L.c1, 1.0), gfo))) && !(tgp < __dmul_rn(L.c2, gfo)));
      conv = sqrt(tgg) < L.tol;
      if (ok) sc[SC_FOLD] = fn;
    } else {
      const float foldf = L.host_fold ? L.foldf : float(sc[SC_FOLDF]);
      const float lnew = float(fn), gdp = float(gfo);
      ok = lnew <= __fadd_rn(foldf, __fmul_rn(__fmul_rn(float(L.c1), L.alphaf), gdp));
      conv = float(sqrt(tgg)) < float(L.tol);
      if (ok) sc[SC_FOLDF] = double(lnew);
    }
    const int status = !ok ? SPEC_REJECT : (conv ? SPEC_CONVERGED : SPEC_ACCEPT);
    if (status != SPEC_ACCEPT) *L.abort = 1;
    SpecRecord *r = L.rec;
    const double alpha0 = sc[SC_ALPHA0], accept_prev = sc[SC_ACCEPT];
    __hip_atomic_store(&r->loss, fn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->tgg, tgg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->alpha0, alpha0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->accept_prev, accept_prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->status, status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&r->seq, L.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s_status = status;
  }
  __syncthreads();
  KT(41);
  // Rejected: history untouched (the host finishes the line search). Converged: the solver stops
  // before the next history update, exactly like the host-driven loop.
  if (s_status != SPEC_ACCEPT) return;
  // ---- accepted: push the pair, coefficients of the next direction ----
  HistStep st;
  st.h = h;
  st.has_pair = a.has_pair;
  st.has_g = 1;
  st.reset = 0;
  st.policy = a.policy;
  st.want_dir = 1;
  st.iter = a.iter_next;
  st.dsign = -1.0;
  hist_prologue(st, sm, h.ist[IST_WSLOT]);
  KT(42);
  const int count0 = sm.count0;
  for (int q = t; q < 6 * count0; q += TF_THREADS) sm.dots[q] = D[q];
  if (t < 6) sm.dots[6 * m + t] = D[6 * m + t];
  __syncthreads();
  KT(43);
  hist_core(st, sm, dyn, 2 * m * m, dyn + 2 * m * m, m * m);
  KT(44);
}

} // namespace

int tail_vpw(int m) {
  const int per_wave = (2 * m + 3) / 4;
  if (m > TAIL_MAXM) return 0;
  return per_wave <= 2 ? 2 : per_wave <= 4 ? 4 : per_wave <= 8 ? 8 : 16;
}

void tail_reduce(hipStream_t s, const TailArgs &a) {
  if (a.nb <= 0) return;
  switch (tail_vpw(a.h.m)) {
  case 2: hipLaunchKernelGGL(tail_reduce_kernel<2>, dim3(unsigned(a.nb)), dim3(256), 0, s, a); break;
  case 4: hipLaunchKernelGGL(tail_reduce_kernel<4>, dim3(unsigned(a.nb)), dim3(256), 0, s, a); break;
  case 8: hipLaunchKernelGGL(tail_reduce_kernel<8>, dim3(unsigned(a.nb)), dim3(256), 0, s, a); break;
  case 16: hipLaunchKernelGGL(tail_reduce_kernel<16>, dim3(unsigned(a.nb)), dim3(256), 0, s, a); break;
  default: throw Error(2, "tail_reduce: history size not supported by the fused tail");
  }
  LBF_KERNEL_CHECK();
  hipLaunchKernelGGL(tail_cols_kernel, dim3(unsigned(a.nc)), dim3(256), 0, s, a);
  LBF_KERNEL_CHECK();
}

void tail_fin(hipStream_t s, const TailArgs &a) {
  const size_t shmem = size_t(3) * a.h.m * a.h.m * sizeof(double);
  hipLaunchKernelGGL(tail_fin_kernel, dim3(1), dim3(TF_THREADS), shmem, s, a);
  LBF_KERNEL_CHECK();
}

} // namespace lbf

#ifdef LBF_KTRACE
extern "C" int lbf_dbg_ktrace_tail(unsigned long long *host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lbf::lbf_kt_buf), size_t(n) * 8) == hipSuccess ? 0 : 1;
}
extern "C" int lbf_dbg_ktrace_tail_blk(unsigned long long *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lbf::lbf_kt_blk), sizeof(lbf::lbf_kt_blk)) == hipSuccess ? 0 : 1;
}
#endif
