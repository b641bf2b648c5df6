// Fused optimizer tail of a speculative L-BFGS iteration (see TailArgs in kernels.hpp).
//
// Replaces, on the fast path (first trial accepted), the sequence reduce_all -> finish -> ls_ctl ->
// gram sweep -> history step by two launches:
//   tail_reduce    (one block per 128-column group): the gradient column from its split-K slabs (or as
//                  written), s = x_t - x_prev and y = g_t - g_prev stored into the ring's write slot,
//                  and the Gram sweep of (s, y, g_t) against every live history vector -> one row of
//                  partial dots per block;
//   tail_cols_fin  (one block per dot column): fixed-order reduction of the rows; the last block to
//                  arrive then runs the one-block fin: loss and status block, the line-search decision
//                  with its host record (ls_ctl's rule), and on acceptance the push + two-loop
//                  coefficients (hist_core.hpp).
// The reference's counterpart is one LBFGS::solve iteration after its line search
// (lbfgs.hpp:77-98 / lbfgs.cuh:143-190) with the gradient of MLPObjective / CudaNetwork.
#include "hist_core.hpp"
#include "internal.hpp"
#include "kernels.hpp"
#include "ls_rule.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace lbf {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double t_wave_sum(double v) { return wave_sum_f64(v); }

// Barriers are LDS-only (wave.hpp lds_barrier): no thread reads global memory that another thread of
// its block wrote in the same launch.
//
// One TAIL_COLS (128) column group per block, lane l owning columns l and l + 64 of it. Wave w owns
// split stripe w of the slab reduction and history vectors v = w + 4j (v < count: S_{L[v]}, else
// Y_{L[v-count]}; VPW per wave). Every global load of the block (history values, slabs, operands)
// is issued before the first use: one round trip, then LDS. The block's dots are then reduced out of
// LDS with four lanes per dot column (32 exact fp64 products each, then a quad DPP add): no
// per-vector 64-lane reductions. Rows are stored transposed, [nc][nb], so tail_cols reads each
// column contiguously. 128-column groups halve the grid (n = 101,770: 796 blocks), which keeps every
// block resident at once (this kernel's SGPR count admits 6 blocks per CU).
template <int VPW, int U>
__global__ __launch_bounds__(256) void tail_reduce_kernel(const TailArgs a) {
  constexpr int TC = TAIL_COLS, C = TAIL_COLS / 64;
  const RedAllArgs &ra = a.ra;
  // the speculative chain's abort flag: requested with the ring header (one round trip for both) and tested
  // before the block's history and slab loads, so an aborted launch exits after that round trip
  const int abf = abort_flag(ra.abort);
  __shared__ double part[4][TC];
  __shared__ float xs[2 * TAIL_MAXM][TC]; // this group's values of the live history vectors
  __shared__ float ops[5][TC];            // s, y, g, p, w
  __shared__ int ist[IST_ORDER + TAIL_MAXM];
  const HistView &h = a.h;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6), stripe = wave; // uniform: scalar branches
  KT(48);
  KTB(0);
#ifdef LBF_KTRACE
  if (t == 0 && blockIdx.x >= 1024 && blockIdx.x < 2048) lbf_kt_blk[5 * 1024 + blockIdx.x - 1024] = wall_clock64();
#endif
  // This block's column group and segment: kernel arguments only, so the loads that need no ring order (the
  // operands and the first round of split-K slabs) go out right behind the ring header's, in the same round trip.
  const int cg = blockIdx.x;
  int si = 0;
  while (si + 1 < ra.nseg && a.tcg0[si + 1] <= cg) ++si;
  const RedSeg &S = ra.seg[si];
  // Every load below is unconditional, from an address clamped into the arrays, and masked after:
  // a per-element "load or zero" select makes the compiler branch around each load and wait for it
  // (one dependent round trip per element).
  long long col[C], colc[C], e[C];
  bool live[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    col[c] = (long long)(cg - a.tcg0[si]) * TC + lane + 64 * c;
    live[c] = col[c] < S.count;
    colc[c] = live[c] ? col[c] : S.count - 1;
    e[c] = S.goff + colc[c];
  }
  // the ring header (count, free slot, order): issued first, so waiting for it waits for nothing issued after
  const int istv = t < IST_ORDER + h.m ? h.ist[t] : 0;
  // ---- operands ----
  // every wave loads them (same lines as wave 0's: L1 hits) so no branch merge forces an early wait;
  // null operands read w instead and are masked where used
  float wv[C], xp[C], gp[C], pv[C], gw[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    wv[c] = ra.w[e[c]];
    xp[c] = (a.x_prev ? a.x_prev : ra.w)[e[c]];
    gp[c] = (a.g_prev ? a.g_prev : ra.w)[e[c]];
    pv[c] = (ra.p ? ra.p : ra.w)[e[c]];
    gw[c] = (a.g_src ? a.g_src : ra.G)[e[c]];
  }
  // ---- gradient columns: split-K slabs in split order (4 stripes); U loads per column in flight per round
  // (clamped duplicates past the end): every slab of the launch in one round where that fits the registers
  // (tail_reduce: U = 24 for up to 96 splits at VPW <= 8). The first round of 8 is requested here; a round of 24
  // held across the header's wait would take the kernel past 128 VGPRs (3 blocks per CU), so it goes out below. ----
  constexpr bool EARLY = U <= 8;
  float x0[EARLY ? U : 1][C];
  if constexpr (EARLY) {
    if (S.splits > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long sp = min(stripe + 4 * u, S.splits - 1);
#pragma unroll
        for (int c = 0; c < C; ++c) x0[u][c] = S.slab[colc[c] + sp * S.stride];
      }
    }
  }
  if (t < IST_ORDER + h.m) ist[t] = istv;
  lds_barrier();
  if (aborted(abf)) return; // uniform for the launch: no store, no arrival
  KTB(1);
  // wave-uniform scalars (SGPRs): the loads below then need no per-lane select or branch
  const int count0 = __builtin_amdgcn_readfirstlane(ist[IST_COUNT]);
  const int w = __builtin_amdgcn_readfirstlane(hist_write_slot(ist, h.m, a.policy, 0));
  const int nvec = 2 * count0;
  // ---- history values of this wave's vectors ----
  const float *Sb = h.S, *Yb = h.Y;
  float vv[VPW][C];
  unsigned zero_mask = 0; // bit j: vector j of this wave is the slot being overwritten (not live)
#pragma unroll
  for (int j = 0; j < VPW; ++j) {
    const int v = wave + 4 * j; // wave-uniform
    const int vi = v < nvec ? v : 0;
    const int slot = __builtin_amdgcn_readfirstlane(ist[IST_ORDER + (vi < count0 ? vi : vi - count0)]);
    const float *base = (vi < count0 ? Sb : Yb) + (long long)slot * h.ld;
#pragma unroll
    for (int c = 0; c < C; ++c) vv[j][c] = base[e[c]];
    if (v >= nvec || (a.has_pair && slot == w)) zero_mask |= 1u << j;
  }
  KT(49);
  double acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.0;
  if (S.splits > 0) {
    int k0 = stripe;
    if constexpr (EARLY) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c)
          if (stripe + 4 * u < S.splits) acc[c] += double(x0[u][c]);
      k0 += 4 * U;
    }
    for (int k = k0; k < S.splits; k += 4 * U) { // (EARLY: the rounds after the first)
      float x[U][C];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long sp = min(k + 4 * u, S.splits - 1);
#pragma unroll
        for (int c = 0; c < C; ++c) x[u][c] = S.slab[colc[c] + sp * S.stride];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c)
          if (k + 4 * u < S.splits) acc[c] += double(x[u][c]);
    }
  }
  if (blockIdx.x == 0 && t == 0) h.ist[IST_WSLOT] = w;
  KT(50);
#pragma unroll
  for (int c = 0; c < C; ++c) part[stripe][lane + 64 * c] = acc[c];
#pragma unroll
  for (int j = 0; j < VPW; ++j) {
    const int v = wave + 4 * j;
    if (v < nvec)
#pragma unroll
      for (int c = 0; c < C; ++c) xs[v][lane + 64 * c] = ((zero_mask >> j) & 1u) || !live[c] ? 0.0f : vv[j][c];
  }
  lds_barrier();
  KT(51);
  KTB(2);
  if (wave == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int q = lane + 64 * c;
      float gv = 0.f, sv = 0.f, yv = 0.f;
      if (live[c]) {
        gv = S.splits > 0 ? float(((part[0][q] + part[1][q]) + part[2][q]) + part[3][q]) : gw[c];
        if (ra.lambda != 0.0) gv = gv + float(ra.lambda) * wv[c]; // finalize_kernel's update
        if (S.splits > 0 || ra.lambda != 0.0 || a.g_src) ra.G[e[c]] = gv;
        if (a.has_pair) {
          sv = wv[c] - xp[c];
          yv = gv - gp[c];
          h.S[(long long)w * h.ld + e[c]] = sv;
          h.Y[(long long)w * h.ld + e[c]] = yv;
        }
      }
      ops[0][q] = sv;
      ops[1][q] = yv;
      ops[2][q] = gv;
      ops[3][q] = ra.p ? pv[c] : 0.f;
      ops[4][q] = live[c] ? wv[c] : 0.f;
    }
  }
  lds_barrier();
  KT(52);
  KTB(3);
  // ---- dot columns: 4 lanes per column, 32 exact fp64 products each, fixed order ----
  // history columns 6i + {0..5}: S_i.s, Y_i.s, S_i.y, Y_i.y, S_i.g, Y_i.g ; then the 8 self columns
  // s.s s.y y.y g.s g.y g.g g.p w.w at 6m + q.
  const int nh = 6 * count0, ncu = nh + 8;
  const int q = t & 3;
  for (int base = 0; base < 4 * ncu; base += 256) {
    const int u = (base + t) >> 2;
    double d = 0.0;
    int c = -1;
    if (u < ncu) {
      const float *A, *B;
      if (u < nh) {
        const int i = u / 6, r = u - 6 * i;
        A = xs[(r & 1) ? count0 + i : i];
        B = ops[r >> 1];
        c = u;
      } else {
        const int z = u - nh; // (s,s) (s,y) (y,y) (g,s) (g,y) (g,g) (g,p) (w,w)
        const int ia = (0x42222100 >> (4 * z)) & 0xF, ib = (0x43210110 >> (4 * z)) & 0xF;
        A = ops[ia];
        B = ops[ib];
        c = 6 * h.m + z;
      }
      const f32x4 *A4 = reinterpret_cast<const f32x4 *>(A + (TC / 4) * q);
      const f32x4 *B4 = reinterpret_cast<const f32x4 *>(B + (TC / 4) * q);
#pragma unroll
      for (int k = 0; k < TC / 16; ++k) {
        const f32x4 x = A4[k], y = B4[k];
        d += double(x[0]) * double(y[0]);
        d += double(x[1]) * double(y[1]);
        d += double(x[2]) * double(y[2]);
        d += double(x[3]) * double(y[3]);
      }
    }
    d += dpp_f64<0xB1, 0xF>(d); // quad_perm [1,0,3,2]
    d += dpp_f64<0x4E, 0xF>(d); // quad_perm [2,3,0,1]: every lane of the quad holds the same sum
    if (c >= 0 && q == 0) a.rows[(long long)c * a.nb + blockIdx.x] = d;
  }
  KT(54);
  KTB(4);
#ifdef LBF_KTRACE
  if (t == 0 && blockIdx.x >= 1024 && blockIdx.x < 2048) lbf_kt_blk[6 * 1024 + blockIdx.x - 1024] = wall_clock64();
#endif
}

// dots[c] = sum over rows in row order (per-thread strided rows, then a fixed tree); rows are stored
// transposed ([nc][nb]), so each block reads one contiguous column. The sum is
// stored write-through (agent-scope relaxed store = sc1) and waited for, so the arrival counter's add
// publishes it without a release fence (MI355X_MICROARCH.md hand-off table, first row).
__device__ __forceinline__ void tail_cols_body(const TailArgs &a, int abf) {
  __shared__ double ws[4];
  const int c = blockIdx.x, t = threadIdx.x;
  const int count0 = a.h.ist[IST_COUNT]; // in flight with the caller's abort flag
  if (aborted(abf)) return;
  // only the columns in use (live pairs and the self block)
  if (c < 6 * a.h.m && c >= 6 * count0) return;
  const double *colp = a.rows + (long long)c * a.nb;
  double v[8];
  double s = 0.0;
  for (int r0 = t; r0 < a.nb; r0 += 256 * 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) { // unconditional loads from clamped rows: all eight in flight at once
      const int r = r0 + 256 * u;
      v[u] = colp[r < a.nb ? r : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (r0 + 256 * u < a.nb) ? v[u] : 0.0;
  }
  s = t_wave_sum(s);
  if ((t & 63) == 0) ws[t >> 6] = s;
  lds_barrier();
  if (t == 0) {
    const double d = ((ws[0] + ws[1]) + ws[2]) + ws[3];
    __hip_atomic_store(&a.dots[c], d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

constexpr int TF_THREADS = 256;

// One block. Every global value it needs (dot columns, SSE partials, status words, ring header, rho,
// SY, YY) is requested up front in one round trip and staged in LDS; hist_core then runs from LDS.
// Wave 0 (decision, then the recurrences) issues no global store until the coefficients: the status
// block, the host record (system-scope stores to host-mapped memory, whose acknowledgement the
// sequence word must wait for) and the history step's ring/Gram writes are made by waves 1..3.
__device__ __forceinline__ void tail_fin_body(const TailArgs &a) {
  const RedAllArgs &ra = a.ra;
  extern __shared__ double dyn[]; // sy [2*m*m] (SY and its transpose) | yy [m*m] | SY, YY [S*S] | rho [S]
  __shared__ HistSmem sm;
  __shared__ double v[4];
  __shared__ double s_rec[4]; // loss, tgg, alpha0, accept_prev
  __shared__ double s_sc[6];  // tgg, tgp, ww, sse, loss, the new f_old
  __shared__ int s_status, s_ok;
  __shared__ int ist_l[IST_ORDER + TAIL_MAXM + 4];
  const HistView &h = a.h;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m = h.m, S_ = h.slots;
  double *SYp = dyn + 3 * m * m, *YYp = SYp + S_ * S_, *rhop = YYp + S_ * S_;
  double *sc = h.scal;
  KTF(40);
  // ---- prefetch (one round trip) ----
  double sse = 0.0;
  if (!a.hilo)
    for (int r = t; r < ra.nsse; r += TF_THREADS) sse += ra.sse_part[r];
  for (int q = t; q < a.nc; q += TF_THREADS) // sc1 loads: written this launch by other blocks (hand-off)
    sm.dots[q] = __hip_atomic_load(&a.dots[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int i = t; i < S_ * S_; i += TF_THREADS) {
    SYp[i] = h.SY[i];
    YYp[i] = h.YY[i];
  }
  if (t < S_) rhop[t] = h.rho[t];
  if (t < IST_ORDER + m) ist_l[t] = h.ist[t];
  double gfo = 0.0, fold = 0.0, alpha0 = 0.0, accept_prev = 0.0;
  if (t == 0) {
    gfo = sc[SC_GTP];
    fold = a.ls.armijo ? sc[SC_FOLDF] : sc[SC_FOLD];
    alpha0 = sc[SC_ALPHA0];
    accept_prev = sc[SC_ACCEPT];
  }
  sse = t_wave_sum(sse);
  if (lane == 0) v[wave] = sse;
  KTF(45);
  lds_barrier();
  KTF(46);
  if (t == 0) { // decide (LDS only: wave 0 issues no global store before the recurrences)
    const double *D = sm.dots;
    const double sse_t = a.hilo ? (double(a.hilo[0]) + double(a.hilo[1])) : ((v[0] + v[1]) + v[2]) + v[3];
    const double tgg = D[6 * m + 5], tgp = D[6 * m + 6], ww = D[6 * m + 7];
    double loss = 0.5 * sse_t * ra.inv_scale;
    if (ra.lambda != 0.0) loss += 0.5 * ra.lambda * ww;
    s_sc[0] = tgg;
    s_sc[1] = tgp;
    s_sc[2] = ww;
    s_sc[3] = sse_t;
    s_sc[4] = loss;
    // ---- the line-search decision (ls_ctl_kernel's rule, vec_kernels.hip) ----
    const LsCtlArgs &L = a.ls;
    const double fn = loss;
    bool ok, conv;
    // (the sufficient-decrease half is ls_rule.hpp's, which the trial's first backward GEMM applied already
    // when EarlyLs was on: a trial that reaches this block passed it there)
    ok = ls_sufficient_decrease(L, fn, fold, gfo);
    if (!L.armijo) {
      ok = L.first || (ok && !(tgp < __dmul_rn(L.c2, gfo)));
      conv = sqrt(tgg) < L.tol;
      s_sc[5] = fn;
    } else {
      conv = float(sqrt(tgg)) < float(L.tol);
      s_sc[5] = double(float(fn));
    }
    s_ok = ok ? 1 : 0;
    s_rec[0] = fn;
    s_rec[1] = tgg;
    s_rec[2] = alpha0;
    s_rec[3] = accept_prev;
    s_status = !ok ? SPEC_REJECT : (conv ? SPEC_CONVERGED : SPEC_ACCEPT);
  }
  lds_barrier();
  KTF(41);
  // status block, abort flag and host record: payload, then (after its acknowledgement) the
  // sequence word. Written by wave 1 after its last barrier (see hist_core<true>).
  auto publish = [&]() {
    sc[SC_TGG] = s_sc[0];
    sc[SC_TGP] = s_sc[1];
    sc[SC_WW] = s_sc[2];
    sc[SC_SSE] = s_sc[3];
    sc[SC_LOSS] = s_sc[4];
    if (s_ok) sc[a.ls.armijo ? SC_FOLDF : SC_FOLD] = s_sc[5];
    if (s_status != SPEC_ACCEPT) *a.ls.abort = 1;
    SpecRecord *r = a.ls.rec;
    __hip_atomic_store(&r->loss, s_rec[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->tgg, s_rec[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->alpha0, s_rec[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->accept_prev, s_rec[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->status, s_status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&r->seq, a.ls.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  // Rejected: history untouched (the host finishes the line search). Converged: the solver stops
  // before the next history update, exactly like the host-driven loop.
  if (s_status != SPEC_ACCEPT) {
    if (t == 64) publish();
    return;
  }
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
  st.ist = ist_l;
  st.rho = rhop;
  st.SY = SYp;
  st.YY = YYp;
  hist_prologue<true>(st, sm, ist_l[IST_WSLOT]);
  KTF(42);
  KTF(43);
  hist_core<true>(st, sm, dyn, 2 * m * m, dyn + 2 * m * m, m * m);
  // waves 1..3 leave hist_core after its deferred stores; wave 1 then publishes
  if (t == 64) publish();
  KTF(44);
}

// tail_cols, then (cols_done) the last block to finish runs the one-block fin: one launch fewer on
// the iteration's critical path. Hand-off without fences (the guide prices __threadfence at ~3.5 us):
// each block's column sum is an sc1 (write-through) store waited for with vmcnt(0) before the same lane's
// agent-scope add; the block whose add returns the last count reads the sums with sc1 loads.
__global__ __launch_bounds__(TF_THREADS) void tail_cols_fin_kernel(const TailArgs a) {
  const int abf = abort_flag(a.ra.abort);
  KT(39);
  tail_cols_body(a, abf);
  if (aborted(abf)) return; // uniform for the launch: nobody arrives, the counter stays 0
  __shared__ int s_last;
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(a.cols_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) *a.cols_done = 0u; // ready for the next launch (stream-ordered)
  tail_fin_body(a);
}

} // namespace

int tail_vpw(int m) {
  const int per_wave = (2 * m + 3) / 4;
  if (m > TAIL_MAXM) return 0;
  return per_wave <= 2 ? 2 : per_wave <= 4 ? 4 : per_wave <= 8 ? 8 : 16;
}

static size_t fin_shmem(const TailArgs &a) {
  return (size_t(3) * a.h.m * a.h.m + 2 * size_t(a.h.slots) * a.h.slots + a.h.slots) * sizeof(double);
}

void tail_reduce(hipStream_t s, const TailArgs &a) {
  if (a.nb <= 0) return;
  int max_splits = 0;
  for (int i = 0; i < a.ra.nseg; ++i) max_splits = std::max(max_splits, a.ra.seg[i].splits);
  // more than 32 slabs (cfg 2: 82): 24 per stripe in one round instead of rounds of 8 (registers: VPW <= 8 only;
  // 13.6 -> 12.8 us at cfg 2, profiles/r06/s/)
  static const bool wide_on = env_int("LBF_TAIL_WIDE", 1) != 0; // A/B switch
  const bool wide = max_splits > 32 && wide_on;
  const dim3 g(unsigned(a.nb)), b(256);
  switch (tail_vpw(a.h.m)) {
  case 2:
    if (wide) hipLaunchKernelGGL((tail_reduce_kernel<2, 24>), g, b, 0, s, a);
    else hipLaunchKernelGGL((tail_reduce_kernel<2, 8>), g, b, 0, s, a);
    break;
  case 4:
    if (wide) hipLaunchKernelGGL((tail_reduce_kernel<4, 24>), g, b, 0, s, a);
    else hipLaunchKernelGGL((tail_reduce_kernel<4, 8>), g, b, 0, s, a);
    break;
  case 8:
    if (wide) hipLaunchKernelGGL((tail_reduce_kernel<8, 24>), g, b, 0, s, a);
    else hipLaunchKernelGGL((tail_reduce_kernel<8, 8>), g, b, 0, s, a);
    break;
  case 16: hipLaunchKernelGGL((tail_reduce_kernel<16, 8>), g, b, 0, s, a); break;
  default: throw Error(2, "tail_reduce: history size not supported by the fused tail");
  }
  LBF_KERNEL_CHECK();
  if (!a.cols_done) throw Error(2, "tail_reduce: needs the arrival counter (cols_done)");
  hipLaunchKernelGGL(tail_cols_fin_kernel, dim3(unsigned(a.nc)), dim3(TF_THREADS), fin_shmem(a), s, a);
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
