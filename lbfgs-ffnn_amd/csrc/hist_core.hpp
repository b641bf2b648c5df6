// Device-side history step shared by hist_step_kernel (vec_kernels.hip) and the fused optimizer tail
// (tail.hip): given the dots of the new pair / gradient against the live history, write the new
// Gram rows, apply the pair acceptance rule of the policy (CPU lbfgs.hpp:77-84 ys > 1e-10; CUDA
// lbfgs.cuh:160 ys > 1e-10; S-LBFGS s_lbfgs.hpp:253 |ys| > 1e-10), push/evict like
// RingBuffer::push_back (ring_buffer.hpp:43-59), and run the two-loop recursion on coefficients.
//
// With q = g - sum_j alpha_j y_j and z = gamma*q + sum_j (alpha_j - beta_j) s_j, the reference's
// loops (lbfgs.hpp:119-136) are two triangular recurrences on Gram entries:
//   backward  alpha_i = rho_i * (gS_i - sum_{j>i} alpha_j SY[i][j])
//   forward   beta_i  = rho_i * (gamma*(gY_i - sum_j alpha_j YY[i][j]) + sum_{j<i} (alpha_j-beta_j) SY[j][i])
// and z = sum_i (alpha_i - beta_i) s_i - gamma*alpha_i y_i + gamma*g. Entries that involve the slot
// written in this step come from the fresh dots (LDS), never from global memory written by this same
// kernel. Lane l of wave 0 owns rows l and l+64 of the recurrences; the per-step scalar is broadcast
// with v_readlane.
//
// Dots layout (sm.dots): live logical index i -> [S_i.s, Y_i.s, S_i.y, Y_i.y, S_i.g, Y_i.g] at
// 6i..6i+5 (i < m), then [s.s, s.y, y.y, g.s, g.y, g.g] at 6m..6m+5.
#pragma once

#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

namespace lbf {

constexpr int COEF_MAXK = 128;

struct HistSmem {
  double dots[6 * COEF_MAXK + 6];
  double gS_l[COEF_MAXK], gY_l[COEF_MAXK], rho_l[COEF_MAXK], alpha_l[COEF_MAXK], c_l[COEF_MAXK];
  int L0[COEF_MAXK + 1], L[COEF_MAXK + 1], inv0[COEF_MAXK + 1];
  int count0, w, k, acc, fslot;
  int iw; // the written slot's index in the new live order (-1: not live)
  double rhow;
};

struct HistStep {
  HistView h;
  int has_pair = 0, has_g = 0, reset = 0, policy = POL_CPU;
  int want_dir = 1; // -1: force the push (explicit upload), 0: no direction, 1: direction (+ CUDA fallback)
  int iter = 1;
  double dsign = -1.0;
  // hist_prologue<true> / hist_core<true>: copies of the ring header, rho, SY and YY already staged
  // in LDS by the caller (the fused tail prefetches them with its first loads). Unused otherwise.
  const int *ist = nullptr;
  const double *rho = nullptr, *SY = nullptr, *YY = nullptr;
  // S-LBFGS pair updates (dir_cols_fin, k <= DIR_MAXM): the live pairs' coefficient map K (slbfgs_kmat) into
  // kmat (global, DIR_KMAT_N doubles), computed by wave 1 beside wave 0's recurrences; kscr: DIR_MAXM^2 doubles
  // of LDS
  double *kmat = nullptr, *kscr = nullptr;
};

// Ring slot the next pair is written to.
__device__ __forceinline__ int hist_write_slot(const int *ist, int m, int policy, int reset) {
  const int count = reset ? 0 : ist[IST_COUNT];
  // CUDA semantics (lbfgs.cuh:149-169): the slot at hist_head is overwritten even when the pair is
  // then rejected; when the ring is full that slot is the oldest live pair.
  if (policy == POL_CUDA && count == m) return ist[IST_ORDER + 0];
  return ist[IST_FREE];
}

__device__ __forceinline__ double hc_wave_sum(double v) { return wave_sum_f64(v); }

// Loads from the step's sources. LDS = true: the HistStep pointers are LDS copies, read with ds_read
// (a generic pointer would be a flat load, whose wait also drains every global store in flight).
typedef const __attribute__((address_space(3))) double *hc_lds_dptr;
typedef const __attribute__((address_space(3))) int *hc_lds_iptr;
template <bool LDS> __device__ __forceinline__ double hc_ld(const double *p, long long i) {
  if constexpr (LDS) return ((hc_lds_dptr)p)[i];
  else return p[i];
}
template <bool LDS> __device__ __forceinline__ int hc_ldi(const int *p, int i) {
  if constexpr (LDS) return ((hc_lds_iptr)p)[i];
  else return p[i];
}

// The two-loop recurrences for k <= 64 (wave 0; lane l owns index l), from LDS: sy = SY of the live
// pairs in order (k x k, row stride k), syT its transpose, yyl = YY; rho_l, gS_l, gY_l per live index.
// Returns this lane's alpha (al0) and alpha - beta (c0). The LDS operands of 8 steps are loaded ahead
// of them (unit stride across lanes), so each step is VALU + v_readlane only. Shared by hist_core and the
// S-LBFGS direction's combine (dir.hip), which rely on it for bitwise the same coefficients.
__device__ __forceinline__ void recur_fast(int k, int lane, const double *rho_l, const double *gS_l,
                                           const double *gY_l, const double *sy, const double *syT,
                                           const double *yyl, double gamma, double &al0, double &c0) {
  // A lane's running sum is read once, at its own step, and is dead after it (backward: steps i < l; forward:
  // steps i > l; lanes >= k never), so every lane updates unconditionally from unconditional (clamped) loads:
  // the live lanes get exactly the masked update, and no select or exec mask sits on the step's chain.
  const int lc = lane < k ? lane : (k > 0 ? k - 1 : 0);
  const double rho_me = lane < k ? rho_l[lane] : 0.0;
  double r = lane < k ? gS_l[lane] : 0.0;
  for (int i0 = k - 1; i0 >= 0; i0 -= 8) { // backward: alpha_i = rho_i (gS_i - sum_{j>i} alpha_j SY[i][j])
    double col[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) col[u] = syT[max(i0 - u, 0) * k + lc];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 - u;
      if (i >= 0) {
        const double ai = lane_f64(rho_me * r, i);
        if (lane == i) al0 = ai;
        r = r - ai * col[u];
      }
    }
  }
  KTC(65);
  KTF(60);
  double acc = lane < k ? gY_l[lane] : 0.0; // gY_l - sum_j alpha_j YY[l][j]  (YY symmetric)
  for (int j0 = 0; j0 < k; j0 += 8) {
    double yv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) yv[u] = yyl[min(j0 + u, k - 1) * k + lc];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (j0 + u < k) acc -= lane_f64(al0, j0 + u) * yv[u];
  }
  double tv = gamma * acc;
  for (int i0 = 0; i0 < k; i0 += 8) { // forward: beta_i = rho_i t_i ; t_l += (alpha_i - beta_i) SY[i][l]
    double row[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) row[u] = sy[min(i0 + u, k - 1) * k + lc];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u;
      if (i < k) {
        const double cand = rho_me * tv;
        const double ci = lane_f64(al0, i) - lane_f64(cand, i);
        if (lane == i) c0 = ci;
        tv = tv + ci * row[u];
      }
    }
  }
}

// The slbfgs gamma (s_lbfgs.hpp:119-126) from the newest pair's ys and yy.
__device__ __forceinline__ double slbfgs_gamma(double ys, double yy) {
  const double g = fabs(yy) < 1e-12 ? 1.0 : ys / yy;
  return fmin(fmax(g, 1e-6), 1e6);
}

// The S-LBFGS direction's coefficient map (round 5). With R the k x k upper-triangular matrix R[i][j] = s_i.y_j
// (i < j), R[i][i] = 1 / rho_i, the two-loop recursion of s_lbfgs.hpp:106-136 is, for ANY rho (checked in
// numpy to 5e-16), H g = gamma g + S cS + Y cY with
//   cY = -gamma R^-1 a,   cS = R^-T ((D + gamma YY) R^-1 a - gamma b),   a = S^T g, b = Y^T g, D = diag(1/rho)
// (the compact form of Byrd, Nocedal & Schnabel 1994): the backward recurrence is R^-1 a, the forward one
// R^-T q. So [cS; cY] = K [a; b] with K = [[R^-T M R^-1, -gamma R^-T], [-gamma R^-1, 0]], M = D + gamma YY,
// and K depends only on the pairs, which change once every L inner steps: one wave computes it at each pair
// update (lane j: column j of R^-1 by back substitution, then column j of M R^-1 and of R^-T M R^-1; no
// cross-lane dependency), and every direction-only step's combine blocks do ONE 2k x 2k mat-vec instead of
// the two k-step recurrences (dir_combine_kernel). Operands from LDS: sy = SY of the live pairs (k x k, row
// stride k), yyl = YY, rho_l; rinv: DIR_MAXM^2 doubles of LDS; K: global, row stride DIR_KS, then gamma and k.
__device__ inline void slbfgs_kmat(int k, int lane, const double *rho_l, const double *sy, const double *yyl,
                                   double *rinv, double *K) {
  constexpr int KM = DIR_MAXM;
  const double gamma = k > 0 ? slbfgs_gamma(sy[(k - 1) * k + (k - 1)], yyl[(k - 1) * k + (k - 1)]) : 1.0;
  const int j = lane;
  double x[KM];
#pragma unroll
  for (int i = 0; i < KM; ++i) x[i] = 0.0;
  if (j < k) {
#pragma unroll
    for (int i = KM - 1; i >= 0; --i) { // back substitution for column j: R x = e_j
      if (i == j) x[i] = rho_l[j];
      if (i < j) {
        double acc = 0.0;
#pragma unroll
        for (int l = i + 1; l < KM; ++l)
          if (l <= j) acc += sy[i * k + l] * x[l];
        x[i] = -rho_l[i] * acc;
      }
    }
  }
  if (j < KM)
#pragma unroll
    for (int i = 0; i < KM; ++i) rinv[i * KM + j] = x[i];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // one wave: its own LDS writes are complete
  __builtin_amdgcn_wave_barrier();
  if (j < k) {
    double tcol[KM]; // column j of M R^-1
#pragma unroll
    for (int i = 0; i < KM; ++i) {
      tcol[i] = 0.0;
      if (i < k) {
        double acc = 0.0;
#pragma unroll
        for (int l = 0; l < KM; ++l)
          if (l < k) acc += yyl[i * k + l] * x[l];
        tcol[i] = x[i] / rho_l[i] + gamma * acc;
      }
    }
#pragma unroll
    for (int i = 0; i < KM; ++i)
      if (i < k) {
        double acc = 0.0; // (R^-T M R^-1)[i][j] = sum_l R^-1[l][i] (M R^-1)[l][j]
#pragma unroll
        for (int l = 0; l < KM; ++l)
          if (l < k) acc += rinv[l * KM + i] * tcol[l];
        K[i * DIR_KS + j] = acc;
        K[i * DIR_KS + k + j] = -gamma * rinv[j * KM + i]; // -gamma R^-T
        K[(k + i) * DIR_KS + j] = -gamma * x[i];           // -gamma R^-1
        K[(k + i) * DIR_KS + k + j] = 0.0;
      }
  }
  if (lane == 0) {
    K[DIR_KS * DIR_KS] = gamma;
    K[DIR_KS * DIR_KS + 1] = double(k); // the layout depends on k: dir_combine checks it against the ring's count
  }
}

// Barriers here are LDS-only (wave.hpp lds_barrier): within a history step no thread reads global
// memory another thread of the block wrote in the same step (fresh entries come from the dots in LDS).
//
// Live order before the step: sm.count0, sm.w (write slot), sm.L0[], sm.inv0[]. Block-wide; ends
// with a barrier. w is the slot the pair was written to (ist[IST_WSLOT] or given).
template <bool LDS = false> __device__ inline void hist_prologue(const HistStep &a, HistSmem &sm, int w) {
  const HistView &h = a.h;
  const int t = threadIdx.x, nt = blockDim.x;
  const int *ist = LDS ? a.ist : h.ist;
  // the count and the first nt order entries in one round trip (entries past the count are loaded and unused)
  const int count0 = a.reset ? 0 : hc_ldi<LDS>(ist, IST_COUNT);
  const int j0 = t < h.m ? hc_ldi<LDS>(ist, IST_ORDER + t) : 0;
  if (t == 0) {
    sm.count0 = count0;
    sm.w = w;
  }
  for (int i = t; i < h.slots; i += nt) sm.inv0[i] = -1;
  lds_barrier();
  for (int i = t; i < count0; i += nt) {
    const int j = i == t ? j0 : hc_ldi<LDS>(ist, IST_ORDER + i);
    sm.L0[i] = j;
    sm.L[i] = j;
    sm.inv0[j] = i;
  }
  lds_barrier();
}

// Steps B and C (see the file comment). Precondition: hist_prologue done and sm.dots filled, then a
// barrier. Must be the last phase of the kernel: waves other than 0 return early.
// sy: sy_cap >= k*k doubles of LDS (SY, plus its transpose when 2*k*k fit); yyl: yy_cap doubles of
// LDS (the YY block is staged when k*k <= yy_cap).
//
// FUSED (the fused tail: sources staged in LDS, want_dir == 1, reset == 0, >= 2 waves): step B only
// decides, in LDS; the global writes of the new Gram rows, rho and the ring header are made by waves
// 1.. while wave 0 runs the recurrences, and the live count by wave 0 with the coefficients. A store
// in flight on wave 0 would stall it at its next vmcnt wait; other waves' stores do not.
template <bool FUSED = false>
__device__ inline void hist_core(const HistStep &a, HistSmem &sm, double *sy, int sy_cap, double *yyl, int yy_cap) {
  constexpr bool LDS = FUSED;
  const HistView &h = a.h;
  const int S_ = h.slots, t = threadIdx.x, nt = blockDim.x, lane = t & 63, wave = t >> 6;
  const int count0 = sm.count0, w = sm.w;
  const double *dots = sm.dots;
  const double *self = dots + 6 * h.m;
  const double *SYsrc = LDS ? a.SY : h.SY, *YYsrc = LDS ? a.YY : h.YY, *rhosrc = LDS ? a.rho : h.rho;
  KTF(56);
  // Gram rows of the new pair and the g-dots -> global (consumed by later steps); u / nu: this
  // thread's index among the writers
  auto write_rows = [&](int u, int nu) {
    for (int i = u; i < count0; i += nu) {
      const int j = sm.L0[i];
      if (a.has_pair && j == w) continue;
      if (a.has_pair) {
        h.SS[w * S_ + j] = dots[6 * i + 0];
        h.SS[j * S_ + w] = dots[6 * i + 0];
        h.SY[w * S_ + j] = dots[6 * i + 1]; // s_w . y_j
        h.SY[j * S_ + w] = dots[6 * i + 2]; // s_j . y_w
        h.YY[w * S_ + j] = dots[6 * i + 3];
        h.YY[j * S_ + w] = dots[6 * i + 3];
      }
      if (a.has_g) {
        h.gS[j] = dots[6 * i + 4];
        h.gY[j] = dots[6 * i + 5];
      }
    }
    if (u == 0 && a.has_pair) {
      h.SS[w * S_ + w] = self[0];
      h.SY[w * S_ + w] = self[1];
      h.YY[w * S_ + w] = self[2];
      if (a.has_g) {
        h.gS[w] = self[3];
        h.gY[w] = self[4];
      }
    }
  };
  // ---- B ----
  if constexpr (!FUSED) write_rows(t, nt);
  if (t == 0) {
    if (!FUSED && a.has_g) h.scal[SC_GG] = self[5];
    int count = count0;
    sm.rhow = (a.has_pair && w < S_) ? hc_ld<LDS>(rhosrc, w) : 0.0;
    sm.acc = 0;
    sm.fslot = -1;
    if (!FUSED && a.reset) h.ist[IST_COUNT] = 0;
    if (a.has_pair) {
      const double ys = self[1];
      bool acc = (a.policy == POL_SLBFGS) ? fabs(ys) > 1e-10 : ys > 1e-10;
      if (a.want_dir < 0) acc = true; // explicit-history upload (lbf_two_loop): always push
      if (!FUSED) {
        h.scal[SC_YS] = ys;
        h.scal[SC_ACCEPT] = acc ? 1.0 : 0.0;
      }
      sm.acc = acc ? 1 : 0;
      if (acc) {
        sm.rhow = 1.0 / ys;
        if (!FUSED) h.rho[w] = sm.rhow;
        int f = -1;
        if (count < h.m) {
          sm.L[count++] = w;
          if (a.policy != POL_CUDA || count < h.m) {
            unsigned long long live[3] = {0ull, 0ull, 0ull}; // next free slot: any of the m+1 not live
            for (int q = 0; q < count; ++q) live[sm.L[q] >> 6] |= 1ull << (sm.L[q] & 63);
            f = S_;
            for (int b = 0; b < 3 && f == S_; ++b)
              if (~live[b]) f = min(S_, b * 64 + __builtin_ctzll(~live[b]));
          }
        } else {
          const int evicted = sm.L[0];
          for (int q = 0; q + 1 < h.m; ++q) sm.L[q] = sm.L[q + 1];
          sm.L[h.m - 1] = w;
          if (w != evicted) f = evicted;
        }
        sm.fslot = f;
        if (!FUSED) {
          if (f >= 0) h.ist[IST_FREE] = f;
          for (int q = 0; q < count; ++q) h.ist[IST_ORDER + q] = sm.L[q];
          h.ist[IST_COUNT] = count;
        }
      }
    }
    if (!FUSED) h.scal[SC_COUNT] = double(count);
    sm.k = count;
    // a pushed pair is last in the live order; a rejected one stays live only where the CUDA semantics
    // overwrite the oldest slot in place (then at its old index)
    sm.iw = !a.has_pair ? -1 : sm.acc ? count - 1 : (w < S_ ? sm.inv0[w] : -1);
    KTF(57);
  }
  lds_barrier();
  // ---- C1: stage the live quantities ----
  const int k = sm.k;
  const int *L = sm.L, *inv0 = sm.inv0;
  auto SYv = [&](int p, int q) -> double { // s_p . y_q
    if (a.has_pair) {
      if (p == w && q == w) return self[1];
      if (p == w) return dots[6 * inv0[q] + 1];
      if (q == w) return dots[6 * inv0[p] + 2];
    }
    return hc_ld<LDS>(SYsrc, p * S_ + q);
  };
  auto YYv = [&](int p, int q) -> double {
    if (a.has_pair) {
      if (p == w && q == w) return self[2];
      if (p == w) return dots[6 * inv0[q] + 3];
      if (q == w) return dots[6 * inv0[p] + 3];
    }
    return hc_ld<LDS>(YYsrc, p * S_ + q);
  };
  const bool yy_lds = k * k <= yy_cap;
  const bool sy_t = 2 * k * k <= sy_cap;
  // No room for SY, its transpose and YY (m = 100): SY with an odd row stride (k + 1, so its column
  // reads are nearly conflict-free and need no transposed copy) and YY's lower triangle, both in the
  // SY area (m = 100: 10100 + 5050 doubles)
  const int kp = k + 1;
  const bool big = !(k <= 64 && sy_t && yy_lds) && k * kp + (k * kp) / 2 <= sy_cap;
  if (big) {
    double *yt = sy + k * kp;
    constexpr int B = 16; // loads in flight per thread: k * k = 10^4 entries in three round trips
    for (int e0 = t; e0 < k * k; e0 += nt * B) {
      double a16[B], b16[B];
#pragma unroll
      for (int u = 0; u < B; ++u) { // every stored entry loaded unconditionally (clamped): one round trip
        const int e = min(e0 + nt * u, k * k - 1);
        const int i = e / k, j = e - i * k;
        const int pq = L[i] * S_ + L[j];
        a16[u] = hc_ld<LDS>(SYsrc, pq);
        b16[u] = hc_ld<LDS>(YYsrc, pq);
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int e = e0 + nt * u;
        if (e < k * k) {
          const int i = e / k, j = e - i * k, p_ = L[i], q_ = L[j];
          double sv = a16[u], yv = b16[u];
          if (a.has_pair && (p_ == w || q_ == w)) { // the pushed pair's row / column: fresh dots (LDS)
            sv = SYv(p_, q_);
            yv = YYv(p_, q_);
          }
          sy[i * kp + j] = sv;
          if (j <= i) yt[(i * (i + 1)) / 2 + j] = yv;
        }
      }
    }
  }
  if (!big) {
    // Every entry not on the written slot's row / column from the sources, then that row and column from the
    // fresh dots (disjoint entries: no barrier between). k <= 64: wave v takes rows v, v + nw, ..., lane j
    // column j; the slot numbers of the rows come from the lanes' own (v_readlane), so the entries of RU rows
    // are loaded in one LDS round trip, with no index division and no per-entry branch.
    const int iw = sm.iw, nw = nt >> 6;
    if (k <= 64) {
      constexpr int RU = 4;
      const int qme = lane < k ? L[lane] : 0;
      for (int i0 = wave; i0 < k; i0 += nw * RU) {
        double sv[RU], yv[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int p = __builtin_amdgcn_readlane(qme, min(i0 + nw * u, k - 1));
          sv[u] = hc_ld<LDS>(SYsrc, p * S_ + qme);
          yv[u] = yy_lds ? hc_ld<LDS>(YYsrc, p * S_ + qme) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int i = i0 + nw * u;
          if (i < k && lane < k && i != iw && lane != iw) {
            sy[i * k + lane] = sv[u];
            if (sy_t) sy[k * k + lane * k + i] = sv[u]; // transposed copy
            if (yy_lds) yyl[i * k + lane] = yv[u];
          }
        }
      }
    } else {
      for (int e = t; e < k * k; e += nt) {
        const int i = e / k, j = e - i * k;
        if (i == iw || j == iw) continue;
        const int pq = L[i] * S_ + L[j];
        sy[e] = hc_ld<LDS>(SYsrc, pq);
        if (sy_t) sy[k * k + j * k + i] = sy[e];
        if (yy_lds) yyl[e] = hc_ld<LDS>(YYsrc, pq);
      }
    }
    // (the row / column and the per-index loop below start on waves 1 and 2: their dependent LDS chains run
    // beside wave 0's rows instead of after them)
    for (int j = (t + nt - 64) % nt; iw >= 0 && j < k; j += nt) { // s_w . y_q, s_q . y_w, y_w . y_q (SYv / YYv)
      const int d = j == iw ? 0 : 6 * inv0[L[j]]; // (the written slot has no old index)
      const double srow = j == iw ? self[1] : dots[d + 1], scol = j == iw ? self[1] : dots[d + 2];
      const double yv = j == iw ? self[2] : dots[d + 3];
      sy[iw * k + j] = srow;
      sy[j * k + iw] = scol;
      if (sy_t) {
        sy[k * k + j * k + iw] = srow;
        sy[k * k + iw * k + j] = scol;
      }
      if (yy_lds) {
        yyl[iw * k + j] = yv;
        yyl[j * k + iw] = yv;
      }
    }
  }
  for (int i = (t + nt - 128 % nt) % nt; i < k; i += nt) {
    const int j = L[i];
    const bool fresh = a.has_pair && j == w;
    if (a.has_g) {
      sm.gS_l[i] = fresh ? self[3] : dots[6 * inv0[j] + 4];
      sm.gY_l[i] = fresh ? self[4] : dots[6 * inv0[j] + 5];
    } else {
      sm.gS_l[i] = h.gS[j];
      sm.gY_l[i] = h.gY[j];
    }
    sm.rho_l[i] = fresh ? sm.rhow : hc_ld<LDS>(rhosrc, j);
  }
  lds_barrier();
  KTF(59);
  if (wave != 0) {
    if (wave == 1 && a.kmat && a.policy == POL_SLBFGS && k <= DIR_MAXM && sy_t && yy_lds)
      slbfgs_kmat(k, lane, sm.rho_l, sy, yyl, a.kscr, a.kmat); // beside wave 0's recurrences
    if constexpr (FUSED) { // the deferred writes of step B (the live count: wave 0, below)
      const int u = t - 64, nu = nt - 64;
      write_rows(u, nu);
      if (u == 0) {
        if (a.has_pair) {
          h.scal[SC_YS] = self[1];
          h.scal[SC_ACCEPT] = sm.acc ? 1.0 : 0.0;
          if (sm.acc) h.rho[w] = sm.rhow;
          if (sm.fslot >= 0) h.ist[IST_FREE] = sm.fslot;
        }
      }
      if (sm.acc)
        for (int q = u; q < sm.k; q += nu) h.ist[IST_ORDER + q] = sm.L[q];
    }
    return;
  }

  // ---- C2: the recurrences (wave 0). Lane l owns indices l and l+64: alpha, c and the running
  // sums live in its registers; the step's scalar is broadcast with v_readlane. LDS reads are
  // unit-stride across lanes: SY^T for the backward sweep, YY by symmetry, SY rows forward. ----
  const double *gS_l = sm.gS_l, *gY_l = sm.gY_l, *rho_l = sm.rho_l;
  const double gg = a.has_g ? self[5] : h.scal[SC_GG];
  double gamma = 1.0;
  if (k > 0) {
    const double ys = big ? sy[(k - 1) * kp + (k - 1)] : sy[(k - 1) * k + (k - 1)];
    const double yy = big ? sy[k * kp + ((k - 1) * k) / 2 + (k - 1)]
                          : (yy_lds ? yyl[(k - 1) * k + (k - 1)] : YYv(L[k - 1], L[k - 1]));
    if (a.policy == POL_CPU) {
      gamma = ys / yy; // lbfgs.hpp:127-128, no guard
    } else if (a.policy == POL_CUDA) {
      gamma = yy > 0.0 ? ys / yy : 1.0; // lbfgs.cuh:247
    } else {
      gamma = slbfgs_gamma(ys, yy); // s_lbfgs.hpp:119-126
    }
  }
  const double *syT = sy + k * k; // syT[i*k + l] = SY[l][i] (when sy_t)
  double al0 = 0.0, al1 = 0.0;     // alpha of indices lane, lane + 64
  double c0 = 0.0, c1 = 0.0;       // alpha - beta of indices lane, lane + 64
  if (k <= 64 && sy_t && yy_lds) {
    KTF(63);
    KTC(64);
    // (the compact form of slbfgs_kmat computed per step in this block, lane j inverting column j of R by
    // back substitution, measured 1.5-2 % slower at cfg 2 than these recurrences: profiles/r05/g/)
    recur_fast(k, lane, rho_l, gS_l, gY_l, sy, syT, yyl, gamma, al0, c0);
  } else if (big) {
    // Two indices per lane (l0 = lane, l1 = lane + 64); the LDS operands of 8 steps are loaded ahead
    // of them, so each step is VALU + v_readlane only (the k <= 64 fast path, widened).
    const double *yt = sy + k * kp;
    const int l0 = lane, l1 = lane + 64;
    const bool in0 = l0 < k, in1 = l1 < k;
    auto tri = [&](int a_, int b_) { return a_ >= b_ ? (a_ * (a_ + 1)) / 2 + b_ : (b_ * (b_ + 1)) / 2 + a_; };
    const double rho0 = in0 ? rho_l[l0] : 0.0, rho1 = in1 ? rho_l[l1] : 0.0;
    double r0 = in0 ? gS_l[l0] : 0.0, r1 = in1 ? gS_l[l1] : 0.0;
    for (int i0 = k - 1; i0 >= 0; i0 -= 8) { // backward: alpha_i = rho_i (gS_i - sum_{j>i} alpha_j SY[i][j])
      double c0v[8], c1v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 - u;
        c0v[u] = (i >= 0 && l0 < i) ? sy[l0 * kp + i] : 0.0; // column i of SY: s_l . y_i
        c1v[u] = (i >= 0 && l1 < i) ? sy[l1 * kp + i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 - u;
        if (i >= 0) { // wave-uniform
          const double ai = (i < 64) ? lane_f64(rho0 * r0, i) : lane_f64(rho1 * r1, i - 64);
          if (i < 64 && lane == i) al0 = ai;
          if (i >= 64 && lane == i - 64) al1 = ai;
          r0 = l0 < i ? r0 - ai * c0v[u] : r0;
          r1 = l1 < i ? r1 - ai * c1v[u] : r1;
        }
      }
    }
    KTF(60);
    double acc0 = in0 ? gY_l[l0] : 0.0, acc1 = in1 ? gY_l[l1] : 0.0; // gY_l - sum_j alpha_j YY[l][j]
    for (int j0 = 0; j0 < k; j0 += 8) {
      double y0v[8], y1v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        y0v[u] = (j < k && in0) ? yt[tri(l0, j)] : 0.0;
        y1v[u] = (j < k && in1) ? yt[tri(l1, j)] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        if (j < k) {
          const double aj = (j < 64) ? lane_f64(al0, j) : lane_f64(al1, j - 64);
          acc0 -= aj * y0v[u];
          acc1 -= aj * y1v[u];
        }
      }
    }
    double t0 = gamma * acc0, t1 = gamma * acc1;
    for (int i0 = 0; i0 < k; i0 += 8) { // forward: beta_i = rho_i t_i ; t_l += (alpha_i - beta_i) SY[i][l]
      double w0v[8], w1v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u;
        w0v[u] = (i < k && l0 > i && in0) ? sy[i * kp + l0] : 0.0;
        w1v[u] = (i < k && l1 > i && in1) ? sy[i * kp + l1] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u;
        if (i < k) {
          double ci;
          if (i < 64) {
            ci = lane_f64(al0, i) - lane_f64(rho0 * t0, i);
            if (lane == i) c0 = ci;
          } else {
            ci = lane_f64(al1, i - 64) - lane_f64(rho1 * t1, i - 64);
            if (lane == i - 64) c1 = ci;
          }
          t0 = (l0 > i && in0) ? t0 + ci * w0v[u] : t0;
          t1 = (l1 > i && in1) ? t1 + ci * w1v[u] : t1;
        }
      }
    }
  } else {
    double r0v = lane < k ? gS_l[lane] : 0.0, r1v = lane + 64 < k ? gS_l[lane + 64] : 0.0;
    for (int i = k - 1; i >= 0; --i) {
      const double cand = rho_l[i] * ((i >> 6) == 0 ? r0v : r1v);
      const double ai = lane_f64(cand, i & 63);
      if (lane == (i & 63)) {
        if (i < 64) al0 = ai;
        else al1 = ai;
      }
      if (lane < i) r0v -= ai * (sy_t ? syT[i * k + lane] : sy[lane * k + i]);
      if (lane + 64 < i) r1v -= ai * (sy_t ? syT[i * k + lane + 64] : sy[(lane + 64) * k + i]);
    }
    KTF(60);
    double t0v = 0.0, t1v = 0.0;
    {
      double acc0 = lane < k ? gY_l[lane] : 0.0, acc1 = lane + 64 < k ? gY_l[lane + 64] : 0.0;
      for (int j = 0; j < k; ++j) {
        const double aj = lane_f64(j < 64 ? al0 : al1, j & 63);
        if (lane < k) acc0 -= aj * (yy_lds ? yyl[j * k + lane] : YYv(L[j], L[lane]));
        if (lane + 64 < k) acc1 -= aj * (yy_lds ? yyl[j * k + lane + 64] : YYv(L[j], L[lane + 64]));
      }
      t0v = gamma * acc0;
      t1v = gamma * acc1;
    }
    for (int i = 0; i < k; ++i) {
      const double cand = rho_l[i] * ((i >> 6) == 0 ? t0v : t1v);
      const double ci = lane_f64(i < 64 ? al0 : al1, i & 63) - lane_f64(cand, i & 63);
      if (lane == (i & 63)) {
        if (i < 64) c0 = ci;
        else c1 = ci;
      }
      if (lane > i && lane < k) t0v += ci * sy[i * k + lane];
      if (lane + 64 > i && lane + 64 < k) t1v += ci * sy[i * k + lane + 64];
    }
  }
  KTF(61);
  const double ds = a.dsign;
  double part = 0.0;
  if (lane < k) part += c0 * gS_l[lane] - gamma * al0 * gY_l[lane];
  if (lane + 64 < k) part += c1 * gS_l[lane + 64] - gamma * al1 * gY_l[lane + 64];
  const double gTz = hc_wave_sum(part) + gamma * gg;
  // lbfgs.cuh:97-104 (CUDA semantics only): not a descent direction -> steepest descent + reset
  const bool fallback = a.policy == POL_CUDA && a.want_dir == 1 && ds * gTz >= 0.0;
  if (lane < k) {
    h.coef[lane] = fallback ? 0.0 : ds * c0;
    h.coef[S_ + lane] = fallback ? 0.0 : ds * (-gamma * al0);
  }
  if (lane + 64 < k) {
    h.coef[lane + 64] = fallback ? 0.0 : ds * c1;
    h.coef[S_ + lane + 64] = fallback ? 0.0 : ds * (-gamma * al1);
  }
  if (lane == 0) {
    h.coef[2 * S_] = fallback ? -1.0 : ds * gamma;
    h.scal[SC_RESET] = fallback ? 1.0 : 0.0;
    h.scal[SC_GTP] = fallback ? -gg : ds * gTz;
    if (FUSED) {
      h.ist[IST_COUNT] = fallback ? 0 : k;
      h.scal[SC_COUNT] = fallback ? 0.0 : double(k);
    } else if (fallback) {
      h.ist[IST_COUNT] = 0;
      h.scal[SC_COUNT] = 0.0;
    }
    h.scal[SC_GG] = gg;
    h.scal[SC_GAMMA] = gamma;
    h.scal[SC_ALPHA0] = (a.iter == 0) ? fmin(1.0, 1.0 / sqrt(gg)) : 1.0;
  }
  KTF(62);
}

} // namespace lbf
