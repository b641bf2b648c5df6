// History update of the S-LBFGS inner step in two launches (the L-BFGS fused tail's pattern, tail.hip,
// with the operands of GramArgs instead of split-K slabs):
//   dir_sweep    one block per 64*C-column group: the new vectors s = sa - sb, y = (ya - yb)*yscale,
//                g = ga - gb + gc of the group (s, y into the ring's write slot, g into g_out), the group's
//                values of every live history vector, all loaded up front (one round trip), then every
//                Gram column of the group reduced out of LDS by four lanes -> one partial row per block,
//                stored transposed ([nc][nb]);
//   dir_cols_fin one block per Gram column: its fixed-order sum; the last block to arrive (arrival
//                counter) runs the history step (hist_core.hpp: push / evict, the two-loop recurrences on
//                coefficients) from those sums.
// The linear-combination sweep (combine_small) follows. Replaces gram_kernel -> fold_rows -> hist_step
// (three launches, the step reading a folded partial table) for S-LBFGS's directions (s_lbfgs.hpp:
// 106-136 two-loop with the VR gradient of :228) and curvature pairs (:245-256).
#include "hist_core.hpp"
#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace lbf {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// C columns per lane (64*C per block) as Q = C/4 quads, lane l owning columns 256q + 4l .. +3 of quad q;
// VPW history vectors per wave (v = wave + 4j). GRED: a.gred_on (the deferred split-K reduction's 16 KB
// of fp64 stripes in LDS are only declared where they are used, so the pair and sliced-DP sweeps keep the
// ~6 KB footprint).
template <int C, int VPW, bool GRED>
__global__ __launch_bounds__(256) void dir_sweep_kernel(const DirArgs a) {
  constexpr int TC = 64 * C, Q = C / 4;
  static_assert(C % 4 == 0, "dir_sweep: whole quads per lane");
  const GramArgs &g = a.g;
  const HistView &h = g.h;
  if (h.abort && *h.abort) return;
  __shared__ float ops[3][TC];      // s, y, g
  __shared__ int ist[IST_ORDER + DIR_MAXM];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  if (t < IST_ORDER + h.m) ist[t] = h.ist[t];
  lds_barrier();
  const int count0 = __builtin_amdgcn_readfirstlane(g.reset ? 0 : ist[IST_COUNT]);
  const int w = __builtin_amdgcn_readfirstlane(hist_write_slot(ist, h.m, g.policy, g.reset));
  if (blockIdx.x == 0 && t == 0) h.ist[IST_WSLOT] = w;
  const int nvec = 2 * count0;
  // 16-B loads (every vector the sweep touches is 16-B aligned and padded to a multiple of 4 floats,
  // History::update checks). Every load is unconditional from a clamped address and masked after
  // (tail.hip's discipline).
  long long col0[Q], e4[Q];
  bool live[Q][4];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    col0[q] = (long long)blockIdx.x * TC + 256 * q + 4 * lane;
    e4[q] = col0[q] < h.n ? col0[q] : ((h.n - 1) & ~3LL); // clamped quad start (inside the padding)
#pragma unroll
    for (int c = 0; c < 4; ++c) live[q][c] = col0[q] + c < h.n;
  }
  f32x4 vv[VPW][Q];
  unsigned zero_mask = 0; // bit j: vector j of this wave is not live (or is the slot being overwritten)
#pragma unroll
  for (int j = 0; j < VPW; ++j) {
    const int v = wave + 4 * j; // wave-uniform: the branch is scalar, no per-lane wait
#pragma unroll
    for (int q = 0; q < Q; ++q) vv[j][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (v < nvec) {
      const int slot = __builtin_amdgcn_readfirstlane(ist[IST_ORDER + (v < count0 ? v : v - count0)]);
      const float *base = (v < count0 ? h.S : h.Y) + (long long)slot * h.ld;
#pragma unroll
      for (int q = 0; q < Q; ++q) vv[j][q] = *reinterpret_cast<const f32x4 *>(base + e4[q]);
      if (g.has_pair && slot == w) zero_mask |= 1u << j;
    } else {
      zero_mask |= 1u << j;
    }
  }
  // g.ga from its split-K slabs (gred_on): wave w sums the splits k = w (mod 4) of this lane's quads in split
  // order (reduce_all_kernel's stripes) into LDS; wave 0 adds the four stripes after the barrier,
  // ((0 + 1) + 2) + 3 as reduce_all does: bitwise its gradient. History::update defers only segment tables
  // whose offsets, counts and strides are multiples of 4 floats (16-B aligned slabs), so a lane's quad lies
  // in one segment and is one 16-B load per split. The segment is found by a loop over the (kernel-argument)
  // table with a wave-uniform index: no lane waits on a load of the table.
  __shared__ double gpart[GRED ? 4 : 1][GRED ? TC : 1];
  auto seg_of = [&](long long e, const float *&base, long long &col, long long &strd, int &nsp) {
    const RedAllArgs &R = a.gred;
    base = R.G;
    col = e;
    strd = 0;
    nsp = 0;
    for (int si = 0; si < R.nseg; ++si) {
      const RedSeg &S = R.seg[si];
      if (e >= S.goff) {
        const bool sp = S.splits > 0;
        base = sp ? S.slab : R.G;
        col = sp ? e - S.goff : e;
        strd = sp ? S.stride : 0;
        nsp = S.splits;
      }
    }
  };
  if (GRED) { // a.gred_on (History::update: has_g, no pair)
    const RedAllArgs &R = a.gred;
    int kmax = 0;
    for (int si = 0; si < R.nseg; ++si) kmax = max(kmax, R.seg[si].splits);
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) gpart[wave][256 * q + 4 * lane + c] = 0.0;
    for (int k0 = wave; k0 < kmax; k0 += 4) { // one round trip per four splits
      f32x4 x[Q];
      int nsp[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) { // unconditional, clamped into the quad's slabs (or G itself)
        const float *base;
        long long col, strd;
        seg_of(e4[q], base, col, strd, nsp[q]);
        const int kc = min(k0, max(nsp[q] - 1, 0));
        x[q] = *reinterpret_cast<const f32x4 *>(base + col + (long long)kc * strd);
      }
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (k0 < nsp[q])
#pragma unroll
          for (int c = 0; c < 4; ++c) gpart[wave][256 * q + 4 * lane + c] += double(x[q][c]);
    }
    lds_barrier();
    if (wave == 0) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const float *base;
        long long col, strd;
        int nsp;
        seg_of(e4[q], base, col, strd, nsp);
        const f32x4 gw = *reinterpret_cast<const f32x4 *>(R.G + e4[q]); // unsplit segments: G as written
        // the other operands of v = g - gb + gc (null operands read G, masked)
        const f32x4 gb4 = *reinterpret_cast<const f32x4 *>((g.gb ? g.gb : R.G) + e4[q]);
        const f32x4 gc4 = *reinterpret_cast<const f32x4 *>((g.gc ? g.gc : R.G) + e4[q]);
        float ww[4] = {0.f, 0.f, 0.f, 0.f};
        if (R.l2 && R.lambda != 0.0) // uniform; w is exactly n long
#pragma unroll
          for (int c = 0; c < 4; ++c) ww[c] = R.w[min(e4[q] + c, h.n - 1)];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int qq = 256 * q + 4 * lane + c;
          float gv = 0.f;
          if (live[q][c]) {
            gv = nsp > 0 ? float(((gpart[0][qq] + gpart[1][qq]) + gpart[2][qq]) + gpart[3][qq]) : gw[c];
            if (R.l2 && R.lambda != 0.0) gv = gv + float(R.lambda) * ww[c]; // finalize_kernel's update
            if (g.gb) gv = gv - gb4[c];
            if (g.gc) gv = gv + gc4[c];
            if (g.g_out) g.g_out[col0[q] + c] = gv;
          }
          ops[0][qq] = 0.f;
          ops[1][qq] = 0.f;
          ops[2][qq] = gv;
        }
      }
    }
  } else if (wave == 0) { // the new vectors of the group (null operands read ga / sa and are masked)
    const float *dflt = g.has_g ? g.ga : g.sa;
    const float ysc = float(g.yscale);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      auto ld4 = [&](const float *p) { return *reinterpret_cast<const f32x4 *>((p ? p : dflt) + e4[q]); };
      const f32x4 sa = ld4(g.sa), sb = ld4(g.sb), ya = ld4(g.ya), yb = ld4(g.yb);
      const f32x4 ga = ld4(g.ga), gb = ld4(g.gb), gc = ld4(g.gc);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int qq = 256 * q + 4 * lane + c;
        const long long e = col0[q] + c;
        float sv = 0.f, yv = 0.f, gv = 0.f;
        if (live[q][c]) {
          if (g.has_pair) { // gram_kernel's arithmetic
            sv = sa[c] - sb[c];
            yv = (ya[c] - yb[c]) * ysc;
            h.S[(long long)w * h.ld + e] = sv;
            h.Y[(long long)w * h.ld + e] = yv;
          }
          if (g.has_g) {
            gv = ga[c];
            if (g.gb) gv = gv - gb[c];
            if (g.gc) gv = gv + gc[c];
            if (g.g_out) g.g_out[e] = gv;
          }
        }
        ops[0][qq] = sv;
        ops[1][qq] = yv;
        ops[2][qq] = gv;
      }
    }
  }
  lds_barrier();
  // ---- dots: every (history vector, new vector) dot is owned by one wave: 4Q exact fp64 products per lane,
  // a DPP wave sum, lane 0 stores the partial row entry (no LDS staging of the history values: staged
  // rows 1 KB apart put every quad of a wave on the same LDS banks) ----
  f32x4 s4[Q], y4[Q], g4[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    s4[q] = *reinterpret_cast<const f32x4 *>(&ops[0][256 * q + 4 * lane]);
    y4[q] = *reinterpret_cast<const f32x4 *>(&ops[1][256 * q + 4 * lane]);
    g4[q] = *reinterpret_cast<const f32x4 *>(&ops[2][256 * q + 4 * lane]);
  }
  double *rows = a.rows + blockIdx.x;
  const long long nb = a.nb;
#pragma unroll
  for (int j = 0; j < VPW; ++j) {
    const int v = wave + 4 * j; // wave-uniform
    if (v >= nvec) break;
    double ds = 0.0, dy = 0.0, dg = 0.0;
    if (!((zero_mask >> j) & 1u)) { // the slot being overwritten contributes zeros (gram_kernel's rule)
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const double x = live[q][c] ? double(vv[j][q][c]) : 0.0;
          ds += x * double(s4[q][c]);
          dy += x * double(y4[q][c]);
          dg += x * double(g4[q][c]);
        }
    }
    ds = wave_sum_f64(ds);
    dy = wave_sum_f64(dy);
    dg = wave_sum_f64(dg);
    if (lane == 0) {
      const int li = v < count0 ? v : v - count0, cc = v < count0 ? 0 : 1;
      rows[(long long)(6 * li + cc + 0) * nb] = ds;
      rows[(long long)(6 * li + cc + 2) * nb] = dy;
      rows[(long long)(6 * li + cc + 4) * nb] = dg;
    }
  }
  if (wave == 3) { // self block 6m + {s.s, s.y, y.y, g.s, g.y, g.g}
    double d[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double sv = s4[q][c], yv = y4[q][c], gv = g4[q][c];
        d[0] += sv * sv;
        d[1] += sv * yv;
        d[2] += yv * yv;
        d[3] += gv * sv;
        d[4] += gv * yv;
        d[5] += gv * gv;
      }
#pragma unroll
    for (int z = 0; z < 6; ++z) d[z] = wave_sum_f64(d[z]);
    if (lane == 0)
#pragma unroll
      for (int z = 0; z < 6; ++z) rows[(long long)(6 * h.m + z) * nb] = d[z];
  }
}

constexpr int DF_THREADS = 256;

// Column sums, then the last block runs the history step. Hand-off without fences (tail.hip's
// tail_cols_fin): sc1 column stores waited for before the arrival add; the last arrival reads them sc1.
__global__ __launch_bounds__(DF_THREADS) void dir_cols_fin_kernel(const DirArgs a) {
  const HistView &h = a.g.h;
  if (h.abort && *h.abort) return; // uniform for the launch: nobody arrives, the counter stays 0
  const int ncols = 6 * h.m + 6; // dir_ncols(m)
  extern __shared__ double dyn[]; // sy [2*m*m] (SY and its transpose) | yy [m*m] | SY, YY [S*S] | rho [S]
  __shared__ HistSmem sm;
  __shared__ double ws[4];
  __shared__ int s_last;
  __shared__ int ist_l[IST_ORDER + GRAM_FIN_MAXM + 4];
  const int t = threadIdx.x;
  KT(49);
  // row-major partials (the Gram sweep's, gram_fin): column c's values are ncols apart, so each XCD (blocks b and
  // b + 8 share one, xcd_tile's bijection) takes a contiguous range of columns and fetches their lines once
  int c = blockIdx.x;
  if (a.row_major) {
    const int q = ncols >> 3, r8 = ncols & 7, x = c & 7;
    c = (x < r8 ? x * (q + 1) : r8 * (q + 1) + (x - r8) * q) + (c >> 3);
  }
  const int count0 = a.g.reset ? 0 : h.ist[IST_COUNT];
  if (!(c < 6 * h.m && c >= 6 * count0)) { // only the columns in use (live pairs and the self block)
    const double *colp = a.rows + (a.row_major ? (long long)c : (long long)c * a.nb);
    const long long rs = a.row_major ? ncols : 1;
    double v[8];
    double s = 0.0;
    for (int r0 = t; r0 < a.nb; r0 += DF_THREADS * 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) { // unconditional loads from clamped rows: all eight in flight at once
        const int r = r0 + DF_THREADS * u;
        v[u] = colp[(r < a.nb ? r : 0) * rs];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (r0 + DF_THREADS * u < a.nb) ? v[u] : 0.0;
    }
    s = wave_sum_f64(s);
    if ((t & 63) == 0) ws[t >> 6] = s;
    lds_barrier();
    if (t == 0) {
      __hip_atomic_store(&a.dots[c], ((ws[0] + ws[1]) + ws[2]) + ws[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  if (t == 0)
    s_last = __hip_atomic_fetch_add(a.cols_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == unsigned(ncols - 1);
  __syncthreads();
  if (!s_last) return;
  if (t == 0) *a.cols_done = 0u; // ready for the next launch (stream-ordered)
  KTF(50);
  // ---- the history step, from LDS: dots, ring header, and (fused) SY, YY, rho ----
  const int m = h.m, S_ = h.slots;
  double *SYp = dyn + 3 * m * m, *YYp = SYp + S_ * S_, *rhop = YYp + S_ * S_;
  for (int q = t; q < 6 * m + 6; q += DF_THREADS) // sc1 loads: written this launch by other blocks
    sm.dots[q] = __hip_atomic_load(&a.dots[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t < IST_ORDER + m) ist_l[t] = h.ist[t];
  const bool fused = a.want_dir == 1 && !a.g.reset;
  if (fused) {
    for (int i = t; i < S_ * S_; i += DF_THREADS) {
      SYp[i] = h.SY[i];
      YYp[i] = h.YY[i];
    }
    if (t < S_) rhop[t] = h.rho[t];
  }
  lds_barrier();
  KTF(51);
  HistStep st;
  st.h = h;
  st.has_pair = a.g.has_pair;
  st.has_g = a.g.has_g;
  st.reset = a.g.reset;
  st.policy = a.g.policy;
  st.want_dir = a.want_dir;
  st.iter = a.iter;
  st.dsign = a.dsign;
  if (a.kmat && a.g.policy == POL_SLBFGS && m <= DIR_MAXM) { // the pair update's coefficient map (hist_core)
    st.kmat = a.kmat;
    st.kscr = rhop + S_; // after SY, YY, rho (cols_fin_launch sizes it)
  }
  if (fused) {
    st.ist = ist_l;
    st.rho = rhop;
    st.SY = SYp;
    st.YY = YYp;
    hist_prologue<true>(st, sm, ist_l[IST_WSLOT]);
    hist_core<true>(st, sm, dyn, 2 * m * m, dyn + 2 * m * m, m * m);
  } else {
    hist_prologue<false>(st, sm, ist_l[IST_WSLOT]);
    hist_core<false>(st, sm, dyn, 2 * m * m, dyn + 2 * m * m, m * m);
  }
}

// Column sums only (the S-LBFGS direction step, followed by dir_combine_kernel): plain stores, read by the
// next launch.
__global__ __launch_bounds__(DF_THREADS) void dir_cols_kernel(const DirArgs a) {
  const HistView &h = a.g.h;
  if (h.abort && *h.abort) return;
  __shared__ double ws[4];
  const int c = blockIdx.x, t = threadIdx.x;
  // The column's loads go out with the live count (one round trip for both): a column not in use (a pair slot
  // not yet live) sums whatever its rows hold and stores nothing.
  const int count0 = h.ist[IST_COUNT];
  const double *colp = a.rows + (long long)c * a.nb;
  double v[8];
  double s = 0.0;
  for (int r0 = t; r0 < a.nb; r0 += DF_THREADS * 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) { // unconditional loads from clamped rows: all eight in flight at once
      const int r = r0 + DF_THREADS * u;
      v[u] = colp[r < a.nb ? r : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (r0 + DF_THREADS * u < a.nb) ? v[u] : 0.0;
  }
  s = wave_sum_f64(s);
  if ((t & 63) == 0) ws[t >> 6] = s;
  lds_barrier();
  if (c < 6 * h.m && c >= 6 * count0) return; // only the columns in use (live pairs and the self block)
  if (t == 0) a.dots[c] = ((ws[0] + ws[1]) + ws[2]) + ws[3]; // dir_cols_fin's order
}

// The S-LBFGS direction step's coefficients and its combine in one launch (direction-only steps: has_g, no
// pair, no reset; k <= KQ live pairs). Every block stages the ring header, the dots and the pairs' coefficient
// map K (slbfgs_kmat, written by the last pair update: [cS; cY] = K [S^T g; Y^T g], one round trip with its g
// and x quads), issues its quads of the live history vectors, and while they are in flight wave 0 computes
// the 2k coefficients as one 2k x 2k mat-vec (the two-loop recursion of s_lbfgs.hpp:106-136 in compact form;
// before round 5 each block ran the two k-step recurrences here); then p = sum c_i basis_i and
// x_out = x + alpha p with combine_small's arithmetic. Block 0 also makes the step's global writes (g-dots,
// coefficients, scalars: hist_core's for this step; no block of the launch reads any of them, and the ring
// header every block reads is not written), so the state after the launch is what dir_cols_fin + combine
// leave.
template <int KQ>
__global__ __launch_bounds__(256) void dir_combine_kernel(const DirArgs a, const CombineArgs cb) {
  const HistView &h = a.g.h;
  if (h.abort && *h.abort) return;
  constexpr int MM = DIR_MAXM;
  __shared__ double sK[DIR_KS * DIR_KS];
  __shared__ double dl[6 * MM + 6], cf[2 * MM + 1];
  __shared__ int Ls[MM];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m = h.m, S_ = h.slots;
  // ---- round trip 1: header, dots, K and gamma; this lane's g and x ----
  // (K is staged for rows and columns < 2m, not < 2k: its loads then need no live count first, one round trip
  // for all; the rows and columns past 2k are not read)
  const int k = __builtin_amdgcn_readfirstlane(h.ist[IST_COUNT]);
  if (t < m) Ls[t] = h.ist[IST_ORDER + t];
  for (int i = t; i < 4 * m * m; i += 256) { // rows and columns < 2m of the DIR_KS-stride map
    const int r = i / (2 * m), c = i - r * (2 * m);
    sK[r * DIR_KS + c] = a.kmat[r * DIR_KS + c];
  }
  const double gamma = k > 0 ? a.kmat[DIR_KS * DIR_KS] : 1.0;
  const double kbuilt = a.kmat[DIR_KS * DIR_KS + 1]; // the live count K was built for (slbfgs_kmat)
  if (t < 6 * m + 6) dl[t] = a.dots[t];
  const long long n = h.n;
  const long long e = ((long long)blockIdx.x * 256 + t) * 4;
  const bool full = e + 3 < n;
  const long long eq = full ? e : 0; // the vector path's quad (clamped; the tail quad goes element-wise)
  const f32x4 g4 = *reinterpret_cast<const f32x4 *>(cb.g + eq);
  const f32x4 x4 = *reinterpret_cast<const f32x4 *>((cb.x_out ? cb.x_in : cb.g) + eq);
  lds_barrier();
  // K's layout depends on the count it was built for: a map out of step with the ring (no pair update since the
  // count changed, which the solver's order rules out) must not be applied. The step then writes NaN (x_out, dir)
  // and block 0 raises SC_KERR, which the solver checks at the epoch's end and fails on.
  const bool kbad = k > 0 && kbuilt != double(k);
  if (kbad && blockIdx.x == 0 && t == 0) h.scal[SC_KERR] = 1.0;
  // ---- round trip 2: this lane's quads of the live history vectors, in flight through the mat-vec ----
  f32x4 sv[KQ], yv[KQ];
  if (k > 0)
#pragma unroll
    for (int i = 0; i < KQ; ++i) {
      const long long off = (long long)Ls[i < k ? i : k - 1] * h.ld + eq;
      sv[i] = *reinterpret_cast<const f32x4 *>(h.S + off);
      yv[i] = *reinterpret_cast<const f32x4 *>(h.Y + off);
    }
  if (wave == 0) {
    // lane i < 2k: c_i = sum_j K[i][j] v_j, v = [S^T g ; Y^T g] (the fresh dots, logical order)
    double c = 0.0;
    if (lane < 2 * k)
      for (int j = 0; j < 2 * k; ++j) c += sK[lane * DIR_KS + j] * (j < k ? dl[6 * j + 4] : dl[6 * (j - k) + 5]);
    const double ds = a.dsign;
    const double gg = dl[6 * m + 5];
    if (lane < k) cf[lane] = ds * c;
    else if (lane < 2 * k) cf[MM + lane - k] = ds * c;
    if (lane == 0) cf[2 * MM] = ds * gamma;
    if (blockIdx.x == 0) { // hist_core's global writes for this step (FUSED, has_g, no pair, want_dir 1)
      const double v = lane < k ? dl[6 * lane + 4] : (lane < 2 * k ? dl[6 * (lane - k) + 5] : 0.0);
      const double gTz = wave_sum_f64(lane < 2 * k ? c * v : 0.0) + gamma * gg;
      if (lane < k) {
        const int j = Ls[lane];
        h.gS[j] = dl[6 * lane + 4];
        h.gY[j] = dl[6 * lane + 5];
        h.coef[lane] = ds * c;
      } else if (lane < 2 * k) {
        h.coef[S_ + lane - k] = ds * c;
      }
      if (lane == 0) {
        h.coef[2 * S_] = ds * gamma;
        h.scal[SC_RESET] = 0.0;
        h.scal[SC_GTP] = ds * gTz;
        // (the live count is unchanged by a direction-only step: the ring header, which every block reads
        // at its start, is not written here)
        h.scal[SC_COUNT] = double(k);
        h.scal[SC_GG] = gg;
        h.scal[SC_GAMMA] = gamma;
        h.scal[SC_ALPHA0] = (a.iter == 0) ? fmin(1.0, 1.0 / sqrt(gg)) : 1.0;
      }
    }
  }
  lds_barrier();
  // ---- combine (combine_small's arithmetic per element) ----
  const double cg = kbad ? __builtin_nan("") : cf[2 * MM];
  const double alpha = cb.alpha;
  if (full) {
    f32x4 d4, o4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double acc = cg * double(g4[c]);
#pragma unroll
      for (int i = 0; i < KQ; ++i)
        if (i < k) acc += cf[i] * double(sv[i][c]) + cf[MM + i] * double(yv[i][c]);
      d4[c] = float(acc);
      o4[c] = x4[c] + float(alpha) * d4[c];
    }
    if (cb.dir) *reinterpret_cast<f32x4 *>(cb.dir + e) = d4;
    if (cb.x_out) {
      *reinterpret_cast<f32x4 *>(cb.x_out + e) = o4;
      if (cb.x_out2) *reinterpret_cast<f32x4 *>(cb.x_out2 + e) = o4;
    }
  } else {
    for (long long q = e; q < n; ++q) { // the tail quad, element-wise (no read past n)
      double acc = cg * double(cb.g[q]);
      for (int i = 0; i < k; ++i) {
        const long long off = (long long)Ls[i] * h.ld + q;
        acc += cf[i] * double(h.S[off]) + cf[MM + i] * double(h.Y[off]);
      }
      const float d = float(acc);
      if (cb.dir) cb.dir[q] = d;
      if (cb.x_out) {
        const float o = cb.x_in[q] + float(alpha) * d;
        cb.x_out[q] = o;
        if (cb.x_out2) cb.x_out2[q] = o;
      }
    }
  }
}

template <int C, bool GRED>
void launch_sweep(hipStream_t s, const DirArgs &a, int vpw) {
  switch (vpw) {
  case 2: hipLaunchKernelGGL((dir_sweep_kernel<C, 2, GRED>), dim3(unsigned(a.nb)), dim3(256), 0, s, a); break;
  case 4: hipLaunchKernelGGL((dir_sweep_kernel<C, 4, GRED>), dim3(unsigned(a.nb)), dim3(256), 0, s, a); break;
  case 6: hipLaunchKernelGGL((dir_sweep_kernel<C, 6, GRED>), dim3(unsigned(a.nb)), dim3(256), 0, s, a); break;
  case 8: hipLaunchKernelGGL((dir_sweep_kernel<C, 8, GRED>), dim3(unsigned(a.nb)), dim3(256), 0, s, a); break;
  default: throw Error(2, "dir_sweep: history size not supported");
  }
}

} // namespace

static int dir_vpw(int m) {
  const int per_wave = (2 * m + 3) / 4;
  return per_wave <= 2 ? 2 : per_wave <= 4 ? 4 : per_wave <= 6 ? 6 : per_wave <= 8 ? 8 : 16;
}
// Columns per block: 256 (one quad per lane) or, by default, 512 (two): at n = 535,818 (cfg 4) 256-column
// blocks are 2093, above the 1792 this kernel's 88 SGPRs admit at once (7 per CU), so the sweep ran in
// two rounds; 1047 blocks of 512 columns run in one, with twice the loads in flight per lane.
// m <= 16.
static int dir_c() { return 8; }
bool dir_supported(int m, long long n) { return m >= 0 && m <= DIR_MAXM && n > 0 && n <= DIR_MAXN; }
int dir_cols_per_block(int m, long long n) {
  (void)m;
  (void)n;
  return 64 * dir_c();
}
int dir_ncols(int m) { return 6 * m + 6; }

void dir_sweep(hipStream_t s, const DirArgs &a) {
  LBF_REQUIRE(dir_supported(a.g.h.m, a.g.h.n), "dir_sweep: history size / vector length");
  LBF_REQUIRE(a.want_dir == 0 || a.want_dir == 1, "dir_sweep: want_dir 0 / 1");
  LBF_REQUIRE(a.nb == int(cdiv(a.g.h.n, dir_cols_per_block(a.g.h.m, a.g.h.n))), "dir_sweep: block count");
  if (a.gred_on) launch_sweep<8, true>(s, a, dir_vpw(a.g.h.m));
  else launch_sweep<8, false>(s, a, dir_vpw(a.g.h.m));
  LBF_KERNEL_CHECK();
}

static void cols_fin_launch(hipStream_t s, const DirArgs &a) {
  // m up to GRAM_FIN_MAXM: ~100 KB of dynamic LDS; once per process, thread-safe
  static const bool attr_set = [] {
    LBF_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(dir_cols_fin_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 16 * 1024));
    return true;
  }();
  (void)attr_set;
  const int m = a.g.h.m, S_ = a.g.h.slots;
  const size_t shmem = (size_t(3) * m * m + 2 * size_t(S_) * S_ + S_ + size_t(DIR_MAXM) * DIR_MAXM) * sizeof(double);
  hipLaunchKernelGGL(dir_cols_fin_kernel, dim3(unsigned(dir_ncols(m))), dim3(DF_THREADS), shmem, s, a);
  LBF_KERNEL_CHECK();
}

void dir_fin(hipStream_t s, const DirArgs &a) { cols_fin_launch(s, a); }

bool dir_combine_supported(const DirArgs &a, const CombineArgs &c) {
  const GramArgs &g = a.g;
  return a.want_dir == 1 && g.has_g && !g.has_pair && !g.reset && g.policy == POL_SLBFGS && g.h.m <= DIR_MAXM &&
         !c.alpha_from_state && g.h.ld % 4 == 0 && a.kmat != nullptr;
}

void dir_cols_combine(hipStream_t s, const DirArgs &a, const CombineArgs &c) {
  LBF_REQUIRE(dir_combine_supported(a, c), "dir_cols_combine: direction-only S-LBFGS step, m <= DIR_MAXM");
  hipLaunchKernelGGL(dir_cols_kernel, dim3(unsigned(dir_ncols(a.g.h.m))), dim3(DF_THREADS), 0, s, a);
  LBF_KERNEL_CHECK();
  const dim3 grid(unsigned(cdiv(a.g.h.n, 1024)));
  const int m = a.g.h.m; // live pairs k <= m
  if (m <= 4) hipLaunchKernelGGL(dir_combine_kernel<4>, grid, dim3(256), 0, s, a, c);
  else if (m <= 8) hipLaunchKernelGGL(dir_combine_kernel<8>, grid, dim3(256), 0, s, a, c);
  else if (m <= 10) hipLaunchKernelGGL(dir_combine_kernel<10>, grid, dim3(256), 0, s, a, c); // cfg 4
  else if (m <= 12) hipLaunchKernelGGL(dir_combine_kernel<12>, grid, dim3(256), 0, s, a, c);
  else hipLaunchKernelGGL(dir_combine_kernel<16>, grid, dim3(256), 0, s, a, c);
  LBF_KERNEL_CHECK();
}

bool gram_fin_supported(int m) { return m >= 0 && m <= GRAM_FIN_MAXM; }

void gram_fin(hipStream_t s, const DirArgs &a) {
  LBF_REQUIRE(gram_fin_supported(a.g.h.m), "gram_fin: history size");
  LBF_REQUIRE(a.want_dir == 0 || a.want_dir == 1, "gram_fin: want_dir 0 / 1");
  LBF_REQUIRE(a.nb == gram_nwg(a.g.h.n), "gram_fin: one partial row per Gram workgroup");
  cols_fin_launch(s, a);
}

} // namespace lbf

#ifdef LBF_KTRACE
extern "C" int lbf_dbg_ktrace_dir(unsigned long long *host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lbf::lbf_kt_buf), size_t(n) * 8) == hipSuccess ? 0 : 1;
}
#endif
