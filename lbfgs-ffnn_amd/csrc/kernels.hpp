// Kernel launcher interfaces (implemented in gemm.hip / vec_kernels.hip) and the device-resident
// L-BFGS history layout shared by host and device code.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace lbf {

enum Act : int { ACT_LINEAR = 0, ACT_TANH = 1, ACT_RELU = 2, ACT_SIGMOID = 3 };

// ------------------------------------------------------------------------------------------------
// GEMM  C[M x N] (row-major, ldc) = op(A)[M x K] * op(B)[K x N]   (fp32 in, fp32 MFMA accumulate)
//   a_kc: A stored k-contiguous   A[m*lda + k]  (else m-contiguous A[k*lda + m])
//   b_kc: B stored k-contiguous   B[n*ldb + k]  (else n-contiguous B[k*ldb + n])
//   a_idx: optional row gather of the stored A rows (k-contiguous: rows = m; m-contiguous: rows = k)
//   a_mvalid / a_ones: m-contiguous A only — columns >= a_mvalid read 0 except column a_ones == 1
//                      (turns dW = A^T dZ into [dW ; db] in one GEMM, the flat layer segment).
// Epilogues: FWD   C = act(acc + bias[n])
//            DX    C = acc * act'(aux[m*ldaux + n])       (act' from the post-activation value)
//            STORE C(+ split*slab_stride) = acc           (split-K partial slabs)
// ------------------------------------------------------------------------------------------------
// Tile shapes: TILE_AUTO = 128 rows x (128 | 64 | 32 by N); TILE_32x128 (few row tiles: a rank's
// shard); TILE_64x64 (split-K weight gradients with fewer, longer splits); TILE_64x128 (mid-size
// shards: two workgroups per CU where 128-row tiles would leave one).
enum GemmTile : int { TILE_AUTO = 0, TILE_32x128 = 1, TILE_64x64 = 2, TILE_64x128 = 3 };
enum GemmEpi : int { EPI_FWD = 0, EPI_DX = 1, EPI_STORE = 2, EPI_HEAD = 3 };

struct EarlyLs;

struct GemmDesc {
  int M = 0, N = 0, K = 0;
  const float *A = nullptr;
  long long lda = 0;
  bool a_kc = true;
  const int *a_idx = nullptr;
  int a_mvalid = 0, a_ones = -1;
  const float *B = nullptr;
  long long ldb = 0;
  bool b_kc = false;
  float *C = nullptr;
  long long ldc = 0, slab_stride = 0;
  int splits = 1, k_chunk = 0;
  int epi = EPI_FWD;
  int tile = TILE_AUTO;
  const float *bias = nullptr;
  int act = ACT_LINEAR;
  const float *aux = nullptr;
  long long ldaux = 0;
  int aux_act = ACT_LINEAR;
  const int *abort = nullptr; // speculative execution: the kernel is a no-op when *abort != 0
  const EarlyLs *early = nullptr; // the trial's first backward launch: its Armijo test first (EarlyLs)
  // A from the previous layer's forward split-K slabs (a_slab non-null; only where gemm_asum_ok): each
  // workgroup forms its A tiles as act(sum_s a_slab[s * a_slab_stride + .] + a_bias) (fwd_reduce_act's
  // arithmetic, splits in order) in its prologue, and the workgroups of column tile 0 also write them to
  // a_out (row stride lda), which replaces the fwd_reduce_act launch of the previous layer.
  const float *a_slab = nullptr;
  int a_splits = 0;
  long long a_slab_stride = 0;
  const float *a_bias = nullptr;
  int a_act = ACT_LINEAR;
  float *a_out = nullptr;
  // Side job riding in an extra z-plane of the launch: side_dst[c] = sum_s side_slab[s*stride + c]
  // (fixed split order, fp64) for c < side_count. Used to finish the fused head's [dW ; db] slabs
  // while the next layer's dW GEMM runs.
  const float *side_slab = nullptr;
  int side_splits = 0;
  long long side_stride = 0, side_count = 0;
  float *side_dst = nullptr;
  // EPI_HEAD (forward GEMM of the last hidden layer, N <= the tile width): bias + activation, then the
  // output layer on each 64-row half in LDS (head_core.hpp) instead of storing the activations.
  const float *head_P = nullptr; // [W ; b] of the output layer
  int head_out = 0, head_act = ACT_LINEAR;
  const float *head_Y = nullptr;
  const int *head_idx = nullptr; // minibatch rows of Y (nullable)
  double head_inv_scale = 1.0;
  float *head_delta = nullptr, *head_slab = nullptr; // slab per workgroup: [(N+1) x head_out]
  double *head_sse = nullptr;                        // SSE partial per workgroup
  // Fold (head_fold >= 0, N <= 128): this layer's [dW ; db] rows head_fold_c0 .. K (input columns
  // head_fold_c0 .. K-1, head_fold = K - head_fold_c0 <= 16 of them, % 4 == 0, then the bias row) are
  // accumulated in the epilogue and written in front of the head's rows: the slab per workgroup is
  // then [(head_fold + 1) x N | (N+1) x head_out], and the dW GEMM covers rows < head_fold_c0 only.
  int head_fold = -1, head_fold_c0 = 0;
};
// Row tiles of the forward GEMM for M rows and N columns (== EPI_HEAD partial slabs).
int gemm_row_tiles(int M, int tile);

// Whether gemm() can take d's A from the previous layer's slabs (a_slab): the 32 x 128 k-contiguous
// forward split-K tile, no row gather, a k-chunk of at most four k-tiles, 16-B aligned operands.
bool gemm_asum_ok(const GemmDesc &d);
// Two GEMMs of the 64 x 64 mn-contiguous split-K dW shape in ONE launch (d1 may carry a side job): the
// S-LBFGS minibatch's dW GEMMs of adjacent layers once both deltas exist.
bool gemm_group_ok(const GemmDesc &d1, const GemmDesc &d2);
void gemm_group(hipStream_t s, const GemmDesc &d1, const GemmDesc &d2);
void gemm(hipStream_t s, const GemmDesc &d);
// Tile (BM, BN) the dispatcher picks for a given N (used by the split-K planner).
void gemm_tile_for(int N, int tile, int *BM, int *BN);

// ------------------------------------------------------------------------------------------------
// Vector / reduction kernels (vec_kernels.hip). All reductions are deterministic: per-workgroup
// fp64 partials written to memory, then summed in a fixed order by reduce_rows.
// ------------------------------------------------------------------------------------------------
// out[c] = sum_r P[r*ncols + c], r in [0, nrows), fixed order.    (one wave per column)
void reduce_rows(hipStream_t s, const double *P, int nrows, int ncols, double *out);
// Partial fold of a tall table: `groups` row groups -> out[g][ncols] (fixed order); returns the number of
// row groups actually written.
int fold_rows(hipStream_t s, const double *P, int nrows, int ncols, int groups, double *out);

// Output layer: d = act_out(Z) already in A_out; diff = A_out - Y[idx? idx[b] : b];
// dZ = diff * act'(A_out) * inv_scale ; per-WG partial of sum(diff^2) -> partials[wg].
int loss_partials_wg(long long B, int Out);
void loss_diff(hipStream_t s, const float *Aout, long long lda, const float *Y, long long ldy, const int *idx,
               long long B, int Out, int act, double inv_scale, float *dZ, long long ldz, double *partials);

// Fused output layer (head.hip): forward + MSE + dZ + delta_prev + per-tile [dW ; db] slabs.
bool head_supported(int H, int Out);
int head_tile(int H);
int head_nwg(long long B, int H);
void head_fused(hipStream_t s, const float *A, int H, const float *P, int Out, const float *Y, const int *idx,
                long long B, int act_out, int act_prev, double inv_scale, float *delta, float *slab,
                double *sse_part, const int *abort = nullptr);

// The same output layer fed straight from the last hidden layer's forward split-K slabs (small batches,
// e.g. S-LBFGS's 256-row minibatches on 784-512-256-10): one wave per sample row finishes the row's
// activations exactly as fwd_reduce_act would (fp32 split order, + bias, act_prev) and runs the head on
// them, so the last hidden layer's reduce launch and the tile-based head become one launch. One
// [dW ; db] partial slab ((H + 1) x Out) and SSE partial per workgroup, like head_fused.
struct RowHeadArgs {
  const float *fslab = nullptr; // [splits][B][H] forward partial slabs of the last hidden layer
  int splits = 0;
  long long stride = 0;         // floats per split (B * H)
  const float *hbias = nullptr; // the hidden layer's bias
  int act_prev = 0;
  const float *P = nullptr;     // the output layer's [W (H x Out) | b]
  int H = 0, Out = 0, act_out = 0;
  const float *Y = nullptr;
  const int *idx = nullptr;
  long long B = 0;
  int rpw = 1;                  // rows per wave
  double inv_scale = 1.0;
  float *delta = nullptr, *slab = nullptr;
  double *sse_part = nullptr;
  const int *abort = nullptr;
};
bool rowhead_supported(int H, int Out);
int rowhead_rpw(long long B);
int rowhead_nwg(long long B); // workgroups == partial slabs
void rowhead(hipStream_t s, const RowHeadArgs &a);

// grad[e] = sum_s slab[s*stride + e] * scale (fixed order), e in [0, count)
// Forward split-K finish: out = act(sum_s slab[s] + bias), slabs summed in split order (fp32, like
// the GEMM's own accumulation).
void fwd_reduce_act(hipStream_t s, const float *slab, int splits, long long stride, int M, int N, const float *bias,
                    int act, float *out, const int *abort);
void reduce_slabs(hipStream_t s, const float *slab, int splits, long long stride, long long count, float *grad,
                  const int *abort = nullptr);

// g += lambda*w (if lambda != 0); per-WG partials of (g.g, g.p, w.w) -> partials[wg*3 + {0,1,2}]
int dots_partials_wg(long long n);
// Two launches for the whole evaluation tail: every layer's [dW ; db] segment is reduced from its
// split-K / head partial slabs (fixed order, fp64), or taken as written (splits == 0). Column groups
// with many slabs are split over several blocks by split range and combined in range order by the
// second launch (one block). With `dots` (single rank) they also apply g += lambda*w and write
// per-group (g.g, g.p, w.w) partials, which the second launch reduces with the SSE partials into the
// status block like eval_tail. No grid-wide ticket: an agent-scope fence right after the GEMM's slab
// writes costs tens of microseconds (dirty-L2 write-back on every XCD).
constexpr int RA_MAXSEG = 17;
struct RedSeg {
  const float *slab = nullptr;
  long long stride = 0, count = 0, goff = 0;
  int splits = 0;
  int parts = 1; // blocks per 64-column group, each over a contiguous range of splits
  int gpb = 1;   // parts == 1: 64-column groups per block (RA_GPB while the splits are few)
  int wg0 = 0;   // first block of the segment (reduce launch)
  int cg0 = 0;   // first column group of the segment (global numbering)
  int fin0 = -1; // parts > 1: first block of the segment in the finishing launch
};
struct RedAllArgs {
  RedSeg seg[RA_MAXSEG];
  int nseg = 0, nwg = 0;
  float *G = nullptr;
  const float *w = nullptr, *p = nullptr;
  double lambda = 0.0;
  int dots = 0;
  int l2 = 0;                   // apply g += lambda w here (single rank; data parallel: after the all-reduce)
  double *partials = nullptr;   // [ncg][3] dot partials
  double *colpart = nullptr;    // [ncg][RA_MAXPART][64] split-range partials
  int ncg = 0;
  int nfin = 0;                 // column groups with parts > 1
  const double *sse_part = nullptr;
  int nsse = 0;
  double inv_scale = 1.0;
  double *scal = nullptr;
  const int *abort = nullptr;
  float *sse_hilo = nullptr;    // data parallel: one extra block packs sum(sse_part[0..nsse)) as fp32 (hi, lo) here
};
constexpr int RA_COLS = 64;
constexpr int RA_GPB = 4; // column groups per reduce_all block for single-pass segments
constexpr int RA_MAXPART = 32;
constexpr int RA_SPLITS_PER_PART = 64; // 4 stripes x 16 loads per thread
constexpr int RA_MAXFIN = 128;         // column groups the one-block finishing launch combines
void reduce_all(hipStream_t s, const RedAllArgs &a);

// Exact Hessian-vector product, elementwise R-steps (hvp.hip; products in Mlp::hvp).
void rop_act(hipStream_t s, long long n, const float *A, const float *RZ, int act, float *RA);
void rop_out(hipStream_t s, long long B, int Out, const float *A, const float *Y, const int *idx, const float *RZ,
             int act, double inv_scale, float *RdZ);
void rop_back(hipStream_t s, long long n, const float *T1, const float *T2, const float *delta, const float *A,
              const float *RZ, int act, float *out);
bool act_has_d2(int act);

// BASELINE config 5's synthetic regression data on the device (synth.hip).
void synth_regression(hipStream_t s, long long row0, long long N, int In, unsigned seed_x, unsigned seed_t, float *X,
                      float *Y);

void finalize_grad_dots(hipStream_t s, long long n, float *g, const float *w, double lambda, const float *p,
                        double *partials, const int *abort = nullptr, const float *g_in = nullptr);
// generic: per-WG partials of x.y -> partials[wg]
void dot_partials(hipStream_t s, long long n, const float *x, const float *y, double *partials);

// scal[LOSS] = 0.5 * sse * inv_scale + 0.5*lambda*ww, with sse from sse_d (double) or, when sse_hilo
// is non-null, sse = hilo[0] + hilo[1] (all-reduced split fp32 pair).
void eval_status(hipStream_t s, const double *sse_d, const float *sse_hilo, double inv_scale, double lambda,
                 double *scal);
// One-workgroup tail: reduce finalize dots (+ SSE partials unless hilo) and write SC_TGG/TGP/WW/SSE/LOSS.
void eval_tail(hipStream_t s, const double *dots_part, int nd, const double *sse_part, int nsse, const float *hilo,
               double inv_scale, double lambda, double *scal, const int *abort = nullptr);
// DP: reduce SSE partials into an fp32 (hi, lo) pair (all-reduced together with the gradient).
// Loss-only status of a forward pass: SC_SSE / SC_LOSS from the SSE partials (reduce_fin's order) or,
// data parallel, from the all-reduced (hi, lo) pair.
void sse_loss(hipStream_t s, const double *sse_part, int nsse, const float *hilo, double inv_scale, double *scal,
              const int *abort);
void sse_pack(hipStream_t s, const double *sse_part, int nsse, float *hilo, const int *abort = nullptr);
// hilo[0] = float(x), hilo[1] = float(x - hilo[0])
void pack_hilo(hipStream_t s, const double *x, float *hilo);

void axpy(hipStream_t s, long long n, float alpha, const float *x, float *y);
void scal(hipStream_t s, long long n, float alpha, float *x);
// y = x + alpha * p
void axpy_to(hipStream_t s, long long n, const float *x, float alpha, const float *p, float *y);
// GD / SGD momentum step and SGD's device-side epoch-loss accumulator (vec_kernels.hip).
void momentum_step(hipStream_t s, long long n, float momentum, float lr, const float *lr_dev, const float *g, float *v,
                   float *x);
void epoch_loss_acc(hipStream_t s, const double *scal, long long rows, float *esum);
// u = (sum_i W[slot_i]) / cnt  in logical order, fp64 accumulation
void average_slots(hipStream_t s, long long n, const float *W, long long ld, const int *h_slots, int cnt, float *u);
// out = a + c*b
void lincomb(hipStream_t s, long long n, const float *a, double c, const float *b, float *out);
// G[r * ld + e] += lambda w[e], r < rows, e < n (finalize_kernel's fp32 update on a block of gradients)
void add_l2_rows(hipStream_t s, long long n, int rows, long long ld, float *G, const float *w, double lambda);
void gather_rows(hipStream_t s, const float *src, long long ld, const int *idx, long long count, int cols,
                 float *dst);
// order-independent fingerprints of x into out[4 slot .. 4 slot + 3] (exact 16-bit halves as floats)
void fingerprint(hipStream_t s, long long n, const float *x, int slot, float *out);
void diff_scale(hipStream_t s, long long n, const float *a, const float *b, float scale, float *out);
void zero_fill(hipStream_t s, long long n, float *x, const int *abort = nullptr);
// dst = sum_i src[i] over the ranks of an in-process group, in rank order (comm.cpp LocalComm)
constexpr int kMaxLocalRanks = 16;
struct RankSrcs {
  int n = 0;
  const float *p[kMaxLocalRanks] = {};
};
void sum_ranks(hipStream_t s, const RankSrcs &r, long long count, float *dst);

// ------------------------------------------------------------------------------------------------
// Device-resident L-BFGS history ("vector-free" two-loop: Chen, Wang & Zhou, NIPS 2014).
// Vectors s_i, y_i live in slots of S/Y (slots = m+1 so a rejected pair never clobbers live data);
// the Gram matrices of all stored vectors are kept in fp64 and the two-loop recursion of the
// reference runs on (2k+1) coefficients, so a direction costs two HBM sweeps of the history
// (dots, then one linear combination) instead of 2k dependent dot/axpy launches.
// ------------------------------------------------------------------------------------------------
enum HistPolicy : int { POL_CPU = 0, POL_CUDA = 1, POL_SLBFGS = 2 };

// istate (int32)
enum { IST_COUNT = 0, IST_FREE = 1, IST_WSLOT = 2, IST_ORDER = 4 };
// scal (fp64) block, read back to the host in one copy
enum {
  SC_GG = 0,      // g.g of the vector the direction was built for
  SC_GTP = 1,     // g^T dir
  SC_ALPHA0 = 2,  // first trial step (min(1, 1/||g||) at iteration 0, else 1)
  SC_GAMMA = 3,
  SC_YS = 4,      // y.s of the last pair
  SC_ACCEPT = 5,  // last pair accepted
  SC_COUNT = 6,   // live pairs
  SC_RESET = 7,   // CUDA descent fallback fired
  SC_LOSS = 8,    // last evaluation: loss
  SC_TGG = 9,     //                  g.g
  SC_TGP = 10,    //                  g.p
  SC_WW = 11,     //                  w.w
  SC_SSE = 12,    //                  local sum of squared errors (before reduction over ranks)
  SC_FOLD = 13,   // speculative line search: loss of the last accepted iterate (fp64, Wolfe)
  SC_FOLDF = 14,  //                          same, as the fp32 value the Armijo test uses
  SC_KERR = 15,   // S-LBFGS: a direction step found the coefficient map K built for another live count (sticky)
  SC_N = 16
};

// Speculative line search (LbfgsSolver::iterate_spec): after the first trial of an iteration, one
// thread applies the host's acceptance test to the device status block, writes the outcome into a
// host-mapped record and, on rejection or convergence, raises the abort flag so every launch already
// queued behind it is a no-op until the host rolls back.
struct SpecRecord {
  double loss;        // trial loss (SC_LOSS)
  double tgg;         // trial g.g  (SC_TGG)
  double alpha0;      // SC_ALPHA0 (first trial step computed on the device)
  double accept_prev; // SC_ACCEPT (whether the previous pair entered the ring)
  int status;         // SPEC_ACCEPT / SPEC_CONVERGED / SPEC_REJECT / SPEC_REJECT_EARLY
  int seq;            // written last
};
// SPEC_REJECT_EARLY: rejected on sufficient decrease by the trial's first backward GEMM (EarlyLs), so the
// trial's backward and tail never ran (tgg is 0; SC_LOSS / SC_SSE of the status block are written)
enum { SPEC_ACCEPT = 1, SPEC_CONVERGED = 2, SPEC_REJECT = 3, SPEC_REJECT_EARLY = 4 };
struct LsCtlArgs {
  double *scal = nullptr;
  int *abort = nullptr;
  SpecRecord *rec = nullptr; // host-mapped
  int seq = 0;
  int armijo = 0;            // 0: Wolfe (lbfgs.hpp:49-70), 1: Armijo (lbfgs.cuh:159-163)
  int first = 0;             // Wolfe: iteration 0 takes alpha0 without a search
  int host_fold = 0;         // use fold/foldf below instead of SC_FOLD/SC_FOLDF
  double fold = 0.0;
  float foldf = 0.0f;
  double c1 = 0.0, c2 = 0.0, tol = 0.0;
  float alphaf = 1.0f;       // Armijo trial step
  double alpha = 1.0;        // Wolfe trial step (1: a speculative first trial; else a host-finished search's)
};
void ls_ctl(hipStream_t s, const LsCtlArgs &a);

// Early Armijo test of a speculative first trial (single rank, lambda = 0; GemmDesc::early): every block of
// the trial's first backward GEMM sums the forward's SSE partials exactly as the fused tail's decision does
// (tail_fin_body), applies ls_rule.hpp's sufficient-decrease test and, when it fails, exits; block 0 then
// publishes the rejection (SC_LOSS, SC_SSE, the abort flag, the host record as SPEC_REJECT_EARLY), so the
// trial's backward GEMMs and tail are skipped. A rejected first trial needs no gradient
// (full_batch_minimizer.hpp:138-141, lbfgs.cuh:159-163), so only the work changes, not the results.
struct EarlyLs {
  const double *sse_part = nullptr; // the forward's SSE partials (Mlp loss_part_)
  int nsse = 0;
  double inv_scale = 0.0;
  LsCtlArgs ls;
};

struct HistView {
  int m = 0, slots = 0;
  long long n = 0, ld = 0; // vector length, slot stride (floats)
  float *S = nullptr, *Y = nullptr;
  int *ist = nullptr;
  double *rho = nullptr, *SS = nullptr, *SY = nullptr, *YY = nullptr, *gS = nullptr, *gY = nullptr;
  double *coef = nullptr; // [2*slots + 1]: cs (logical), cy (logical), cg
  double *scal = nullptr; // SC_N
  const int *abort = nullptr; // speculative execution flag (nullable)
};

struct GramArgs {
  HistView h;
  // pair: s = sa - sb ; y = (ya - yb) * yscale, written into slot ist[IST_WSLOT] (set by gram_select)
  const float *sa = nullptr, *sb = nullptr, *ya = nullptr, *yb = nullptr;
  double yscale = 1.0;
  int has_pair = 0;
  // vector: g = ga - gb + gc (gb, gc nullable), optionally materialised into g_out
  const float *ga = nullptr, *gb = nullptr, *gc = nullptr;
  float *g_out = nullptr;
  int has_g = 0;
  int reset = 0; // treat the history as empty before the push (CUDA reset_history)
  int policy = POL_CPU;
};
// Number of fp64 partial columns per workgroup and the workgroup count for a given n.
int gram_ncols(int m);
int gram_nwg(long long n);
// Chooses the write slot (device), then streams the history once computing all new dots. Partials
// [gram_nwg(n)][gram_ncols(m)], or transposed ([gram_ncols(m)][gram_nwg(n)], gram_fin's input).
void gram_update(hipStream_t s, const GramArgs &a, double *partials, int transposed = 0);

struct CoefArgs {
  HistView h;
  const double *partials = nullptr; // gram_update's per-workgroup partials [nwg][gram_ncols(m)]
  int nwg = 0;
  int has_pair = 0, has_g = 0, reset = 0, policy = POL_CPU;
  int want_dir = 1;
  int iter = 1;
  int stage = 0;  // LDS doubles for staging partial rows (set by hist_coef)
  int sy_cap = 0; // LDS doubles for SY (and its transpose) (set by hist_coef)
  int fused = 0;  // hist_core<true>: SY, YY, rho prefetched into LDS, stores off wave 0 (set by hist_coef)
  double dsign = -1.0;
};
int hist_stage_rows(int m);
void hist_coef(hipStream_t s, const CoefArgs &a);

// Fused optimizer tail of a speculative L-BFGS iteration (tail.hip): the evaluation's gradient
// columns, the new pair s = x_t - x_prev, y = g_t - g_prev written into the ring's write slot, the
// Gram sweep of (s, y, g_t) against the live history (one partial row per block), then one block
// that takes the line-search decision and, on acceptance, pushes the pair and computes the next
// direction's coefficients (hist_core.hpp). Row layout (nc = 6m + 8 doubles): the Gram sweep's
// columns (see hist_core.hpp), then g.p and w.w.
constexpr int TAIL_MAXM = 32;
constexpr int TAIL_COLS = 128; // columns per tail_reduce block
struct TailArgs {
  RedAllArgs ra;                // every segment with parts == 1; ra.w = x_t, ra.p = direction
  const float *hilo = nullptr;  // data parallel: all-reduced SSE (hi, lo) behind the gradient
  // data parallel: the all-reduced gradient words to read the columns from (segments taken as written);
  // the tail then writes ra.G. Never ra.G itself: an aborted speculative iteration's collective still
  // runs, so it must not land in a buffer that may hold the live gradient.
  const float *g_src = nullptr;
  HistView h;
  int has_pair = 0;
  const float *x_prev = nullptr, *g_prev = nullptr;
  int policy = POL_CPU;
  int iter_next = 1;
  LsCtlArgs ls;
  double *rows = nullptr; // [nb][nc]
  double *dots = nullptr; // [nc]
  int tcg0[RA_MAXSEG] = {}; // first TAIL_COLS column group of each segment
  int nb = 0, nc = 0;       // nb: TAIL_COLS column groups over all segments (one block each)
  // Arrival counter (zero between launches): the last tail_cols block to finish runs the one-block fin.
  unsigned *cols_done = nullptr;
};
void tail_reduce(hipStream_t s, const TailArgs &a); // tail_reduce + tail_cols_fin launches
int tail_vpw(int m);                                // vectors per wave of the Gram sweep (0: unsupported)

// S-LBFGS history update in two launches (dir.hip): a one-round-trip Gram sweep of the new s / y / g
// against the live history (one block per 64*C columns, a partial row each, stored [nc][nb]), then one
// block per Gram column whose last arrival runs the history step (hist_core.hpp) from the column sums.
constexpr int DIR_MAXM = 16;
// The S-LBFGS direction's coefficient map K ([cS; cY] = K [S^T g; Y^T g], hist_core.hpp slbfgs_kmat): row stride
// DIR_KS, then gamma at [DIR_KS * DIR_KS] and the live count k it was built for at [DIR_KS * DIR_KS + 1]
constexpr int DIR_KS = 2 * DIR_MAXM;
constexpr int DIR_KMAT_N = DIR_KS * DIR_KS + 4;
constexpr long long DIR_MAXN = 1LL << 22;
struct CombineArgs {
  HistView h;
  const float *g = nullptr; // the vector the direction was built for
  float *dir = nullptr;     // nullable
  const float *x_in = nullptr;
  float *x_out = nullptr, *x_out2 = nullptr; // x_out = x_in + alpha*dir ; x_out2 = copy of x_out
  int alpha_from_state = 1;                  // alpha = scal[SC_ALPHA0]
  double alpha = 1.0;
};
struct DirArgs {
  GramArgs g;               // operands, policy, has_pair / has_g, reset; g.h carries the abort flag
  int want_dir = 1;         // 0 (pair only) or 1
  int iter = 1;
  double dsign = 1.0;
  double *rows = nullptr;   // [dir_ncols(m)][nb], or [nb][dir_ncols(m)] when row_major (gram_fin)
  int row_major = 0;
  double *dots = nullptr;   // [dir_ncols(m)]
  int nb = 0;               // cdiv(n, dir_cols_per_block(m, n))
  unsigned *cols_done = nullptr; // arrival counter, zero between launches
  // gred_on: g.ga's values are finished here from split-K slabs (reduce_all's arithmetic: per column the
  // splits in four stripes k = 0, 4, ..., then ((s0 + s1) + s2) + s3 in fp64, float, + lambda w in fp32)
  // instead of read; segments without splits (finished by the dW launch's side blocks) read gred.G
  RedAllArgs gred;
  int gred_on = 0;
  // S-LBFGS (POL_SLBFGS, k <= DIR_MAXM): the coefficient map of the live pairs, written by every pair update
  // (dir_fin) and read by the direction-only steps (dir_cols_combine); DIR_KMAT_N doubles
  double *kmat = nullptr;
};
bool dir_supported(int m, long long n);
int dir_cols_per_block(int m, long long n);
int dir_ncols(int m);
void dir_sweep(hipStream_t s, const DirArgs &a);
void dir_fin(hipStream_t s, const DirArgs &a);
// The direction-only S-LBFGS step (has_g, no pair, want_dir 1) as column sums + one launch that runs the
// coefficient recurrences in every block and combines (x_out = x_in + alpha p): replaces dir_fin + the
// combine. c.h = a.g.h; alpha not from state.
bool dir_combine_supported(const DirArgs &a, const CombineArgs &c);
void dir_cols_combine(hipStream_t s, const DirArgs &a, const CombineArgs &c);
// The same column sums + last-block history step for gram_update's transposed partials (the unfused
// L-BFGS path: n > 2M or m > TAIL_MAXM), replacing fold_rows + hist_step: a.rows = the partials,
// a.nb = gram_nwg(n). m <= GRAM_FIN_MAXM (LDS of the fused step).
constexpr int GRAM_FIN_MAXM = 52;
bool gram_fin_supported(int m);
void gram_fin(hipStream_t s, const DirArgs &a);

void hist_combine(hipStream_t s, const CombineArgs &a);
void hist_reset(hipStream_t s, const HistView &h);

} // namespace lbf
