// Host runtime of liblbfgs_amd_abi3.so: context (device, stream, RCCL communicator), the MLP evaluation
// plan, the device-resident L-BFGS history, and the solver drivers.
#pragma once

#include "internal.hpp"
#include "comm.hpp"
#include "kernels.hpp"

#include <memory>
#include <vector>

namespace lbf {

// Per-kernel-class timing with HIP events on the launch stream (enabled by the benchmark only).
enum ProfKind : int { PK_FWD = 0, PK_DW = 1, PK_DX = 2, PK_LOSS = 3, PK_SLAB = 4, PK_FINAL = 5, PK_GRAM = 6,
                      PK_COEF = 7, PK_COMBINE = 8, PK_AXPY = 9, PK_ALLREDUCE = 10 };
struct ProfRec { int id; size_t a, b; double work; };
struct Profiler {
  bool on = false;
  int only = -1; // section filter (-1: all)
  int every = 1;  // sample every k-th launch of a wanted section
  long long seen = 0;
  bool want(int id) {
    if (!on || (only >= 0 && only != id)) return false;
    return every <= 1 || (seen++ % every) == 0;
  }
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  using Rec = ProfRec;
  std::vector<Rec> recs;
  std::vector<double> ms;      // by section id
  std::vector<long long> cnt;  // by section id
  std::vector<double> work;    // by section id: the caller's work units of the timed launches (GEMMs: rows)
  ~Profiler();
  size_t mark(hipStream_t s);
  void resolve();
  void merge_into(Profiler &dst); // resolve this one and add its totals to dst's
  void add(const Rec &r, float t);
};

struct Ctx {
  int device = 0;
  int cus = 256; // compute units (workgroup slots = 2 per CU for the GEMM tiles, see Mlp::plan)
  Profiler prof;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::unique_ptr<Comm> comm; // RCCL (lbf_comm_init) or an in-process rank group (lbf_comm_init_local)
  int rank = 0, nranks = 1;
  const int *abort = nullptr; // set by a solver while it runs speculatively (see LbfgsSolver)
  // evaluate as a single rank although a communicator exists (replicated S-LBFGS inner steps, LocalOnly)
  bool local_only = false;
  // scratch for the BLAS-1 ABI helpers
  DevBuf<double> part, red;
  PinnedBuf<double> host;
  ~Ctx();
  void set_device() const;
  // data-parallel evaluation path: taken whenever a communicator exists, including a 1-rank one
  // (lbf_comm_init(ctx, 1, 0, id)), which is how the RCCL path is exercised on a single GPU
  bool dp() const { return comm != nullptr && !local_only; }
  void allreduce(float *buf, size_t count);
};

// Scoped Ctx::local_only (when `on`).
struct LocalOnly {
  Ctx *c;
  bool prev;
  LocalOnly(Ctx *ctx, bool on) : c(ctx), prev(ctx->local_only) {
    if (on) c->local_only = true;
  }
  ~LocalOnly() { c->local_only = prev; }
};

// Fused optimizer tail request (speculative L-BFGS fast path, tail.hip): the pair inputs, the
// history and the line-search decision taken after the evaluation.
struct TailFuse {
  HistView h;
  int has_pair = 0;
  const float *x_prev = nullptr, *g_prev = nullptr;
  int policy = POL_CPU;
  int iter_next = 1;
  LsCtlArgs ls;
  int early = 0; // a speculative first trial: its Armijo test in the first backward launch (EarlyLs)
};

struct Layer {
  int in, out, act;
  size_t off;      // flat offset of the [(in+1) x out] segment
  int splits = 1;  // split-K factor of the dW GEMM at the planned batch
  int k_chunk = 0;
  size_t slab_off = 0; // this layer's partial slabs inside the shared slab buffer
  int fsplits = 1;     // split-K factor of the forward GEMM (few row tiles: small per-rank batches)
  int fk_chunk = 0;
  int ftile = 0;       // forward GEMM tile (GemmTile)
  int dtile = 0;       // dW GEMM tile (GemmTile)
};

// RAII section: records an event pair around the enclosed launches when profiling is on.
struct ProfScope {
  Ctx *c;
  int id;
  size_t a = 0;
  bool on;
  double work;
  ProfScope(Ctx *ctx, int kind, int layer = 0, double w = 0.0)
      : c(ctx), id(kind * 16 + layer), on(ctx->prof.want(id)), work(w) {
    if (on) a = c->prof.mark(c->stream);
  }
  ~ProfScope() {
    if (on) c->prof.recs.push_back({id, a, c->prof.mark(c->stream), work});
  }
};

// Dense MLP (the reference's CudaNetwork, src/cuda/network.cuh:21-158) with a cached workspace.
class Mlp {
public:
  Mlp(Ctx *ctx, int nl, const int *dims, const int *acts);
  size_t nparams() const { return nparams_; }
  const std::vector<Layer> &layers() const { return layers_; }
  Ctx *ctx() const { return ctx_; }

  // Forward only: activations of every layer into the workspace; returns the output buffer.
  // raw_last: the last layer run stays as its split-K slabs in fslab_buf(l) (no fwd_reduce_act; rowhead reads them)
  const float *forward(const float *P, const float *X, const int *idx, long long B, int nrun = -1,
                       bool raw_last = false);
  // Fused loss + gradient (+ all-reduce over the communicator) + line-search dots.
  //   G    : gradient output, must hold nparams()+2 floats (two extra words carry the loss for the
  //          all-reduce).
  //   pdir : optional direction for the g.p dot.
  //   scal : device fp64 status block (SC_LOSS, SC_TGG, SC_TGP, SC_WW, SC_SSE written).
  void loss_grad(const float *P, float *G, const float *X, const float *Y, const int *idx, long long B,
                 double inv_scale, double lambda, const float *pdir, double *scal, const TailFuse *tf = nullptr);
  // loss_grad without the last launch (a single rank's gradient only: scal == nullptr): the split-K slabs
  // are left for the consumer, which finishes each gradient value with reduce_all's arithmetic (the S-LBFGS
  // direction sweep, dir.hip). *red describes the slabs; red->nseg == 0 when a segment needs the multi-part
  // reduction (then G is complete as with loss_grad). When red->nseg > 0, G is left INCOMPLETE: the split
  // segments of G keep whatever they held (the consumer forms those values in registers and does not store
  // them back; the S-LBFGS sweep writes only v = g - gb + mu). No reader of G exists on that route.
  void loss_grad_deferred(const float *P, float *G, const float *X, const float *Y, const int *idx, long long B,
                          double inv_scale, double lambda, RedAllArgs *red);
  // The same evaluation in two steps (a line-search trial needs f first and the gradient only once
  // Armijo holds, full_batch_minimizer.hpp:136-146): loss_only runs the forward phase and writes
  // SC_SSE / SC_LOSS (lambda == 0); grad_after_loss then runs the backward phase of that same forward
  // state. loss_only followed by grad_after_loss == loss_grad, bit for bit.
  void loss_only(const float *P, const float *X, const float *Y, const int *idx, long long B, double inv_scale,
                 double *scal);
  void grad_after_loss(const float *P, float *G, const float *X, const int *idx, long long B, double inv_scale,
                       double lambda, const float *pdir, double *scal, const TailFuse *tf = nullptr);
  // Packed data-parallel evaluation in two halves: loss_grad_local stops before the all-reduce, leaving
  // this rank's gradient (no lambda w) and its SSE as fp32 (hi, lo) words in G[0 .. n+2); the caller
  // all-reduces one or more such blocks in a single collective and then finishes each with
  // finish_reduced (+ lambda w, status block). Together bitwise equal to loss_grad on the same rank.
  void loss_grad_local(const float *P, float *G, const float *X, const float *Y, const int *idx, long long B,
                       double inv_scale);
  // g_src (nullable): the reduced words are there and the finished gradient is written to G
  void finish_reduced(const float *P, float *G, double inv_scale, double lambda, const float *pdir, double *scal,
                      const float *hilo_in = nullptr, const float *g_src = nullptr);
  // Per-minibatch gradients at one point P (S-LBFGS's anchor gradients: w is fixed for an epoch): rows
  // [t cnt, (t+1) cnt) of the gathered X / Y are minibatch t (t < nmb); its gradient, scaled by inv_scale,
  // goes to G + t ldg (+ lambda P unless local: a data-parallel rank's partial sums). One evaluation over
  // the nmb cnt rows (full-batch GEMM tiles), whose dW GEMMs split K exactly at the minibatch boundaries
  // and write split t in place as minibatch t's [dW ; db]: no slab reduction. cnt % 32 == 0.
  void batch_grads(const float *P, const float *X, const float *Y, int nmb, long long cnt, double inv_scale,
                   double lambda, float *G, long long ldg, bool local);
  long long loss_only_evals() const { return loss_only_; }
  long long grad_after_loss_evals() const { return gal_; } // backward phases run after a loss_only
  // Exact Hessian-vector product Hv = H(P) V of the same batch loss (+ lambda V), Pearlmutter's
  // R-operator (hvp.hip); with a communicator the shards' products are all-reduced. Hv: nparams().
  void hvp(const float *P, const float *V, const float *X, const float *Y, const int *idx, long long B,
           double inv_scale, double lambda, float *Hv);
  long long evals() const { return evals_; }
  long long rows() const { return rows_; } // batch rows evaluated (sum of B over loss_grad calls)
  void discard_evals(long long k, long long B) { // speculative evaluations (B rows each) that were aborted
    evals_ -= k;
    rows_ -= k * B;
  }
  void backward_skipped() { // a trial rejected by EarlyLs ran its forward only: a loss-only trial
    --evals_;
    ++loss_only_;
  }

private:
  void forward_phase(const float *P, const float *X, const float *Y, const int *idx, long long B, double inv_scale);
  void backward_phase(const float *P, float *G, const float *X, const int *idx, long long B, double inv_scale,
                      double lambda, const float *pdir, double *scal, const TailFuse *tf, bool local,
                      const float *hilo_in, RedAllArgs *defer = nullptr);
  struct FwdState {
    long long B = -1;
    bool fused = false;
    int fold = -1, nloss = 0, lstart = 0;
  } fs_;
  DevBuf<float> hilo_, words_; // loss-only (hi, lo); data parallel: this rank's [grad | hi | lo] for the collective
  long long loss_only_ = 0, gal_ = 0;
  void ensure(long long B);
  bool side_reduced(int l, bool fused, int nloss) const;
  GemmDesc fwd_desc(size_t l, const float *P, const float *in, const int *idx, long long B) const;
  GemmDesc fwd_launch_desc(size_t l, const float *P, const float *in, const int *idx, long long B);
  void set_asum(GemmDesc &d, size_t l, const float *P, long long B);
  Ctx *ctx_;
  std::vector<Layer> layers_;
  size_t nparams_ = 0;
  long long cap_ = -1, planned_ = -1;
  std::vector<DevBuf<float>> A_, D_;
  DevBuf<float> slab_, head_slab_, fslab_, fslab2_;
  float *fslab_buf(size_t l) const { return (l & 1) ? fslab2_.get() : fslab_.get(); } // forward slabs of layer l
  bool group_dw_ = true;      // dW of layers 1 and 0 in one launch (LBF_NO_GROUP=1: separate launches)
  bool fold_on_ = true;       // fold into the EPI_HEAD epilogue (LBF_NO_FOLD=1: the unfolded route, tests)
  bool rowhead_on(long long B) const; // the standalone head fed by the last hidden layer's slabs
  // Planned fold: the last hidden layer's [dW ; db] rows fold_c0_ .. in (fold_ input columns and the
  // bias row) are computed in the forward GEMM's EPI_HEAD epilogue instead of a mostly empty last
  // row tile of its dW GEMM; fold_ = -1: none.
  int fold_ = -1, fold_c0_ = 0;
  bool gemm_head_on() const; // the output layer runs inside the last hidden layer's forward GEMM
  int dx_tile(long long B, int N) const;
  DevBuf<double> loss_part_, dots_part_, sse_, colpart_, trows_, tdots_;
  DevBuf<unsigned> cols_done_; // tail_cols arrival counter (zero between launches)
  // R-pass workspace (hvp): R{Z}, R{A}, R{dZ} and delta per layer, two products, one segment
  std::vector<DevBuf<float>> RZ_, RA_, RD_, DL_;
  DevBuf<float> T1_, T2_, seg_;
  long long rcap_ = -1;
  long long evals_ = 0, rows_ = 0;
  void plan(long long B);
};

// Device-resident history of (s, y) pairs and its fp64 Gram state.
// Row groups the Gram sweep's partial table is folded into before the history step (large n).
constexpr int kGramFold = 32;

class History {
public:
  History(Ctx *ctx, int m, long long n);
  HistView view() const { return v_; }
  void reset();
  // Gram sweep + bookkeeping (+ direction coefficients when want_dir > 0).
  // gred (nullable, nseg > 0): g.ga's values are still split-K slabs (Mlp::loss_grad_deferred); the fused
  // S-LBFGS sweep finishes them in place of reduce_all, other routes launch reduce_all first.
  void update(const GramArgs &g, int want_dir, int iter, double dsign, const RedAllArgs *gred = nullptr) {
    (void)update_impl(g, want_dir, iter, dsign, gred, nullptr);
  }
  void combine(const float *g, float *dir, const float *x_in, float *x_out, float *x_out2, bool alpha_from_state,
               double alpha);
  // update(g, 1, iter, dsign) then combine(g.g_out, nullptr, x_in, x_out, x_out2, false, alpha)
  bool update_combine(const GramArgs &g, int iter, double dsign, const float *x_in, float *x_out, float *x_out2,
                      double alpha, const RedAllArgs *gred = nullptr);
  double *scal() const { return v_.scal; }
  int m() const { return v_.m; }

private:
  // cmb: the combine to fuse into the update when the S-LBFGS direction path can (dir_cols_combine);
  // returns whether it did
  bool update_impl(const GramArgs &g, int want_dir, int iter, double dsign, const RedAllArgs *gred,
                   const CombineArgs *cmb);

  Ctx *ctx_;
  HistView v_;
  DevBuf<float> S_, Y_;
  DevBuf<int> ist_;
  DevBuf<double> dstate_, part_, red_;
  // two-launch S-LBFGS update (dir.hip): partial rows, column sums, arrival counter
  DevBuf<double> drows_, ddots_, dkmat_;
  DevBuf<unsigned> dcount_;
  bool dir_on_ = false;
  // unfused path: Gram sweep (transposed partials in part_) + column sums whose last block runs the step
  DevBuf<double> gdots_;
  DevBuf<unsigned> gcount_;
  bool gfin_on_ = false;
};

struct LbfgsRecordRow {
  double loss, gnorm, time_ms, alpha;
  int trials, accepted;
};

} // namespace lbf
