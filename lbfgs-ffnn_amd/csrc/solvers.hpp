// Solver drivers: full-batch L-BFGS (CPU/Wolfe and CUDA/Armijo semantics) and S-LBFGS.
#pragma once

#include "../../include/lbfgs_amd.h"
#include "host_sync.hpp"
#include "runtime.hpp"
#include "sampler.hpp"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <random>
#include <thread>

namespace lbf {

// What the minimizer evaluates: the reference's LossGradFun (src/cuda/minimizer_base.cuh:15-16) plus the
// dots the line search needs. eval() writes the gradient into g (n+2 floats) and SC_LOSS / SC_TGG /
// SC_TGP (g.pdir) into the device status block scal, all on ctx()->stream.
struct Objective {
  virtual ~Objective() = default;
  virtual Ctx *ctx() const = 0;
  virtual long long n() const = 0;
  virtual void eval(const float *x, float *g, const float *pdir, double *scal) = 0;
  virtual long long evals() const = 0;
  virtual long long rows() const { return 0; } // batch rows evaluated (0: not an MLP objective)
  // Asynchronous objectives can be enqueued ahead of the host's line-search decisions.
  virtual bool async() const { return false; }
  virtual void discard_evals(long long) {}
  virtual void backward_skipped() {} // the last trial's backward was skipped (SPEC_REJECT_EARLY)
  // Two-step evaluation of a line-search trial (split_eval()): the loss alone (SC_LOSS, SC_SSE), then the
  // gradient and dots of that same point; together bitwise equal to eval().
  virtual bool split_eval() const { return false; }
  virtual void eval_loss(const float *, double *) {}
  virtual void eval_grad_after_loss(const float *, float *, const float *, double *) {}
  virtual long long loss_only_evals() const { return 0; }
  virtual long long grad_after_loss_evals() const { return 0; }
  // Evaluation followed by the fused optimizer tail (tail.hip); only when fused_tail() is true.
  virtual bool fused_tail() const { return false; }
  virtual void eval_fused(const float *, float *, const float *, double *, const TailFuse &) {}
  // eval_grad_after_loss followed by the fused tail (fused_tail() objectives)
  virtual void eval_grad_after_loss_fused(const float *, float *, const float *, double *, const TailFuse &) {}
};

// The MLP's fused loss+grad over the rank's shard (mean over n_global samples).
struct MlpObjective : Objective {
  Mlp *net;
  const float *X, *Y;
  long long nloc, nglob;
  MlpObjective(Mlp *m, const float *x, const float *y, long long nl, long long ng)
      : net(m), X(x), Y(y), nloc(nl), nglob(ng) {}
  Ctx *ctx() const override { return net->ctx(); }
  long long n() const override { return (long long)net->nparams(); }
  void eval(const float *x, float *g, const float *pdir, double *scal) override {
    net->loss_grad(x, g, X, Y, nullptr, nloc, 1.0 / double(nglob), 0.0, pdir, scal);
  }
  long long evals() const override { return net->evals(); }
  long long rows() const override { return net->rows(); }
  bool async() const override { return true; }
  void discard_evals(long long k) override { net->discard_evals(k, nloc); }
  void backward_skipped() override { net->backward_skipped(); }
  bool split_eval() const override { return true; }
  void eval_loss(const float *x, double *scal) override {
    net->loss_only(x, X, Y, nullptr, nloc, 1.0 / double(nglob), scal);
  }
  void eval_grad_after_loss(const float *x, float *g, const float *pdir, double *scal) override {
    net->grad_after_loss(x, g, X, nullptr, nloc, 1.0 / double(nglob), 0.0, pdir, scal);
  }
  long long loss_only_evals() const override { return net->loss_only_evals(); }
  long long grad_after_loss_evals() const override { return net->grad_after_loss_evals(); }
  bool fused_tail() const override { return true; }
  void eval_fused(const float *x, float *g, const float *pdir, double *scal, const TailFuse &tf) override {
    net->loss_grad(x, g, X, Y, nullptr, nloc, 1.0 / double(nglob), 0.0, pdir, scal, &tf);
  }
  void eval_grad_after_loss_fused(const float *x, float *g, const float *pdir, double *scal,
                                  const TailFuse &tf) override {
    net->grad_after_loss(x, g, X, nullptr, nloc, 1.0 / double(nglob), 0.0, pdir, scal, &tf);
  }
};

// A user callback with the reference's LossGradFun contract: returns the loss, writes the gradient
// (device) for the device parameters it is given. Host-driven, so the stream is synchronised first.
struct CallbackObjective : Objective {
  Ctx *c;
  long long nn;
  double (*fn)(void *, const float *, float *);
  void *user;
  DevBuf<double> part;
  PinnedBuf<double> hl;
  long long count = 0;
  CallbackObjective(Ctx *cx, long long n_, double (*f)(void *, const float *, float *), void *u)
      : c(cx), nn(n_), fn(f), user(u) {
    part.resize(size_t(dots_partials_wg(n_)) * 3);
    hl.ensure(1);
  }
  Ctx *ctx() const override { return c; }
  long long n() const override { return nn; }
  void eval(const float *x, float *g, const float *pdir, double *scal) override;
  long long evals() const override { return count; }
};

// Full-batch L-BFGS on the MLP. All vectors, the (s, y) ring and its Gram state stay on the device;
// the host only reads a 16-double status block once per line-search trial.
class LbfgsSolver {
public:
  LbfgsSolver(Objective *obj, const lbf_lbfgs_params &prm, float *d_params);
  ~LbfgsSolver();
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
  int iterate_spec(int iters, lbf_record *rec);
  bool entry_converged() const;
  // First trial of an iteration (history update, direction, x + alpha p, evaluation), enqueued only.
  // Returns the Armijo trial step (Wolfe takes alpha0 from the device status block). With `ls`, the
  // evaluation carries the fused tail: decision + (on acceptance) the next direction's coefficients.
  float begin_iteration(const LsCtlArgs *ls = nullptr);
  // Rest of the iteration once hs_ holds the first trial's status: further trials, role rotation,
  // record.
  void finish_wolfe(lbf_record *rec, bool spec = false);
  int grad_fused(double alpha, SpecRecord *r); // finish_wolfe's gradient phase through the fused tail
  void finish_armijo(float alpha, lbf_record *rec, bool spec = false);
  void accept_roles();
  void mark_prev_accepted(lbf_record *rec, double flag);
  void record(lbf_record *rec, double loss, double gnorm, double alpha, int trials, int accepted);

  // speculative pipeline state
  struct Roles {
    float *x, *xp, *xt, *g, *gp, *gt;
    int iter;
    bool pair, reset;
  };
  Roles roles() const { return {x_, xp_, xt_, g_, gp_, gt_, iter_, pending_pair_, pending_reset_}; }
  void restore(const Roles &r);
  struct Flight {
    Roles roles;
    float alpha;
    int seq;
    size_t prof_end;
  };
  void drain(std::deque<Flight> &q, size_t prof_end, bool status = false);
  void wait_record(int seq, SpecRecord *out);
  static constexpr int kSpecRing = 32;
  static constexpr long long kFusedTailMaxN = 1LL << 21;
  int depth_ = 0;
  int seq_ = 0;
  bool fuse_ = false;      // fused optimizer tail on the speculative path
  bool dir_ready_ = false; // the last fused tail left the next direction's coefficients on the device
  DevBuf<int> abort_;
  SpecRecord *spec_rec_ = nullptr;

  Objective *obj_;
  Ctx *ctx_;
  lbf_lbfgs_params prm_;
  float *user_params_;
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
  long long evals0_ = 0, rows0_ = 0, lonly0_ = 0, gal0_ = 0; // the objective's counters when this solve began
  std::chrono::steady_clock::time_point t0_;
};

class SlbfgsSolver {
public:
  SlbfgsSolver(Mlp *net, const lbf_slbfgs_params &prm, float *d_params, const float *X, const float *Y,
               long long N);
  ~SlbfgsSolver();
  int run(lbf_record *rec);                 // prm.max_epochs epochs (lbf_slbfgs_solve)
  int iterate(int epochs, lbf_record *rec); // up to `epochs` more (lbf_slbfgs_begin / iterate / end)
  void info(lbf_solve_info *out) const;
  // copies the first traced curvature-pair candidate's iterate w_t, average u, s and y (n floats each);
  // false when no candidate was traced yet
  bool pair0(float *wt, float *u, float *s, float *y) const;
  // Diagnostics (lbf_slbfgs_pair_io): at curvature event e (each inner step t > 0 with t % L == 0, the first,
  // which offers no pair, included) record [w_{t+1} | u | g(u + eps s) | g(u - eps s)] into rec + 4 e ld, and
  // force u, g(u + eps s), g(u - eps s) to force + 4 e ld's before use (ld = round4(n); NULL: off)
  void pair_io(int cap, float *rec, const float *force) {
    pio_cap_ = cap;
    pio_rec_ = rec;
    pio_force_ = force;
  }

private:
  int pio_cap_ = 0, nev_ = 0;
  float *pio_rec_ = nullptr;
  const float *pio_force_ = nullptr;
  struct Slice {
    long long off = 0, cnt = 0, total = 0; // offset / count in this rank's flat list, whole batch size
  };
  // An epoch's index lists: every minibatch, the Hessian batches (only once a u exists), then the anchor
  // pick, in the reference's RNG order (s_lbfgs.hpp:212-266); `flat` holds this rank's slices.
  struct EpochDraw {
    std::vector<int> flat, hflat, batch;
    std::vector<Slice> mb, hb;
    int pick = -1;
    bool u_seen = false; // have_u after the epoch
  };
  void draw_epoch(bool u_seen, EpochDraw &d);
  // The epoch's inner steps (s_lbfgs.hpp:218-262) enqueued on the streams.
  void epoch_steps(const EpochDraw &d);
  int wh_slot(int logical) const { return (wh_head_ + logical) % (prm_.L + 1); }
  int wh_push_slot();
  std::mt19937 rng_;
  std::unique_ptr<MinibatchSampler> sampler_;
  bool started_ = false, have_u_ = false, mu_valid_ = false, next_ready_ = false, converged_ = false;
  EpochDraw cur_, next_;
  int wh_head_ = 0, wh_count_ = 0; // ring of L+1 iterates (w_history)
  int rec_i_ = 0;
  // Data parallel (a communicator), LBF_SLBFGS_DP_REPLICATED: every rank runs the epoch's whole inner-step
  // chain (identical inputs, identical bits) with no collective; only the full-batch gradient at the
  // anchor (s_lbfgs.hpp:206, 274-284) is sharded, one all-reduce per epoch. LBF_SLBFGS_DP_SLICED: each rank
  // evaluates its 1/p slice of every minibatch and Hessian batch, one all-reduce per inner step.
  bool repl_ = false;
  bool dp_inner() const { return ctx_->dp() && !repl_; }
  // Replicated mode's guard: every epoch, fingerprints of each rank's new anchor w are all-reduced before
  // the sharded full-batch evaluation, and a mismatch (ranks whose inner chains drifted apart, which would
  // make that all-reduce sum gradients taken at different points) fails the solve.
  DevBuf<float> fp_;
  PinnedBuf<float> hfp_;
  void replica_fingerprints();
  void replica_check() const;
  std::chrono::steady_clock::time_point t0_;
  // Two independent batch gradients of one step (the FD pair at u +- eps s) into one [ga | gb] block
  // (gb = gab + ng_): the second on the twin's stream when there is one, joined before the next launch.
  // Data parallel: both evaluations stop before the all-reduce and ONE collective sums the block.
  void eval_pair(const float *wa, const float *wb, float *gab, long long off, long long count,
                 double inv_scale); // rows off .. off+count-1 of this rank's gathered block
  // Data parallel: all-reduce a [ga | gb] block once, then finish both gradients (+ lambda w).
  void reduce_pair(const float *wa, const float *wb, float *gab, double inv_scale);
  void trace_pair(int epoch, int t);
  int npairs_ = 0;
  // diagnostics (pair_trace on): the first traced candidate's w_t, u, s, y (lbf_slbfgs_pair0)
  DevBuf<float> p0_;
  bool p0_set_ = false;
  Mlp *net_;
  Ctx *ctx_;
  lbf_slbfgs_params prm_;
  float *user_params_;
  const float *X_, *Y_;
  long long N_, n_;
  History hist_;
  DevBuf<float> w_, wt_, mu_, v_, r_, u_, up_, s_, wp_, wm_, wh_;
  // [g(w_t) | g(w)] of an inner step, double-buffered (the twin fills the anchor half one step ahead),
  // and [g(u + eps s) | g(u - eps s)] of a Hessian step: one all-reduce per block under data parallelism
  DevBuf<float> gpair_[2], fdpair_;
  long long ng_ = 0; // floats per gradient in a block (n + 2 loss words, rounded to 4)
  DevBuf<int> idx_;
  PinnedBuf<int> idx_host_; // pinned staging of an epoch's index lists
  PinnedBuf<double> hs_;
  int iters_ = 0;
  double last_loss_ = 0, last_gnorm_ = 0;
  long long evals0_ = 0, rows0_ = 0; // the net's counters when this solve began
  // Twin evaluator: a second workspace of the same network on its own stream, so the two latency-bound
  // minibatch evaluations of a step run concurrently (results unchanged: each is the same launch
  // sequence on its own buffers). Data parallel: the twin's evaluations stop before the all-reduce
  // (it has no communicator) and the context stream's one collective per block sums both.
  std::unique_ptr<Ctx> tctx_;
  std::unique_ptr<Mlp> tnet_;
  // The twin stream's launches enqueued by a helper host thread: the inner step's host enqueue (≈ 100-130 µs, ~40 % of it the twin's evaluation) bounds the epoch on slower
  // hosts. Tasks run in posting order (one FIFO, so the twin stream sees the single-thread launch order);
  // the context thread waits for a task's ticket before it waits on an event that task records, and records
  // an event the twin waits on only after the waiting task has been enqueued (see epoch_steps).
  std::unique_ptr<TaskFifo> tw_; // host_sync.hpp
  long long twin_post(std::function<void()> f);
  void twin_wait(long long ticket); // returns once task `ticket` (1-based) has run; rethrows its error
  // this rank's slices of the epoch's sampled rows, gathered once (all minibatches and Hessian batches)
  DevBuf<float> xg_, yg_;
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
  // free-running twin (no per-step collective): anchor gradient of step t in ganc_ + t ng_, its event
  // ev_anc_[t]; off for good once its buffer does not fit in free device memory (double-buffered twin)
  bool free_twin_ = true;
  DevBuf<float> ganc_;
  std::vector<hipEvent_t> ev_anc_;
  hipEvent_t ev_g2_[2] = {nullptr, nullptr}, ev_free_[2] = {nullptr, nullptr}; // anchor gradients ahead (twin)
  // The epoch-end full-batch evaluation at the next anchor (s_lbfgs.hpp:265-284: the recorder's loss and
  // gradient, which are the next epoch's mu) started as soon as the picked iterate exists: the pick is drawn
  // with the epoch's index lists, before the epoch runs, and the picked entry of w_history stays in its ring
  // slot to the end. A third workspace of the network on its own stream evaluates it beside the epoch's last
  // inner steps into mu_next_ and its own status block; the context stream joins it where the ordered route
  // evaluated. Same launches on the same inputs: bitwise the ordered route. Single rank only (data parallel
  // keeps the ordered, sharded evaluation and its fingerprint check). Opt-in (LBF_FULL_AHEAD=1): measured
  // slower at cfg 4, 35.27-35.59 against 35.88-36.16 epochs/s interleaved (profiles/r05/n/): the full-batch
  // GEMMs occupy the chip for ~1.2 ms and the latency-bound inner steps beside them slow down by more than
  // the evaluation's ~0.6 ms average window (the pick lands mid-ring) saves.
  std::unique_ptr<Ctx> fctx_;
  std::unique_ptr<Mlp> fnet_;
  DevBuf<float> mu_next_;
  DevBuf<double> fscal_;
  hipEvent_t ev_anchor_ = nullptr, ev_full_ = nullptr;
  bool full_posted_ = false;
  // inner step after whose combine the picked iterate exists (-1: the epoch's start, -2: no pick)
  int full_ahead_step(const EpochDraw &d) const;
  void post_full(const float *anchor);
};

// CudaGD / CudaSGD (src/cuda/gd.cuh:38-106, sgd.cuh:50-153) on the MLP; return the iterations done.
int run_gd(Mlp *net, const lbf_gd_params &prm, float *d_params, const float *X, const float *Y, long long n_local,
           long long n_global, lbf_record *rec, lbf_solve_info *info);
int run_sgd(Mlp *net, const lbf_sgd_params &prm, float *d_params, const float *X, const float *Y, long long N,
            lbf_record *rec, lbf_solve_info *info);

// finite_difference_hvp_batch (s_lbfgs.hpp:88-101) up to the last step: wp/wm = u +- eps s, gp/gm = the
// batch gradients there (1/count scale, + lambda w). y = (gp - gm) / (2 eps) is formed by the caller (the
// S-LBFGS pair sweep, or diff_scale) in fp32 with the factor rounded once.
void fd_hvp_grads(Mlp *net, const float *u, const float *s, const float *X, const float *Y, const int *idx,
                  long long count, double inv_scale, double lambda, double eps, float *wp, float *wm, float *gp,
                  float *gm, double *scal);


} // namespace lbf
