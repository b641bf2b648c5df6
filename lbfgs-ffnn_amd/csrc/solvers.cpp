// L-BFGS / S-LBFGS drivers (see solvers.hpp).
#include "solvers.hpp"

#include <algorithm>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>

// Host-side acceptance tests must round like ls_ctl_kernel (and the reference's host code).
#pragma clang fp contract(off)

namespace lbf {

namespace {
long long round4(long long n) { return cdiv(n, 4) * 4; }
} // namespace

// ================================================================================================
// Full-batch L-BFGS
// ================================================================================================
void CallbackObjective::eval(const float *x, float *g, const float *pdir, double *scal) {
  LBF_HIP(hipStreamSynchronize(c->stream)); // x is complete before the host callback reads it
  hl[0] = fn(user, x, g);
  ++count;
  const int nd = dots_partials_wg(nn);
  finalize_grad_dots(c->stream, nn, g, x, 0.0, pdir, part.get());
  eval_tail(c->stream, part.get(), nd, part.get(), 0, nullptr, 0.0, 0.0, scal);
  LBF_HIP(hipMemcpyAsync(scal + SC_LOSS, hl.get(), sizeof(double), hipMemcpyHostToDevice, c->stream));
}

LbfgsSolver::LbfgsSolver(Objective *obj, const lbf_lbfgs_params &prm, float *d_params)
    : obj_(obj), ctx_(obj->ctx()), prm_(prm), user_params_(d_params), n_(obj->n()),
      hist_(obj->ctx(), prm.m, obj->n()) {
  LBF_REQUIRE(d_params, "null pointer");
  LBF_REQUIRE(prm.max_line_iters >= 1, "max_line_iters >= 1");
  for (int i = 0; i < 3; ++i) {
    xbuf_[i].resize(size_t(round4(n_)));
    gbuf_[i].resize(size_t(round4(n_ + 2)));
  }
  p_.resize(size_t(round4(n_)));
  x_ = xbuf_[0].get();
  xp_ = xbuf_[1].get();
  xt_ = xbuf_[2].get();
  g_ = gbuf_[0].get();
  gp_ = gbuf_[1].get();
  gt_ = gbuf_[2].get();
  hs_.ensure(SC_N);
  // Speculation depth: iterations enqueued ahead of the host's line-search decision
  // (LBF_SPEC_DEPTH, default 3; 0 = host-driven). Host callbacks synchronise anyway.
  depth_ = 3;
  if (const char *e = std::getenv("LBF_SPEC_DEPTH")) depth_ = std::max(0, std::min(16, std::atoi(e)));
  if (!obj_->async()) depth_ = 0;
  // Fused optimizer tail on the speculative path (LBF_FUSED_TAIL=0 disables). It is a latency design
  // (one block per 64 coordinates, a partial row each): past kFusedTailMaxN the classic Gram sweep +
  // folded history step moves fewer bytes.
  fuse_ = depth_ > 0 && obj_->fused_tail() && prm_.m > 0 && prm_.m <= TAIL_MAXM && n_ <= kFusedTailMaxN;
  if (const char *e = std::getenv("LBF_FUSED_TAIL")) fuse_ = fuse_ && e[0] != '0';
  if (depth_ > 0) {
    abort_.resize(1);
    LBF_HIP(hipMemsetAsync(abort_.get(), 0, sizeof(int), ctx_->stream));
    LBF_HIP(hipHostMalloc(reinterpret_cast<void **>(&spec_rec_), kSpecRing * sizeof(SpecRecord),
                          hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(spec_rec_, 0xff, kSpecRing * sizeof(SpecRecord));
  }
  LBF_HIP(hipMemcpyAsync(x_, d_params, size_t(n_) * sizeof(float), hipMemcpyDeviceToDevice, ctx_->stream));
  evals0_ = obj_->evals();
  rows0_ = obj_->rows();
  lonly0_ = obj_->loss_only_evals();
  gal0_ = obj_->grad_after_loss_evals();
  // initial evaluation (lbfgs.hpp:44 / lbfgs.cuh:147)
  eval(x_, g_, nullptr);
  read_status();
  loss_ = hs_[SC_LOSS];
  lossf_ = float(loss_);
  gg_ = hs_[SC_TGG];
  t0_ = std::chrono::steady_clock::now();
}

LbfgsSolver::~LbfgsSolver() {
  if (spec_rec_) (void)hipHostFree(spec_rec_);
}

void LbfgsSolver::eval(const float *x, float *g, const float *pdir) { obj_->eval(x, g, pdir, hist_.scal()); }

void LbfgsSolver::read_status() {
  LBF_HIP(hipMemcpyAsync(hs_.get(), hist_.scal(), SC_N * sizeof(double), hipMemcpyDeviceToHost, ctx_->stream));
  LBF_HIP(hipStreamSynchronize(ctx_->stream));
}

void LbfgsSolver::writeback() {
  LBF_HIP(hipMemcpyAsync(user_params_, x_, size_t(n_) * sizeof(float), hipMemcpyDeviceToDevice, ctx_->stream));
  LBF_HIP(hipStreamSynchronize(ctx_->stream));
}

void LbfgsSolver::record(lbf_record *rec, double loss, double gnorm, double alpha, int trials, int accepted) {
  if (!rec) return;
  const int i = rec_idx_++;
  if (i >= rec->cap) return;
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count();
  if (rec->loss) rec->loss[i] = loss;
  if (rec->grad_norm) rec->grad_norm[i] = gnorm;
  if (rec->time_ms) rec->time_ms[i] = ms;
  if (rec->alpha) rec->alpha[i] = alpha;
  if (rec->ls_trials) rec->ls_trials[i] = trials;
  if (rec->accepted) rec->accepted[i] = accepted;
  rec->size = std::max(rec->size, i + 1);
}

// The accepted flag of a pair is only known when the next iteration's history step has run.
void LbfgsSolver::mark_prev_accepted(lbf_record *rec, double flag) {
  if (rec && rec->accepted && rec_idx_ > 0 && rec_idx_ - 1 < rec->cap) rec->accepted[rec_idx_ - 1] = int(flag);
}

bool LbfgsSolver::entry_converged() const {
  if (prm_.line_search == LBF_LS_ARMIJO) return float(std::sqrt(gg_)) < float(prm_.tol); // lbfgs.cuh:143
  return std::sqrt(gg_) < prm_.tol;                                                     // lbfgs.hpp:42
}

int LbfgsSolver::iterate(int iters, lbf_record *rec) {
  ctx_->set_device();
  rec_idx_ = rec ? rec->size : 0;
  int done;
  if (depth_ > 0)
    done = iterate_spec(iters, rec);
  else
    done = prm_.line_search == LBF_LS_ARMIJO ? iterate_armijo(iters, rec) : iterate_wolfe(iters, rec);
  writeback();
  return done;
}

// x <- trial, xp <- old x, xt <- free (same rotation for g)
void LbfgsSolver::accept_roles() {
  std::swap(xp_, x_);
  std::swap(x_, xt_);
  std::swap(gp_, g_);
  std::swap(g_, gt_);
  pending_pair_ = prm_.m > 0;
  ++iter_;
}

void LbfgsSolver::restore(const Roles &r) {
  x_ = r.x;
  xp_ = r.xp;
  xt_ = r.xt;
  g_ = r.g;
  gp_ = r.gp;
  gt_ = r.gt;
  iter_ = r.iter;
  pending_pair_ = r.pair;
  pending_reset_ = r.reset;
}

float LbfgsSolver::begin_iteration(const LsCtlArgs *ls) {
  const bool armijo = prm_.line_search == LBF_LS_ARMIJO;
  if (ls && dir_ready_) { // the previous fused tail computed this direction's coefficients
    float alpha = 1.0f;
    hist_.combine(g_, p_.get(), x_, xt_, nullptr, !armijo, armijo ? double(alpha) : 0.0);
    TailFuse tf;
    tf.h = hist_.view();
    tf.has_pair = prm_.m > 0;
    tf.x_prev = x_;
    tf.g_prev = g_;
    tf.policy = armijo ? POL_CUDA : POL_CPU;
    tf.iter_next = iter_ + 1;
    tf.ls = *ls;
    tf.ls.alphaf = alpha;
    tf.early = ls->first ? 0 : 1; // (Wolfe iteration 0 takes its trial without a test)
    obj_->eval_fused(xt_, gt_, p_.get(), hist_.scal(), tf);
    return alpha;
  }
  GramArgs ga;
  ga.policy = armijo ? POL_CUDA : POL_CPU;
  ga.has_g = 1;
  ga.ga = g_;
  ga.reset = (armijo && pending_reset_) ? 1 : 0;
  if (pending_pair_) {
    ga.has_pair = 1;
    ga.sa = x_;
    ga.sb = xp_;
    ga.ya = g_;
    ga.yb = gp_;
  }
  hist_.update(ga, 1, iter_, -1.0);
  float alpha = 1.0f;
  if (armijo) {
    if (iter_ == 0) alpha = std::min(1.0f, 1.0f / float(std::sqrt(gg_))); // lbfgs.cuh:149
    hist_.combine(g_, p_.get(), x_, xt_, nullptr, false, double(alpha));
  } else {
    hist_.combine(g_, p_.get(), x_, xt_, nullptr, true, 0.0); // xt = x + alpha0 p
  }
  if (ls) {
    TailFuse tf;
    tf.h = hist_.view();
    tf.has_pair = prm_.m > 0;
    tf.x_prev = x_;
    tf.g_prev = g_;
    tf.policy = armijo ? POL_CUDA : POL_CPU;
    tf.iter_next = iter_ + 1;
    tf.ls = *ls;
    tf.ls.alphaf = alpha;
    tf.early = ls->first ? 0 : 1; // (Wolfe iteration 0 takes its trial without a test)
    obj_->eval_fused(xt_, gt_, p_.get(), hist_.scal(), tf);
  } else {
    eval(xt_, gt_, p_.get());
  }
  return alpha;
}

// CPU semantics: LBFGS::solve (lbfgs.hpp:38-100) + FullBatchMinimizer::line_search
// (full_batch_minimizer.hpp:126-157). Every f / Gradient call of the reference maps to a cached
// fused evaluation: line_search's f(x), Gradient(x) are the previous accepted trial, the trial's
// Gradient(x+ap) comes with its f, the post-search Gradient(x_new) and the recorder's f(x) are the
// accepted trial's. Only an exhausted search (returns an alpha it never evaluated) costs one more.
// The host-finished search's gradient phase on the speculative route (finish_wolfe / finish_armijo): the backward
// of the loss-only trial just taken, then the fused tail with the host's decision rule at this alpha
// (tail.hip): on acceptance it pushes the pair
// and computes the next direction's coefficients, as a speculative iteration's tail does, so the next
// iteration speculates at once on the fused route. Returns the record's status; anything but SPEC_ACCEPT has
// raised the abort flag, which is cleared here (stream-ordered), and leaves the history untouched.
int LbfgsSolver::grad_fused(double alpha, SpecRecord *r) {
  const bool armijo = prm_.line_search == LBF_LS_ARMIJO;
  LsCtlArgs a;
  a.scal = hist_.scal();
  a.abort = abort_.get();
  a.seq = seq_++;
  a.rec = spec_rec_ + a.seq % kSpecRing;
  a.armijo = armijo ? 1 : 0;
  a.first = 0;
  a.host_fold = 1;
  a.fold = loss_;
  a.foldf = lossf_;
  a.c1 = prm_.c1;
  a.c2 = prm_.c2;
  a.tol = prm_.tol;
  a.alpha = alpha;
  TailFuse tf;
  tf.h = hist_.view();
  tf.has_pair = prm_.m > 0;
  tf.x_prev = x_;
  tf.g_prev = g_;
  tf.policy = armijo ? POL_CUDA : POL_CPU;
  tf.iter_next = iter_ + 1;
  tf.ls = a;
  tf.ls.alphaf = float(alpha); // Armijo: the fp32 trial step itself
  obj_->eval_grad_after_loss_fused(xt_, gt_, p_.get(), hist_.scal(), tf);
  wait_record(a.seq, r);
  if (r->seq != a.seq) throw Error(2, "speculative line search: record out of sequence");
  if (r->status != SPEC_ACCEPT) LBF_HIP(hipMemsetAsync(abort_.get(), 0, sizeof(int), ctx_->stream));
  return r->status;
}

void LbfgsSolver::finish_wolfe(lbf_record *rec, bool spec) {
  const double inf = std::numeric_limits<double>::infinity();
  double alpha = hs_[SC_ALPHA0];
  int trials = 0;
  bool fused_done = false; // the accepted trial's tail pushed the pair and built the next direction
  SpecRecord fr{};
  if (iter_ > 0) {
    const double f_old = loss_, gfo = hs_[SC_GTP];
    double amin = 0.0, amax = inf;
    alpha = 1.0;
    bool evaluated = true, have_grad = true;
    const bool split = obj_->split_eval();
    for (int i = 0; i < prm_.max_line_iters; ++i) {
      if (!evaluated) {
        {
          ProfScope ps(ctx_, PK_AXPY);
          axpy_to(ctx_->stream, n_, x_, float(alpha), p_.get(), xt_);
        }
        if (split) { // f(x + alpha p) first; the gradient only once Armijo holds (:136-146)
          obj_->eval_loss(xt_, hist_.scal());
          have_grad = false;
        } else {
          eval(xt_, gt_, p_.get());
        }
        read_status();
        evaluated = true;
      }
      ++trials;
      const double fn = hs_[SC_LOSS];
      if (fn > f_old + prm_.c1 * alpha * gfo) {
        amax = alpha;
        alpha = prm_.rho * (amin + amax);
        evaluated = false;
        continue;
      }
      if (!have_grad) { // backward phase of the forward pass just taken: bitwise the full evaluation
        have_grad = true;
        if (spec && fuse_) {
          if (grad_fused(alpha, &fr) == SPEC_ACCEPT) { // the host's tests below would pass alike
            fused_done = true;
            break;
          }
          read_status(); // rejected on curvature (or converged): the host's search goes on from the status
        } else {
          obj_->eval_grad_after_loss(xt_, gt_, p_.get(), hist_.scal());
          read_status();
        }
      }
      const double gnp = hs_[SC_TGP];
      if (gnp < prm_.c2 * gfo) {
        amin = alpha;
        alpha = (amax == inf) ? alpha * 2 : prm_.rho * (amin + amax);
        evaluated = false;
        continue;
      }
      break;
    }
    if (!evaluated) { // exhausted: the returned alpha was never evaluated (lbfgs.hpp:67-70)
      axpy_to(ctx_->stream, n_, x_, float(alpha), p_.get(), xt_);
      eval(xt_, gt_, p_.get());
      read_status();
    } else if (!have_grad) { // exhausted on an Armijo failure: x_new's gradient is still needed
      obj_->eval_grad_after_loss(xt_, gt_, p_.get(), hist_.scal());
      read_status();
    }
  }
  accept_roles();
  loss_ = fused_done ? fr.loss : hs_[SC_LOSS];
  gg_ = fused_done ? fr.tgg : hs_[SC_TGG];
  dir_ready_ = fused_done;
  record(rec, loss_, std::sqrt(gg_), alpha, trials, -1);
}

int LbfgsSolver::iterate_wolfe(int iters, lbf_record *rec) {
  int k = 0;
  for (; k < iters; ++k) {
    if (entry_converged()) {
      converged_ = true;
      break;
    }
    const bool had_pair = pending_pair_;
    begin_iteration();
    read_status();
    if (had_pair) mark_prev_accepted(rec, hs_[SC_ACCEPT]);
    finish_wolfe(rec);
  }
  return k;
}

// CUDA semantics: CudaLBFGS::solve (lbfgs.cuh:39-194), host scalars in fp32 like the reference.
void LbfgsSolver::finish_armijo(float alpha, lbf_record *rec, bool spec) {
  const float c1 = float(prm_.c1), rho = float(prm_.rho);
  const float gdp = float(hs_[SC_GTP]);
  bool ok = false;
  int trials = 0;
  float lnew = 0.f, a_eval = alpha;
  const bool split = obj_->split_eval();
  bool have_grad = true;
  for (int ls = 0; ls < prm_.max_line_iters; ++ls) {
    if (ls > 0) { // loss only; the accepted (or last) trial's gradient afterwards (lbfgs.cuh:115-140)
      axpy_to(ctx_->stream, n_, x_, alpha, p_.get(), xt_);
      if (split) {
        obj_->eval_loss(xt_, hist_.scal());
        have_grad = false;
      } else {
        eval(xt_, gt_, p_.get());
      }
      read_status();
    }
    ++trials;
    a_eval = alpha;
    lnew = float(hs_[SC_LOSS]);
    if (lnew <= lossf_ + c1 * alpha * gdp) {
      ok = true;
      break;
    }
    const float den = 2.0f * (lnew - lossf_ - gdp * alpha);
    bool fb = true;
    if (std::fabs(den) > 1e-20f) {
      const float na = -(gdp * alpha * alpha) / den;
      if (na >= 0.1f * alpha && na <= 0.9f * alpha) {
        alpha = na;
        fb = false;
      }
    }
    if (fb) alpha *= rho;
  }
  bool fused_done = false; // the accepted trial's tail pushed the pair and built the next direction
  SpecRecord fr{};
  if (!have_grad) {
    if (spec && fuse_ && ok && grad_fused(double(a_eval), &fr) == SPEC_ACCEPT) {
      fused_done = true;
    } else {
      if (!(spec && fuse_ && ok)) obj_->eval_grad_after_loss(xt_, gt_, p_.get(), hist_.scal());
      read_status(); // (after a fused tail that did not accept: its status block)
    }
  }
  accept_roles();
  pending_reset_ = !ok; // lbfgs.cuh:147
  lossf_ = lnew;
  loss_ = fused_done ? fr.loss : hs_[SC_LOSS];
  gg_ = fused_done ? fr.tgg : hs_[SC_TGG];
  dir_ready_ = fused_done;
  record(rec, double(lnew), double(float(std::sqrt(gg_))), double(a_eval), trials, -1);
}

int LbfgsSolver::iterate_armijo(int iters, lbf_record *rec) {
  int k = 0;
  for (; k < iters; ++k) {
    if (entry_converged()) {
      converged_ = true;
      break;
    }
    const bool had_pair = pending_pair_;
    const float alpha = begin_iteration();
    read_status();
    if (had_pair) mark_prev_accepted(rec, hs_[SC_ACCEPT]);
    finish_armijo(alpha, rec);
  }
  return k;
}

// Spins on the host-mapped record of speculative iteration `seq` (no event: an event record costs
// ~5 us of idle GPU per iteration). Only after 5 ms of spinning is the stream queried, so a failed
// launch or an already-drained queue surfaces instead of spinning forever: hipStreamQuery enqueues a
// marker packet behind the last launch, and a query per iteration put a ~6 us idle gap (the marker's
// release) in front of the first kernel of the iterations enqueued after it (profiles/r03/README.md).
void LbfgsSolver::wait_record(int seq, SpecRecord *out) {
  volatile SpecRecord *r = spec_rec_ + seq % kSpecRing;
  auto t0 = std::chrono::steady_clock::now();
  for (long long spin = 0;; ++spin) {
    if (__atomic_load_n(&spec_rec_[seq % kSpecRing].seq, __ATOMIC_ACQUIRE) == seq) break;
    if ((spin & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5)) {
      const hipError_t q = hipStreamQuery(ctx_->stream);
      if (q == hipSuccess) { // queue drained: the record must be there now
        if (__atomic_load_n(&spec_rec_[seq % kSpecRing].seq, __ATOMIC_ACQUIRE) == seq) break;
        throw Error(2, "speculative line search: record missing after the stream drained");
      }
      if (q != hipErrorNotReady) LBF_HIP(q);
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
        throw Error(2, "speculative line search: timed out waiting for the device");
    }
  }
  out->loss = r->loss;
  out->tgg = r->tgg;
  out->alpha0 = r->alpha0;
  out->accept_prev = r->accept_prev;
  out->status = r->status;
  out->seq = r->seq;
}

// Waits for everything queued, clears the abort flag and forgets the aborted iterations. status: the
// status block is copied to the host behind the aborted launches, in the same wait (read_status's copy).
void LbfgsSolver::drain(std::deque<Flight> &q, size_t prof_end, bool status) {
  if (status)
    LBF_HIP(hipMemcpyAsync(hs_.get(), hist_.scal(), SC_N * sizeof(double), hipMemcpyDeviceToHost, ctx_->stream));
  LBF_HIP(hipStreamSynchronize(ctx_->stream));
  LBF_HIP(hipMemsetAsync(abort_.get(), 0, sizeof(int), ctx_->stream));
  obj_->discard_evals((long long)q.size());
  if (ctx_->prof.on && ctx_->prof.recs.size() > prof_end) ctx_->prof.recs.resize(prof_end);
  q.clear();
}

// Speculative pipeline. Almost every accepted step is the first trial (alpha = 1), so the host
// enqueues up to depth_ iterations assuming it will be, and a one-thread ls_ctl kernel after each first
// trial decides on the device with the host's own test. A rejected (or converged) trial raises the
// abort flag: every launch queued behind it exits at entry, the host waits, restores the buffer roles
// of that iteration (the history, Gram state and status block are exactly as that trial left them)
// and finishes it host-driven, then speculates again. Results are identical to the host-driven loop.
int LbfgsSolver::iterate_spec(int iters, lbf_record *rec) {
  const bool armijo = prm_.line_search == LBF_LS_ARMIJO;
  std::deque<Flight> q;
  int done = 0, issued = 0;
  bool host_fold = true;
  ctx_->abort = abort_.get();
  struct Clear {
    Ctx *c;
    ~Clear() { c->abort = nullptr; }
  } clear{ctx_};
  // LBF_HOST_TIMING=1: where the host thread spends an iteration (enqueue vs waiting for the device)
  static const int host_timing = env_int("LBF_HOST_TIMING", 0);
  double t_enq = 0.0, t_wait = 0.0;
  long long n_wait = 0, n_ready = 0;
  using clk = std::chrono::steady_clock;
  while (done < iters) {
    if (q.empty() && entry_converged()) {
      converged_ = true;
      break;
    }
    const auto te0 = clk::now();
    while (issued < iters && int(q.size()) < depth_) {
      Flight f;
      f.roles = roles();
      f.seq = seq_++;
      LsCtlArgs a;
      a.scal = hist_.scal();
      a.abort = abort_.get();
      a.rec = spec_rec_ + f.seq % kSpecRing;
      a.seq = f.seq;
      a.armijo = armijo ? 1 : 0;
      a.first = iter_ == 0 ? 1 : 0;
      a.host_fold = host_fold ? 1 : 0;
      a.fold = loss_;
      a.foldf = lossf_;
      a.c1 = prm_.c1;
      a.c2 = prm_.c2;
      a.tol = prm_.tol;
      if (fuse_) {
        f.alpha = begin_iteration(&a); // decision inside the fused tail
        dir_ready_ = true;
      } else {
        f.alpha = begin_iteration();
        a.alphaf = f.alpha;
        ls_ctl(ctx_->stream, a);
      }
      f.prof_end = ctx_->prof.recs.size();
      q.push_back(f);
      host_fold = false;
      accept_roles(); // assume the first trial is taken
      pending_reset_ = false;
      ++issued;
    }
    const Flight f = q.front();
    q.pop_front();
    SpecRecord r;
    const auto tw0 = clk::now();
    if (host_timing) {
      t_enq += std::chrono::duration<double>(tw0 - te0).count();
      n_ready += __atomic_load_n(&spec_rec_[f.seq % kSpecRing].seq, __ATOMIC_ACQUIRE) == f.seq ? 1 : 0;
    }
    wait_record(f.seq, &r);
    if (host_timing) {
      t_wait += std::chrono::duration<double>(clk::now() - tw0).count();
      ++n_wait;
    }
    if (r.seq != f.seq) throw Error(2, "speculative line search: record out of sequence");
    if (f.roles.pair) mark_prev_accepted(rec, r.accept_prev);
    if (r.status == SPEC_REJECT || r.status == SPEC_REJECT_EARLY) {
      if (r.status == SPEC_REJECT_EARLY) obj_->backward_skipped();
      drain(q, f.prof_end, true); // + the status block as the rejected trial left it (one wait)
      dir_ready_ = false;         // the host finishes this iteration; the next one builds its direction
      restore(f.roles);
      if (armijo)
        finish_armijo(f.alpha, rec, true);
      else
        finish_wolfe(rec, true);
      ++done;
      issued = done;
      host_fold = true;
      continue;
    }
    loss_ = r.loss;
    gg_ = r.tgg;
    if (armijo) {
      lossf_ = float(r.loss);
      record(rec, double(lossf_), double(float(std::sqrt(gg_))), double(f.alpha), 1, -1);
    } else {
      record(rec, loss_, std::sqrt(gg_), f.roles.iter == 0 ? r.alpha0 : 1.0, f.roles.iter == 0 ? 0 : 1, -1);
    }
    ++done;
    if (r.status == SPEC_CONVERGED) {
      // the iterations queued behind were aborted: return to the roles right after this step
      if (!q.empty()) restore(q.front().roles);
      drain(q, f.prof_end);
      dir_ready_ = false; // the fused tail does not push the pair of a converged step
      issued = done;
      host_fold = true;
    }
  }
  if (host_timing && n_wait)
    std::fprintf(stderr, "[lbf host] spec: %lld records, enqueue %.2f us/iter, wait %.2f us/iter, %lld already there\n",
                 n_wait, 1e6 * t_enq / double(n_wait), 1e6 * t_wait / double(n_wait), n_ready);
  return done;
}

void LbfgsSolver::info(lbf_solve_info *out) const {
  if (!out) return;
  std::memset(out, 0, sizeof(*out));
  out->iterations = iter_;
  out->n_evals = obj_->evals() - evals0_;
  out->n_rows = obj_->rows() - rows0_;
  out->n_loss_only = obj_->loss_only_evals() - lonly0_;
  out->n_grad_after_loss = obj_->grad_after_loss_evals() - gal0_;
  out->final_loss = loss_;
  out->final_grad_norm = std::sqrt(gg_);
}

// ================================================================================================
// S-LBFGS
// ================================================================================================
void fd_hvp_grads(Mlp *net, const float *u, const float *s, const float *X, const float *Y, const int *idx,
                  long long count, double inv_scale, double lambda, double eps, float *wp, float *wm, float *gp,
                  float *gm, double *scal) {
  hipStream_t st = net->ctx()->stream;
  const long long n = (long long)net->nparams();
  lincomb(st, n, u, eps, s, wp);
  lincomb(st, n, u, -eps, s, wm);
  net->loss_grad(wp, gp, X, Y, idx, count, inv_scale, lambda, nullptr, scal);
  net->loss_grad(wm, gm, X, Y, idx, count, inv_scale, lambda, nullptr, scal);
}

SlbfgsSolver::SlbfgsSolver(Mlp *net, const lbf_slbfgs_params &prm, float *d_params, const float *X, const float *Y,
                           long long N)
    : net_(net), ctx_(net->ctx()), prm_(prm), user_params_(d_params), X_(X), Y_(Y), N_(N),
      n_((long long)net->nparams()), hist_(net->ctx(), prm.M, (long long)net->nparams()) {
  LBF_REQUIRE(d_params && X && Y && N > 0, "null pointer / empty data");
  LBF_REQUIRE(prm.b > 0 && prm.L > 0 && prm.L + 1 <= 64, "b > 0, 1 <= L <= 63");
  const size_t nv = size_t(round4(n_)), ng = size_t(round4(n_ + 2));
  w_.resize(nv);
  wt_.resize(nv);
  v_.resize(nv);
  r_.resize(nv);
  u_.resize(nv);
  up_.resize(nv);
  s_.resize(nv);
  wp_.resize(nv);
  wm_.resize(nv);
  mu_.resize(ng);
  ng_ = (long long)ng;
  // zeroed once: the pads between the two halves of a block are summed by the all-reduce too
  for (auto *b : {&gpair_[0], &gpair_[1], &fdpair_}) {
    b->resize(2 * ng);
    LBF_HIP(hipMemsetAsync(b->get(), 0, 2 * ng * sizeof(float), ctx_->stream));
  }
  wh_.resize(nv * size_t(prm.L + 1));
  hs_.ensure(SC_N);
  evals0_ = net->evals();
  rows0_ = net->rows();
  rng_.seed(prm.seed);
  sampler_.reset(new MinibatchSampler(size_t(N)));
  repl_ = ctx_->dp() && prm.dp_mode == LBF_SLBFGS_DP_REPLICATED;
  LBF_REQUIRE(prm.dp_mode == LBF_SLBFGS_DP_REPLICATED || prm.dp_mode == LBF_SLBFGS_DP_SLICED, "dp_mode 0 / 1");
  // Twin evaluator (see tnet_). Epoch hipGraphs of both streams were built and measured slower on ROCm
  // 7.2: hipGraphLaunch spends about as much host time per node as an eager launch, and the replay runs
  // every node on one queue, so the twin's anchor gradients stopped overlapping the context stream's chain
  // (profiles/r03b/cfg4_graph*). Precomputing an epoch's anchor gradients in one evaluation measured no
  // faster than the twin (profiles/r03/bench_cfg4_{pre,twin}_*.json).
  {
    tctx_.reset(new Ctx());
    tctx_->device = ctx_->device;
    tctx_->cus = ctx_->cus;
    // the lowest priority: the anchor gradients are off the critical path, the context stream's chain is on it
    // (the twin confined to 32-128 of the CUs measured the same, profiles/r04/e/)
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest < least)
      LBF_HIP(hipStreamCreateWithPriority(&tctx_->stream, hipStreamNonBlocking, least));
    else
      LBF_HIP(hipStreamCreateWithFlags(&tctx_->stream, hipStreamNonBlocking));
    tctx_->own_stream = true;
    tctx_->prof.on = ctx_->prof.on; // the benchmark's section timing covers the twin's launches too
    tctx_->prof.only = ctx_->prof.only;
    tctx_->prof.every = ctx_->prof.every;
    std::vector<int> dims, acts;
    for (const Layer &L : net->layers()) {
      dims.push_back(L.in);
      acts.push_back(L.act);
    }
    dims.push_back(net->layers().back().out);
    tnet_.reset(new Mlp(tctx_.get(), int(acts.size()), dims.data(), acts.data()));
    LBF_HIP(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming | event_release_flags()));
    LBF_HIP(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming | event_release_flags()));
    for (int i = 0; i < 2; ++i) {
      LBF_HIP(hipEventCreateWithFlags(&ev_g2_[i], hipEventDisableTiming | event_release_flags()));
      LBF_HIP(hipEventCreateWithFlags(&ev_free_[i], hipEventDisableTiming | event_release_flags()));
    }
    const int dev = ctx_->device;
    tw_.reset(new TaskFifo([dev]() { LBF_HIP(hipSetDevice(dev)); }));
    // the epoch-end full-batch evaluation ahead (see fnet_): single rank, opt-in (LBF_FULL_AHEAD=1)
    if (!ctx_->dp() && env_int("LBF_FULL_AHEAD", 0) != 0) {
      fctx_.reset(new Ctx());
      fctx_->device = ctx_->device;
      fctx_->cus = ctx_->cus;
      if (greatest < least) LBF_HIP(hipStreamCreateWithPriority(&fctx_->stream, hipStreamNonBlocking, least));
      else LBF_HIP(hipStreamCreateWithFlags(&fctx_->stream, hipStreamNonBlocking));
      fctx_->own_stream = true;
      fctx_->prof.on = ctx_->prof.on;
      fctx_->prof.only = ctx_->prof.only;
      fctx_->prof.every = ctx_->prof.every;
      fnet_.reset(new Mlp(fctx_.get(), int(acts.size()), dims.data(), acts.data()));
      mu_next_.resize(ng);
      fscal_.resize(SC_N);
      LBF_HIP(hipMemsetAsync(fscal_.get(), 0, SC_N * sizeof(double), ctx_->stream));
      LBF_HIP(hipEventCreateWithFlags(&ev_anchor_, hipEventDisableTiming | event_release_flags()));
      LBF_HIP(hipEventCreateWithFlags(&ev_full_, hipEventDisableTiming | event_release_flags()));
    }
  }
}

int SlbfgsSolver::full_ahead_step(const EpochDraw &d) const {
  if (!fnet_ || d.pick < 0) return -2;
  // w_history at the epoch's end holds iterates w_{m+1-W} .. w_m (w_0: the anchor copy, w_{t+1}: after step t),
  // W = min(m + 1, L + 1) entries, the same count draw_epoch drew the pick over (s_lbfgs.hpp:265-266)
  const int m_inner = int(std::max(1LL, N_ / prm_.b));
  const int W = std::min(m_inner + 1, prm_.L + 1);
  const int j = m_inner + 1 - W + d.pick;
  return j - 1;
}

void SlbfgsSolver::post_full(const float *anchor) {
  hipStream_t s = ctx_->stream;
  LBF_HIP(hipEventRecord(ev_anchor_, s));
  LBF_HIP(hipStreamWaitEvent(fctx_->stream, ev_anchor_, 0));
  fnet_->loss_grad(anchor, mu_next_.get(), X_, Y_, nullptr, N_, 1.0 / double(N_), prm_.lambda, nullptr, fscal_.get());
  LBF_HIP(hipEventRecord(ev_full_, fctx_->stream));
  full_posted_ = true;
}

long long SlbfgsSolver::twin_post(std::function<void()> f) {
  if (!tw_) {
    f();
    return 0;
  }
  return tw_->post(std::move(f));
}

void SlbfgsSolver::twin_wait(long long ticket) {
  if (tw_) tw_->wait(ticket);
}

SlbfgsSolver::~SlbfgsSolver() {
  tw_.reset(); // runs what is queued, joins the helper thread
  for (auto e : ev_anc_) (void)hipEventDestroy(e);
  if (ev_fork_) (void)hipEventDestroy(ev_fork_);
  if (ev_join_) (void)hipEventDestroy(ev_join_);
  for (int i = 0; i < 2; ++i) {
    if (ev_g2_[i]) (void)hipEventDestroy(ev_g2_[i]);
    if (ev_free_[i]) (void)hipEventDestroy(ev_free_[i]);
  }
  if (fctx_) (void)hipStreamSynchronize(fctx_->stream);
  if (ev_anchor_) (void)hipEventDestroy(ev_anchor_);
  if (ev_full_) (void)hipEventDestroy(ev_full_);
}

void SlbfgsSolver::reduce_pair(const float *wa, const float *wb, float *gab, double inv_scale) {
  {
    ProfScope ps(ctx_, PK_ALLREDUCE);
    ctx_->allreduce(gab, size_t(2 * ng_)); // [ga | hi | lo | pad | gb | hi | lo | pad]
  }
  net_->finish_reduced(wa, gab, inv_scale, prm_.lambda, nullptr, nullptr);
  net_->finish_reduced(wb, gab + ng_, inv_scale, prm_.lambda, nullptr, nullptr);
}

void SlbfgsSolver::eval_pair(const float *wa, const float *wb, float *gab, long long off, long long count,
                             double inv_scale) {
  // the step's rows were gathered for the whole epoch (contiguous slices, same values in the same order
  // as the gathering GEMMs would read), which also lets the dW GEMM of layer 0 take the LDS-DMA path
  const int In = net_->layers().front().in, Out = net_->layers().back().out;
  const float *X = xg_.get() + off * In, *Y = yg_.get() + off * Out;
  float *ga = gab, *gb = gab + ng_;
  const bool dp = dp_inner();
  // gradients only: nobody reads a minibatch evaluation's loss or dots (scal = nullptr skips them)
  auto one = [&](Mlp *m, const float *w, float *g) {
    if (dp) m->loss_grad_local(w, g, X, Y, nullptr, count, inv_scale);
    else m->loss_grad(w, g, X, Y, nullptr, count, inv_scale, prm_.lambda, nullptr, nullptr);
  };
  if (!tnet_) {
    one(net_, wa, ga);
    one(net_, wb, gb);
  } else {
    LBF_HIP(hipEventRecord(ev_fork_, ctx_->stream)); // wa, wb, the gathered rows and gb's last reader are done
    const long long tk = twin_post([=]() {
      LBF_HIP(hipStreamWaitEvent(tctx_->stream, ev_fork_, 0));
      one(tnet_.get(), wb, gb);
      LBF_HIP(hipEventRecord(ev_join_, tctx_->stream));
    });
    try {
      one(net_, wa, ga);
    } catch (...) { // the task refers to this frame: let it finish first
      try {
        twin_wait(tk);
      } catch (...) {
      }
      throw;
    }
    twin_wait(tk); // ev_join_ recorded (and ev_fork_ waited for: it may be re-recorded after this)
    LBF_HIP(hipStreamWaitEvent(ctx_->stream, ev_join_, 0));
  }
  if (dp) reduce_pair(wa, wb, gab, inv_scale);
}

// SLBFGS::stochastic_solve (s_lbfgs.hpp:165-290) with the UnifiedSLBFGS_CPU closures
// (unified_optimization.hpp:343-400). The host RNG stream is consumed in exactly the reference's
// order; because no sample depends on device values, each epoch's index lists are drawn up front
// and uploaded once, and the epoch then runs without a host synchronisation.
int SlbfgsSolver::run(lbf_record *rec) {
  iterate(prm_.max_epochs, rec);
  return iters_;
}

// An epoch's index lists in the reference's RNG order (s_lbfgs.hpp:212-266). Every rank draws the same
// lists; with sliced data parallelism it keeps only its slice [b*rk/nr, b*(rk+1)/nr) of each batch (a
// replicated rank keeps every index). The minibatch slices come first
// in `flat` (minibatch t's rows right after minibatch t-1's, as Mlp::batch_grads reads them), the
// Hessian-batch slices after them; the draws stay in RNG order.
void SlbfgsSolver::draw_epoch(bool u_seen, EpochDraw &d) {
  const int nr = dp_inner() ? ctx_->nranks : 1, rk = dp_inner() ? ctx_->rank : 0;
  const int m_inner = int(std::max(1LL, N_ / prm_.b));
  const int L = prm_.L;
  d.flat.clear();
  d.hflat.clear();
  d.mb.assign(size_t(m_inner), Slice{});
  d.hb.assign(size_t(m_inner), Slice{-1, 0, 0});
  auto take = [&](size_t bsz, std::vector<int> &dst) {
    d.batch.clear();
    const long long tot = (long long)sampler_->draw(bsz, rng_, d.batch);
    const long long a0 = tot * rk / nr, a1 = tot * (rk + 1) / nr;
    Slice sl{(long long)dst.size(), a1 - a0, tot};
    dst.insert(dst.end(), d.batch.begin() + a0, d.batch.begin() + a1);
    return sl;
  };
  int whist_size = 1;
  for (int t = 0; t < m_inner; ++t) {
    d.mb[t] = take(size_t(prm_.b), d.flat);
    whist_size = std::min(whist_size + 1, L + 1);
    if (t > 0 && t % L == 0) {
      if (u_seen) d.hb[t] = take(size_t(prm_.b_H), d.hflat);
      u_seen = true;
    }
  }
  const long long nmb_rows = (long long)d.flat.size();
  for (Slice &h : d.hb)
    if (h.off >= 0) h.off += nmb_rows;
  d.flat.insert(d.flat.end(), d.hflat.begin(), d.hflat.end());
  d.pick = -1;
  if (whist_size >= 2) {
    std::uniform_int_distribution<size_t> pk(0, size_t(whist_size) - 2); // s_lbfgs.hpp:266
    d.pick = int(pk(rng_));
  }
  d.u_seen = u_seen;
}

int SlbfgsSolver::wh_push_slot() {
  const int L = prm_.L;
  int slot;
  if (wh_count_ < L + 1) {
    slot = (wh_head_ + wh_count_) % (L + 1);
    ++wh_count_;
  } else {
    slot = wh_head_;
    wh_head_ = (wh_head_ + 1) % (L + 1);
  }
  return slot;
}

// The inner steps of one epoch (s_lbfgs.hpp:218-262), from the anchor copy to the last step; the epoch's
// rows are gathered (xg_, yg_) and the context stream is idle when this is called.
void SlbfgsSolver::epoch_steps(const EpochDraw &d) {
  hipStream_t s = ctx_->stream;
  const long long In = net_->layers().front().in, Out = net_->layers().back().out;
  const long long ld = round4(n_);
  const int m_inner = int(std::max(1LL, N_ / prm_.b));
  const int L = prm_.L;
  const bool dp = dp_inner();
  const auto &mb = d.mb, &hb = d.hb;
  LBF_HIP(hipMemcpyAsync(wt_.get(), w_.get(), size_t(n_) * sizeof(float), hipMemcpyDeviceToDevice, s));
  wh_head_ = 0;
  wh_count_ = 0;
  const int full_at = full_ahead_step(d);
  {
    const int slot = wh_push_slot();
    LBF_HIP(hipMemcpyAsync(wh_.get() + slot * ld, wt_.get(), size_t(n_) * sizeof(float), hipMemcpyDeviceToDevice,
                           s));
    if (full_at == -1) post_full(wh_.get() + slot * ld);
  }
  // The minibatch gradients at the anchor w (fixed for the epoch, and independent of the iterates) run one
  // step ahead on the twin stream: step t's evaluation at w_t and its direction on the context stream then
  // overlap the twin's gradient of minibatch t + 1 at w, instead of joining the two evaluations of each
  // step. Same evaluations on the same inputs: bitwise the same.
  // Free-running (no per-step collective): the anchor half of step t goes to its own buffer ganc_ + t ng_
  // (the epoch's 234 anchor gradients, 501 MB at cfg 4), so the twin never waits for the context stream to
  // release a block: no ev_free_ record on the context stream (≈ 5 µs of its time per step,
  // profiles/r03/launch_floor.txt) and no wait on the twin. When that buffer does not fit in free device
  // memory (keeping a quarter of it free), or its allocation fails, the twin falls back for good to two
  // blocks, double-buffered in the second half of gpair_[t & 1]. Sliced data parallelism keeps that packed
  // [g(w_t) | g(w)] block: both halves are this rank's partial sums until the step's one all-reduce.
  bool twin_free = !dp && free_twin_;
  if (twin_free) {
    const size_t need = size_t(m_inner) * size_t(ng_);
    if (ganc_.size() < need) {
      size_t fr = 0, tot = 0;
      const bool fits = hipMemGetInfo(&fr, &tot) == hipSuccess &&
                        double(need - ganc_.size()) * sizeof(float) <= 0.75 * double(fr);
      try {
        if (fits) ganc_.resize(need);
      } catch (const Error &) {
        (void)hipGetLastError();
      }
      if (ganc_.size() < need) {
        ganc_.resize(0);
        free_twin_ = twin_free = false;
      }
    }
  }
  if (twin_free) {
    while (ev_anc_.size() < size_t(m_inner)) {
      hipEvent_t e;
      LBF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | event_release_flags()));
      ev_anc_.push_back(e);
    }
  }
  auto g1 = [&](int t) { return gpair_[t & 1].get(); };
  auto g2 = [&](int t) { return twin_free ? ganc_.get() + (long long)t * ng_ : gpair_[t & 1].get() + ng_; };
  auto rows_x = [&](const Slice &sl) { return xg_.get() + sl.off * In; };
  auto rows_y = [&](const Slice &sl) { return yg_.get() + sl.off * Out; };
  // Tickets of the twin tasks (0: ran inline). Event order across the two host threads: task t + 2 (which
  // waits on ev_free_[t & 1]) is posted at step t + 1, after step t recorded that event; step t + 2
  // re-records it only after twin_wait(task t + 2), i.e. after that wait was enqueued. Task t records
  // ev_g2_[t & 1] and the context thread waits on it after twin_wait(task t); task t + 2 re-records it
  // only after being posted at step t + 1, after that wait.
  std::vector<long long> tk(size_t(std::max(m_inner, 1)), 0);
  auto anchor_ahead = [&](int t) { // twin stream: the anchor half of step t's block
    const Slice sl = mb[t];
    float *gdst = g2(t);
    const float *xr = rows_x(sl), *yr = rows_y(sl);
    hipEvent_t efree = twin_free ? nullptr : ev_free_[t & 1], eg2 = twin_free ? ev_anc_[size_t(t)] : ev_g2_[t & 1];
    tk[size_t(t)] = twin_post([=]() {
      if (efree) LBF_HIP(hipStreamWaitEvent(tctx_->stream, efree, 0)); // step t - 2's direction read it
      if (dp)
        tnet_->loss_grad_local(w_.get(), gdst, xr, yr, nullptr, sl.cnt, 1.0 / double(sl.total));
      else
        tnet_->loss_grad(w_.get(), gdst, xr, yr, nullptr, sl.cnt, 1.0 / double(sl.total), prm_.lambda, nullptr,
                         nullptr);
      LBF_HIP(hipEventRecord(eg2, tctx_->stream));
    });
  };
  // LBF_HOST_TIMING=2: host time of each part of the inner step's enqueue (where the epoch's host-bound
  // ~130 us per step go)
  static const int host_timing = env_int("LBF_HOST_TIMING", 0);
  using hclk = std::chrono::steady_clock;
  double ht[6] = {0, 0, 0, 0, 0, 0}; // twin, main eval, events, direction, combine, Hessian step
  auto tick = [&]() { return host_timing >= 2 ? hclk::now() : hclk::time_point(); };
  auto tock = [&](int i, hclk::time_point a) {
    if (host_timing >= 2) ht[i] += std::chrono::duration<double, std::micro>(hclk::now() - a).count();
  };
  if (!twin_free) {
    // the twin may reuse block t & 1 once the direction of step t - 2 has read it: nothing of this epoch
    // has yet
    LBF_HIP(hipEventRecord(ev_free_[0], s));
    LBF_HIP(hipEventRecord(ev_free_[1], s));
  } else {
    // the twin's first launch must follow this epoch's gather and w (same role as ev_free_ above)
    LBF_HIP(hipEventRecord(ev_fork_, s));
    LBF_HIP(hipStreamWaitEvent(tctx_->stream, ev_fork_, 0));
  }
  anchor_ahead(0);
  RedAllArgs gred; // the main evaluation's split-K slabs, finished by the direction sweep
  for (int t = 0; t < m_inner; ++t) {
    const Slice &sl = mb[t];
    const double inv_b = 1.0 / double(sl.total);
    const float *gb = g2(t);
    {
      auto h0 = tick();
      if (t + 1 < m_inner) anchor_ahead(t + 1);
      tock(0, h0);
      h0 = tick();
      if (dp)
        net_->loss_grad_local(wt_.get(), g1(t), rows_x(sl), rows_y(sl), nullptr, sl.cnt, inv_b);
      else // the gradient's last reduction runs inside the direction sweep (one launch fewer per step)
        net_->loss_grad_deferred(wt_.get(), g1(t), rows_x(sl), rows_y(sl), nullptr, sl.cnt, inv_b, prm_.lambda,
                                 &gred);
      tock(1, h0);
      h0 = tick();
      twin_wait(tk[size_t(t)]); // task t recorded ev_g2_[t & 1] / ev_anc_[t]
      LBF_HIP(hipStreamWaitEvent(ctx_->stream, twin_free ? ev_anc_[size_t(t)] : ev_g2_[t & 1], 0));
      tock(2, h0);
      if (dp) reduce_pair(wt_.get(), w_.get(), g1(t), inv_b);
    }
    GramArgs ga;
    ga.policy = POL_SLBFGS;
    ga.has_g = 1;
    ga.ga = g1(t);
    ga.gb = gb;
    ga.gc = mu_.get();
    ga.g_out = v_.get();
    auto h0 = tick();
    const int slot = wh_push_slot();
    // r = H v (two-loop), then wt = wt - step * r ; w_history.push_back(wt)
    hist_.update_combine(ga, 1, +1.0, wt_.get(), wt_.get(), wh_.get() + slot * ld, -prm_.step, dp ? nullptr : &gred);
    tock(3, h0);
    h0 = tick();
    if (!twin_free) LBF_HIP(hipEventRecord(ev_free_[t & 1], ctx_->stream)); // block t & 1 read (v formed)
    tock(2, h0);
    if (t == full_at) post_full(wh_.get() + slot * ld); // the picked iterate w_{t+1} now exists
    h0 = tick();
    if (t > 0 && t % L == 0) {
      int slots[64];
      for (int i = 0; i < wh_count_; ++i) slots[i] = wh_slot(i);
      average_slots(s, n_, wh_.get(), ld, slots, wh_count_, u_.get());
      // diagnostics (lbf_slbfgs_pair_io): this event's record [w_{t+1} | u | g+ | g-] and forced inputs
      const int ev = nev_++;
      float *pr = pio_rec_ && ev < pio_cap_ ? pio_rec_ + size_t(ev) * 4 * size_t(ld) : nullptr;
      const float *pf = pio_force_ && ev < pio_cap_ ? pio_force_ + size_t(ev) * 4 * size_t(ld) : nullptr;
      const size_t nb = size_t(n_) * sizeof(float);
      if (pr) {
        LBF_HIP(hipMemcpyAsync(pr, wt_.get(), nb, hipMemcpyDeviceToDevice, s));
        LBF_HIP(hipMemcpyAsync(pr + ld, u_.get(), nb, hipMemcpyDeviceToDevice, s));
        LBF_HIP(hipMemsetAsync(pr + 2 * ld, 0, 2 * nb + 2 * (size_t(ld) - size_t(n_)) * sizeof(float), s));
      }
      if (pf) LBF_HIP(hipMemcpyAsync(u_.get(), pf + ld, nb, hipMemcpyDeviceToDevice, s));
      if (have_u_) {
        const Slice &hs = hb[t];
        const double eps = prm_.fd_eps;
        lincomb(s, n_, u_.get(), -1.0, up_.get(), s_.get()); // s = u - u_prev
        GramArgs pa;
        pa.policy = POL_SLBFGS;
        pa.has_pair = 1;
        pa.sa = u_.get();
        pa.sb = up_.get();
        float *gp = fdpair_.get(), *gm = fdpair_.get() + ng_;
        if (prm_.hvp_exact) { // y = H(u) s on the b_H batch, R-operator (hvp.hip)
          net_->hvp(u_.get(), s_.get(), X_, Y_, idx_.get() + hs.off, hs.cnt, 1.0 / double(hs.total), prm_.lambda,
                    gp);
          LBF_HIP(hipMemsetAsync(gm, 0, size_t(n_) * sizeof(float), s));
          pa.yscale = 1.0;
        } else { // s_lbfgs.hpp:88-101: central difference of two batch gradients
          lincomb(s, n_, u_.get(), eps, s_.get(), wp_.get()); // fd_hvp_grads, the two evaluations paired
          lincomb(s, n_, u_.get(), -eps, s_.get(), wm_.get());
          eval_pair(wp_.get(), wm_.get(), fdpair_.get(), hs.off, hs.cnt, 1.0 / double(hs.total));
          pa.yscale = 1.0 / (2.0 * eps);
        }
        if (pr) {
          LBF_HIP(hipMemcpyAsync(pr + 2 * ld, gp, nb, hipMemcpyDeviceToDevice, s));
          LBF_HIP(hipMemcpyAsync(pr + 3 * ld, gm, nb, hipMemcpyDeviceToDevice, s));
        }
        if (pf) {
          LBF_HIP(hipMemcpyAsync(gp, pf + 2 * ld, nb, hipMemcpyDeviceToDevice, s));
          LBF_HIP(hipMemcpyAsync(gm, pf + 3 * ld, nb, hipMemcpyDeviceToDevice, s));
        }
        pa.ya = gp;
        pa.yb = gm;
        hist_.update(pa, 0, 1, +1.0);
        if (prm_.pair_trace && npairs_ < prm_.pair_trace_cap) trace_pair(iters_, t);
      }
      LBF_HIP(hipMemcpyAsync(up_.get(), u_.get(), size_t(n_) * sizeof(float), hipMemcpyDeviceToDevice, s));
      have_u_ = true;
    }
    tock(5, h0);
  }
  if (tw_) tw_->wait_all(); // every twin task of the epoch enqueued
  if (host_timing >= 2)
    std::fprintf(stderr, "[lbf host] per inner step (us): twin %.1f, main eval %.1f, events %.1f, direction %.1f, "
                 "combine %.1f, Hessian step %.1f\n", ht[0] / m_inner, ht[1] / m_inner, ht[2] / m_inner,
                 ht[3] / m_inner, ht[4] / m_inner, ht[5] / m_inner);
}

int SlbfgsSolver::iterate(int epochs, lbf_record *rec) {
  ctx_->set_device();
  hipStream_t s = ctx_->stream;
  const long long In = net_->layers().front().in, Out = net_->layers().back().out;
  const long long ld = round4(n_);
  const int nr = ctx_->nranks, rk = ctx_->rank;
  const int m_inner = int(std::max(1LL, N_ / prm_.b));
  for (Ctx *c : {tctx_.get(), fctx_.get()}) { // the benchmark's section timing covers the side streams' launches
    if (!c) continue;                          // too (settings may change per call)
    c->prof.on = ctx_->prof.on;
    c->prof.only = ctx_->prof.only;
    if (c->prof.every != ctx_->prof.every) c->prof.seen = 0;
    c->prof.every = ctx_->prof.every;
  }
  if (!started_) {
    LBF_HIP(hipMemcpyAsync(w_.get(), user_params_, size_t(n_) * sizeof(float), hipMemcpyDeviceToDevice, s));
    t0_ = std::chrono::steady_clock::now();
    rec_i_ = rec ? rec->size : 0;
    started_ = true;
  }
  // full-batch shard of this rank
  const long long lo = N_ * rk / nr, hi = N_ * (rk + 1) / nr;
  const float *Xs = X_ + lo * In, *Ys = Y_ + lo * Out;
  const double inv_full = 1.0 / double(N_);
  auto eval_full = [&](const float *w, float *g) {
    net_->loss_grad(w, g, Xs, Ys, nullptr, hi - lo, inv_full, prm_.lambda, nullptr, hist_.scal());
  };
  auto read = [&]() {
    LBF_HIP(hipMemcpyAsync(hs_.get(), hist_.scal(), SC_N * sizeof(double), hipMemcpyDeviceToHost, s));
    LBF_HIP(hipStreamSynchronize(s));
  };
  const int target = iters_ + std::max(0, epochs);
  const int done0 = iters_;
  while (iters_ < target && !converged_) {
    if (!mu_valid_) {
      if (repl_ && nr > 1) replica_fingerprints(); // the caller's parameters must agree too
      eval_full(w_.get(), mu_.get());
      read();
      if (repl_ && nr > 1) replica_check();
    }
    if (std::sqrt(hs_[SC_TGG]) < prm_.tol) { // s_lbfgs.hpp:208
      converged_ = true;
      break;
    }
    // --- this epoch's samples in reference order (drawn during the previous epoch when it ran) -------
    if (next_ready_) std::swap(cur_, next_);
    else draw_epoch(have_u_, cur_);
    next_ready_ = false;
    const std::vector<int> &flat = cur_.flat;
    const int pick = cur_.pick;
    idx_.ensure(std::max<size_t>(1, flat.size()));
    if (!flat.empty()) { // through pinned staging: an asynchronous copy (the stream was synchronised by read())
      idx_host_.ensure(flat.size());
      std::memcpy(idx_host_.get(), flat.data(), flat.size() * sizeof(int));
      LBF_HIP(hipMemcpyAsync(idx_.get(), idx_host_.get(), flat.size() * sizeof(int), hipMemcpyHostToDevice, s));
    }
    // this rank's sampled rows of the epoch gathered once, in sampling order: step t's minibatch slice (and
    // its Hessian batch slice) is then contiguous (batch_g's column gather, unified_optimization.hpp:361-364)
    xg_.ensure(std::max<size_t>(1, flat.size()) * size_t(In));
    yg_.ensure(std::max<size_t>(1, flat.size()) * size_t(Out));
    gather_rows(s, X_, In, idx_.get(), (long long)flat.size(), int(In), xg_.get());
    gather_rows(s, Y_, Out, idx_.get(), (long long)flat.size(), int(Out), yg_.get());
    // No host synchronisation here: the upload reads pinned staging (rewritten only after the next read()),
    // and every consumer of the gathered rows is ordered after the gathers (the context stream, and the
    // twin through the event it waits on at the epoch's start), so the host enqueues the first inner step
    // while the gathers run.
    // --- epoch -----------------------------------------------------------------------------------
    static const int host_timing = env_int("LBF_HOST_TIMING", 0);
    const auto th0 = std::chrono::steady_clock::now();
    {
      // replicated data parallelism: the inner steps evaluate without the communicator
      LocalOnly lo_guard(ctx_, repl_);
      epoch_steps(cur_);
    }
    if (host_timing) { // host time to enqueue the epoch's inner steps vs the epoch on the device
      const auto th1 = std::chrono::steady_clock::now();
      LBF_HIP(hipStreamSynchronize(s));
      const auto th2 = std::chrono::steady_clock::now();
      std::fprintf(stderr, "[lbf host] epoch %d: %d inner steps enqueued in %.3f ms, device done %.3f ms later\n",
                   iters_, m_inner, std::chrono::duration<double, std::milli>(th1 - th0).count(),
                   std::chrono::duration<double, std::milli>(th2 - th1).count());
    }
    // the next epoch's lists, drawn while the GPU runs this epoch's queued steps
    if (iters_ + 1 < target || iters_ + 1 < prm_.max_epochs) {
      draw_epoch(cur_.u_seen, next_);
      next_ready_ = true;
    }
    // anchor reset (s_lbfgs.hpp:265-270)
    const float *anchor = pick >= 0 ? wh_.get() + wh_slot(pick) * ld : wt_.get();
    LBF_HIP(hipMemcpyAsync(w_.get(), anchor, size_t(n_) * sizeof(float), hipMemcpyDeviceToDevice, s));
    if (repl_ && nr > 1) replica_fingerprints(); // compared after read(): no extra host wait
    // recorder (s_lbfgs.hpp:274-284): full loss and gradient at the new anchor == next epoch's mu
    if (full_posted_) { // evaluated ahead on the third stream (fnet_): join, take its gradient and status words
      LBF_HIP(hipStreamWaitEvent(s, ev_full_, 0));
      std::swap(mu_, mu_next_);
      double *hsc = hist_.scal();
      LBF_HIP(hipMemcpyAsync(hsc + SC_LOSS, fscal_.get() + SC_LOSS, 2 * sizeof(double), hipMemcpyDeviceToDevice, s));
      LBF_HIP(hipMemcpyAsync(hsc + SC_WW, fscal_.get() + SC_WW, 2 * sizeof(double), hipMemcpyDeviceToDevice, s));
      full_posted_ = false;
    } else {
      eval_full(w_.get(), mu_.get());
    }
    read();
    if (repl_ && nr > 1) replica_check();
    if (hs_[SC_KERR] != 0.0) // dir_combine_kernel's check of the coefficient map against the ring's live count
      throw Error(LBF_ERR_STATE, "S-LBFGS: a direction step found the coefficient map K out of step with the "
                                 "history ring's live count (epoch " + std::to_string(iters_) + ")");
    mu_valid_ = true;
    last_loss_ = hs_[SC_LOSS];
    last_gnorm_ = std::sqrt(hs_[SC_TGG]);
    if (rec && rec_i_ < rec->cap) {
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count();
      if (rec->loss) rec->loss[rec_i_] = last_loss_;
      if (rec->grad_norm) rec->grad_norm[rec_i_] = last_gnorm_;
      if (rec->time_ms) rec->time_ms[rec_i_] = ms;
      if (rec->alpha) rec->alpha[rec_i_] = prm_.step;
      if (rec->ls_trials) rec->ls_trials[rec_i_] = 0;
      if (rec->accepted) rec->accepted[rec_i_] = int(hs_[SC_COUNT]);
      rec->size = std::max(rec->size, ++rec_i_);
    }
    ++iters_;
  }
  LBF_HIP(hipMemcpyAsync(user_params_, w_.get(), size_t(n_) * sizeof(float), hipMemcpyDeviceToDevice, s));
  LBF_HIP(hipStreamSynchronize(s));
  if (tctx_) {
    LBF_HIP(hipStreamSynchronize(tctx_->stream));
    tctx_->prof.merge_into(ctx_->prof);
  }
  if (fctx_) {
    LBF_HIP(hipStreamSynchronize(fctx_->stream));
    fctx_->prof.merge_into(ctx_->prof);
  }
  return iters_ - done0;
}

void SlbfgsSolver::replica_fingerprints() {
  hipStream_t s = ctx_->stream;
  const size_t cnt = 4 * size_t(ctx_->nranks);
  fp_.ensure(cnt);
  hfp_.ensure(cnt);
  LBF_HIP(hipMemsetAsync(fp_.get(), 0, cnt * sizeof(float), s));
  fingerprint(s, n_, w_.get(), ctx_->rank, fp_.get());
  ctx_->allreduce(fp_.get(), cnt);
  LBF_HIP(hipMemcpyAsync(hfp_.get(), fp_.get(), cnt * sizeof(float), hipMemcpyDeviceToHost, s));
}

void SlbfgsSolver::replica_check() const {
  const float *f = hfp_.get();
  for (int r = 1; r < ctx_->nranks; ++r)
    for (int i = 0; i < 4; ++i)
      if (f[4 * r + i] != f[i])
        throw Error(LBF_ERR_STATE, "S-LBFGS replicated data parallelism: rank " + std::to_string(r) +
                                       "'s anchor differs from rank 0's at the full-batch evaluation of epoch " +
                                       std::to_string(iters_) + " (the replicated ranks' parameters drifted apart)");
}

// Diagnostics row of the pair just offered to the ring (lbf_slbfgs_params.pair_trace): synchronous.
void SlbfgsSolver::trace_pair(int epoch, int t) {
  hipStream_t s = ctx_->stream;
  const HistView v = hist_.view();
  LBF_HIP(hipMemcpyAsync(hs_.get(), v.scal, SC_N * sizeof(double), hipMemcpyDeviceToHost, s));
  int wslot = 0;
  LBF_HIP(hipMemcpyAsync(&wslot, v.ist + IST_WSLOT, sizeof(int), hipMemcpyDeviceToHost, s));
  LBF_HIP(hipStreamSynchronize(s));
  double ss = 0.0, yy = 0.0;
  const size_t d = size_t(wslot) * size_t(v.slots) + size_t(wslot);
  LBF_HIP(hipMemcpyAsync(&ss, v.SS + d, sizeof(double), hipMemcpyDeviceToHost, s));
  LBF_HIP(hipMemcpyAsync(&yy, v.YY + d, sizeof(double), hipMemcpyDeviceToHost, s));
  LBF_HIP(hipStreamSynchronize(s));
  if (npairs_ == 0) { // the iterate after step t, u, s = u - u_prev and the y just stored in the ring
    const size_t nb = size_t(n_) * sizeof(float), ld = size_t(round4(n_));
    p0_.resize(4 * ld);
    const float *src[4] = {wt_.get(), u_.get(), s_.get(), v.Y + size_t(wslot) * size_t(v.ld)};
    for (int i = 0; i < 4; ++i)
      LBF_HIP(hipMemcpyAsync(p0_.get() + i * ld, src[i], nb, hipMemcpyDeviceToDevice, s));
    LBF_HIP(hipStreamSynchronize(s));
    p0_set_ = true;
  }
  double *row = prm_.pair_trace + size_t(npairs_++) * LBF_PAIR_TRACE_COLS;
  const double vals[LBF_PAIR_TRACE_COLS] = {double(epoch), double(t), hs_[SC_YS], ss, yy, hs_[SC_ACCEPT],
                                            hs_[SC_COUNT], 0.0};
  for (int i = 0; i < LBF_PAIR_TRACE_COLS; ++i) row[i] = vals[i];
}

bool SlbfgsSolver::pair0(float *wt, float *u, float *s, float *y) const {
  if (!p0_set_) return false;
  const size_t nb = size_t(n_) * sizeof(float), ld = size_t(round4(n_));
  float *dst[4] = {wt, u, s, y};
  for (int i = 0; i < 4; ++i)
    if (dst[i]) LBF_HIP(hipMemcpyAsync(dst[i], p0_.get() + i * ld, nb, hipMemcpyDeviceToDevice, ctx_->stream));
  LBF_HIP(hipStreamSynchronize(ctx_->stream));
  return true;
}

void SlbfgsSolver::info(lbf_solve_info *out) const {
  if (!out) return;
  std::memset(out, 0, sizeof(*out));
  out->iterations = iters_;
  out->n_evals = net_->evals() - evals0_ + (tnet_ ? tnet_->evals() : 0) + (fnet_ ? fnet_->evals() : 0);
  out->n_rows = net_->rows() - rows0_ + (tnet_ ? tnet_->rows() : 0) + (fnet_ ? fnet_->rows() : 0);
  out->final_loss = last_loss_;
  out->final_grad_norm = last_gnorm_;
}

// ================================================================================================
// GD / SGD with momentum
// ================================================================================================
namespace {
void put_record(lbf_record *rec, int i, double loss, double gnorm, double ms, double lr) {
  if (!rec || i >= rec->cap) return;
  if (rec->loss) rec->loss[i] = loss;
  if (rec->grad_norm) rec->grad_norm[i] = gnorm;
  if (rec->time_ms) rec->time_ms[i] = ms;
  if (rec->alpha) rec->alpha[i] = lr;
  if (rec->ls_trials) rec->ls_trials[i] = 0;
  if (rec->accepted) rec->accepted[i] = -1;
  rec->size = std::max(rec->size, i + 1);
}
} // namespace

// CudaGD::solve (gd.cuh:38-106): the loss/grad callback is one fused evaluation; the reference's
// blocking cublasSnrm2 becomes the evaluation's g.g, read with the loss once per iteration.
int run_gd(Mlp *net, const lbf_gd_params &prm, float *d_params, const float *X, const float *Y, long long n_local,
           long long n_global, lbf_record *rec, lbf_solve_info *info) {
  LBF_REQUIRE(d_params && n_local >= 0 && n_global > 0 && (n_local == 0 || (X && Y)), "bad argument");
  Ctx *c = net->ctx();
  c->set_device();
  hipStream_t s = c->stream;
  const long long n = (long long)net->nparams();
  DevBuf<float> g(size_t(round4(n + 2))), v(size_t(std::max(1LL, n)));
  DevBuf<double> scal(SC_N);
  PinnedBuf<double> hs;
  hs.ensure(SC_N);
  LBF_HIP(hipMemsetAsync(v.get(), 0, size_t(n) * sizeof(float), s));
  const long long evals0 = net->evals(), rows0 = net->rows();
  auto eval = [&]() {
    net->loss_grad(d_params, g.get(), X, Y, nullptr, n_local, 1.0 / double(n_global), 0.0, nullptr, scal.get());
    LBF_HIP(hipMemcpyAsync(hs.get(), scal.get(), SC_N * sizeof(double), hipMemcpyDeviceToHost, s));
    LBF_HIP(hipStreamSynchronize(s));
  };
  const float lr = float(prm.lr), mom = float(prm.momentum), tol = float(prm.tol);
  eval();
  const auto t0 = std::chrono::steady_clock::now();
  int done = 0, ri = rec ? rec->size : 0;
  for (int it = 0; it < prm.max_iters; ++it) {
    if (float(std::sqrt(hs[SC_TGG])) < tol) break; // gd.cuh:73
    momentum_step(s, n, mom, lr, nullptr, g.get(), v.get(), d_params);
    eval();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    put_record(rec, ri++, double(float(hs[SC_LOSS])), double(float(std::sqrt(hs[SC_TGG]))), ms, double(lr));
    ++done;
  }
  if (info) {
    std::memset(info, 0, sizeof(*info));
    info->iterations = done;
    info->n_evals = net->evals() - evals0;
    info->n_rows = net->rows() - rows0;
    info->final_loss = hs[SC_LOSS];
    info->final_grad_norm = std::sqrt(hs[SC_TGG]);
  }
  return done;
}

// CudaSGD::solve (sgd.cuh:50-153). Batch losses accumulate on the device (epoch_loss_acc, fp32 like
// the reference's host sum), so an epoch synchronises once, not once per batch.
int run_sgd(Mlp *net, const lbf_sgd_params &prm, float *d_params, const float *X, const float *Y, long long N,
            lbf_record *rec, lbf_solve_info *info) {
  LBF_REQUIRE(d_params && X && Y && N > 0 && prm.batch > 0, "bad argument");
  Ctx *c = net->ctx();
  LBF_REQUIRE(!c->dp(), "SGD runs on one rank (the reference's contiguous batches have no shard split)");
  c->set_device();
  hipStream_t s = c->stream;
  const long long n = (long long)net->nparams();
  const int In = net->layers().front().in, Out = net->layers().back().out;
  DevBuf<float> g(size_t(round4(n + 2))), v(size_t(std::max(1LL, n))), esum(1);
  DevBuf<double> scal(SC_N);
  PinnedBuf<double> hs;
  hs.ensure(SC_N);
  PinnedBuf<float> he;
  he.ensure(1);
  LBF_HIP(hipMemsetAsync(v.get(), 0, size_t(n) * sizeof(float), s));
  const long long evals0 = net->evals(), rows0 = net->rows();
  auto full = [&]() {
    net->loss_grad(d_params, g.get(), X, Y, nullptr, N, 1.0 / double(N), 0.0, nullptr, scal.get());
    LBF_HIP(hipMemcpyAsync(hs.get(), scal.get(), SC_N * sizeof(double), hipMemcpyDeviceToHost, s));
    LBF_HIP(hipStreamSynchronize(s));
  };
  const float mom = float(prm.momentum), tol = float(prm.tol);
  float cur_lr = float(prm.lr);
  const long long nb = cdiv(N, prm.batch);
  float prev = std::numeric_limits<float>::infinity();
  const auto t0 = std::chrono::steady_clock::now();
  int done = 0, ri = rec ? rec->size : 0;
  auto ms_now = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  if (rec) { // sgd.cuh:93-98
    full();
    put_record(rec, ri++, double(float(hs[SC_LOSS])), double(float(std::sqrt(hs[SC_TGG]))), 0.0, double(cur_lr));
    ++done;
  }
  for (int it = 0; it < prm.max_epochs; ++it) {
    if (prm.decay_step > 0 && it > 0 && it % prm.decay_step == 0) cur_lr *= float(prm.decay_rate); // :101-103
    LBF_HIP(hipMemsetAsync(esum.get(), 0, sizeof(float), s));
    for (long long b = 0; b < nb; ++b) { // :107-127
      const long long r0 = b * prm.batch, bs = std::min<long long>(prm.batch, N - r0);
      net->loss_grad(d_params, g.get(), X + r0 * In, Y + r0 * Out, nullptr, bs, 1.0 / double(bs), 0.0, nullptr,
                     scal.get());
      epoch_loss_acc(s, scal.get(), bs, esum.get());
      momentum_step(s, n, mom, cur_lr, nullptr, g.get(), v.get(), d_params);
    }
    LBF_HIP(hipMemcpyAsync(he.get(), esum.get(), sizeof(float), hipMemcpyDeviceToHost, s));
    LBF_HIP(hipStreamSynchronize(s));
    const float avg = he[0] / float(N);
    if (tol > 0.0f && std::isfinite(prev)) { // :129-135
      const float rel = std::fabs(prev - avg) / std::max(1.0f, std::fabs(prev));
      if (rel < tol) break;
    }
    prev = avg;
    if (rec) { // :138-148
      full();
      put_record(rec, ri++, double(float(hs[SC_LOSS])), double(float(std::sqrt(hs[SC_TGG]))), ms_now(),
                 double(cur_lr));
    }
    ++done;
  }
  if (info) {
    std::memset(info, 0, sizeof(*info));
    info->iterations = done;
    info->n_evals = net->evals() - evals0;
    info->n_rows = net->rows() - rows0;
    info->final_loss = rec ? hs[SC_LOSS] : double(prev);
    info->final_grad_norm = rec ? std::sqrt(hs[SC_TGG]) : 0.0;
  }
  return done;
}

} // namespace lbf
