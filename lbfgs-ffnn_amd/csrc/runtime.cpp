// Context, MLP evaluation plan and device history (see runtime.hpp).
#include "runtime.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace lbf {

// ------------------------------------------------------------------------------------------------
// Ctx
// ------------------------------------------------------------------------------------------------
Ctx::~Ctx() {
  comm.reset();
  if (own_stream && stream) (void)hipStreamDestroy(stream);
}

Profiler::~Profiler() {
  for (auto e : pool) (void)hipEventDestroy(e);
}

size_t Profiler::mark(hipStream_t s) {
  if (used == pool.size()) {
    hipEvent_t e;
    LBF_HIP(hipEventCreateWithFlags(&e, hipEventDefault | event_release_flags()));
    pool.push_back(e);
  }
  LBF_HIP(hipEventRecord(pool[used], s));
  return used++;
}

void Profiler::add(const Rec &r, float t) {
  if (size_t(r.id) >= ms.size()) {
    ms.resize(r.id + 1, 0.0);
    cnt.resize(r.id + 1, 0);
    work.resize(r.id + 1, 0.0);
  }
  ms[r.id] += t;
  cnt[r.id] += 1;
  work[r.id] += r.work;
}

void Profiler::resolve() {
  if (recs.empty()) return;
  LBF_HIP(hipEventSynchronize(pool[used - 1]));
  for (auto &r : recs) {
    float t = 0.f;
    LBF_HIP(hipEventElapsedTime(&t, pool[r.a], pool[r.b]));
    add(r, t);
  }
  recs.clear();
  used = 0;
}

void Profiler::merge_into(Profiler &dst) {
  resolve();
  if (dst.ms.size() < ms.size()) {
    dst.ms.resize(ms.size(), 0.0);
    dst.cnt.resize(ms.size(), 0);
    dst.work.resize(ms.size(), 0.0);
  }
  for (size_t i = 0; i < ms.size(); ++i) {
    dst.ms[i] += ms[i];
    dst.cnt[i] += cnt[i];
    dst.work[i] += work[i];
  }
  ms.assign(ms.size(), 0.0);
  cnt.assign(cnt.size(), 0);
  work.assign(work.size(), 0.0);
}

void Ctx::set_device() const { LBF_HIP(hipSetDevice(device)); }

void Ctx::allreduce(float *buf, size_t count) {
  if (!dp()) return;
  comm->allreduce(buf, count, stream);
}

// ------------------------------------------------------------------------------------------------
// Mlp
// ------------------------------------------------------------------------------------------------
Mlp::Mlp(Ctx *ctx, int nl, const int *dims, const int *acts) : ctx_(ctx) {
  LBF_REQUIRE(nl >= 1 && nl <= 16, "1..16 layers");
  size_t off = 0;
  for (int l = 0; l < nl; ++l) {
    LBF_REQUIRE(dims[l] > 0 && dims[l + 1] > 0, "layer dims must be positive");
    LBF_REQUIRE(acts[l] >= 0 && acts[l] <= 3, "activation id 0..3");
    Layer L;
    L.in = dims[l];
    L.out = dims[l + 1];
    L.act = acts[l];
    L.off = off;
    off += size_t(L.in + 1) * L.out;
    layers_.push_back(L);
  }
  nparams_ = off;
  if (const char *e = std::getenv("LBF_NO_FOLD")) fold_on_ = e[0] != '1'; // tests: the unfolded route
  if (const char *e = std::getenv("LBF_NO_GROUP")) group_dw_ = e[0] != '1';
}

// Split-K factor for `tiles` output tiles over a K of `K` rows: the GEMM tiles run two workgroups per
// CU, so a launch is ceil(tiles * s / slots) waves of equal-length workgroups; choose s (chunks of at
// least min_chunk rows, slabs within a memory cap) to maximise tiles * s / (waves * slots), the
// smallest s within half a percent of the best. A count just past a multiple of the slots (e.g. 520
// workgroups on 512 slots) would otherwise cost a whole extra wave.
static long long split_factor(long long tiles, long long K, long long min_chunk, long long slots,
                              long long slab_elems_per_split) {
  const long long cap_elems = 1LL << 29; // 2 GiB of fp32 slabs
  long long smax = std::max(1LL, std::min(cdiv(K, min_chunk), 4 * slots));
  if (slab_elems_per_split > 0) smax = std::max(1LL, std::min(smax, cap_elems / slab_elems_per_split));
  long long best = 1;
  double best_eff = 0.0;
  for (long long s = 1; s <= smax; ++s) {
    const long long wg = tiles * s, waves = cdiv(wg, slots);
    const double eff = double(wg) / double(waves * slots);
    if (eff > best_eff + 0.005) {
      best_eff = eff;
      best = s;
    }
  }
  return best;
}

// Batches up to this many rows are "small" for the dW plan (64x64 tiles, k chunks of two k-tiles).
constexpr long long DW_SMALL_BATCH = 2048;

// Forward plan (split-K for few row tiles), the EPI_HEAD fold, then the split-K plan of every dW GEMM
// for batch B (workgroup-slot aware, split_factor), k chunks a multiple of the 32-deep LDS tile.
void Mlp::plan(long long B) {
  if (planned_ == B) return;
  size_t slab = 0, fslab = 0;
  const int nl = int(layers_.size());
  const bool fused = nl >= 2 && head_supported(layers_[nl - 1].in, layers_[nl - 1].out);
  const long long slots = 2LL * ctx_->cus;
  for (auto &L : layers_) {
    // forward GEMM: with fewer row tiles than CUs (a data-parallel rank's shard), split K so the chip
    // fills; the partial slabs are summed in split order with the bias and activation afterwards
    int fBM, fBN;
    gemm_tile_for(L.out, TILE_AUTO, &fBM, &fBN);
    const long long ftiles = cdiv(B, 128) * cdiv(L.out, fBN);
    L.fsplits = 1;
    L.fk_chunk = L.in;
    L.ftile = TILE_AUTO;
    // Row-tile height for layers 65..128 wide (one column tile of 128, where the head can fuse). A small
    // tile is bound by its per-CU operand delivery (~22 GB/s per CU for the LDS-DMA stream,
    // profiles/r02/gemm_small_tiles.txt), a 128-row tile by the MFMA issue, so the plan takes the tile
    // with the shortest estimated launch: n = the most tiles any CU gets, each costing a measured time per
    // 32-deep k-tile, plus one epilogue per round of co-resident workgroups (one per CU for 32 x 128,
    // two otherwise). Constants: 784 -> 128 with the fused head on MI355X (profiles/r02/
    // gemm_fwd_tiles_by_shard.txt, tile64_*.json, tilemodel_*.json): 32 x 128 at 7500 rows (one round),
    // 64 x 128 at 15000-40000 rows (forward 63.5 -> 48.4 us at 15000, 120.4 -> 77.9 at 30000,
    // 132.4 -> 112.7 at 40000), 128 x 128 at 60000 (137 against 144.5 with 64-row tiles). Layers up to 64
    // wide keep the round-1 rule (32-row tiles below 256 row tiles of 128, else 128 x 64 / 128 x 32).
    const long long cus = ctx_->cus, nkt = cdiv(L.in, 32);
    auto est_us = [&](long long bm, double per_ktile, long long per_round, double epi) {
      const long long n = cdiv(cdiv(B, bm), cus);
      return double(n) * per_ktile * double(nkt) + double(cdiv(n, per_round)) * epi;
    };
    if (L.out > 64 && L.out <= 128) {
      const double t32 = est_us(32, 0.93, 1, 8.0), t64 = est_us(64, 1.25, 2, 12.0), t128 = est_us(128, 2.3, 2, 20.0);
      if (t32 <= t64 && t32 <= t128) L.ftile = TILE_32x128; // full rows (the head can still fuse), no split
      else if (t64 <= t128) L.ftile = TILE_64x128;
    } else if (L.out <= 64 && cdiv(B, 128) < 256) {
      L.ftile = TILE_32x128;
    }
    if (L.ftile != TILE_AUTO) {
      // no split: the fused head and the activation need the full K
    } else if (ftiles < 192 && L.in >= 256) {
      // Few rows of a wide layer (S-LBFGS minibatches: 256 x 784 -> 512 is 8 tiles of 128 x 128): split
      // K. With 32 x 128 tiles the rows make 4x the tiles, so fewer, longer splits fill the chip (one
      // workgroup per CU) and the slabs are a quarter of the bytes of 128 x 128 tiles at the same count.
      const long long tiles32 = cdiv(B, 32) * cdiv(L.out, 128);
      long long fs;
      if (2 * tiles32 <= cus) {
        L.ftile = TILE_32x128;
        fs = std::max(2LL, std::min(cus / tiles32, cdiv(L.in, 64))); // splits of >= 2 k-tiles
        static const int fs_cap = env_int("LBF_FSPLIT_CAP", 0); // A/B of the split count (slab bytes vs depth)
        if (fs_cap > 0) fs = std::min<long long>(fs, fs_cap);
      } else {
        fs = std::min(cdiv(384, ftiles), (long long)L.in / 128);
      }
      long long fkc = cdiv(cdiv(L.in, fs), 32) * 32;
      fs = cdiv(L.in, fkc);
      if (fs > 1) {
        L.fsplits = int(fs);
        L.fk_chunk = int(fkc);
        fslab = std::max(fslab, size_t(fs) * size_t(B) * L.out);
      }
    }
    // dW: 64x64 tiles over narrow outputs -> fewer, longer K splits (a third of the slab traffic)
    // (only for short K: at long K the 128x128 tile's reuse wins over the slab savings). Small batches
    // (S-LBFGS minibatches, K = 128 / 256 rows) take 64x64 tiles at any width: four times the tiles of
    // 128x128 at the same K, where 128x128 tiles filled a fifth of the chip (784 -> 512: 56 workgroups).
    L.dtile = ((L.out <= 128 && L.in + 1 <= 1024 && B <= 16384) || B <= DW_SMALL_BATCH) ? TILE_64x64 : TILE_AUTO;
    // (128 x 128 tiles with two k-groups and one workgroup per CU, half the split-K slabs, measured slower at
    // cfg 2: dW 128.5 against 112.2 us, profiles/r04/a/bench_400{,_nok2}.json; not kept)
  }
  // The last hidden layer's dW GEMM has in + 1 rows; when they pass a multiple of its tile height by
  // at most 16 input columns + the bias row (784 + 1 = 6 x 128 + 17 at cfg 2), those rows go to the
  // EPI_HEAD epilogue, which holds delta in registers, instead of a last row tile that would be
  // mostly padding (a seventh of the dW GEMM's MFMA work at cfg 2).
  fold_ = -1;
  fold_c0_ = 0;
  if (fold_on_ && gemm_head_on()) {
    const Layer &L = layers_[size_t(nl - 2)];
    int BM, BN;
    gemm_tile_for(L.out, L.dtile, &BM, &BN);
    const int c0 = L.in / BM * BM;
    if (c0 > 0 && L.in - c0 <= 16 && L.in % 4 == 0 && L.out <= 128) {
      fold_ = L.in - c0;
      fold_c0_ = c0;
    }
  }
  // dW tiles and split-K, last layer first: layer l's launch also carries the side blocks that finish
  // layer l+1's slabs (side_reduced), and those take workgroup slots too
  for (int l = nl - 1; l >= 0; --l) {
    Layer &L = layers_[l];
    int BM, BN;
    const long long M = (fold_ >= 0 && l == nl - 2) ? fold_c0_ : L.in + 1;
    gemm_tile_for(L.out, L.dtile, &BM, &BN);
    const long long tiles = cdiv(M, BM) * cdiv(L.out, BN);
    const long long min_chunk = L.dtile == TILE_64x64 ? (B <= DW_SMALL_BATCH ? 64 : 256) : 128;
    long long side = 0;
    if (side_reduced(l + 1, fused, 0)) {
      const Layer &N1 = layers_[l + 1];
      long long cols = (long long)(N1.in + 1) * N1.out;
      if (fold_ >= 0 && l == nl - 2) cols += (long long)(fold_ + 1) * L.out;
      side = cdiv(cdiv(cols, 256), tiles) * tiles; // gemm.hip SIDE_COLS per side block
    }
    long long splits = split_factor(tiles, B, min_chunk, std::max(slots - side, slots / 2), M * L.out);
    long long kc = cdiv(cdiv(B, splits), 32) * 32;
    if (kc <= 0) kc = 32;
    splits = std::max(1LL, cdiv(B, kc));
    L.splits = int(splits);
    L.k_chunk = int(kc);
  }
  for (auto &L : layers_) {
    L.slab_off = slab;
    if (L.splits > 1) slab += size_t(L.splits) * size_t(L.in + 1) * L.out; // every layer keeps its own slabs
  }
  static const int show = env_int("LBF_SHOW_PLAN", 0);
  if (show) {
    for (int l = 0; l < nl; ++l)
      std::fprintf(stderr, "[lbf plan] B=%lld layer %d: dW tile %d splits %d k_chunk %d | fwd tile %d splits %d\n", B,
                   l, layers_[l].dtile, layers_[l].splits, layers_[l].k_chunk, layers_[l].ftile, layers_[l].fsplits);
    std::fprintf(stderr, "[lbf plan] B=%lld fold %d from column %d\n", B, fold_, fold_c0_);
  }
  slab_.ensure(slab);
  fslab_.ensure(std::max<size_t>(fslab, 1));
  fslab2_.ensure(std::max<size_t>(fslab, 1)); // odd layers' slabs: the next layer may read the previous one's
  planned_ = B;
}

// dX GEMM tile: 128-row tiles unless they leave most CUs idle (a minibatch of a few hundred rows:
// S-LBFGS's b = 256 gives 8 tiles of 128 x 128 for a 512-wide layer), then 32 x 128 (four times the
// row tiles; the epilogue needs the full K, so no split-K here).
int Mlp::dx_tile(long long B, int N) const {
  if (N >= 128 && cdiv(B, 128) * cdiv((long long)N, 128) < ctx_->cus / 2) return TILE_32x128;
  return TILE_AUTO;
}

bool Mlp::rowhead_on(long long B) const {
  const int nl = int(layers_.size());
  if (nl < 2 || B <= 0) return false;
  const Layer &Lo = layers_[size_t(nl - 1)], &Lh = layers_[size_t(nl - 2)];
  return Lh.fsplits > 1 && rowhead_supported(Lo.in, Lo.out) && head_supported(Lo.in, Lo.out);
}

bool Mlp::gemm_head_on() const {
  const int nl = int(layers_.size());
  if (nl < 2) return false;
  const Layer &Lo = layers_[size_t(nl - 1)];
  return head_supported(Lo.in, Lo.out) && layers_[size_t(nl - 2)].fsplits == 1 && Lo.in <= 128;
}

void Mlp::ensure(long long B) {
  if (B > cap_) {
    A_.clear();
    D_.clear();
    for (auto &L : layers_) {
      A_.emplace_back(size_t(std::max(1LL, B)) * L.out);
      D_.emplace_back(size_t(std::max(1LL, B)) * L.out);
    }
    cap_ = B;
  }
  plan(B);
  const int nl = int(layers_.size());
  const Layer &Lo = layers_[nl - 1];
  size_t nloss = size_t(loss_partials_wg(std::max(1LL, B), Lo.out));
  if (nl >= 2 && head_supported(Lo.in, Lo.out)) {
    const size_t hw = size_t(std::max({head_nwg(B, Lo.in), gemm_row_tiles(int(std::max(1LL, B)), layers_[nl - 2].ftile),
                                       rowhead_nwg(B)}));
    nloss = std::max(nloss, hw);
    head_slab_.ensure(hw * (size_t(Lo.in + 1) * Lo.out + (fold_ >= 0 ? size_t(fold_ + 1) * Lo.in : 0)));
  }
  loss_part_.ensure(nloss);
  long long ncg = 0;
  for (auto &L : layers_) ncg += cdiv((long long)(L.in + 1) * L.out, RA_COLS);
  dots_part_.ensure(size_t(std::max<long long>(dots_partials_wg(nparams_), ncg)) * 3);
  colpart_.ensure(size_t(ncg) * RA_MAXPART * RA_COLS);
  sse_.ensure(1);
}

// Layer l's dW slabs are reduced by side blocks of layer l-1's dW launch: the fused head's always,
// other layers' when they have many split-K slabs over few columns.
bool Mlp::side_reduced(int l, bool fused, int nloss) const {
  if (l <= 0 || l >= int(layers_.size())) return false;
  (void)nloss;
  if (fused && l == int(layers_.size()) - 1) return true;
  return layers_[l].splits > 2 * RA_SPLITS_PER_PART;
}

GemmDesc Mlp::fwd_desc(size_t l, const float *P, const float *in, const int *idx, long long B) const {
  const Layer &L = layers_[l];
  GemmDesc d;
  d.M = int(B);
  d.N = L.out;
  d.K = L.in;
  d.A = in;
  d.lda = L.in;
  d.a_kc = true;
  d.a_idx = (l == 0) ? idx : nullptr;
  d.B = P + L.off; // W as [In][Out] row-major (column-major Out x In)
  d.ldb = L.out;
  d.b_kc = false;
  d.C = A_[l].get();
  d.ldc = L.out;
  d.epi = EPI_FWD;
  d.bias = P + L.off + size_t(L.in) * L.out;
  d.act = L.act;
  d.abort = ctx_->abort;
  d.tile = L.ftile;
  return d;
}

// Layer l's forward GEMM as forward() launches it (split-K slabs into fslab_buf(l) when split).
GemmDesc Mlp::fwd_launch_desc(size_t l, const float *P, const float *in, const int *idx, long long B) {
  const Layer &L = layers_[l];
  GemmDesc d = fwd_desc(l, P, in, idx, B);
  if (L.fsplits > 1) {
    d.epi = EPI_STORE;
    d.C = fslab_buf(l);
    d.splits = L.fsplits;
    d.k_chunk = L.fk_chunk;
    d.slab_stride = B * L.out;
  }
  return d;
}

// d (layer l + 1's GEMM) takes its A, layer l's activations, from layer l's split-K slabs
void Mlp::set_asum(GemmDesc &d, size_t l, const float *P, long long B) {
  const Layer &L = layers_[l];
  d.a_slab = fslab_buf(l);
  d.a_splits = L.fsplits;
  d.a_slab_stride = B * L.out;
  d.a_bias = P + L.off + size_t(L.in) * L.out;
  d.a_act = L.act;
  d.a_out = A_[l].get();
}

const float *Mlp::forward(const float *P, const float *X, const int *idx, long long B, int nrun, bool raw_last) {
  ensure(B);
  hipStream_t s = ctx_->stream;
  const float *in = X;
  const size_t nr = nrun < 0 ? layers_.size() : size_t(nrun);
  bool pending = false; // layer l - 1's slabs are reduced by layer l's GEMM (its A prologue)
  for (size_t l = 0; l < nr; ++l) {
    const Layer &L = layers_[l];
    GemmDesc d = fwd_launch_desc(l, P, in, idx, B);
    if (pending) set_asum(d, l - 1, P, B);
    {
      ProfScope ps(ctx_, PK_FWD, int(l), double(B));
      gemm(s, d);
    }
    pending = false;
    if (L.fsplits > 1 && !(raw_last && l + 1 == nr)) {
      // The split-K slabs summed in split order with the bias and activation: by the next layer's GEMM while
      // it loads its A (one launch fewer; the 32 x 128 split tile of S-LBFGS minibatches), else by
      // fwd_reduce_act. (An in-launch reduction by each tile's last split measured slower: the reducer's
      // serial slab read lengthened the GEMM more than the launch it saved, profiles/r03/bench_cfg4_*_fin.json.)
      if (l + 1 < nr) {
        GemmDesc dn = fwd_launch_desc(l + 1, P, A_[l].get(), nullptr, B);
        set_asum(dn, l, P, B);
        pending = gemm_asum_ok(dn);
      }
      if (!pending)
        fwd_reduce_act(s, fslab_buf(l), L.fsplits, B * L.out, int(B), L.out, d.bias, L.act, A_[l].get(), ctx_->abort);
    }
    in = A_[l].get();
  }
  return in;
}

// Forward phase of an evaluation: every forward GEMM, the output layer (fused head or loss_diff) with
// its SSE partials, delta of the last layer the head covers, and the head's [dW ; db] partial slabs.
// What the backward phase needs is kept in fs_.
void Mlp::forward_phase(const float *P, const float *X, const float *Y, const int *idx, long long B,
                        double inv_scale) {
  hipStream_t s = ctx_->stream;
  const int nl = int(layers_.size());
  const Layer &Lo = layers_[nl - 1];
  const bool fused = nl >= 2 && head_supported(Lo.in, Lo.out);
  ensure(B);
  // the output layer inside the last hidden layer's forward GEMM (EPI_HEAD), when that GEMM is one
  // unsplit tile column: its activations then never reach HBM
  const bool gemm_head = gemm_head_on();
  // the fold reads the last hidden layer's input with 16-byte loads; an unaligned caller X (2-layer
  // nets) takes the unfolded route instead
  const float *head_in = nl >= 3 ? A_[nl - 3].get() : X;
  const int fold = (gemm_head && (reinterpret_cast<uintptr_t>(head_in) & 15u) == 0) ? fold_ : -1;
  const bool row_head = fused && !gemm_head && rowhead_on(B);
  forward(P, X, idx, B, fused ? (gemm_head ? nl - 2 : nl - 1) : nl, row_head);
  int nloss, lstart;
  if (row_head) {
    // last layer straight from the last hidden layer's split-K slabs: its fwd_reduce_act and the tile head
    // in one launch (head.hip rowhead)
    const Layer &Lh = layers_[nl - 2];
    RowHeadArgs r;
    r.fslab = fslab_buf(size_t(nl - 2));
    r.splits = Lh.fsplits;
    r.stride = B * Lh.out;
    r.hbias = P + Lh.off + size_t(Lh.in) * Lh.out;
    r.act_prev = Lh.act;
    r.P = P + Lo.off;
    r.H = Lo.in;
    r.Out = Lo.out;
    r.act_out = Lo.act;
    r.Y = Y;
    r.idx = idx;
    r.B = B;
    r.rpw = rowhead_rpw(B);
    r.inv_scale = inv_scale;
    r.delta = D_[nl - 2].get();
    r.slab = head_slab_.get();
    r.sse_part = loss_part_.get();
    r.abort = ctx_->abort;
    nloss = rowhead_nwg(B);
    {
      ProfScope ps(ctx_, PK_LOSS);
      rowhead(s, r);
    }
    lstart = nl - 2;
  } else if (gemm_head) {
    nloss = gemm_row_tiles(int(B), layers_[nl - 2].ftile);
    GemmDesc d = fwd_desc(size_t(nl - 2), P, head_in, idx, B);
    d.epi = EPI_HEAD;
    d.C = nullptr;
    d.head_P = P + Lo.off;
    d.head_out = Lo.out;
    d.head_act = Lo.act;
    d.head_Y = Y;
    d.head_idx = idx;
    d.head_inv_scale = inv_scale;
    d.head_delta = D_[nl - 2].get();
    d.head_slab = head_slab_.get();
    d.head_sse = loss_part_.get();
    d.head_fold = fold;
    d.head_fold_c0 = fold_c0_;
    ProfScope ps(ctx_, PK_FWD, nl - 2, double(B));
    gemm(s, d);
    lstart = nl - 2;
  } else if (fused) {
    // last layer: forward + loss + dZ + delta + [dW ; db] partials in one kernel (head.hip)
    nloss = head_nwg(B, Lo.in);
    {
      ProfScope ps(ctx_, PK_LOSS);
      head_fused(s, A_[nl - 2].get(), Lo.in, P + Lo.off, Lo.out, Y, idx, B, Lo.act, layers_[nl - 2].act, inv_scale,
                 D_[nl - 2].get(), head_slab_.get(), loss_part_.get(), ctx_->abort);
    }
    lstart = nl - 2;
  } else {
    nloss = loss_partials_wg(std::max(1LL, B), Lo.out);
    ProfScope ps(ctx_, PK_LOSS);
    loss_diff(s, A_[nl - 1].get(), Lo.out, Y, Lo.out, idx, B, Lo.out, Lo.act, inv_scale, D_[nl - 1].get(), Lo.out,
              loss_part_.get());
    lstart = nl - 1;
  }
  fs_.B = B;
  fs_.fused = fused;
  fs_.fold = fold;
  fs_.nloss = nloss;
  fs_.lstart = lstart;
}

// Loss only (forward phase + the SSE reduction; the reference's f(x) of a line-search trial,
// full_batch_minimizer.hpp:136): SC_SSE / SC_LOSS of scal, bitwise the values a full evaluation of
// the same point writes (same partials, same reduction order). The forward state stays for
// grad_after_loss. lambda must be 0 (the L-BFGS objectives).
void Mlp::loss_only(const float *P, const float *X, const float *Y, const int *idx, long long B, double inv_scale,
                    double *scal) {
  LBF_REQUIRE(B >= 0, "negative batch");
  hipStream_t s = ctx_->stream;
  const float *hilo = nullptr;
  if (B > 0) forward_phase(P, X, Y, idx, B, inv_scale);
  if (ctx_->dp() || B == 0) {
    hilo_.ensure(4);
    if (B > 0) sse_pack(s, loss_part_.get(), fs_.nloss, hilo_.get(), ctx_->abort);
    else zero_fill(s, 2, hilo_.get(), ctx_->abort);
    if (ctx_->dp()) {
      ProfScope ps(ctx_, PK_ALLREDUCE);
      ctx_->allreduce(hilo_.get(), 2);
    }
    hilo = hilo_.get();
  }
  ProfScope ps(ctx_, PK_FINAL, 2);
  sse_loss(s, loss_part_.get(), B > 0 ? fs_.nloss : 0, hilo, inv_scale, scal, ctx_->abort);
  ++loss_only_;
}

void Mlp::loss_grad(const float *P, float *G, const float *X, const float *Y, const int *idx, long long B,
                    double inv_scale, double lambda, const float *pdir, double *scal, const TailFuse *tf) {
  LBF_REQUIRE(B >= 0, "negative batch");
  if (B > 0) forward_phase(P, X, Y, idx, B, inv_scale);
  backward_phase(P, G, X, idx, B, inv_scale, lambda, pdir, scal, tf, false, nullptr);
}

void Mlp::loss_grad_deferred(const float *P, float *G, const float *X, const float *Y, const int *idx, long long B,
                             double inv_scale, double lambda, RedAllArgs *red) {
  LBF_REQUIRE(B >= 0 && red, "loss_grad_deferred: batch / output");
  LBF_REQUIRE(!ctx_->dp(), "loss_grad_deferred: single rank (or replicated) only");
  red->nseg = 0;
  if (B > 0) forward_phase(P, X, Y, idx, B, inv_scale);
  backward_phase(P, G, X, idx, B, inv_scale, lambda, nullptr, nullptr, nullptr, false, nullptr, red);
}

void Mlp::loss_grad_local(const float *P, float *G, const float *X, const float *Y, const int *idx, long long B,
                          double inv_scale) {
  LBF_REQUIRE(B >= 0, "negative batch");
  if (B > 0) forward_phase(P, X, Y, idx, B, inv_scale);
  backward_phase(P, G, X, idx, B, inv_scale, 0.0, nullptr, nullptr, nullptr, true, nullptr);
}

void Mlp::grad_after_loss(const float *P, float *G, const float *X, const int *idx, long long B, double inv_scale,
                          double lambda, const float *pdir, double *scal, const TailFuse *tf) {
  LBF_REQUIRE(B == 0 || fs_.B == B, "grad_after_loss: no forward phase of this batch");
  ++gal_;
  // the reduced route reports the loss of the loss-only trial's own all-reduced words, so the Armijo
  // decision and the recorded loss are one value whatever order the collective sums the two buffers in
  const bool reduced = ctx_->dp() || B == 0;
  backward_phase(P, G, X, idx, B, inv_scale, lambda, pdir, scal, tf, false, reduced ? hilo_.get() : nullptr);
}

// Backward phase: the dW / dX GEMMs below the head, every layer's slab reduction, the gradient
// finish (+ all-reduce, dots, status block) or the fused optimizer tail.
void Mlp::backward_phase(const float *P, float *G, const float *X, const int *idx, long long B, double inv_scale,
                         double lambda, const float *pdir, double *scal, const TailFuse *tf, bool local,
                         const float *hilo_in, RedAllArgs *defer) {
  hipStream_t s = ctx_->stream;
  const int nl = int(layers_.size());
  const Layer &Lo = layers_[nl - 1];
  const bool empty = B == 0; // a data-parallel rank whose share of a small batch is empty
  const bool reduced = ctx_->dp() || empty || local;
  const bool fused = fs_.fused;
  const int fold = empty ? -1 : fs_.fold, nloss = empty ? 0 : fs_.nloss, lstart = empty ? -1 : fs_.lstart;
  const long long nfold = fold >= 0 ? (long long)(fold + 1) * Lo.in : 0; // fold rows in the head slab
  // Where this rank's gradient lands before the collective: G itself on a single rank and for a packed
  // local evaluation (its caller reduces the block), else the private words buffer. The collective of a
  // speculative iteration that was aborted still runs (RCCL cannot skip it; every rank aborts alike), and
  // G of a queued iteration can be the buffer of the live gradient: only abort-aware kernels (the tail,
  // finalize) may write G from the reduced words.
  float *Gl = G;
  if (reduced && !local) {
    words_.ensure(size_t(cdiv((long long)nparams_ + 2, 4) * 4));
    Gl = words_.get();
  }
  if (empty) zero_fill(s, (long long)nparams_ + 2, Gl, ctx_->abort);
  // [dW ; db] = [A_in | 1]^T dZ  (layer.cuh:81-84 + sum_rows_kernel kernels.cuh:144-153)
  auto dw_desc = [&](int l) {
    const Layer &L = layers_[l];
    GemmDesc d;
    d.M = L.in + 1;
    d.N = L.out;
    d.K = int(B);
    d.A = (l == 0) ? X : A_[l - 1].get();
    d.lda = L.in;
    d.a_kc = false;
    d.a_idx = (l == 0) ? idx : nullptr;
    d.a_mvalid = L.in;
    d.a_ones = L.in;
    d.B = D_[l].get();
    d.ldb = L.out;
    d.b_kc = false;
    d.epi = EPI_STORE;
    d.ldc = L.out;
    d.splits = L.splits;
    d.k_chunk = L.k_chunk;
    d.abort = ctx_->abort;
    d.tile = L.dtile;
    const bool folded = fold >= 0 && l == nl - 2; // rows >= fold_c0_ come from the EPI_HEAD epilogue
    if (folded) {
      d.M = fold_c0_;
      d.a_mvalid = fold_c0_;
      d.a_ones = -1;
    }
    if (l + 1 < nl && side_reduced(l + 1, fused, nloss)) {
      // finish layer l+1's [dW ; db] slabs (the fused head's, or many split-K slabs) in side blocks
      // of this launch, while its GEMM runs; the head's slab starts with this layer's folded rows
      const Layer &N1 = layers_[l + 1];
      const bool head = fused && l + 1 == nl - 1;
      // the segment exactly as layer l+1's launch wrote its slabs: a folded layer's GEMM has fold_c0_
      // rows (its remaining rows live in the head's segment)
      const long long n1rows = (fold >= 0 && l + 1 == nl - 2) ? fold_c0_ : N1.in + 1;
      const long long nseg = head ? (long long)(N1.in + 1) * N1.out + nfold : n1rows * N1.out;
      d.side_slab = head ? head_slab_.get() : slab_.get() + N1.slab_off;
      d.side_splits = head ? nloss : N1.splits;
      d.side_stride = nseg;
      d.side_count = nseg;
      d.side_dst = Gl + N1.off - (head ? nfold : 0);
    }
    if (L.splits > 1) {
      d.C = slab_.get() + L.slab_off;
      d.slab_stride = (long long)d.M * L.out;
    } else {
      d.C = Gl + L.off;
    }
    return d;
  };
  // dX = dZ W^T .* act'(A_prev)   (layer.cuh:89-103 fused with activation_deriv of layer l-1)
  auto dx_desc = [&](int l) {
    const Layer &L = layers_[l];
    const Layer &P0 = layers_[l - 1];
    GemmDesc x;
    x.M = int(B);
    x.N = L.in;
    x.K = L.out;
    x.A = D_[l].get();
    x.lda = L.out;
    x.a_kc = true;
    x.B = P + L.off; // B[n=i][k=o] = W[i][o]
    x.ldb = L.out;
    x.b_kc = true;
    x.C = D_[l - 1].get();
    x.ldc = L.in;
    x.epi = EPI_DX;
    x.aux = A_[l - 1].get();
    x.ldaux = L.in;
    x.aux_act = P0.act;
    x.abort = ctx_->abort;
    x.tile = dx_tile(B, L.in);
    return x;
  };
  // A speculative first trial (tf->early: single rank, lambda = 0) takes its Armijo test in the first backward
  // launch (EarlyLs, gemm.hip gemm_early_exit): on a failure that launch, the rest of the backward and the tail
  // exit at entry, and the host finishes the search as after the tail's own rejection (LBF_NO_EARLY=1: off).
  const bool early_on = env_int("LBF_NO_EARLY", 0) == 0; // read per evaluation: tests switch it in-process
  EarlyLs early;
  const EarlyLs *early_p = nullptr;
  if (early_on && tf && tf->early && !reduced && lambda == 0.0 && nloss > 0) {
    early.sse_part = loss_part_.get();
    early.nsse = nloss;
    early.inv_scale = inv_scale;
    early.ls = tf->ls;
    early_p = &early;
  }
  auto first_launch = [&](GemmDesc d) { // the early test rides on the first launch only
    d.early = early_p;
    early_p = nullptr;
    return d;
  };
  for (int l = lstart; l >= 0; --l) {
    if (l == 1 && group_dw_ && !side_reduced(1, fused, nloss)) {
      // the last two dW GEMMs in one launch (S-LBFGS minibatches: two small split-K grids that each
      // leave most of the chip idle at its tail): dX of layer 1 first, since dW of layer 0 reads it
      const GemmDesc d1 = dw_desc(1), d0 = dw_desc(0);
      if (gemm_group_ok(d1, d0)) {
        {
          ProfScope ps(ctx_, PK_DX, 1, double(B));
          gemm(s, first_launch(dx_desc(1)));
        }
        ProfScope ps(ctx_, PK_DW, 1, double(B));
        gemm_group(s, first_launch(d1), d0);
        break;
      }
    }
    {
      ProfScope ps(ctx_, PK_DW, l, double(B));
      gemm(s, first_launch(dw_desc(l)));
    }
    if (l > 0) {
      ProfScope ps(ctx_, PK_DX, l, double(B));
      gemm(s, first_launch(dx_desc(l)));
    }
  }
  // every layer's partial slabs -> gradient (+ dots and the status block on a single rank)
  RedAllArgs ra;
  ra.G = Gl;
  ra.w = P;
  ra.p = pdir;
  ra.lambda = lambda;
  // scal == nullptr (S-LBFGS minibatch / Hessian-batch gradients, whose status nobody reads): the
  // gradient only, no dot partials and no finishing launch. The reduced route (data parallel, an empty
  // share, or a packed local evaluation) finishes the gradient from [G | hi | lo] after the all-reduce.
  ra.dots = (reduced || !scal) ? 0 : 1;
  ra.l2 = reduced ? 0 : 1;
  ra.partials = dots_part_.get();
  ra.colpart = colpart_.get();
  ra.sse_part = loss_part_.get();
  ra.nsse = empty ? 0 : nloss;
  ra.inv_scale = inv_scale;
  ra.scal = scal;
  ra.abort = ctx_->abort;
  for (int l = 0; l < nl; ++l) {
    const Layer &L = layers_[l];
    RedSeg &g = ra.seg[l];
    g.count = (long long)(L.in + 1) * L.out;
    g.goff = (long long)L.off;
    if (fold >= 0 && l == nl - 2) g.count = (long long)fold_c0_ * L.out; // the rest is the head's segment
    if (fold >= 0 && l == nl - 1) {
      g.count += nfold;
      g.goff -= nfold;
    }
    g.stride = g.count;
    if (empty || side_reduced(l, fused, nloss)) {
      // zero-filled (an empty share) / finished by the side blocks of the next dW launch: as written
    } else if (L.splits > 1) {
      g.slab = slab_.get() + L.slab_off;
      g.splits = L.splits;
    }
    const int ncols = int(cdiv(g.count, RA_COLS));
    // many slabs over few columns (the head's): split ranges over blocks, finished by one block
    if (g.splits > 2 * RA_SPLITS_PER_PART && ra.nfin + ncols <= RA_MAXFIN)
      g.parts = int(std::min<long long>(RA_MAXPART, cdiv(g.splits, RA_SPLITS_PER_PART)));
    g.wg0 = ra.nwg;
    g.cg0 = ra.ncg;
    if (g.parts > 1) {
      g.fin0 = ra.nfin;
      ra.nfin += ncols;
    }
    // few splits: RA_GPB groups per block (a block's loads are few, blocks the cost); many: one group per
    // block, so the splits' loads spread over four times the blocks (the 20-slab shard gradient)
    g.gpb = g.parts == 1 && g.splits <= 8 ? RA_GPB : 1;
    ra.nwg += g.parts > 1 ? ncols * g.parts : int(cdiv(ncols, g.gpb));
    ra.ncg += ncols;
  }
  ra.nseg = nl;
  // this rank's gradient (no lambda w) and its SSE as an fp32 (hi, lo) pair: [G | hi | lo]
  auto local_words = [&]() {
    if (empty) return; // zero-filled at entry
    RedAllArgs loc = ra;
    loc.dots = 0;
    loc.sse_part = loss_part_.get(); // the SSE words in an extra block of the same launch
    loc.nsse = nloss;
    loc.sse_hilo = Gl + nparams_;
    ProfScope ps(ctx_, PK_SLAB, 0);
    reduce_all(s, loc);
  };
  bool tail_ok = tf != nullptr && !local;
  for (int l = 0; l < nl && tail_ok; ++l) tail_ok = ra.seg[l].parts == 1;
  if (tail_ok) {
    // fused optimizer tail (tail.hip); data parallel: local reduce -> all-reduce -> tail over G
    TailArgs ta;
    const float *hilo = nullptr;
    if (reduced) {
      local_words();
      if (ctx_->dp()) {
        ProfScope ps(ctx_, PK_ALLREDUCE);
        ctx_->allreduce(Gl, nparams_ + 2);
      }
      hilo = hilo_in ? hilo_in : Gl + nparams_;
      for (int l = 0; l < nl; ++l) {
        ra.seg[l].slab = nullptr;
        ra.seg[l].splits = 0;
      }
    }
    ta.ra = ra;
    ta.ra.G = G;
    ta.g_src = Gl != G ? Gl : nullptr;
    ta.hilo = hilo;
    ta.h = tf->h;
    ta.h.abort = ctx_->abort;
    ta.has_pair = tf->has_pair;
    ta.x_prev = tf->x_prev;
    ta.g_prev = tf->g_prev;
    ta.policy = tf->policy;
    ta.iter_next = tf->iter_next;
    ta.ls = tf->ls;
    ta.nc = 6 * tf->h.m + 8;
    ta.nb = 0; // one TAIL_COLS column group per block: latency-bound work wants every CU busy
    for (int l = 0; l < nl; ++l) {
      ta.tcg0[l] = ta.nb;
      ta.nb += int(cdiv(ra.seg[l].count, (long long)TAIL_COLS));
    }
    trows_.ensure(size_t(ta.nb) * ta.nc);
    tdots_.ensure(size_t(ta.nc));
    ta.rows = trows_.get();
    ta.dots = tdots_.get();
    if (!cols_done_.get()) {
      cols_done_.resize(1);
      LBF_HIP(hipMemsetAsync(cols_done_.get(), 0, sizeof(unsigned), s));
    }
    ta.cols_done = cols_done_.get();
    {
      ProfScope ps(ctx_, PK_GRAM, 1);
      tail_reduce(s, ta); // + the fin in the last tail_cols block (cols_done)
    }
    ++evals_;
    rows_ += B;
    return;
  }
  ++evals_;
  rows_ += B;
  if (!reduced) {
    if (defer && !ra.dots) {
      bool one_pass = true;
      for (int l = 0; l < nl; ++l) one_pass = one_pass && ra.seg[l].parts == 1;
      if (one_pass) { // the consumer finishes the gradient from the slabs (Mlp::loss_grad_deferred)
        *defer = ra;
        return;
      }
    }
    ProfScope ps(ctx_, PK_SLAB, 0);
    reduce_all(s, ra);
    return;
  }
  local_words();
  if (local) return; // the caller all-reduces [G | hi | lo] (with other blocks) and calls finish_reduced
  if (ctx_->dp()) {
    ProfScope ps(ctx_, PK_ALLREDUCE);
    ctx_->allreduce(Gl, nparams_ + 2); // one RCCL all-reduce of [grad | sse_hi | sse_lo]
  }
  finish_reduced(P, G, inv_scale, lambda, pdir, scal, hilo_in, Gl != G ? Gl : nullptr);
}

void Mlp::batch_grads(const float *P, const float *X, const float *Y, int nmb, long long cnt, double inv_scale,
                      double lambda, float *G, long long ldg, bool local) {
  LBF_REQUIRE(nmb > 0 && cnt > 0 && cnt % 32 == 0, "batch_grads: minibatches of a multiple of 32 rows");
  LBF_REQUIRE(ldg >= (long long)nparams_, "batch_grads: gradient stride below the parameter count");
  hipStream_t s = ctx_->stream;
  const int nl = int(layers_.size());
  const Layer &Lo = layers_[nl - 1];
  const long long R = (long long)nmb * cnt;
  ensure(R);
  // forward over every row (no fused head: its [dW ; db] partials are per 64-row tile, not per minibatch)
  forward(P, X, nullptr, R, nl);
  {
    ProfScope ps(ctx_, PK_LOSS);
    loss_diff(s, A_[nl - 1].get(), Lo.out, Y, Lo.out, nullptr, R, Lo.out, Lo.act, inv_scale, D_[nl - 1].get(),
              Lo.out, loss_part_.get());
  }
  for (int l = nl - 1; l >= 0; --l) {
    const Layer &L = layers_[l];
    GemmDesc d; // [dW ; db] of minibatch t = split t of [A_in | 1]^T dZ
    d.M = L.in + 1;
    d.N = L.out;
    d.K = int(R);
    d.A = (l == 0) ? X : A_[l - 1].get();
    d.lda = L.in;
    d.a_kc = false;
    d.a_mvalid = L.in;
    d.a_ones = L.in;
    d.B = D_[l].get();
    d.ldb = L.out;
    d.b_kc = false;
    d.epi = EPI_STORE;
    d.ldc = L.out;
    d.splits = nmb;
    d.k_chunk = int(cnt);
    d.C = G + L.off;
    d.slab_stride = ldg;
    d.abort = ctx_->abort;
    d.tile = TILE_64x64;
    {
      ProfScope ps(ctx_, PK_DW, l, double(R));
      gemm(s, d);
    }
    if (l > 0) {
      const Layer &P0 = layers_[l - 1];
      GemmDesc x; // dX = dZ W^T .* act'(A_prev), as backward_phase
      x.M = int(R);
      x.N = L.in;
      x.K = L.out;
      x.A = D_[l].get();
      x.lda = L.out;
      x.a_kc = true;
      x.B = P + L.off;
      x.ldb = L.out;
      x.b_kc = true;
      x.C = D_[l - 1].get();
      x.ldc = L.in;
      x.epi = EPI_DX;
      x.aux = A_[l - 1].get();
      x.ldaux = L.in;
      x.aux_act = P0.act;
      x.abort = ctx_->abort;
      x.tile = dx_tile(R, L.in);
      ProfScope ps(ctx_, PK_DX, l, double(R));
      gemm(s, x);
    }
  }
  if (!local) {
    ProfScope ps(ctx_, PK_FINAL, 0);
    add_l2_rows(s, (long long)nparams_, nmb, ldg, G, P, lambda);
  }
  evals_ += nmb;
  rows_ += R;
}

// The gradient and status of an all-reduced [G | hi | lo] block: G += lambda w, the dots of the status
// block, and the loss from the (hi, lo) words (or from hilo_in: a loss-only trial's reduced words).
void Mlp::finish_reduced(const float *P, float *G, double inv_scale, double lambda, const float *pdir, double *scal,
                         const float *hilo_in, const float *g_src) {
  hipStream_t s = ctx_->stream;
  ProfScope ps(ctx_, PK_FINAL, 1);
  const int nd = dots_partials_wg(nparams_);
  dots_part_.ensure(size_t(nd) * 3);
  finalize_grad_dots(s, nparams_, G, P, lambda, pdir, dots_part_.get(), ctx_->abort, g_src);
  if (scal)
    eval_tail(s, dots_part_.get(), nd, loss_part_.get(), 0, hilo_in ? hilo_in : (g_src ? g_src : G) + nparams_,
              inv_scale, lambda, scal, ctx_->abort);
}

// ------------------------------------------------------------------------------------------------
// Exact Hessian-vector product (R-operator; hvp.hip has the derivation). An unfused forward/backward
// of the batch, then the R-forward and R-backward with the same GEMM kernels: every product that
// involves the direction V is one more GEMM whose B operand is V's layer block.
// ------------------------------------------------------------------------------------------------
void Mlp::hvp(const float *P, const float *V, const float *X, const float *Y, const int *idx, long long B,
              double inv_scale, double lambda, float *Hv) {
  LBF_REQUIRE(P && V && Hv && B >= 0 && (B == 0 || (X && Y)), "hvp: bad argument");
  hipStream_t s = ctx_->stream;
  const int nl = int(layers_.size());
  if (B == 0) { // a data-parallel rank with an empty share still joins the all-reduce
    LBF_HIP(hipMemsetAsync(Hv, 0, nparams_ * sizeof(float), s));
    if (ctx_->dp()) ctx_->allreduce(Hv, nparams_);
    if (lambda != 0.0) lincomb(s, (long long)nparams_, Hv, lambda, V, Hv);
    return;
  }
  ensure(B);
  if (B > rcap_) {
    RZ_.clear();
    RA_.clear();
    RD_.clear();
    DL_.clear();
    size_t wmax = 1, segmax = 1;
    for (auto &L : layers_) {
      RZ_.emplace_back(size_t(B) * L.out);
      RA_.emplace_back(size_t(B) * L.out);
      RD_.emplace_back(size_t(B) * L.out);
      DL_.emplace_back(act_has_d2(L.act) ? size_t(B) * L.out : size_t(1));
      // T1_ holds R{A} W_l (B x out) in the R-forward and (dZ W^T) (B x in) in the R-backward
      wmax = std::max(wmax, size_t(std::max(L.in, L.out)));
      segmax = std::max(segmax, size_t(L.in + 1) * L.out);
    }
    T1_.resize(size_t(B) * wmax);
    T2_.resize(size_t(B) * wmax);
    seg_.resize(segmax);
    rcap_ = B;
  }
  // Z = in * W + bias (no activation) for layer l, with the forward's tile / split-K plan
  auto linear_fwd = [&](int l, const float *Wsrc, const float *in, const int *rows, bool with_bias, float *out) {
    const Layer &L = layers_[size_t(l)];
    GemmDesc d = fwd_desc(size_t(l), Wsrc, in, rows, B);
    d.act = ACT_LINEAR;
    if (!with_bias) d.bias = nullptr;
    if (L.fsplits > 1) {
      const float *bias = d.bias;
      d.epi = EPI_STORE;
      d.C = fslab_.get();
      d.splits = L.fsplits;
      d.k_chunk = L.fk_chunk;
      d.slab_stride = B * L.out;
      gemm(s, d);
      fwd_reduce_act(s, fslab_.get(), L.fsplits, B * L.out, int(B), L.out, bias, ACT_LINEAR, out, ctx_->abort);
    } else {
      d.C = out;
      gemm(s, d);
    }
  };
  // [in | ones?]^T dZ for layer l into dst (the dW GEMM's plan: split-K slabs summed in split order)
  auto weight_grad = [&](int l, const float *in, const int *rows, bool ones, const float *dZ, float *dst) {
    const Layer &L = layers_[size_t(l)];
    GemmDesc d;
    d.M = L.in + 1;
    d.N = L.out;
    d.K = int(B);
    d.A = in;
    d.lda = L.in;
    d.a_kc = false;
    d.a_idx = rows;
    d.a_mvalid = L.in;
    d.a_ones = ones ? L.in : -1; // no ones column: the bias row is zero
    d.B = dZ;
    d.ldb = L.out;
    d.b_kc = false;
    d.epi = EPI_STORE;
    d.ldc = L.out;
    d.splits = L.splits;
    d.k_chunk = L.k_chunk;
    d.abort = ctx_->abort;
    d.tile = L.dtile;
    const long long seg = (long long)(L.in + 1) * L.out;
    if (L.splits > 1) {
      d.C = slab_.get() + L.slab_off;
      d.slab_stride = seg;
      gemm(s, d);
      reduce_slabs(s, slab_.get() + L.slab_off, L.splits, seg, seg, dst, ctx_->abort);
    } else {
      d.C = dst;
      gemm(s, d);
    }
  };
  // (dZ W^T) .* act'(aux) for layer l (aux_act linear: the plain product)
  auto back_prod = [&](int l, const float *dZ, const float *Wsrc, int aux_act, float *out) {
    const Layer &L = layers_[size_t(l)];
    GemmDesc x;
    x.M = int(B);
    x.N = L.in;
    x.K = L.out;
    x.A = dZ;
    x.lda = L.out;
    x.a_kc = true;
    x.B = Wsrc + L.off;
    x.ldb = L.out;
    x.b_kc = true;
    x.C = out;
    x.ldc = L.in;
    x.epi = EPI_DX;
    x.aux = A_[size_t(l - 1)].get();
    x.ldaux = L.in;
    x.aux_act = aux_act;
    x.abort = ctx_->abort;
    x.tile = dx_tile(B, L.in);
    gemm(s, x);
  };
  // ---- forward and the plain backward (dZ_l; delta_l where act'' != 0) ----
  forward(P, X, idx, B, nl);
  const Layer &Lo = layers_[size_t(nl - 1)];
  loss_diff(s, A_[size_t(nl - 1)].get(), Lo.out, Y, Lo.out, idx, B, Lo.out, Lo.act, inv_scale,
            D_[size_t(nl - 1)].get(), Lo.out, loss_part_.get());
  for (int l = nl - 1; l >= 1; --l) {
    const int pa = layers_[size_t(l - 1)].act;
    back_prod(l, D_[size_t(l)].get(), P, pa, D_[size_t(l - 1)].get());
    if (act_has_d2(pa)) back_prod(l, D_[size_t(l)].get(), P, ACT_LINEAR, DL_[size_t(l - 1)].get());
  }
  // ---- R-forward ----
  for (int l = 0; l < nl; ++l) {
    const Layer &L = layers_[size_t(l)];
    const long long nz = B * L.out;
    if (l == 0) {
      linear_fwd(0, V, X, idx, true, RZ_[0].get()); // X V_0 + v_0
    } else {
      linear_fwd(l, V, A_[size_t(l - 1)].get(), nullptr, true, RZ_[size_t(l)].get()); // A V_l + v_l
      linear_fwd(l, P, RA_[size_t(l - 1)].get(), nullptr, false, T1_.get());         // R{A} W_l
      lincomb(s, nz, RZ_[size_t(l)].get(), 1.0, T1_.get(), RZ_[size_t(l)].get());
    }
    rop_act(s, nz, A_[size_t(l)].get(), RZ_[size_t(l)].get(), L.act, RA_[size_t(l)].get());
  }
  // ---- R-backward ----
  rop_out(s, B, Lo.out, A_[size_t(nl - 1)].get(), Y, idx, RZ_[size_t(nl - 1)].get(), Lo.act, inv_scale,
          RD_[size_t(nl - 1)].get());
  for (int l = nl - 1; l >= 0; --l) {
    const Layer &L = layers_[size_t(l)];
    float *dst = Hv + L.off;
    const long long seg = (long long)(L.in + 1) * L.out;
    weight_grad(l, l == 0 ? X : A_[size_t(l - 1)].get(), l == 0 ? idx : nullptr, true, RD_[size_t(l)].get(), dst);
    if (l > 0) {
      weight_grad(l, RA_[size_t(l - 1)].get(), nullptr, false, D_[size_t(l)].get(), seg_.get());
      lincomb(s, seg, dst, 1.0, seg_.get(), dst);
      const int pa = layers_[size_t(l - 1)].act;
      back_prod(l, RD_[size_t(l)].get(), P, pa, T1_.get());
      back_prod(l, D_[size_t(l)].get(), V, pa, T2_.get());
      rop_back(s, B * L.in, T1_.get(), T2_.get(), act_has_d2(pa) ? DL_[size_t(l - 1)].get() : nullptr,
               A_[size_t(l - 1)].get(), RZ_[size_t(l - 1)].get(), pa, RD_[size_t(l - 1)].get());
    }
  }
  if (ctx_->dp()) ctx_->allreduce(Hv, nparams_);
  if (lambda != 0.0) lincomb(s, (long long)nparams_, Hv, lambda, V, Hv);
}

// ------------------------------------------------------------------------------------------------
// History
// ------------------------------------------------------------------------------------------------
History::History(Ctx *ctx, int m, long long n) : ctx_(ctx) {
  LBF_REQUIRE(m >= 0 && m <= 128, "history size m must be in [0, 128]");
  const int slots = m + 1;
  // Slot stride n rounded to 4 floats. (Rounded up to 2 MiB, the many-stream reads of the old combine pattern went
  // 5.45 -> 5.88 TB/s in profiles/micro/ring_ld.hip, but the Gram sweep slowed 5.43 -> 5.25 TB/s at n = 10.49M and the
  // chunked combine below needs no help: 65.4-65.7 % against 65.9-66.0 % of HBM at m = 50, profiles/r06/f/.)
  const long long ld = cdiv(n, 4) * 4;
  S_.resize(size_t(slots) * ld);
  Y_.resize(size_t(slots) * ld);
  ist_.resize(IST_ORDER + slots + 4);
  // dstate: rho | SS | SY | YY | gS | gY | coef(2*slots+1) | scal
  const size_t nd = slots + 3 * size_t(slots) * slots + 2 * slots + (2 * slots + 1) + SC_N;
  dstate_.resize(nd);
  part_.resize(size_t(gram_nwg(n)) * gram_ncols(m));
  red_.resize(size_t(kGramFold) * gram_ncols(m));
  v_.m = m;
  v_.slots = slots;
  v_.n = n;
  v_.ld = ld;
  v_.S = S_.get();
  v_.Y = Y_.get();
  v_.ist = ist_.get();
  double *p = dstate_.get();
  v_.rho = p;
  p += slots;
  v_.SS = p;
  p += size_t(slots) * slots;
  v_.SY = p;
  p += size_t(slots) * slots;
  v_.YY = p;
  p += size_t(slots) * slots;
  v_.gS = p;
  p += slots;
  v_.gY = p;
  p += slots;
  v_.coef = p;
  p += 2 * slots + 1;
  v_.scal = p;
  LBF_HIP(hipMemsetAsync(ist_.get(), 0, ist_.size() * sizeof(int), ctx_->stream));
  LBF_HIP(hipMemsetAsync(dstate_.get(), 0, dstate_.size() * sizeof(double), ctx_->stream));
  // the ring vectors are only ever read for live slots, but keep them defined
  LBF_HIP(hipMemsetAsync(S_.get(), 0, S_.size() * sizeof(float), ctx_->stream));
  LBF_HIP(hipMemsetAsync(Y_.get(), 0, Y_.size() * sizeof(float), ctx_->stream));
  dir_on_ = dir_supported(m, n);
  if (dir_on_) {
    const int nb = int(cdiv(n, dir_cols_per_block(m, n)));
    drows_.resize(size_t(dir_ncols(m)) * size_t(nb));
    ddots_.resize(size_t(dir_ncols(m)));
    dkmat_.resize(size_t(DIR_KMAT_N));
    LBF_HIP(hipMemsetAsync(dkmat_.get(), 0, dkmat_.size() * sizeof(double), ctx_->stream));
    dcount_.resize(1);
    LBF_HIP(hipMemsetAsync(dcount_.get(), 0, sizeof(unsigned), ctx_->stream));
  }
  // Column sums + last-block step (gram_fin) for short histories; for m > 20 the fold_rows + hist_step route, which
  // measured faster there (two-loop at n = 10.49M: m = 10 58.0 against 57.5 %, m = 50 67.7 against 68.1 %,
  // profiles/r06/j/). LBF_GRAM_FIN=1 / 0 forces either route (tests compare them).
  const int gf = env_int("LBF_GRAM_FIN", -1);
  gfin_on_ = gram_fin_supported(m) && (gf == 1 || (gf < 0 && m <= 20));
  if (gfin_on_) {
    gdots_.resize(size_t(gram_ncols(m)));
    gcount_.resize(1);
    LBF_HIP(hipMemsetAsync(gcount_.get(), 0, sizeof(unsigned), ctx_->stream));
  }
}

void History::reset() { hist_reset(ctx_->stream, v_); }

bool History::update_impl(const GramArgs &g0, int want_dir, int iter, double dsign, const RedAllArgs *gred,
                          const CombineArgs *cmb) {
  GramArgs g = g0;
  g.h = v_;
  g.h.abort = ctx_->abort;
  hipStream_t s = ctx_->stream;
  auto al16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  const bool aligned = al16(g.sa) && al16(g.sb) && al16(g.ya) && al16(g.yb) && al16(g.ga) && al16(g.gb) &&
                       al16(g.gc) && al16(g.g_out); // 16-B lanes in dir_sweep (null pointers pass)
  const bool defer = gred && gred->nseg > 0;
  const bool dir = dir_on_ && aligned && g.policy == POL_SLBFGS && (want_dir == 0 || want_dir == 1);
  // the sweep reads a lane's four columns of a segment's slabs as one 16-B load per split
  bool quads = true;
  for (int i = 0; defer && i < gred->nseg; ++i) {
    const RedSeg &S = gred->seg[i];
    quads = quads && S.goff % 4 == 0 && S.parts == 1 &&
            (S.splits == 0 || (S.count % 4 == 0 && S.stride % 4 == 0 && al16(S.slab)));
  }
  const bool in_sweep = defer && dir && quads && g.has_g && !g.has_pair && gred->G == g.ga;
  if (defer && !in_sweep) { // only the fused sweep finishes deferred slabs
    ProfScope ps(ctx_, PK_SLAB, 0);
    reduce_all(s, *gred);
  }
  if (dir) {
    // S-LBFGS: sweep + column sums whose last block runs the step (dir.hip), two launches instead of
    // gram -> fold -> hist_step
    DirArgs d;
    d.g = g;
    if (in_sweep) { // g.ga finished inside the sweep from its split-K slabs
      d.gred = *gred;
      d.gred_on = 1;
    }
    d.want_dir = want_dir;
    d.iter = iter;
    d.dsign = dsign;
    d.rows = drows_.get();
    d.dots = ddots_.get();
    d.nb = int(cdiv(v_.n, dir_cols_per_block(v_.m, v_.n)));
    d.cols_done = dcount_.get();
    d.kmat = dkmat_.get();
    {
      ProfScope ps(ctx_, PK_GRAM);
      dir_sweep(s, d);
    }
    if (cmb && dir_combine_supported(d, *cmb)) {
      // direction-only step: column sums, then the coefficients computed in every block of the combine
      ProfScope ps(ctx_, PK_COMBINE);
      dir_cols_combine(s, d, *cmb);
      return true;
    }
    ProfScope ps(ctx_, PK_COEF);
    dir_fin(s, d);
    return false;
  }
  if (gfin_on_ && (want_dir == 0 || want_dir == 1)) {
    // Gram sweep with transposed partials, then one block per column whose last arrival runs the step:
    // two launches instead of gram -> fold_rows -> hist_step
    DirArgs d;
    d.g = g;
    d.want_dir = want_dir;
    d.iter = iter;
    d.dsign = dsign;
    d.rows = part_.get();
    d.dots = gdots_.get();
    d.nb = gram_nwg(v_.n);
    d.cols_done = gcount_.get();
    // the sweep's partial rows stored row-major (one contiguous row per workgroup): its transposed stores, three
    // scattered doubles per history vector per workgroup, cost the sweep 13 % in profiles/micro/ring_ld.hip
    // (gram3_tr1 / tr0) and 5.44 against 5.59 TB/s in the engine (LBF_GRAM_FIN=1 / 0, profiles/r06/i/)
    d.row_major = 1;
    {
      ProfScope ps(ctx_, PK_GRAM);
      gram_update(s, g, part_.get(), 0);
    }
    ProfScope ps(ctx_, PK_COEF);
    gram_fin(s, d);
    return false;
  }
  {
    ProfScope ps(ctx_, PK_GRAM);
    gram_update(s, g, part_.get());
  }
  CoefArgs c;
  c.h = v_;
  c.h.abort = ctx_->abort;
  c.partials = part_.get();
  c.nwg = gram_nwg(v_.n);
  // tall partial table (large n, or a large m whose rows fill the step's staging area): fold it on many
  // blocks first, so the single-workgroup history step reads one staging round of rows, not thousands
  const int fold_to = std::min(kGramFold, hist_stage_rows(v_.m));
  if (c.nwg > 2 * fold_to) {
    ProfScope pf(ctx_, PK_COEF);
    c.nwg = fold_rows(s, part_.get(), c.nwg, gram_ncols(v_.m), fold_to, red_.get());
    c.partials = red_.get();
  }
  c.has_pair = g.has_pair;
  c.has_g = g.has_g;
  c.reset = g.reset;
  c.policy = g.policy;
  c.want_dir = want_dir;
  c.iter = iter;
  c.dsign = dsign;
  ProfScope ps(ctx_, PK_COEF);
  hist_coef(s, c);
  return false;
}

bool History::update_combine(const GramArgs &g0, int iter, double dsign, const float *x_in, float *x_out,
                             float *x_out2, double alpha, const RedAllArgs *gred) {
  // (the combine inside the column-sum launch measured slower: its waiting blocks slowed the column sums
  // and the one-block step, profiles/r03b/README.md)
  CombineArgs c;
  c.h = v_;
  c.h.abort = ctx_->abort;
  c.g = g0.g_out;
  c.x_in = x_in;
  c.x_out = x_out;
  c.x_out2 = x_out2;
  c.alpha_from_state = 0;
  c.alpha = alpha;
  if (update_impl(g0, 1, iter, dsign, gred, &c)) return true; // dir_cols_combine ran (coefficients from K)
  combine(g0.g_out, nullptr, x_in, x_out, x_out2, false, alpha);
  return false;
}

void History::combine(const float *g, float *dir, const float *x_in, float *x_out, float *x_out2,
                      bool alpha_from_state, double alpha) {
  CombineArgs a;
  a.h = v_;
  a.h.abort = ctx_->abort;
  a.g = g;
  a.dir = dir;
  a.x_in = x_in;
  a.x_out = x_out;
  a.x_out2 = x_out2;
  a.alpha_from_state = alpha_from_state ? 1 : 0;
  a.alpha = alpha;
  ProfScope ps(ctx_, PK_COMBINE);
  hist_combine(ctx_->stream, a);
}

} // namespace lbf
