// Communicators (see comm.hpp).
#include "comm.hpp"

#include "host_sync.hpp"
#include "kernels.hpp"

#include <rccl/rccl.h>

#include <cstring>
#include <memory>

namespace lbf {

namespace {

struct RcclComm : Comm {
  ncclComm_t c = nullptr;
  ~RcclComm() override {
    if (c) (void)ncclCommDestroy(c);
  }
  void allreduce(float *buf, size_t count, hipStream_t s) override {
    const ncclResult_t r = ncclAllReduce(buf, buf, count, ncclFloat, ncclSum, c, s);
    if (r != ncclSuccess) throw Error(3, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  }
  const char *kind() const override { return "rccl"; }
};

// Shared state of an in-process group: one slot per rank for the current collective, and a reusable
// generation barrier (host_sync.hpp). A rank that never arrives (an error on its thread) turns into an error
// on the others after RankBarrier's timeout instead of a hang.
struct LocalGroup {
  int n = 0, device = 0;
  std::unique_ptr<RankBarrier> bar;
  std::vector<float *> bufs;
  std::vector<size_t> counts;
  std::vector<hipEvent_t> ready, read; // per rank: its buffer is complete / its sum has read every buffer

  ~LocalGroup() {
    for (auto e : ready)
      if (e) (void)hipEventDestroy(e);
    for (auto e : read)
      if (e) (void)hipEventDestroy(e);
  }
  void fail(const std::string &why) {
    bar->break_all();
    throw Error(3, "local rank group: " + why);
  }
  void barrier() {
    try {
      bar->arrive_and_wait();
    } catch (const std::runtime_error &e) {
      throw Error(3, e.what());
    }
  }
};

struct LocalComm : Comm {
  std::shared_ptr<LocalGroup> g;
  int rank = 0;
  DevBuf<float> sum;
  void allreduce(float *buf, size_t count, hipStream_t s) override {
    LocalGroup &G = *g;
    // 1. publish this rank's buffer and the point on its stream where the buffer is complete
    LBF_HIP(hipEventRecord(G.ready[size_t(rank)], s));
    G.bufs[size_t(rank)] = buf;
    G.counts[size_t(rank)] = count;
    G.barrier(); // every rank's event is recorded before anyone waits on it
    RankSrcs src;
    src.n = G.n;
    for (int j = 0; j < G.n; ++j) {
      if (G.counts[size_t(j)] != count) G.fail("ranks called allreduce with different counts");
      src.p[j] = G.bufs[size_t(j)];
    }
    // 2. sum every rank's buffer in rank order into this rank's private sum buffer
    for (int j = 0; j < G.n; ++j)
      if (j != rank) LBF_HIP(hipStreamWaitEvent(s, G.ready[size_t(j)], 0));
    sum.ensure(std::max<size_t>(count, 1));
    sum_ranks(s, src, (long long)count, sum.get());
    LBF_HIP(hipEventRecord(G.read[size_t(rank)], s));
    G.barrier(); // nobody overwrites its buffer before every rank's sum has read it
    // 3. the result into this rank's buffer
    for (int j = 0; j < G.n; ++j)
      if (j != rank) LBF_HIP(hipStreamWaitEvent(s, G.read[size_t(j)], 0));
    if (count) LBF_HIP(hipMemcpyAsync(buf, sum.get(), count * sizeof(float), hipMemcpyDeviceToDevice, s));
  }
  const char *kind() const override { return "local"; }
};

} // namespace

std::unique_ptr<Comm> make_rccl_comm(int nranks, int rank, const char id[128]) {
  std::unique_ptr<RcclComm> c(new RcclComm());
  ncclUniqueId uid;
  static_assert(sizeof(uid) <= 128, "unique id size");
  std::memcpy(&uid, id, sizeof(uid));
  const ncclResult_t r = ncclCommInitRank(&c->c, nranks, uid, rank);
  if (r != ncclSuccess) throw Error(3, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  return c;
}

std::vector<std::unique_ptr<Comm>> make_local_group(int nranks, int device) {
  LBF_REQUIRE(nranks >= 1 && nranks <= kMaxLocalRanks, "local rank group: 1..16 ranks");
  auto g = std::make_shared<LocalGroup>();
  g->n = nranks;
  g->bar.reset(new RankBarrier(nranks));
  g->device = device;
  g->bufs.assign(size_t(nranks), nullptr);
  g->counts.assign(size_t(nranks), 0);
  g->ready.assign(size_t(nranks), nullptr);
  g->read.assign(size_t(nranks), nullptr);
  LBF_HIP(hipSetDevice(device));
  for (int r = 0; r < nranks; ++r) {
    LBF_HIP(hipEventCreateWithFlags(&g->ready[size_t(r)], hipEventDisableTiming));
    LBF_HIP(hipEventCreateWithFlags(&g->read[size_t(r)], hipEventDisableTiming));
  }
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < nranks; ++r) {
    std::unique_ptr<LocalComm> c(new LocalComm());
    c->g = g;
    c->rank = r;
    out.push_back(std::move(c));
  }
  return out;
}

} // namespace lbf
