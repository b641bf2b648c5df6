// Data-parallel communicators of a context (new in this engine: the reference has no collective,
// SURVEY.md §2.1). The evaluation path (runtime.cpp) only needs one operation: an in-place fp32 sum
// all-reduce on the context stream, once per loss+grad evaluation.
//
//   RcclComm   the product route: one process per GPU, ncclAllReduce over xGMI.
//   LocalComm  an in-process group of ranks that share one device, each driven by its own host
//              thread (lbf_comm_init_local). RCCL refuses two ranks on one GPU, so this is how the
//              multi-rank code path (rank > 0 shard offsets, n_global scaling, minibatch slices,
//              replicated line-search decisions over summed data) executes on a one-GPU box. The sum
//              is a device kernel over every rank's buffer in rank order, ordered by HIP events and a
//              host barrier; no data leaves the device.
#pragma once

#include "internal.hpp"

#include <memory>
#include <vector>

namespace lbf {

struct Comm {
  virtual ~Comm() = default;
  // buf[0 .. count) <- sum over the ranks of their buf[0 .. count), enqueued on s
  virtual void allreduce(float *buf, size_t count, hipStream_t s) = 0;
  virtual const char *kind() const = 0;
};

// RCCL communicator from a 128-byte unique id (lbf_comm_unique_id); the context's device is current.
std::unique_ptr<Comm> make_rccl_comm(int nranks, int rank, const char id[128]);
// An in-process group of nranks ranks on `device`: element r belongs to rank r. Every rank must call
// allreduce the same number of times with the same counts, each from its own host thread.
std::vector<std::unique_ptr<Comm>> make_local_group(int nranks, int device);

} // namespace lbf
