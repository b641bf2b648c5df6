// include/lbfgs_amd/hip_backend.hpp — header-only C++ mirror of the reference's unified API for a
// HipBackend, written purely against the C ABI (include/lbfgs_amd.h; link -llbfgs_amd). Plain C++17:
// no HIP, Eigen or torch headers are needed to compile it.
//
// Reference interfaces mirrored (paths relative to SignorB/lbfgs-FFNN):
//   hip_mlp::HipMinimizerBase / HipLBFGS     <- cuda_mlp::CudaMinimizerBase / CudaLBFGS
//                                               (src/cuda/minimizer_base.cuh:12-67, src/cuda/lbfgs.cuh:25-266)
//   hip_mlp::HipNetwork                      <- cuda_mlp::CudaNetwork (src/cuda/network.cuh:21-158)
//   hip_mlp::DeviceBuffer<T>                 <- cuda_mlp::DeviceBuffer (src/cuda/device_buffer.cuh:7-96)
//   hip_mlp::HipHandle                       <- cuda_mlp::CublasHandle (src/cuda/cublas_handle.cuh:22-39)
//   IterationRecorder<HipBackend>            <- IterationRecorder<CudaBackend> (src/iteration_recorder.hpp:98-146)
//   NetworkWrapper<HipBackend>               <- NetworkWrapper<CudaBackend> (src/network_wrapper.hpp:92-110)
//   UnifiedOptimizer<HipBackend>, UnifiedLBFGS_HIP, UnifiedSLBFGS_HIP
//                                            <- UnifiedOptimizer<CudaBackend>, UnifiedLBFGS_CUDA
//                                               (src/unified_optimization.hpp:420-592; S-LBFGS is CPU-only there)
//   UnifiedLauncher<HipBackend>              <- UnifiedLauncher<CudaBackend> (src/unified_launcher.hpp:83-205)
// Standalone, the header also defines UnifiedConfig / UnifiedDataset (same fields as
// src/unified_optimization.hpp:26-59) with a column-major HostMatrix in place of Eigen::MatrixXd.
// Dropped in next to the reference headers, define LBF_USE_REFERENCE_UNIFIED_TYPES first so the
// reference's own UnifiedConfig / UnifiedDataset (Eigen) are used.
#pragma once

#include "../lbfgs_amd.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

/// @brief Backend tag for the MI355X (HIP) implementation.
struct HipBackend {};

template <typename Backend> class IterationRecorder;
template <typename Backend> class NetworkWrapper;
template <typename Backend> class UnifiedOptimizer;
template <typename Backend> class UnifiedLauncher;

namespace hip_mlp {

using HipScalar = float; // fp32 like CudaScalar (src/cuda/common.cuh:11)

/// Abort with a message on any engine error, like cuda_check (src/cuda/common.cuh:18-23).
inline void hip_check(int rc, const char *msg) {
  if (rc != LBF_OK) {
    std::cerr << "HIP engine error: " << msg << " -> " << lbf_last_error() << std::endl;
    std::abort();
  }
}

/// Activation tags (the reference uses cpu_mlp::{Linear,ReLU,Sigmoid,Tanh}, src/layer.hpp:16-47).
struct Linear { static constexpr int id = LBF_ACT_LINEAR; };
struct Tanh { static constexpr int id = LBF_ACT_TANH; };
struct ReLU { static constexpr int id = LBF_ACT_RELU; };
struct Sigmoid { static constexpr int id = LBF_ACT_SIGMOID; };

/// Maps an activation tag type to the engine's id; specialise for other tag types.
template <typename T> struct ActivationId { static constexpr int value = T::id; };

/// Owns the device context (stream, optional RCCL communicator): CublasHandle analogue.
class HipHandle {
public:
  explicit HipHandle(int device = 0) { hip_check(lbf_ctx_create(device, nullptr, &h_), "lbf_ctx_create"); }
  ~HipHandle() { lbf_ctx_destroy(h_); }
  HipHandle(const HipHandle &) = delete;
  HipHandle &operator=(const HipHandle &) = delete;
  lbf_ctx *get() const { return h_; }
  void sync() const { hip_check(lbf_ctx_sync(h_), "lbf_ctx_sync"); }
  /// Data parallelism: call on every rank with the id from rank 0's unique_id().
  static std::vector<char> unique_id() {
    std::vector<char> id(128);
    hip_check(lbf_comm_unique_id(id.data()), "lbf_comm_unique_id");
    return id;
  }
  void comm_init(int nranks, int rank, const std::vector<char> &id) {
    hip_check(lbf_comm_init(h_, nranks, rank, id.data()), "lbf_comm_init");
  }

private:
  lbf_ctx *h_ = nullptr;
};

/// RAII device buffer (src/cuda/device_buffer.cuh:7-96).
template <typename T> class DeviceBuffer {
public:
  explicit DeviceBuffer(HipHandle &h, size_t n = 0) : h_(&h) { resize(n); }
  ~DeviceBuffer() { release(); }
  DeviceBuffer(const DeviceBuffer &) = delete;
  DeviceBuffer &operator=(const DeviceBuffer &) = delete;
  void resize(size_t n) {
    if (n == n_) return;
    release();
    if (n) {
      void *p = nullptr;
      hip_check(lbf_device_alloc(h_->get(), n * sizeof(T), &p), "lbf_device_alloc");
      p_ = static_cast<T *>(p);
    }
    n_ = n;
  }
  T *data() { return p_; }
  const T *data() const { return p_; }
  size_t size() const { return n_; }
  void copy_from_host(const T *src, size_t n) {
    hip_check(lbf_memcpy(h_->get(), p_, src, n * sizeof(T), 0), "copy_from_host");
  }
  void copy_to_host(T *dst, size_t n) const {
    hip_check(lbf_memcpy(h_->get(), dst, p_, n * sizeof(T), 1), "copy_to_host");
  }

private:
  void release() {
    if (p_) lbf_device_free(h_->get(), p_);
    p_ = nullptr;
    n_ = 0;
  }
  HipHandle *h_;
  T *p_ = nullptr;
  size_t n_ = 0;
};

/// Dense MLP on the device (CudaNetwork, src/cuda/network.cuh:21-158).
class HipNetwork {
public:
  explicit HipNetwork(HipHandle &h) : h_(h), params_(h), grads_(h) {}
  ~HipNetwork() {
    if (net_) lbf_mlp_destroy(net_);
  }
  void addLayer(int in, int out, int act) {
    if (dims_.empty()) dims_.push_back(in);
    dims_.push_back(out);
    acts_.push_back(act);
  }
  /// init_mode LBF_INIT_CUDA reproduces network.cuh:36-59; LBF_INIT_CPU reproduces network.hpp:45-71.
  void bindParams(unsigned seed = 123, int init_mode = LBF_INIT_CUDA) {
    if (!net_) {
      hip_check(lbf_mlp_create(h_.get(), int(acts_.size()), dims_.data(), acts_.data(), &net_), "lbf_mlp_create");
      params_.resize(size_t(lbf_mlp_param_count(net_)));
      grads_.resize(params_.size());
    }
    hip_check(lbf_mlp_init_params(net_, seed, init_mode, params_.data()), "lbf_mlp_init_params");
  }
  size_t params_size() const { return params_.size(); }
  int output_size() const { return dims_.empty() ? 0 : dims_.back(); }
  HipScalar *params_data() { return params_.data(); }
  HipScalar *grads_data() { return grads_.data(); }
  void forward_only(const HipScalar *input, int batch, HipScalar *out) {
    hip_check(lbf_mlp_forward(net_, params_.data(), input, batch, out), "lbf_mlp_forward");
  }
  /// Mean MSE loss and gradient into grads_data() (network.cuh:97-119).
  HipScalar compute_loss_and_grad(const HipScalar *input, const HipScalar *target, int batch) {
    double loss = 0.0;
    hip_check(lbf_mlp_loss_grad(net_, params_.data(), grads_.data(), input, target, nullptr, batch, 1.0 / batch, 0.0,
                                &loss),
              "lbf_mlp_loss_grad");
    return HipScalar(loss);
  }
  lbf_mlp *raw() const { return net_; }
  HipHandle &handle() { return h_; }
  const std::vector<int> &dims() const { return dims_; }

private:
  HipHandle &h_;
  lbf_mlp *net_ = nullptr;
  std::vector<int> dims_, acts_;
  DeviceBuffer<HipScalar> params_, grads_;
};

/// Abstract minimizer (CudaMinimizerBase, src/cuda/minimizer_base.cuh:12-67).
class HipMinimizerBase {
public:
  using LossGradFun = std::function<HipScalar(const HipScalar *params, HipScalar *grad, const HipScalar *input,
                                              const HipScalar *target, int batch)>;
  using IterHook = std::function<void(int)>;
  explicit HipMinimizerBase(HipHandle &handle) : handle_(handle) {}
  virtual ~HipMinimizerBase() = default;
  int iterations() const noexcept { return last_iterations_; }
  void setRecorder(::IterationRecorder<HipBackend> *recorder) { recorder_ = recorder; }
  void setMaxIterations(int iters) { max_iters_ = iters; }
  void setTolerance(HipScalar tol) { tol_ = tol; }
  void setLineSearchParams(int max_iters, HipScalar c1, HipScalar rho) {
    max_line_iters_ = (max_iters < 1) ? 1 : max_iters;
    c1_ = c1;
    rho_ = rho;
  }
  virtual void solve(int n, HipScalar *params, const HipScalar *input, const HipScalar *target, int batch,
                     const LossGradFun &loss_grad) = 0;

protected:
  HipHandle &handle_;
  int max_iters_ = 200, max_line_iters_ = 20;
  HipScalar tol_ = 1e-6f, c1_ = 1e-4f, rho_ = 0.5f;
  int last_iterations_ = 0;
  ::IterationRecorder<HipBackend> *recorder_ = nullptr;
};

} // namespace hip_mlp

/// Host-side history of (loss, ||g||, cumulative ms) per iteration (iteration_recorder.hpp:13-146;
/// the device records in bulk instead of three H2D copies per iteration).
template <> class IterationRecorder<HipBackend> {
public:
  void init(int capacity) {
    if (capacity <= 0) return;
    capacity_ = capacity;
    loss_.assign(size_t(capacity), 0.0);
    grad_norm_.assign(size_t(capacity), 0.0);
    time_ms_.assign(size_t(capacity), 0.0);
    size_ = 0;
  }
  void reset() { size_ = 0; }
  void record(int idx, double loss, double grad_norm, double time_ms = 0.0) {
    if (idx < 0 || idx >= capacity_) return;
    loss_[size_t(idx)] = loss;
    grad_norm_[size_t(idx)] = grad_norm;
    time_ms_[size_t(idx)] = time_ms;
    size_ = std::max(size_, idx + 1);
  }
  void copy_to_host(std::vector<double> &l, std::vector<double> &g) const {
    l.assign(loss_.begin(), loss_.begin() + size_);
    g.assign(grad_norm_.begin(), grad_norm_.begin() + size_);
  }
  void copy_to_host(std::vector<double> &l, std::vector<double> &g, std::vector<double> &t) const {
    copy_to_host(l, g);
    t.assign(time_ms_.begin(), time_ms_.begin() + size_);
  }
  int size() const { return size_; }
  // the engine writes its record here (lbf_record views the recorder's arrays)
  lbf_record view() {
    lbf_record r{};
    r.loss = loss_.data();
    r.grad_norm = grad_norm_.data();
    r.time_ms = time_ms_.data();
    r.cap = capacity_;
    r.size = 0;
    return r;
  }
  void set_size(int s) { size_ = s; }

private:
  std::vector<double> loss_, grad_norm_, time_ms_;
  int capacity_ = 0, size_ = 0;
};

namespace hip_mlp {

/// L-BFGS with the reference's CUDA semantics by default (Armijo + interpolation, lbfgs.cuh:39-194);
/// setLineSearch(LBF_LS_WOLFE) selects the CPU semantics (lbfgs.hpp:38-100). Any LossGradFun works:
/// the engine keeps the (s, y) history, two-loop and line search on the device.
class HipLBFGS : public HipMinimizerBase {
public:
  explicit HipLBFGS(HipHandle &handle) : HipMinimizerBase(handle) {}
  void setMemory(size_t m) { m_ = m; }
  void setLineSearch(int ls) { ls_ = ls; }

  void solve(int n, HipScalar *params, const HipScalar *input, const HipScalar *target, int batch,
             const LossGradFun &loss_grad) override {
    if (n <= 0 || params == nullptr) { // lbfgs.cuh:45-48
      last_iterations_ = 0;
      return;
    }
    struct Closure {
      const LossGradFun *f;
      const HipScalar *in, *tg;
      int batch;
    } cl{&loss_grad, input, target, batch};
    auto tramp = [](void *u, const float *p, float *g) -> double {
      auto *c = static_cast<Closure *>(u);
      return double((*c->f)(p, g, c->in, c->tg, c->batch));
    };
    lbf_lbfgs_params prm;
    lbf_lbfgs_default_params(&prm, ls_);
    prm.m = int(m_);
    prm.max_iters = max_iters_;
    prm.tol = tol_;
    if (ls_ == LBF_LS_ARMIJO) {
      prm.max_line_iters = max_line_iters_;
      prm.c1 = c1_;
      prm.rho = rho_;
    }
    lbf_record rec{};
    lbf_record *rp = nullptr;
    if (recorder_) {
      recorder_->reset();
      rec = recorder_->view();
      rp = &rec;
    }
    lbf_solve_info info{};
    hip_check(lbf_lbfgs_solve_fn(handle_.get(), &prm, n, params, tramp, &cl, rp, &info), "lbf_lbfgs_solve_fn");
    if (recorder_) recorder_->set_size(rec.size);
    last_iterations_ = info.iterations;
  }

private:
  size_t m_ = 16; // lbfgs.cuh:264
  int ls_ = LBF_LS_ARMIJO;
};

/// Column-major host matrix with the subset of Eigen::MatrixXd's interface the launcher uses.
class HostMatrix {
public:
  HostMatrix() = default;
  HostMatrix(long rows, long cols) : r_(rows), c_(cols), d_(size_t(rows * cols), 0.0) {}
  long rows() const { return r_; }
  long cols() const { return c_; }
  long size() const { return r_ * c_; }
  double *data() { return d_.data(); }
  const double *data() const { return d_.data(); }
  double &operator()(long i, long j) { return d_[size_t(i + j * r_)]; }
  double operator()(long i, long j) const { return d_[size_t(i + j * r_)]; }

private:
  long r_ = 0, c_ = 0;
  std::vector<double> d_;
};

/// The reference's MNISTLoader (tests/mnist/mnist_loader.hpp:8-100) over lbf_idx_read_*: images as a
/// (rows*cols) x N matrix scaled to [0, 1], labels one-hot 10 x N, column-major like the Eigen version.
struct MNISTLoader {
  static HostMatrix loadImages(const std::string &path, int max_images = 0) {
    long long n = 0;
    int r = 0, c = 0;
    hip_check(lbf_idx_read_images(path.c_str(), max_images, nullptr, &n, &r, &c), "lbf_idx_read_images");
    std::vector<float> buf(size_t(n) * size_t(r) * size_t(c));
    hip_check(lbf_idx_read_images(path.c_str(), max_images, buf.data(), &n, &r, &c), "lbf_idx_read_images");
    HostMatrix m(long(r) * c, long(n));
    for (size_t i = 0; i < buf.size(); ++i) m.data()[i] = double(buf[i]);
    return m;
  }
  static HostMatrix loadLabels(const std::string &path, int max_images = 0) {
    long long n = 0;
    hip_check(lbf_idx_read_labels(path.c_str(), max_images, 10, nullptr, &n), "lbf_idx_read_labels");
    std::vector<float> buf(size_t(n) * 10);
    hip_check(lbf_idx_read_labels(path.c_str(), max_images, 10, buf.data(), &n), "lbf_idx_read_labels");
    HostMatrix m(10, long(n));
    for (size_t i = 0; i < buf.size(); ++i) m.data()[i] = double(buf[i]);
    return m;
  }
};

} // namespace hip_mlp

#ifndef LBF_USE_REFERENCE_UNIFIED_TYPES
/// src/unified_optimization.hpp:26-48
struct UnifiedConfig {
  std::string name = "Experiment";
  int max_iters = 100;
  double tolerance = 1e-4;
  double learning_rate = 0.01;
  double momentum = 0.0;
  double lr_decay = 0.0;
  int lr_decay_rate = 1;
  int batch_size = 128;
  int m_param = 10;
  int L_param = 10;
  int b_H_param = 0;
  int log_interval = 10;
  bool reset_params = true;
  unsigned int seed = 123u;
};
/// src/unified_optimization.hpp:54-59 (HostMatrix instead of Eigen::MatrixXd)
struct UnifiedDataset {
  hip_mlp::HostMatrix train_x, train_y, test_x, test_y;
};
#endif

/// NetworkWrapper<HipBackend> (src/network_wrapper.hpp:92-110).
template <> class NetworkWrapper<HipBackend> {
public:
  using InternalNetwork = hip_mlp::HipNetwork;
  explicit NetworkWrapper(hip_mlp::HipHandle &handle) : network_(handle) {}
  template <int In, int Out, typename Activation> void addLayer() {
    network_.addLayer(In, Out, hip_mlp::ActivationId<Activation>::value);
  }
  void bindParams() { network_.bindParams(); }
  void bindParams(unsigned int seed, int init_mode = LBF_INIT_CUDA) { network_.bindParams(seed, init_mode); }
  InternalNetwork &getInternal() { return network_; }
  const InternalNetwork &getInternal() const { return network_; }
  size_t getParamsSize() const { return network_.params_size(); }

private:
  InternalNetwork network_;
};

inline std::string hip_log_filename(const UnifiedConfig &config) {
  return (config.name.empty() ? std::string("run") : config.name) + "_history.csv";
}

/// CSV schema Iteration,Loss,GradNorm,TimeMs (unified_optimization.hpp:446-465).
inline void write_hip_history_csv(const std::string &filename, const IterationRecorder<HipBackend> &recorder,
                                  int log_interval) {
  if (log_interval <= 0) return;
  std::vector<double> l, g, t;
  recorder.copy_to_host(l, g, t);
  if (l.empty()) return;
  std::ofstream f(filename);
  if (!f.is_open()) return;
  f << "Iteration,Loss,GradNorm,TimeMs\n";
  for (size_t i = 0; i < l.size(); i += size_t(std::max(1, log_interval)))
    f << i << "," << l[i] << "," << g[i] << "," << t[i] << "\n";
}

/// UnifiedOptimizer<HipBackend> (unified_optimization.hpp:420-439): the reference strategy's parameter list,
/// (handle, net, host_data, d_train_x, d_train_y, config), so a strategy written against
/// UnifiedOptimizer<CudaBackend>::optimize overrides this one with its backend types renamed. host_data is the
/// host dataset (for dimensions: n_train = host_data.train_x.cols()); the device data are fp32 rows of In / Out
/// floats per sample (== the reference's column-major matrices).
template <> class UnifiedOptimizer<HipBackend> {
public:
  virtual ~UnifiedOptimizer() = default;
  virtual void optimize(hip_mlp::HipHandle &handle, NetworkWrapper<HipBackend> &net, const UnifiedDataset &host_data,
                        hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &d_train_x,
                        hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &d_train_y, const UnifiedConfig &config) = 0;
  IterationRecorder<HipBackend> recorder;
  int line_search = LBF_LS_ARMIJO; // UnifiedLBFGS_CUDA's semantics unless set to LBF_LS_WOLFE
};

/// UnifiedLBFGS_CUDA counterpart (unified_optimization.hpp:560-592): full-batch L-BFGS of the MLP,
/// all on the device (no per-evaluation callback or D2D gradient copy, cf. :483-491).
class UnifiedLBFGS_HIP : public UnifiedOptimizer<HipBackend> {
public:
  void optimize(hip_mlp::HipHandle &, NetworkWrapper<HipBackend> &net, const UnifiedDataset &host_data,
                hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &dx, hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &dy,
                const UnifiedConfig &c) override {
    const long n_train = long(host_data.train_x.cols());
    auto &nw = net.getInternal();
    lbf_lbfgs_params prm;
    lbf_lbfgs_default_params(&prm, line_search);
    prm.m = c.m_param > 0 ? c.m_param : 10;
    prm.max_iters = c.max_iters;
    prm.tol = c.tolerance;
    recorder.init(c.max_iters);
    lbf_record rec = recorder.view();
    lbf_solve_info info{};
    hip_mlp::hip_check(lbf_lbfgs_solve(nw.raw(), &prm, nw.params_data(), dx.data(), dy.data(), n_train, n_train,
                                       &rec, &info),
                       "lbf_lbfgs_solve");
    recorder.set_size(rec.size);
    write_hip_history_csv(hip_log_filename(c), recorder, c.log_interval);
  }
};

/// S-LBFGS on the device (the reference's is CPU-only: unified_optimization.hpp:306-408, 688-696).
class UnifiedSLBFGS_HIP : public UnifiedOptimizer<HipBackend> {
public:
  void optimize(hip_mlp::HipHandle &, NetworkWrapper<HipBackend> &net, const UnifiedDataset &host_data,
                hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &dx, hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &dy,
                const UnifiedConfig &c) override {
    const long n_train = long(host_data.train_x.cols());
    auto &nw = net.getInternal();
    lbf_slbfgs_params prm;
    lbf_slbfgs_default_params(&prm);
    prm.max_epochs = c.max_iters;
    prm.tol = c.tolerance;
    prm.M = c.m_param;
    prm.L = c.L_param;
    prm.b = c.batch_size;
    prm.b_H = c.b_H_param > 0 ? c.b_H_param : c.batch_size / 2;
    prm.step = c.learning_rate;
    recorder.init(c.max_iters);
    lbf_record rec = recorder.view();
    lbf_solve_info info{};
    hip_mlp::hip_check(lbf_slbfgs_solve(nw.raw(), &prm, nw.params_data(), dx.data(), dy.data(), n_train, &rec, &info),
                       "lbf_slbfgs_solve");
    recorder.set_size(rec.size);
    write_hip_history_csv(hip_log_filename(c), recorder, c.log_interval);
  }
};

/// UnifiedGD_CUDA counterpart (unified_optimization.hpp:518-554): CudaGD with lr, momentum,
/// max_iters, tolerance from the config (gd.cuh:38-106), on the device.
class UnifiedGD_HIP : public UnifiedOptimizer<HipBackend> {
public:
  void optimize(hip_mlp::HipHandle &, NetworkWrapper<HipBackend> &net, const UnifiedDataset &host_data,
                hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &dx, hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &dy,
                const UnifiedConfig &c) override {
    const long n_train = long(host_data.train_x.cols());
    auto &nw = net.getInternal();
    lbf_gd_params prm;
    lbf_gd_default_params(&prm);
    prm.lr = c.learning_rate;
    prm.momentum = c.momentum;
    prm.max_iters = c.max_iters;
    prm.tol = c.tolerance;
    recorder.init(c.max_iters);
    lbf_record rec = recorder.view();
    lbf_solve_info info{};
    hip_mlp::hip_check(lbf_gd_solve(nw.raw(), &prm, nw.params_data(), dx.data(), dy.data(), n_train, n_train, &rec,
                                    &info),
                       "lbf_gd_solve");
    recorder.set_size(rec.size);
    write_hip_history_csv(hip_log_filename(c), recorder, c.log_interval);
  }
};

/// UnifiedSGD_CUDA counterpart (unified_optimization.hpp:595-632): CudaSGD with the config's lr,
/// momentum, batch size, max_iters (epochs) and setLearningRateDecay(lr_decay, lr_decay_rate)
/// (sgd.cuh:50-153; the reference does not pass the tolerance, so CudaSGD keeps its 1e-6).
class UnifiedSGD_HIP : public UnifiedOptimizer<HipBackend> {
public:
  void optimize(hip_mlp::HipHandle &, NetworkWrapper<HipBackend> &net, const UnifiedDataset &host_data,
                hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &dx, hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &dy,
                const UnifiedConfig &c) override {
    const long n_train = long(host_data.train_x.cols());
    auto &nw = net.getInternal();
    lbf_sgd_params prm;
    lbf_sgd_default_params(&prm);
    prm.lr = c.learning_rate;
    prm.momentum = c.momentum;
    prm.batch = c.batch_size;
    prm.max_epochs = c.max_iters;
    prm.decay_rate = c.lr_decay;
    prm.decay_step = c.lr_decay_rate;
    recorder.init(c.max_iters + 1);
    lbf_record rec = recorder.view();
    lbf_solve_info info{};
    hip_mlp::hip_check(lbf_sgd_solve(nw.raw(), &prm, nw.params_data(), dx.data(), dy.data(), n_train, &rec, &info),
                       "lbf_sgd_solve");
    recorder.set_size(rec.size);
    write_hip_history_csv(hip_log_filename(c), recorder, c.log_interval);
  }
};

/// UnifiedLauncher<HipBackend> (src/unified_launcher.hpp:83-205).
template <> class UnifiedLauncher<HipBackend> {
public:
  explicit UnifiedLauncher(int device = 0)
      : handle_(device), net_wrapper_(handle_), d_train_x_(handle_), d_train_y_(handle_), d_test_x_(handle_),
        d_test_y_(handle_) {}
  template <int In, int Out, typename Activation> void addLayer() { net_wrapper_.addLayer<In, Out, Activation>(); }
  void buildNetwork() { net_wrapper_.bindParams(); }

  /// Host -> device upload with the fp64 -> fp32 conversion of unified_launcher.hpp:105-128; like the reference
  /// it keeps a copy of the dataset, which train() hands to the strategy as host_data.
  /// Works with the reference's Eigen-based UnifiedDataset and with the standalone HostMatrix one.
  void setData(const UnifiedDataset &data) {
    dataset_ = data;
    upload(dataset_.train_x, d_train_x_, train_x_);
    upload(dataset_.train_y, d_train_y_, train_y_);
    upload(dataset_.test_x, d_test_x_, test_x_);
    upload(dataset_.test_y, d_test_y_, test_y_);
    n_train_ = long(dataset_.train_x.cols());
    n_test_ = long(dataset_.test_x.cols());
    std::cout << "Data Uploaded to GPU. Train: " << n_train_ << " samples." << std::endl;
  }

  void train(UnifiedOptimizer<HipBackend> &optimizer, const UnifiedConfig &config) {
    std::cout << ">>> Running HIP Experiment: " << config.name << std::endl;
    if (config.reset_params) net_wrapper_.bindParams(config.seed);
    optimizer.optimize(handle_, net_wrapper_, dataset_, d_train_x_, d_train_y_, config);
    last_train_ = evaluate(train_y_, d_train_x_, n_train_, "Training Results");
  }
  void test() { last_test_ = evaluate(test_y_, d_test_x_, n_test_, "Test Results"); }
  NetworkWrapper<HipBackend> &getWrapper() { return net_wrapper_; }
  std::pair<double, double> lastTrain() const { return last_train_; }
  std::pair<double, double> lastTest() const { return last_test_; }

private:
  template <typename M>
  void upload(const M &mat, hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &buf, std::vector<double> &host) {
    const size_t n = size_t(mat.rows() * mat.cols());
    host.assign(mat.data(), mat.data() + n);
    std::vector<hip_mlp::HipScalar> tmp(n);
    for (size_t i = 0; i < n; ++i) tmp[i] = hip_mlp::HipScalar(host[i]);
    buf.resize(n);
    if (n) buf.copy_from_host(tmp.data(), n);
    rows_.push_back(long(mat.rows()));
  }
  /// Accuracy + mean MSE (unified_launcher.hpp:154-199).
  std::pair<double, double> evaluate(const std::vector<double> &y, hip_mlp::DeviceBuffer<hip_mlp::HipScalar> &d_x,
                                     long batch, const char *label) {
    auto &net = net_wrapper_.getInternal();
    const int out_dim = net.output_size();
    if (batch <= 0) return {0.0, 0.0};
    hip_mlp::DeviceBuffer<hip_mlp::HipScalar> d_out(handle_, size_t(batch) * out_dim);
    net.forward_only(d_x.data(), int(batch), d_out.data());
    std::vector<hip_mlp::HipScalar> out(size_t(batch) * out_dim);
    d_out.copy_to_host(out.data(), out.size());
    double mse = 0.0;
    long correct = 0;
    for (long i = 0; i < batch; ++i) {
      int pi = 0, ti = 0;
      double pm = -1e20, tm = -1e20;
      for (int r = 0; r < out_dim; ++r) {
        const size_t idx = size_t(r + i * out_dim);
        const double v = out[idx], t = y[idx];
        mse += (v - t) * (v - t);
        if (v > pm) { pm = v; pi = r; }
        if (t > tm) { tm = t; ti = r; }
      }
      if (pi == ti) ++correct;
    }
    mse /= double(batch * out_dim);
    const double acc = double(correct) / double(batch) * 100.0;
    std::cout << label << ": MSE=" << mse << ", Accuracy=" << acc << "%" << std::endl;
    return {mse, acc};
  }

  hip_mlp::HipHandle handle_;
  NetworkWrapper<HipBackend> net_wrapper_;
  UnifiedDataset dataset_;
  hip_mlp::DeviceBuffer<hip_mlp::HipScalar> d_train_x_, d_train_y_, d_test_x_, d_test_y_;
  std::vector<double> train_x_, train_y_, test_x_, test_y_;
  std::vector<long> rows_;
  long n_train_ = 0, n_test_ = 0;
  std::pair<double, double> last_train_{0, 0}, last_test_{0, 0};
};
