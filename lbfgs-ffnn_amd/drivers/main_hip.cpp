// C++ driver through include/lbfgs_amd/hip_backend.hpp, structured like the reference's
// tests/mnist/main-gpu.cpp (UnifiedLauncher<Backend> + UnifiedConfig + train/test) with
// Backend = HipBackend. The MNIST images are absent from the reference snapshot, so it uses the
// synthetic MNIST-shaped data of SURVEY.md §8(d) (lbf_synth_mnist). Plain C++17, links liblbfgs_amd_abi3.so.
//   usage: main_hip [N_train] [max_iters] [mnist_dir]
#include "lbfgs_amd/hip_backend.hpp"

#include <cstdlib>
#include <iostream>

using Backend = HipBackend;

static void fill(long N, hip_mlp::HostMatrix &X, hip_mlp::HostMatrix &Y, unsigned seed) {
  std::vector<float> x(size_t(N) * 784), y(size_t(N) * 10);
  hip_mlp::hip_check(lbf_synth_mnist(N, 784, 10, seed, x.data(), y.data()), "lbf_synth_mnist");
  X = hip_mlp::HostMatrix(784, N); // column-major In x N, one sample per column
  Y = hip_mlp::HostMatrix(10, N);
  for (size_t i = 0; i < x.size(); ++i) X.data()[i] = x[i];
  for (size_t i = 0; i < y.size(); ++i) Y.data()[i] = y[i];
}

int main(int argc, char **argv) {
  const long train_size = argc > 1 ? std::atol(argv[1]) : 60000;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 50;
  UnifiedLauncher<Backend> launcher;
  std::cout << "Building Network..." << std::endl;
  launcher.addLayer<784, 128, hip_mlp::ReLU>();
  launcher.addLayer<128, 10, hip_mlp::Linear>();
  launcher.buildNetwork();

  UnifiedDataset dataset;
  if (argc > 3) { // an MNIST directory, as tests/mnist/main-gpu.cpp reads it (train-/t10k- idx files)
    const std::string dir = argv[3];
    dataset.train_x = hip_mlp::MNISTLoader::loadImages(dir + "/train-images.idx3-ubyte", int(train_size));
    dataset.train_y = hip_mlp::MNISTLoader::loadLabels(dir + "/train-labels.idx1-ubyte", int(train_size));
    dataset.test_x = hip_mlp::MNISTLoader::loadImages(dir + "/t10k-images.idx3-ubyte");
    dataset.test_y = hip_mlp::MNISTLoader::loadLabels(dir + "/t10k-labels.idx1-ubyte");
  } else { // the reference snapshot has no image files: synthetic MNIST-shaped data
    fill(train_size, dataset.train_x, dataset.train_y, 123);
    fill(10000, dataset.test_x, dataset.test_y, 124);
  }
  launcher.setData(dataset);

  {
    UnifiedConfig config;
    config.name = "HIP_LBFGS_m10";
    config.max_iters = iters;
    config.tolerance = 1e-3;
    config.m_param = 10;
    config.log_interval = 1;
    std::cout << "Running LBFGS..." << std::endl;
    UnifiedLBFGS_HIP optimizer; // CUDA-backend semantics (Armijo), as UnifiedLBFGS<CudaBackend>
    launcher.train(optimizer, config);
    launcher.test();
    std::cout << "[RESULT] lbfgs_armijo iters=" << optimizer.recorder.size() << std::endl;
    std::vector<double> l, g;
    optimizer.recorder.copy_to_host(l, g);
    if (l.size() < 2 || !(l.back() < l.front())) {
      std::cerr << "loss did not decrease" << std::endl;
      return 1;
    }
    std::cout << "[RESULT] first_loss=" << l.front() << " last_loss=" << l.back() << std::endl;
  }
  {
    UnifiedConfig config;
    config.name = "HIP_LBFGS_wolfe_m10";
    config.max_iters = iters;
    config.tolerance = 1e-3;
    config.m_param = 10;
    config.log_interval = 1;
    UnifiedLBFGS_HIP optimizer;
    optimizer.line_search = LBF_LS_WOLFE; // CPU-backend semantics
    launcher.train(optimizer, config);
    launcher.test();
  }
  {
    UnifiedConfig config;
    config.name = "HIP_SLBFGS";
    config.max_iters = 2;
    config.tolerance = 1e-4;
    config.learning_rate = 0.02;
    config.batch_size = 256;
    config.m_param = 10;
    config.L_param = 10;
    config.b_H_param = 128;
    config.log_interval = 1;
    UnifiedSLBFGS_HIP optimizer; // GPU S-LBFGS (CPU-only in the reference)
    launcher.train(optimizer, config);
    launcher.test();
  }
  {
    UnifiedConfig config; // tests/mnist/main-gpu.cpp's GD block
    config.name = "HIP_GD";
    config.max_iters = iters;
    config.tolerance = 1e-4;
    config.learning_rate = 0.1;
    config.momentum = 0.9;
    config.log_interval = 1;
    UnifiedGD_HIP optimizer;
    launcher.train(optimizer, config);
    launcher.test();
    std::cout << "[RESULT] gd iters=" << optimizer.recorder.size() << std::endl;
  }
  {
    UnifiedConfig config; // tests/mnist/main-gpu.cpp's SGD block
    config.name = "HIP_SGD";
    config.max_iters = 3;
    config.learning_rate = 0.05;
    config.momentum = 0.9;
    config.batch_size = 256;
    config.lr_decay = 0.5;
    config.lr_decay_rate = 2;
    config.log_interval = 1;
    UnifiedSGD_HIP optimizer;
    launcher.train(optimizer, config);
    launcher.test();
    std::vector<double> l, g;
    optimizer.recorder.copy_to_host(l, g);
    if (l.size() != 4 || !(l.back() < l.front())) {
      std::cerr << "SGD: expected 4 records and a decrease" << std::endl;
      return 1;
    }
    std::cout << "[RESULT] sgd epochs=" << l.size() - 1 << " last_loss=" << l.back() << std::endl;
  }
  std::cout << "[RESULT] ok" << std::endl;
  return 0;
}
