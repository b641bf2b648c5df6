// IDX dataset reader: the reference's MNISTLoader (tests/mnist/
// mnist_loader.hpp:8-100) — big-endian header, magic 2051 (images: count, rows, cols, then one byte
// per pixel, scaled by 1/255) or 2049 (labels: count, then one byte per label, one-hot over 10
// classes, labels >= 10 left all-zero) — into row-major fp32 [N][rows*cols] / [N][classes], the
// layout lbf_mlp_* take (== the reference's column-major feature x sample matrices). Host code: the
// files are read once, before any device work.
#include "host_rng.hpp"
#include "internal.hpp"

#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

namespace lbf {

namespace {

struct File {
  std::FILE *f = nullptr;
  explicit File(const char *path) : f(std::fopen(path, "rb")) {
    if (!f) throw Error(1, std::string("cannot open file: ") + path);
  }
  ~File() {
    if (f) std::fclose(f);
  }
  uint32_t be32() {
    unsigned char b[4];
    if (std::fread(b, 1, 4, f) != 4) throw Error(1, "IDX: truncated header");
    return (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | uint32_t(b[3]);
  }
  void bytes(unsigned char *dst, size_t n) {
    if (std::fread(dst, 1, n, f) != n) throw Error(1, "IDX: truncated data");
  }
};

} // namespace

void idx_read_images(const char *path, long long max_images, float *h_out, long long *count, int *rows, int *cols) {
  LBF_REQUIRE(path && count, "null argument");
  File f(path);
  if (f.be32() != 2051) throw Error(1, "Invalid MNIST image file!"); // mnist_loader.hpp:34
  const uint32_t n = f.be32(), r = f.be32(), c = f.be32();
  long long cnt = n;
  if (max_images > 0 && max_images < cnt) cnt = max_images; // :44-47
  *count = cnt;
  if (rows) *rows = int(r);
  if (cols) *cols = int(c);
  if (!h_out) return;
  const size_t px = size_t(r) * c;
  std::vector<unsigned char> buf(px);
  for (long long i = 0; i < cnt; ++i) {
    f.bytes(buf.data(), px);
    for (size_t j = 0; j < px; ++j) h_out[size_t(i) * px + j] = float(buf[j]) / 255.0f; // :55-57
  }
}

void idx_read_labels(const char *path, long long max_labels, int classes, float *h_onehot, long long *count) {
  LBF_REQUIRE(path && count && classes > 0, "bad argument");
  File f(path);
  if (f.be32() != 2049) throw Error(1, "Invalid MNIST label file!"); // mnist_loader.hpp:76
  const uint32_t n = f.be32();
  long long cnt = n;
  if (max_labels > 0 && max_labels < cnt) cnt = max_labels;
  *count = cnt;
  if (!h_onehot) return;
  std::vector<unsigned char> buf(static_cast<size_t>(cnt));
  f.bytes(buf.data(), buf.size());
  for (long long i = 0; i < cnt; ++i) {
    for (int k = 0; k < classes; ++k) h_onehot[size_t(i) * classes + k] = 0.0f;
    if (buf[size_t(i)] < classes) h_onehot[size_t(i) * classes + buf[size_t(i)]] = 1.0f; // :91-94
  }
}

} // namespace lbf
