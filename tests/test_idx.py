"""IDX dataset reader (the reference's tests/mnist/mnist_loader.hpp) on the CPU.

Golden fixture: tests/golden/mnist-t10k-labels.idx1-ubyte is the MNIST test-label file the reference
ships (tests/mnist/t10k-labels.idx1-ubyte, data): 10,000 labels with the well-known class counts.
The reference ships no image files, so images are checked on a synthetic IDX file written here.
"""
import os
import struct

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_mnist_test_labels(pkg):
    Y = pkg.load_idx_labels(os.path.join(GOLDEN, "mnist-t10k-labels.idx1-ubyte"))
    assert Y.shape == (10000, 10) and Y.dtype == np.float32
    assert np.all(Y.sum(1) == 1.0)
    assert Y.sum(0).astype(int).tolist() == [980, 1135, 1032, 1010, 982, 892, 958, 1028, 974, 1009]
    Y5 = pkg.load_idx_labels(os.path.join(GOLDEN, "mnist-t10k-labels.idx1-ubyte"), max_labels=5)
    assert np.array_equal(Y5, Y[:5])
    assert np.argmax(Y[:10], 1).tolist() == [7, 2, 1, 0, 4, 1, 4, 9, 5, 9]   # the first MNIST test digits


def test_images_and_errors(pkg, tmp_path):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (7, 5, 3), dtype=np.uint8)
    p = tmp_path / "x.idx3-ubyte"
    p.write_bytes(struct.pack(">IIII", 2051, 7, 5, 3) + img.tobytes())
    X = pkg.load_idx_images(str(p))
    assert X.shape == (7, 15)
    assert np.array_equal(X, img.reshape(7, 15).astype(np.float32) / np.float32(255.0))
    assert np.array_equal(pkg.load_idx_images(str(p), max_images=2), X[:2])
    lab = tmp_path / "y.idx1-ubyte"
    lab.write_bytes(struct.pack(">II", 2049, 4) + bytes([3, 11, 0, 9]))
    Y = pkg.load_idx_labels(str(lab))
    assert Y.tolist()[1] == [0.0] * 10 and np.argmax(Y, 1).tolist() == [3, 0, 0, 9]   # label >= 10: all zero
    with pytest.raises(pkg.LbfError, match="Invalid MNIST image file"):
        pkg.load_idx_images(str(lab))
    with pytest.raises(pkg.LbfError, match="Invalid MNIST label file"):
        pkg.load_idx_labels(str(p))
    trunc = tmp_path / "t.idx3-ubyte"
    trunc.write_bytes(struct.pack(">IIII", 2051, 7, 5, 3) + img.tobytes()[:20])
    with pytest.raises(pkg.LbfError, match="truncated"):
        pkg.load_idx_images(str(trunc))
    with pytest.raises(pkg.LbfError, match="cannot open"):
        pkg.load_idx_images(str(tmp_path / "missing"))
