"""IDX file reader (the MNIST / FashionMNIST container format torchvision downloads,
distributed_cnn.py:90-106).  Used when real FashionMNIST files are present on disk; otherwise
recipes fall back to :func:`sparkmi.data.synthetic.fashion_mnist_like`."""
import gzip
import os

import numpy as np

_DTYPES = {0x08: np.uint8, 0x09: np.int8, 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4", 0x0E: ">f8"}


def read_idx(path):
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    if len(data) < 4 or data[0] != 0 or data[1] != 0:
        raise ValueError(f"{path}: not an IDX file")
    dt, nd = data[2], data[3]
    if dt not in _DTYPES:
        raise ValueError(f"{path}: unknown IDX dtype 0x{dt:02x}")
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(nd)]
    off = 4 + 4 * nd
    arr = np.frombuffer(data, dtype=np.dtype(_DTYPES[dt]), offset=off, count=int(np.prod(dims)) if dims else 1)
    return arr.reshape(dims).astype(arr.dtype.newbyteorder("=")) if arr.dtype.byteorder == ">" else arr.reshape(dims)


def write_idx(path, arr):
    arr = np.ascontiguousarray(arr)
    code = {np.dtype(np.uint8): 0x08, np.dtype(np.int8): 0x09, np.dtype(np.int16): 0x0B, np.dtype(np.int32): 0x0C,
            np.dtype(np.float32): 0x0D, np.dtype(np.float64): 0x0E}[arr.dtype]
    hdr = bytes([0, 0, code, arr.ndim]) + b"".join(int(d).to_bytes(4, "big") for d in arr.shape)
    body = arr.astype(arr.dtype.newbyteorder(">")).tobytes() if arr.dtype.itemsize > 1 else arr.tobytes()
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(hdr + body)


def _find(root, stem):
    for sub in ("", "FashionMNIST/raw", "raw"):
        for ext in ("", ".gz"):
            p = os.path.join(root, sub, stem + ext)
            if os.path.exists(p):
                return p
    return None


def load_fashion_mnist(root):
    """((train_images uint8 [N,1,28,28], train_labels int64), (test_images, test_labels)) or None."""
    names = ["train-images-idx3-ubyte", "train-labels-idx1-ubyte", "t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"]
    paths = [_find(root, n) for n in names] if root else [None]
    if not root or any(p is None for p in paths):
        return None
    xtr, ytr, xte, yte = (read_idx(p) for p in paths)
    return ((xtr.reshape(-1, 1, 28, 28), ytr.astype(np.int64)), (xte.reshape(-1, 1, 28, 28), yte.astype(np.int64)))


FASHION_MNIST_CLASSES = ["T-shirt/top", "Trouser", "Pullover", "Dress", "Coat", "Sandal", "Shirt", "Sneaker", "Bag",
                         "Ankle boot"]
