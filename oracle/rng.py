"""Test infrastructure (never imported by the product package): the dropout
mask stream of the HIP kernels restated in numpy, so the oracle can replay the
exact masks a GPU run drew.  Element i of a tensor dropped with `seed` is kept
iff u01(seed, i) >= p; kept elements are scaled by 1 / (1 - p)
(csrc/common.h u01 / drop_scale: 16-bit field i % 4 of the splitmix64
finaliser of seed + golden * (i // 4 + 1))."""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def u01(seed, n):
    """u01(seed, i) for i < n: 16-bit field i % 4 of the finaliser of
    seed + golden * (i // 4 + 1) (four elements per 64-bit hash)."""
    with np.errstate(over='ignore'):
        i = np.arange(n, dtype=np.uint64)
        q = (i >> np.uint64(2)) + np.uint64(1)
        z = np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * q
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        f = (z >> (np.uint64(16) * (i & np.uint64(3)))) & np.uint64(0xFFFF)
    return f.astype(np.float32) * np.float32(1.0 / 65536.0)


def dropout_scale(seed, shape, p):
    """Multiplicative mask (0 or 1/(1-p)) of a contiguous tensor of `shape`."""
    n = int(np.prod(shape))
    keep = u01(seed, n) >= np.float32(p)
    return (keep.astype(np.float32) / np.float32(1.0 - p)).reshape(shape)
