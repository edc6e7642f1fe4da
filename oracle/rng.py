"""Test infrastructure (never imported by the product package): the dropout
mask stream of the HIP kernels restated in numpy, so the oracle can replay the
exact masks a GPU run drew.  Element i of a tensor dropped with `seed` is kept
iff u01(seed, i) >= p; kept elements are scaled by 1 / (1 - p)
(csrc/common.h u01 / drop_scale: 16-bit field i % 2 of a 32-bit lowbias32
hash of ((i // 2) * 0x9E3779B9) xor the seed's hashed 32-bit key)."""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _lowbias32(x):
    M32 = np.uint64(0xFFFFFFFF)
    x = x & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def u01(seed, n):
    """u01(seed, i) for i < n: 16-bit field i % 2 of lowbias32(((i // 2) *
    0x9E3779B9) xor key) in 32-bit arithmetic, key = lowbias32(low 32 bits of
    seed xor high 32 bits * 0x85EBCA6B), divided by 65536 (two elements per
    hash)."""
    M32 = np.uint64(0xFFFFFFFF)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    key = _lowbias32(np.uint64(((seed & 0xFFFFFFFF) ^ (((seed >> 32) * 0x85EBCA6B) & 0xFFFFFFFF))))
    i = np.arange(n, dtype=np.uint64)
    x = _lowbias32(((i >> np.uint64(1)) * np.uint64(0x9E3779B9) & M32) ^ key)
    f = (x >> (np.uint64(16) * (i & np.uint64(1)))) & np.uint64(0xFFFF)
    return f.astype(np.float32) * np.float32(1.0 / 65536.0)


def dropout_scale(seed, shape, p):
    """Multiplicative mask (0 or 1/(1-p)) of a contiguous tensor of `shape`."""
    n = int(np.prod(shape))
    keep = u01(seed, n) >= np.float32(p)
    return (keep.astype(np.float32) / np.float32(1.0 - p)).reshape(shape)
