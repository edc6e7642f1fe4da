"""The dropout mask stream of the HIP kernels (csrc/common.h u01 / drop_scale,
asr_dropout) against its numpy restatement (oracle/rng.py), bitwise: seeds
with high bits set, an odd length, p at and between 16-bit steps.  Every
kernel that applies or regenerates a mask (GEMM epilogues, the VGG row passes,
the fused forward's hand-off) draws from the same function, so the oracle's
replays of GPU runs rely on this identity.  (nn.Dropout's own mask stream is
torch's RNG, which no reimplementation reproduces; the reference tests run
dropout-free, see tests/golden/make_golden.py.)"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import rng


@pytest.mark.gpu
@pytest.mark.parametrize('seed', [1, 0xDEADBEEFCAFEBABE, 2 ** 63 + 12345])
@pytest.mark.parametrize('p', [0.2, 0.5, 13107.0 / 65536.0])
def test_asr_dropout_mask_matches_oracle(seed, p, cuda_dev):
    from pytorch_end2end_speech_recognition_amd import _native as N
    n = 100003
    x = torch.ones(n, device=cuda_dev)
    y = torch.empty_like(x)
    N.call('asr_dropout', N.ptr(x), N.ptr(y), n, ctypes.c_float(p), ctypes.c_ulonglong(seed),
           N.stream_handle(cuda_dev))
    torch.cuda.synchronize()
    got = y.cpu().numpy()
    keep = rng.u01(seed, n) >= np.float32(p)
    np.testing.assert_array_equal(got > 0, keep)
    np.testing.assert_allclose(got[keep], 1.0 / (1.0 - np.float32(p)), rtol=1e-6)
    assert abs(float(keep.mean()) - (1 - p)) < 0.01
