"""A/B timing of the BLSTM recurrence variants in ONE process (interleaved
rounds, cdna_hip_programming.md §5.4 rule 24).  Each variant is a set of
environment switches read by libasr_hip per call (ASR_LSTM_PERSIST,
ASR_LSTM_PUBW, ...).  Times the persistent pass kernels with the library's
HIP-event hooks and the whole layer fwd+bwd with torch events.

usage: python tools/lstm_ab.py [--rounds 5] [--T 1000] [--B 32] [--H 512]
       [--variant NAME:VAR=VAL,VAR=VAL ...]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_end2end_speech_recognition_amd import _native as N  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--B', type=int, default=32)
    ap.add_argument('--T', type=int, default=1000)
    ap.add_argument('--H', type=int, default=512)
    ap.add_argument('--Din', type=int, default=1024)
    ap.add_argument('--variant', action='append', default=[])
    args = ap.parse_args()
    variants = []
    for v in args.variant or ['default:']:
        name, _, kv = v.partition(':')
        env = dict(x.split('=') for x in kv.split(',') if x)
        variants.append((name, env))
    dev = torch.device('cuda:0')
    ops.set_compute_dtype('bf16')
    B, T, H, Din = args.B, args.T, args.H, args.Din
    rng = np.random.RandomState(0)
    x = torch.from_numpy(rng.randn(B, T, Din).astype(np.float32)).to(dev).requires_grad_(True)
    ws = [torch.from_numpy(rng.uniform(-0.1, 0.1, s).astype(np.float32)).to(dev).requires_grad_(True)
          for s in ((8 * H, Din), (8 * H, H), (8 * H,), (8 * H,))]
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    R = torch.randn(B, T, 2 * H, device=dev)
    res = {n: {'fwd': [], 'bwd': [], 'layer': []} for n, _ in variants}
    base_env = dict(os.environ)
    for rnd in range(args.rounds + 1):
        for name, env in variants:
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(env)
            torch.cuda.synchronize()
            N.call('asr_prof_begin', 1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            y = ops.blstm_layer(x, lens, T, *ws)
            (y * R).sum().backward()
            e1.record()
            torch.cuda.synchronize()
            mean_us = (ctypes.c_double * 5)()
            launches = (ctypes.c_longlong * 5)()
            N.call('asr_prof_end', ctypes.cast(mean_us, ctypes.c_void_p),
                   ctypes.cast(launches, ctypes.c_void_p), None, 5)
            if rnd == 0:
                continue  # warm-up round
            fwd = mean_us[2] if launches[2] else mean_us[0] * launches[0]
            bwd = mean_us[3] if launches[3] else mean_us[1] * launches[1]
            res[name]['fwd'].append(fwd)
            res[name]['bwd'].append(bwd)
            res[name]['layer'].append(e0.elapsed_time(e1) * 1000.0)
    st = ctypes.c_int(0)
    N.call('asr_lstm_persist_status', ctypes.byref(st), 1, N.stream_handle())
    print('persist_status', st.value)
    for name, _ in variants:
        r = res[name]
        print('%-14s fwd pass %8.1f us (min %8.1f)  bwd pass %8.1f us (min %8.1f)  layer %8.1f us'
              % (name, np.median(r['fwd']), np.min(r['fwd']), np.median(r['bwd']),
                 np.min(r['bwd']), np.median(r['layer'])))


if __name__ == '__main__':
    main()
