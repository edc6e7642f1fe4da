"""bench.py host logic that needs no GPU: `--gpus N` starts N ranks itself
(one process per GPU, torch.distributed.run on 127.0.0.1) before anything
touches the GPU, refuses a world size that disagrees with --gpus, and the
parity samples are built as documented."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_gpus_n_launches_ranks(monkeypatch):
    bench = _bench()
    calls = []
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setattr(subprocess, 'call', lambda cmd: calls.append(cmd) or 0)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '4', '--steps', '3', '--warmup', '1'])
    # no GPU call may happen in the launching process
    monkeypatch.setattr(torch.cuda, 'set_device', lambda *a: pytest.fail('GPU touched'))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    (cmd,) = calls
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    i = cmd.index('--nproc-per-node')
    assert cmd[i + 1] == '4'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-6:] == [os.path.join(ROOT, 'bench.py'), '--gpus', '4', '--steps', '3',
                        '--warmup', '1'][-6:]


def test_world_size_must_match_gpus(monkeypatch):
    bench = _bench()
    monkeypatch.setenv('WORLD_SIZE', '2')
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '4'])
    monkeypatch.setattr(torch.cuda, 'set_device', lambda *a: pytest.fail('GPU touched'))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert 'WORLD_SIZE=2' in str(e.value.code)


def test_parity_samples():
    bench = _bench()
    b = bench.synthetic_batch(6, 1000, 80, 28, seed=0)
    t = bench._truncate(b, 200)
    assert t['xs'].shape == (6, 200, 80) and int(t['x_lens'].max()) == 200
    assert np.array_equal(t['ys'], b['ys'])
    sd = {'encoder.lstm.weight_hh_l0': torch.full((8, 2), 0.1),
          'encoder.lstm.weight_ih_l0': torch.full((8, 3), 0.1)}
    s = bench._small_whh(sd)
    assert float(s['encoder.lstm.weight_hh_l0'].abs().max()) <= 0.03
    assert torch.equal(s['encoder.lstm.weight_ih_l0'], sd['encoder.lstm.weight_ih_l0'])
    assert torch.equal(bench._small_whh(sd)['encoder.lstm.weight_hh_l0'],
                       s['encoder.lstm.weight_hh_l0'])      # seeded


def test_repeat_batches_are_fresh_copies():
    bench = _bench()
    b = bench.synthetic_batch(4, 1000, 8, 28, seed=1)
    r = bench._RepeatBatches(b, 2)
    x1, _ = r.next()
    x2, _ = r.next()
    assert x1['xs'] is not x2['xs'] and np.array_equal(x1['xs'], b['xs'])
    with pytest.raises(StopIteration):
        r.next()


def test_roofline_rows_per_kernel_instantiation():
    """The roofline is reported per kernel instantiation (kind x prof tag), the
    dominant row names ONE kernel (not the GEMM family), and each CTC head
    gets its own rows plus a whole-op row against 8 * V bytes per frame."""
    bench = _bench()
    import argparse
    args = argparse.Namespace(batch=32, frames=1000, precision='bf16')
    p = dict(bench.CONFIGS['vgg_hier']['params'])
    V, rows = 10001, 32 * 250
    samples = {
        3: [(3, 0.0, 1000.0)] * 4,                                  # lstm_bwd_xg
        4: ([(4 * 1 + 3, 2e11, 300.0)] * 10 +                       # gemm_bf16_8r<1, 1>
            [(4 * 9, 5e10, 120.0)] * 6),                            # conv3x3_tr
        5: [(V, 4.0 * V * rows, 100.0), (29, 4.0 * 29 * rows * 4, 50.0)],
        6: [(V, 8.0 * V * rows, 120.0), (29, 8.0 * 29 * rows * 4, 20.0)],
    }
    launches = [0, 0, 0, 4, 16, 2, 2, 0, 0]
    r = bench.roofline_report(args, p, samples, launches, 'x')
    assert r['kernel'] == 'lstm_bwd_xg<*>' and r['launches_timed'] == 4
    assert r['bound'] == 'mfma' and r['us_per_time_step'] > 0
    o = r['other_kernels']
    assert 'gemm_bf16_8r<1, 1>' in o and o['gemm_bf16_8r<1, 1>']['launches'] == 10
    assert abs(o['gemm_bf16_8r<1, 1>']['achieved'] - 2e11 / 300e-6 / 1e12) < 0.01
    assert 'conv3x3_tr<*>' in o
    assert 'ctc_grad [V=10001]' in o and 'ctc_grad [V=29]' in o
    op = o['ctc_op [V=10001]']
    assert op['algorithmic_bytes_per_call'] == int(8.0 * V * rows)
    assert abs(op['mean_call_us'] - 220.0) < 1e-9
    assert abs(sum(v['share_of_timed_kernel_time'] for k, v in o.items() if 'ctc_op' not in k)
               + r['share_of_timed_kernel_time'] - 1.0) < 0.01
