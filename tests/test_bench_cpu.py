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
