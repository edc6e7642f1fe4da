"""The data-parallel bucket path on the REAL model, on one GPU.

torch.distributed is replaced by a recording shim (world size reported as 2,
every collective a no-op that snapshots its segment on the compute stream at
issue time), so the whole production backward runs with the bucket hooks
installed: the BLSTMLayerFn 'recurrence' / 'grads' notifications, the
side-stream weight gradients joined into the compute stream, the remainder
bucket and the device-guard MAX all-reduce.  Checked:

  * every flat-gradient element is issued exactly once (buckets disjoint,
    covering the buffer), the per-layer buckets top layer first;
  * each bucket's snapshot -- what RCCL would read when its collective runs,
    stream-ordered after everything enqueued before it -- equals the final
    gradient of that range: no weight-gradient GEMM (main or side stream)
    writes a range after its collective was issued;
  * the guard all-reduce is issued (MAX) and the update equals the plain
    single-process step bitwise (SUM over one rank is the identity).
"""
import numpy as np
import pytest
import torch
import torch.distributed as dist

from test_model_ctc import _build


class _Work(object):
    def wait(self):
        pass


def _kw(H=512, L=5):
    return dict(input_size=80, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=H, encoder_num_proj=0, encoder_num_layers=L, fc_list=[],
                dropout_input=0, dropout_encoder=0, num_classes=28, parameter_init=0.1,
                subsample_list=[], subsample_type='drop')


def _batch(B=32, T=240, seed=0):
    rng = np.random.RandomState(seed)
    x_lens = np.sort(rng.randint(int(T * 0.8), T + 1, B))[::-1].astype(np.int32)
    x_lens[0] = T
    xs = rng.randn(B, T, 80).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    y_lens = rng.randint(15, 30, B).astype(np.int32)
    ys = np.full((B, int(y_lens.max())), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 28, y_lens[b])
    return dict(xs=xs, ys=ys, x_lens=x_lens, y_lens=y_lens)


@pytest.mark.gpu
@pytest.mark.parametrize('overlap,H,L', [('auto', 512, 5), ('auto', 320, 4), ('3', 256, 3),
                                         ('0', 320, 4)])
def test_buckets_on_real_model(overlap, H, L, cuda_dev, monkeypatch):
    """ctc5x512's encoder (auto: mode 3 with 32-unit backward work-groups, the
    weight gradients on the side stream beside the next recurrence), the 4x320
    encoder of configs[2]-[4] (auto: mode 3 with 16 units), a 3x256 encoder in
    mode 3 and the 4x320 one on the compute stream (mode 0); the side-stream
    gradients are joined into the compute stream before their bucket is
    issued.  Within each parametrisation the bucketed step updates the weights
    bitwise like the plain single-process step in the SAME overlap mode (run
    to run, not across modes: tests/test_coresidency_gpu.py compares modes 2
    and 3 with mode 0 bitwise); the bucket checks are exact."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training import training_loop as TL
    monkeypatch.setenv('ASR_OVERLAP_WGRAD', overlap)
    batch = _batch()
    native_ops.set_compute_dtype('bf16')
    try:
        torch.manual_seed(1623)
        sd = {k: v.clone() for k, v in _build(_kw(H, L)).state_dict().items()}

        def fresh():
            m = _build(_kw(H, L))
            m.load_state_dict(sd)
            m.set_cuda()
            m.set_optimizer('adam', 1e-3, weight_decay=1e-6)
            return m

        ref = fresh()
        native_ops.recurrence_status(cuda_dev)
        ref, lv_ref = TL.train_step(ref, batch, clip_grad_norm=5.0)
        torch.cuda.synchronize()

        m = fresh()
        flat = m._flat_grad
        base, es = flat.data_ptr(), flat.element_size()
        issued, guards = [], []

        def all_reduce(t, op=None, async_op=False, **kw):
            if t.data_ptr() >= base and t.data_ptr() < base + flat.numel() * es:
                a = (t.data_ptr() - base) // es
                issued.append((a, a + t.numel(), t.clone()))   # stream-ordered snapshot
            else:
                guards.append((op, t.numel()))
            return _Work() if async_op else None

        monkeypatch.setattr(TL, '_world', lambda: 2)
        monkeypatch.setattr(dist, 'all_reduce', all_reduce)
        m, lv = TL.train_step(m, batch, clip_grad_norm=5.0, grad_scale=None)
        torch.cuda.synchronize()
        monkeypatch.undo()
        native_ops.set_compute_dtype('bf16')

        # exactly once, disjoint, covering the whole flat buffer
        cover = np.zeros(flat.numel(), np.int32)
        for a, b, _ in issued:
            cover[a:b] += 1
        assert cover.min() == 1 and cover.max() == 1
        # per-layer buckets first, top layer first (L layers + the remainder)
        enc = m.encoder
        starts = []
        for l in range(enc.num_layers):
            ps = [p for pair in enc._layer_params(l) for p in pair]
            starts.append(min((p.grad.data_ptr() - base) // es for p in ps))
        assert [a for a, _, _ in issued[:enc.num_layers]] == sorted(starts, reverse=True)
        # what each collective would read == the final gradient of its range
        for a, b, snap in issued:
            assert torch.equal(snap, flat[a:b]), (a, b, float((snap - flat[a:b]).abs().max()))
        assert guards and all(op == dist.ReduceOp.MAX for op, _ in guards)
        assert lv == lv_ref
        assert torch.equal(m._flat_param, ref._flat_param)
    finally:
        native_ops.set_compute_dtype('fp32')
