"""Per-step recurrence workspace arena (round 6, native_ops.rec_arena_begin).

The encoder forward clears one buffer holding a granule workspace for every
BLSTM layer pass of the step, and those launches skip their own memset.  The
recurrences must compute bitwise what they compute with a fresh, memset
workspace per launch (ASR_REC_ARENA=0), also when a second forward clears the
arena again before the first one's backward ran (its reservations are then
stale and its backward takes a private workspace).
"""
import pytest
import torch

from test_grad_buckets_gpu import _batch, _kw
from test_model_ctc import _build


def _loss_grad(m, batch):
    m.zero_grad()
    loss = m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'])
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), m._flat_grad.clone()


@pytest.fixture
def bf16_mode():
    from pytorch_end2end_speech_recognition_amd import native_ops
    native_ops.set_compute_dtype('bf16')
    yield
    native_ops.set_compute_dtype('fp32')


@pytest.mark.gpu
def test_arena_bitwise_equals_per_launch_memset(cuda_dev, monkeypatch, bf16_mode):
    from pytorch_end2end_speech_recognition_amd import native_ops
    H, L = 256, 3
    torch.manual_seed(1623)
    sd = {k: v.clone() for k, v in _build(_kw(H, L)).state_dict().items()}
    b1, b2 = _batch(T=160, seed=1), _batch(T=200, seed=2)

    def fresh():
        m = _build(_kw(H, L))
        m.load_state_dict(sd)
        m.set_cuda()
        return m

    monkeypatch.setenv('ASR_REC_ARENA', '0')
    m = fresh()
    ref = [_loss_grad(m, b1), _loss_grad(m, b2)]

    monkeypatch.setenv('ASR_REC_ARENA', '1')
    m = fresh()
    got = [_loss_grad(m, b1), _loss_grad(m, b2), _loss_grad(m, b1)]
    for (l0, g0), (l1, g1) in zip(ref + ref[:1], got):
        assert l0 == l1
        assert torch.equal(g0, g1), int((g0 != g1).sum())

    # two forwards, then the two backwards: the first forward's backward
    # reservations are stale once the second forward cleared the arena
    m.zero_grad()
    la = m(b1['xs'], b1['ys'], b1['x_lens'], b1['y_lens'])
    gen_a = native_ops._arena['gen']
    lb = m(b2['xs'], b2['ys'], b2['x_lens'], b2['y_lens'])
    assert native_ops._arena['gen'] == gen_a + 1
    la.backward()
    torch.cuda.synchronize()
    ga = m._flat_grad.clone()
    m.zero_grad()
    lb.backward()
    torch.cuda.synchronize()
    gb = m._flat_grad.clone()
    assert la.item() == ref[0][0] and lb.item() == ref[1][0]
    assert torch.equal(ga, ref[0][1]), int((ga != ref[0][1]).sum())
    assert torch.equal(gb, ref[1][1]), int((gb != ref[1][1]).sum())
