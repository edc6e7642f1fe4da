"""The data-parallel form of train_step over torch.distributed (gloo, world
size 2, CPU): round-robin sharding of a length-sorted batch, ONE all-reduce of
the flat gradient, the collective skip-batch flag, and equality of the
data-parallel update with the single-process update of the global batch.

The MI355X kernels cannot run here (no GPU); the model in this test is a tiny
ModelBase with a CPU torch forward, used only to exercise the collective logic
the GPU path shares (flat buffers, train_step, shard_batch)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pytorch_end2end_speech_recognition_amd import native_ops
from pytorch_end2end_speech_recognition_amd.models.pytorch_v3.base import ModelBase
from pytorch_end2end_speech_recognition_amd.utils.training import training_loop as TL


class _LayerFn(torch.autograd.Function):
    """Stand-in for BLSTMLayerFn: weight gradients written by the op itself into
    the flat-buffer views, with the same 'recurrence' / 'grads' notifications."""

    @staticmethod
    def forward(ctx, x, w, gviews):
        ctx.save_for_backward(x, w)
        ctx.gviews = gviews
        return torch.tanh(x @ w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        y = torch.tanh(x @ w.t())
        dz = dy * (1 - y * y)
        native_ops.notify_grad_event('pre_recurrence')
        native_ops.notify_grad_event('recurrence')
        for g in ctx.gviews:
            g.add_(dz.t() @ x)
        native_ops.notify_grad_event('grads', ctx.gviews)
        return dz @ w, None, None


class TinyEncoder(torch.nn.Module):
    """Two 'layers', each a (forward, reverse) parameter pair kept adjacent in
    the flat buffer like encoders/rnn.py."""

    def __init__(self):
        super().__init__()
        self.num_layers = 2
        for l in range(2):
            setattr(self, 'w%d_f' % l, torch.nn.Parameter(torch.randn(3, 3) * 0.3))
            setattr(self, 'w%d_r' % l, torch.nn.Parameter(torch.randn(3, 3) * 0.3))

    def _layer_params(self, l):
        return [(getattr(self, 'w%d_f' % l), getattr(self, 'w%d_r' % l))]

    def flat_order(self):
        return [list(pair) for l in range(2) for pair in self._layer_params(l)]


class TinyModel(ModelBase):
    def __init__(self, fail_rank=-1):
        super(ModelBase, self).__init__()
        torch.manual_seed(0)
        self.encoder = TinyEncoder()
        self.lin = torch.nn.Linear(3, 2)
        self.num_stack = 1
        self.fail_rank = fail_rank
        self.flatten_parameters_()

    def forward(self, xs, ys, x_lens, y_lens, is_eval=False):
        if dist.is_initialized() and dist.get_rank() == self.fail_rank:
            raise RuntimeError('simulated OOM')
        h = torch.from_numpy(np.asarray(xs, np.float32)).sum(1)      # [B, 3]
        for l in range(2):
            wf, wr = self.encoder._layer_params(l)[0]
            h = _LayerFn.apply(h, wf + wr, (wf.grad, wr.grad))
        out = self.lin(h)
        return ((out - 1.0) ** 2).mean().reshape(1)


def _batch(B=6):
    rng = np.random.RandomState(0)
    T = 5
    x_lens = np.array([5, 5, 4, 3, 3, 2][:B], np.int32)
    xs = rng.randn(B, T, 3).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    return dict(xs=xs, ys=np.zeros((B, 2), np.int32), x_lens=x_lens,
                y_lens=np.ones(B, np.int32))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fail_rank, out, B, clip):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    model = TinyModel(fail_rank)
    model.optimizer = torch.optim.SGD(model.parameters(), lr=0.1)
    local, scale = TL.shard_batch(_batch(B), rank, world)
    # per-rank loss is a mean over the local batch -> scale by local/global
    issued = []
    orig = TL.GradBuckets.finish

    def finish(self, ok=1):
        issued.append(self.issued_during_backward)
        return orig(self, ok)
    TL.GradBuckets.finish = finish
    _, lv = TL.train_step(model, local, clip_grad_norm=clip, grad_scale=scale)
    out[rank] = (model._flat_param.clone(), issued[0] if issued else -1)
    dist.destroy_process_group()


def _run(world, fail_rank=-1, B=6, clip=0.0):
    ctx = mp.get_context('spawn')
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, out, B, clip))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    return [out[r] for r in range(world)]


def test_shard_batch_round_robin():
    b = _batch()
    l0, s0 = TL.shard_batch(b, 0, 2)
    l1, s1 = TL.shard_batch(b, 1, 2)
    np.testing.assert_array_equal(l0['x_lens'], [5, 4, 3])
    np.testing.assert_array_equal(l1['x_lens'], [5, 3, 2])
    assert l1['xs'].shape[1] == 5 and s0 == s1 == 0.5


@pytest.mark.parametrize('B,clip', [(6, 0.0), (5, 0.0), (5, 0.05)])
def test_data_parallel_update_equals_single_process(B, clip):
    """Equal (3/3) and unequal (3/2) shards, without and with the global-norm
    clip: the data-parallel update equals the single-process update of the
    global batch on every rank."""
    res = _run(2, B=B, clip=clip)
    params = [r[0] for r in res]
    torch.testing.assert_close(params[0], params[1])
    # the layer-1 bucket went out during the backward (after layer 0's
    # 'recurrence'), the layer-0 bucket and the remainder at the end
    assert all(r[1] == 1 for r in res)
    model = TinyModel()
    model.optimizer = torch.optim.SGD(model.parameters(), lr=0.1)
    TL.train_step(model, _batch(B), clip_grad_norm=clip)
    torch.testing.assert_close(params[0], model._flat_param, rtol=1e-5, atol=1e-6)
    assert not torch.equal(model._flat_param, TinyModel()._flat_param)


def test_grad_buckets_partition_the_flat_buffer():
    model = TinyModel()
    gb = TL.GradBuckets(model, 0.5)
    spans = sorted(gb.order + gb.rest)
    assert spans[0][0] == 0 and spans[-1][1] == model._flat_grad.numel()
    for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
        assert b0 == a1
    assert len(gb.order) == 2 and gb.order[0][0] > gb.order[1][0]    # top layer first


def test_skip_batch_is_collective():
    res = _run(2, fail_rank=1)
    init = TinyModel()._flat_param
    for p, _ in res:                 # both ranks skipped the update
        torch.testing.assert_close(p, init)
