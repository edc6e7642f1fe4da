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

from pytorch_end2end_speech_recognition_amd.models.pytorch_v3.base import ModelBase
from pytorch_end2end_speech_recognition_amd.utils.training import training_loop as TL


class TinyModel(ModelBase):
    def __init__(self, fail_rank=-1):
        super(ModelBase, self).__init__()
        torch.manual_seed(0)
        self.lin = torch.nn.Linear(3, 2)
        self.num_stack = 1
        self.fail_rank = fail_rank
        self.flatten_parameters_()

    def forward(self, xs, ys, x_lens, y_lens, is_eval=False):
        if dist.is_initialized() and dist.get_rank() == self.fail_rank:
            raise RuntimeError('simulated OOM')
        x = torch.from_numpy(np.asarray(xs, np.float32)).sum(1)      # [B, 3]
        out = self.lin(x)
        return ((out - 1.0) ** 2).mean().reshape(1)


def _batch():
    rng = np.random.RandomState(0)
    B, T = 6, 5
    x_lens = np.array([5, 5, 4, 3, 3, 2], np.int32)
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


def _worker(rank, world, port, fail_rank, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    model = TinyModel(fail_rank)
    model.optimizer = torch.optim.SGD(model.parameters(), lr=0.1)
    local, scale = TL.shard_batch(_batch(), rank, world)
    # per-rank loss is a mean over the local batch -> scale by local/global
    _, lv = TL.train_step(model, local, clip_grad_norm=0, grad_scale=scale)
    out[rank] = model._flat_param.clone()
    dist.destroy_process_group()


def _run(world, fail_rank=-1):
    ctx = mp.get_context('spawn')
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, out))
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


def test_data_parallel_update_equals_single_process():
    params = _run(2)
    torch.testing.assert_close(params[0], params[1])
    # single-process reference on the global batch
    model = TinyModel()
    model.optimizer = torch.optim.SGD(model.parameters(), lr=0.1)
    b = _batch()
    # the 1-GPU gradient of the global batch = mean of the two shard means here
    # (equal shard sizes), i.e. the global-batch mean loss
    TL.train_step(model, b, clip_grad_norm=0)
    torch.testing.assert_close(params[0], model._flat_param, rtol=1e-5, atol=1e-6)


def test_skip_batch_is_collective():
    params = _run(2, fail_rank=1)
    init = TinyModel()._flat_param
    for p in params:                 # both ranks skipped the update
        torch.testing.assert_close(p, init)
