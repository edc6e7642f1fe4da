"""train_step: the reference's training-step contract
(utils/training/training_loop.py:27-83) on the MI355X path, plus its
data-parallel form over RCCL.

Single GPU: zero_grad -> forward -> backward -> fused clip + optimizer step
(the global-norm clip coefficient is computed on device; no host sync until
the loss value is read).  Data parallel (torch.distributed initialised, world
size > 1): each rank runs forward/backward on its shard, the flat gradient
buffer is summed over ranks with ONE RCCL all-reduce (the shard losses are
scaled so the sum equals the 1-GPU gradient of the global batch), then every
rank clips with the same global norm and applies the same update.  A RuntimeError
on any rank skips the batch on every rank (a 1-int all-reduce keeps the ranks
in lock step), mirroring training_loop.py:69-76.
"""
import logging

import torch
import torch.distributed as dist

logger = logging.getLogger('training')
INF = float('inf')


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def allreduce_gradients(model, grad_scale=None):
    """Sum the flat gradient over ranks (one contiguous RCCL collective)."""
    if _world() > 1:
        dist.all_reduce(model._flat_grad, op=dist.ReduceOp.SUM)
        if grad_scale is not None:
            model._flat_grad.mul_(grad_scale)


def train_step(model, batch, clip_grad_norm, backend='pytorch', grad_scale=None):
    """Returns (model, loss_value) like training_loop.py:27-83.

    grad_scale: optional factor applied to the all-reduced gradient (data
    parallel: pass local_batch / global_batch when every rank divides its loss
    by its local batch size, so the update equals the 1-GPU update)."""
    loss_val = 0.
    ok = 1
    try:
        model.optimizer.zero_grad()
        loss = model(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'])
        loss.backward()
    except RuntimeError as e:
        logger.warning('!!!Skip mini-batch!!! (max_frame_num: %d, batch: %d) %s' %
                       (max(batch['x_lens']) * model.num_stack, len(batch['xs']), e))
        ok = 0
        loss = None
    if _world() > 1:
        flag = torch.tensor([ok], dtype=torch.int32, device=model.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = int(flag.item())
    if not ok:
        model.optimizer.zero_grad()
        return model, 0.
    allreduce_gradients(model, grad_scale)
    if hasattr(model.optimizer, 'clip_and_step'):
        model.optimizer.clip_and_step(clip_grad_norm if clip_grad_norm > 0 else 0.0)
    else:
        if clip_grad_norm > 0:
            torch.nn.utils.clip_grad_norm_(model.parameters(), clip_grad_norm)
        model.optimizer.step()
    loss_val = float(loss.item())
    if loss_val == INF or loss_val == -INF:
        logger.warning('WARNING: received an inf loss, setting loss value to 0.')
        loss_val = 0
    return model, loss_val
