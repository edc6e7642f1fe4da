"""train_step: the reference's training-step contract
(utils/training/training_loop.py:27-83) on the MI355X path, plus its
data-parallel form over RCCL.

Single GPU: zero_grad -> forward -> backward -> fused clip + optimizer step
(the global-norm clip coefficient is computed on device; no host sync until
the loss value is read).  Data parallel (torch.distributed initialised, world
size > 1): each rank runs forward/backward on its shard; each rank's gradient
(of its per-rank mean loss) is scaled by local_B / global_B BEFORE the SUM
all-reduce, so the reduced gradient is the 1-GPU gradient of the global batch
for any split (unequal shards included).  The flat gradient buffer is reduced
in buckets (utils/training/grad_buckets.py): one per BLSTM layer, issued while
the backward of the layers below still runs, plus the remainder at the end.
Then every rank clips with the same global norm and applies the same update.
A RuntimeError on any rank skips the batch on every rank (a 1-int all-reduce
keeps the ranks in lock step), mirroring training_loop.py:69-76.
"""
import logging

import torch
import torch.distributed as dist

from .grad_buckets import GradBuckets

logger = logging.getLogger('training')
INF = float('inf')

# Per-process counters of the training steps this module ran (VERDICT r05 #7:
# a skipped step is never silent): 'skipped' counts every step whose update
# was dropped -- a RuntimeError on some rank, or a persistent recurrence that
# gave up a bounded wait (its status word folded into the device guard) --
# and 'recurrence_give_ups' the subset whose guard carried a recurrence status
# word rather than an exception on this rank.  bench.py reports both.
STEP_STATS = {'steps': 0, 'skipped': 0, 'recurrence_give_ups': 0}


def reset_step_stats():
    for k in STEP_STATS:
        STEP_STATS[k] = 0


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def shard_batch(batch, rank, world):
    """Deal a length-sorted global batch round-robin to the ranks:
    rank r takes utterances r, r + world, ...  Every rank's longest utterance is
    within one position of the global order, so per-rank Tmax (the recurrence
    length, i.e. the step time) stays balanced; contiguous chunks would hand
    rank 0 all the longest utterances.  Returns (local batch, grad_scale) where
    grad_scale = local_B / global_B makes the summed gradient of the
    per-rank-mean losses equal the 1-GPU gradient of the global batch."""
    import numpy as np
    B = len(batch['xs'])
    if world <= 1:
        return batch, None
    idx = np.arange(rank, B, world)
    if len(idx) == 0:
        raise ValueError('global batch %d smaller than world size %d' % (B, world))
    local = {}
    for k, v in batch.items():
        v = np.asarray(v)
        local[k] = v[idx] if v.ndim >= 1 and len(v) == B else v
    # trim padding to the local maxima (the reference pads per batch)
    tmax = int(np.max(local['x_lens']))
    local['xs'] = local['xs'][:, :tmax]
    if 'ys' in local and 'y_lens' in local:
        local['ys'] = local['ys'][:, :max(1, int(np.max(local['y_lens'])))]
    if 'ys_sub' in local and 'y_lens_sub' in local:
        local['ys_sub'] = local['ys_sub'][:, :max(1, int(np.max(local['y_lens_sub'])))]
    return local, float(len(idx)) / float(B)


def allreduce_gradients(model, grad_scale=None):
    """Scale this rank's flat gradient by grad_scale (local_B / global_B), then
    SUM it over ranks (one contiguous RCCL collective).  Scaling before the sum
    is what makes unequal shards correct: SUM_r (n_r / N) g_r is the gradient
    of the global-batch mean loss on every rank."""
    if _world() > 1:
        if grad_scale is not None:
            model._flat_grad.mul_(grad_scale)
        dist.all_reduce(model._flat_grad, op=dist.ReduceOp.SUM)


def _status_guard(model):
    """Device int32[2]: the recurrence status words of this step (a bounded
    spin that gave up), gathered and cleared stream-ordered (no host sync);
    None on a CPU model (the gloo tests) or without the library."""
    if model.device.type != 'cuda':
        return None
    from ... import native_ops
    return native_ops.recurrence_status(model.device)


class PendingLosses(object):
    """The losses of a train_step(..., sync=False), read back one step late.

    The step's loss values and skip guard are copied (stream-ordered) into a
    pinned host buffer; nothing waits for them until value() is called -- or
    until the NEXT step reaches its optimizer, which resolves the previous
    step first (so a skipped batch undoes its Adam step count before the next
    update, exactly as the synchronous path does).  The host therefore runs
    one step ahead of the GPU instead of idling it at every step boundary
    (the reference's loss.item() per step, training_loop.py:78)."""

    def __init__(self, model, host, event, n_losses, n_guard, has_losses):
        self._model, self._host, self._event = model, host, event
        self._n, self._ng, self._has = n_losses, n_guard, has_losses
        self._vals = None

    def value(self):
        if self._vals is None:
            self._event.synchronize()
            host = self._host.tolist()
            # no zero_grad on a skip here: the flat gradient already belongs to
            # the next step (which zeroes it itself before its backward)
            self._vals = _finish(self._model, host, self._n, self._ng, self._has, zero=False)
            if getattr(self._model, '_pending_losses', None) is self:
                self._model._pending_losses = None
        return self._vals

    def __float__(self):
        return float(self.value()[0])


def _finish(model, host, n_losses, n_guard, has_losses, zero=True):
    """Loss values from the step's host read-back (skip / inf semantics of
    training_loop.py:69-83)."""
    vals = host[:n_losses] if has_losses else [0.] * n_losses
    if n_guard and max(host[-n_guard:]) > 0:
        if has_losses:    # no exception on this rank: the guard is a status word
            STEP_STATS['recurrence_give_ups'] += 1
        # the fused step left the weights untouched; undo its step count
        if hasattr(model.optimizer, 'undo_step_count'):
            model.optimizer.undo_step_count()
        return _skipped(model, n_losses, 'a rank failed or a persistent recurrence gave up '
                        '(status %s)' % host[-n_guard:], zero=zero)
    if vals[0] == INF or vals[0] == -INF:
        logger.warning('WARNING: received an inf loss, setting loss value to 0.')
        vals = [0.] * n_losses
    return vals


def _step(model, forward, clip_grad_norm, n_losses, grad_scale, sync=True):
    """zero_grad -> forward (returns n_losses loss tensors, the first is the
    total) -> backward -> collective skip flag -> gradient all-reduce ->
    fused clip + optimizer step.  Returns the losses as floats (0 on skip).

    Skips (training_loop.py:69-76): a RuntimeError on any rank, or a
    persistent recurrence whose bounded spin gave up (its gradients are
    invalid).  On the GPU both are folded into a device guard (MAX-reduced
    over ranks) that the fused optimizer kernel checks, so the step needs no
    host sync before the optimizer; the host reads the guard with the loss."""
    ok = 1
    world = _world()
    STEP_STATS['steps'] += 1
    if model.device.type == 'cuda':
        from ... import native_ops
        # weight gradients a failed backward outside train_step left pending
        # are joined and forgotten; status words set outside a training step
        # (an eval pass the caller did not check) are dropped, so the guard
        # below covers only this step's own recurrences
        native_ops.discard_side_wgrads()
        native_ops.recurrence_status(model.device)
    buckets = GradBuckets.for_model(model, grad_scale) if world > 1 else None
    try:
        # ModelBase.zero_grad zeroes the flat gradient and re-binds every
        # param.grad view (torch.optim's zero_grad would set them to None and
        # detach them from the buffer the all-reduce / fused step work on)
        model.zero_grad()
        losses = forward()
        if buckets is not None:
            with buckets:                 # per-layer collectives during the backward
                losses[0].backward()
        else:
            losses[0].backward()
    except RuntimeError as e:
        logger.warning('!!!Skip mini-batch!!! %s' % e)
        ok = 0
        losses = None
        if model.device.type == 'cuda':
            # side-stream weight gradients of the failed backward: the zero of
            # the flat gradient (skip path / next step) must wait for them, and
            # no bucket may report them ready
            from ... import native_ops
            native_ops.discard_side_wgrads()
    if buckets is not None:
        buckets.finish(ok)                # remainder + wait; never skipped, so every
    guard = _status_guard(model)          # rank pairs the others' collectives
    if guard is not None:
        if not ok:
            guard[0:1].fill_(1)
        if world > 1:
            dist.all_reduce(guard, op=dist.ReduceOp.MAX)
    elif world > 1:
        flag = torch.tensor([ok], dtype=torch.int32, device=model.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = int(flag.item())
    if not ok and (guard is None or world == 1):
        STEP_STATS['skipped'] += 1
        model.zero_grad()
        return [0.] * n_losses
    prev = getattr(model, '_pending_losses', None)
    if prev is not None:     # the previous step's read-back (its skip undoes its step count)
        prev.value()
    if hasattr(model.optimizer, 'clip_and_step'):
        model.optimizer.clip_and_step(clip_grad_norm if clip_grad_norm > 0 else 0.0, guard=guard)
    else:
        if guard is not None and int(guard.max().item()):
            if ok:
                STEP_STATS['recurrence_give_ups'] += 1
            return _skipped(model, n_losses, 'persistent recurrence gave up')
        if clip_grad_norm > 0:
            torch.nn.utils.clip_grad_norm_(model.parameters(), clip_grad_norm)
        model.optimizer.step()
    # ONE host read for the losses and the guard (each .item() is a full sync)
    parts = [l.detach().reshape(-1)[:1].float() for l in losses] if losses is not None else []
    if guard is not None:
        parts.append(guard.float())
    n_guard = guard.numel() if guard is not None else 0
    if not sync and parts and model.device.type == 'cuda':
        dev_vals = torch.cat(parts)
        host = torch.empty(dev_vals.numel(), dtype=torch.float32, pin_memory=True)
        host.copy_(dev_vals, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        pend = PendingLosses(model, host, ev, n_losses, n_guard, losses is not None)
        model._pending_losses = pend
        return pend
    host = torch.cat(parts).tolist() if parts else []
    vals = _finish(model, host, n_losses, n_guard, losses is not None)
    return vals if sync else _Resolved(vals)


class _Resolved(object):
    """PendingLosses' interface for a step that was read back synchronously."""

    def __init__(self, vals):
        self._vals = vals

    def value(self):
        return self._vals

    def __float__(self):
        return float(self._vals[0])


def _skipped(model, n_losses, why, zero=True):
    STEP_STATS['skipped'] += 1
    logger.warning('!!!Skip mini-batch!!! %s' % why)
    if zero:
        model.zero_grad()
    return [0.] * n_losses


def train_step(model, batch, clip_grad_norm, backend='pytorch', grad_scale=None, sync=True):
    """Returns (model, loss_value) like training_loop.py:27-83.

    grad_scale: data parallel only -- the factor applied to this rank's
    gradient before the sum over ranks: pass shard_batch's local_B / global_B
    (every rank's loss is a mean over its local batch), so the update equals
    the 1-GPU update of the global batch.
    sync=False: loss_value is a PendingLosses (float() / value() read it);
    the step does not wait for the GPU, so consecutive steps queue back to
    back (the update sequence is identical)."""
    vals = _step(model, lambda: [model(batch['xs'], batch['ys'], batch['x_lens'],
                                       batch['y_lens'])], clip_grad_norm, 1, grad_scale, sync)
    if sync:
        return model, vals[0]
    return model, (_Resolved(vals) if isinstance(vals, list) else vals)


def train_hierarchical_step(model, batch, clip_grad_norm, backend='pytorch', grad_scale=None,
                            sync=True):
    """Returns (model, loss, loss_main, loss_sub) like training_loop.py:86-153
    (batch carries ys_sub / y_lens_sub for the sub task).  sync=False:
    returns (model, PendingLosses) (see train_step)."""
    vals = _step(model, lambda: list(model(batch['xs'], batch['ys'], batch['x_lens'],
                                           batch['y_lens'], batch['ys_sub'],
                                           batch['y_lens_sub'])), clip_grad_norm, 3, grad_scale,
                 sync)
    if sync:
        return (model,) + tuple(vals)
    return model, (_Resolved(vals) if isinstance(vals, list) else vals)
