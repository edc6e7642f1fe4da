"""Bucketed gradient all-reduce overlapped with the backward pass.

The flat gradient buffer (models/pytorch_v3/base.py) holds every BLSTM layer's
weights as one contiguous range (encoders/rnn.py flat_order), so a layer is a
natural bucket: its gradients are final once its weight-gradient GEMMs are
enqueued (native_ops.BLSTMLayerFn.backward notifies 'grads').  The bucket's
collective is issued right after the NEXT layer's backward recurrence has been
enqueued (notification 'recurrence'), so on the device it starts when that
persistent recurrence has finished and runs beside the GEMMs and the
recurrences that follow it.  The stream semantics are RCCL's own:
ProcessGroupNCCL makes its stream wait for the current (compute) stream at
issue time, and ``wait()`` makes the compute stream wait for the collective.

Before each backward recurrence ('pre_recurrence') the compute stream waits
for every collective issued so far (the default; ASR_DP_SERIALIZE=0 lets them
run beside the recurrences).  Rounds 3-4 introduced the wait because
co-resident kernels changed the recurrence's results; round 5 found that
cause -- a gfx950 packed-FP32 operand-selection hazard the library no longer
contains (tools/isa_check.py).  The wait stays the default for
the second reason: the persistent recurrence needs every one of
its work-groups resident at once, and an RCCL kernel spinning on its peer can
hold CUs while the next recurrence registers.  What a timeout does then: the
registered work-groups give up their bounded wait, the recurrence's status
word is set and the step is skipped on EVERY rank (the status word is folded
into the MAX-reduced device guard the fused optimizer reads; train_step counts
it in STEP_STATS['recurrence_give_ups'] / ['skipped'] and logs it) -- never a
silently wrong update.  tests/test_coresidency_gpu.py holds CUs beside a
5x512 backward recurrence for shorter and longer than that wait and checks
both outcomes.  Without RCCL on more than one GPU here, the overlapped form is
measured only with memory traffic and held CUs in its place.

Every rank issues the same buckets in the same canonical order (top layer
first, then the remainder of the buffer), whatever happens during its backward:
buckets are issued strictly in that order, and ``finish`` issues whatever is
left.  A rank whose backward raised still pairs every collective of the others
(its values do not matter: the skip flag that follows discards the step).

Each bucket is scaled by grad_scale (local_B / global_B) on the compute stream
before its SUM, so the reduced gradient equals the 1-GPU gradient of the
global batch for any shard sizes.
"""
import os

import torch
import torch.distributed as dist

from ... import native_ops


class GradBuckets(object):
    def __init__(self, model, grad_scale):
        self.model = model
        self.scale = grad_scale
        flat = model._flat_grad
        self.flat = flat
        base = flat.data_ptr()
        es = flat.element_size()
        total = flat.numel()
        layers = []           # (start, end) element ranges of the BLSTM layers
        enc = getattr(model, 'encoder', None)
        if enc is not None and hasattr(enc, 'flat_order') and hasattr(enc, '_layer_params'):
            for l in range(enc.num_layers):
                ps = [p for pair in enc._layer_params(l) for p in pair]
                starts = [(p.grad.data_ptr() - base) // es for p in ps if p.grad is not None]
                ends = [(p.grad.data_ptr() - base) // es + p.numel() for p in ps
                        if p.grad is not None]
                if len(starts) == len(ps):
                    layers.append((min(starts), max(ends)))
        # canonical order: top layer first (the order the backward produces them)
        self.order = list(reversed(layers))
        covered = sorted(layers)
        rest, pos = [], 0
        for a, b in covered:
            if a > pos:
                rest.append((pos, a))
            pos = max(pos, b)
        if pos < total:
            rest.append((pos, total))
        self.rest = rest
        self.by_start = {a: i for i, (a, b) in enumerate(self.order)}
        self.base, self.es = base, es
        self.ready = [False] * len(self.order)
        self.next = 0          # next bucket (canonical order) to issue
        self.works = []
        self.waited = 0
        self.issued_during_backward = 0

    @classmethod
    def for_model(cls, model, grad_scale):
        return cls(model, grad_scale)

    # ---------------------------------------------------------------- hooks
    def __enter__(self):
        # weight gradients left pending by an earlier failed backward must not
        # be reported into this step's buckets
        native_ops.discard_side_wgrads()
        native_ops.set_grad_ready_hook(self._on_event)
        return self

    def __exit__(self, *exc):
        native_ops.set_grad_ready_hook(None)
        return False

    def _on_event(self, event, arg=None):
        if event == 'pre_recurrence':
            # default (ASR_DP_SERIALIZE=0 turns it off): the compute stream
            # waits for every collective issued so far, so none holds CUs when
            # the persistent recurrence about to be enqueued registers its
            # work-groups (module docstring)
            if os.environ.get('ASR_DP_SERIALIZE', '1') == '0':
                return
            for w in self.works[self.waited:]:
                w.wait()
            self.waited = len(self.works)
        elif event == 'grads':
            start = (arg[0].data_ptr() - self.base) // self.es
            i = self.by_start.get(start)
            if i is not None:
                self.ready[i] = True
        elif event == 'recurrence':
            n = self._issue_ready()
            self.issued_during_backward += n

    def _issue(self, a, b):
        seg = self.flat[a:b]
        if self.scale is not None:
            seg.mul_(self.scale)
        self.works.append(dist.all_reduce(seg, op=dist.ReduceOp.SUM, async_op=True))

    def _issue_ready(self):
        n = 0
        while self.next < len(self.order) and self.ready[self.next]:
            self._issue(*self.order[self.next])
            self.next += 1
            n += 1
        return n

    def finish(self, ok=1):
        """Issue every bucket not issued yet (canonical order), then make the
        compute stream wait for all of them."""
        while self.next < len(self.order):
            self._issue(*self.order[self.next])
            self.next += 1
        for a, b in self.rest:
            self._issue(a, b)
        for w in self.works[self.waited:]:
            w.wait()
        self.works = []
        self.waited = 0
