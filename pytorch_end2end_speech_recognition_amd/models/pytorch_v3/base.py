"""ModelBase: the reference's model base class (models/pytorch_v3/base.py:36-408),
re-designed around ONE flat f32 parameter buffer and ONE flat gradient buffer.

Why flat: the fused optimizer kernel updates every parameter in one HBM pass,
the gradient all-reduce over RCCL is one (or a few large) contiguous
collectives, and the two directions of each bidirectional LSTM layer are laid
out adjacently so one GEMM covers both.  Parameters stay individually named
``nn.Parameter`` views (same state_dict keys as the reference), so checkpoints
interchange.

There is no CPU compute path: models are constructed on the host (parameter
initialisation uses torch's CPU RNG like the reference), then ``set_cuda()``
moves the flat buffers to the GPU.  Calling ``forward`` on a CPU model raises.
"""
import logging
import os
from glob import glob
from os.path import basename, isfile, join

import numpy as np
import torch
import torch.nn as nn

from ... import _native as N
from ... import native_ops as ops

logger = logging.getLogger('training')

_ALIGN = 64  # elements: every flat group starts 256-B aligned

OPTIMIZER_KINDS = {'adam': 0, 'sgd': 1, 'momentum': 2, 'nesterov': 3}
TORCH_ONLY = ('adadelta', 'adagrad', 'rmsprop')


def resolve_pending_losses(model):
    """Read back a train_step(..., sync=False) still in flight, so a skipped
    last step has undone its optimizer step count before anyone records it."""
    pend = getattr(model, '_pending_losses', None)
    if pend is not None:
        pend.value()


def eval_retry(fn):
    """Eval / decode entry points (the is_eval forward the reference's training
    scripts call for the dev loss every print_step, decode, posteriors): when a
    persistent recurrence gives up its bounded wait during the pass
    (check_recurrences raises RecurrenceGaveUp), the pass -- side-effect free:
    BatchNorm on its running statistics, no dropout, no optimizer state -- runs
    once more with a warning; a second give-up raises.  A training forward
    never raises it (its give-ups are handled by the step's device guard), so
    the wrapper changes nothing there."""
    import functools

    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        from ...native_ops import RecurrenceGaveUp
        try:
            return fn(self, *args, **kwargs)
        except RecurrenceGaveUp as e:
            logger.warning('%s: %s; running the pass once more', fn.__name__, e)
        return fn(self, *args, **kwargs)
    return wrapper


def check_recurrences(model):
    """Eval / decode entry points: a persistent recurrence that gave up its
    bounded wait during this pass left invalid outputs -- raise instead of
    returning them (and the status words are consumed here, so the next
    train_step's guard does not skip a healthy batch for it)."""
    if getattr(model, 'device', None) is not None and model.device.type == 'cuda':
        from ... import native_ops
        native_ops.raise_if_recurrence_failed(model.device)


class ModelBase(nn.Module):
    """Base class of CTC / AttentionSeq2seq (reference base.py:36)."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError

    def forward(self, inputs):
        raise NotImplementedError

    # ------------------------------------------------------------------ init
    def init_weights(self, parameter_init, distribution, keys=[None], ignore_keys=[None]):
        """base.py:45-73 (same key filters and distributions)."""
        for name, param in self.named_parameters():
            if keys != [None] and len([k for k in keys if k in name]) == 0:
                continue
            if ignore_keys != [None] and len([k for k in ignore_keys if k in name]) > 0:
                continue
            with torch.no_grad():
                if distribution == 'uniform':
                    nn.init.uniform_(param, a=-parameter_init, b=parameter_init)
                elif distribution == 'normal':
                    assert parameter_init > 0
                    nn.init.normal_(param, mean=0, std=parameter_init)
                elif distribution == 'orthogonal':
                    if param.dim() >= 2:
                        nn.init.orthogonal_(param, gain=1)
                elif distribution == 'constant':
                    nn.init.constant_(param, val=parameter_init)
                else:
                    raise NotImplementedError

    def init_forget_gate_bias_with_one(self):
        """base.py:75-83: forget slice of BOTH bias_ih and bias_hh set to 1."""
        for name, param in self.named_parameters():
            if 'lstm' in name and 'bias' in name:
                n = param.size(0)
                with torch.no_grad():
                    param[n // 4:n // 2].fill_(1.)

    # ------------------------------------------------------------ flat buffer
    def _flat_groups(self):
        """Groups of parameters that must be contiguous, in buffer order."""
        groups, seen = [], set()
        for mod in self.modules():
            fo = getattr(mod, 'flat_order', None)
            if fo is None:
                continue
            for grp in fo():
                groups.append(list(grp))
                seen.update(id(p) for p in grp)
        for _, p in self.named_parameters():
            if id(p) not in seen:
                groups.append([p])
                seen.add(id(p))
        return groups

    def flatten_parameters_(self):
        """Pack every parameter into one flat buffer (call at the end of __init__)."""
        groups = self._flat_groups()
        offsets, off = [], 0
        for grp in groups:
            off = (off + _ALIGN - 1) // _ALIGN * _ALIGN
            for p in grp:
                offsets.append((p, off))
                off += p.numel()
        total = (off + _ALIGN - 1) // _ALIGN * _ALIGN
        dev = next(self.parameters()).device
        flat = torch.zeros(total, dtype=torch.float32, device=dev)
        for p, o in offsets:
            flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
        self._flat_param = flat
        self._flat_grad = torch.zeros_like(flat)
        self._flat_index = [(p, o) for p, o in offsets]
        self._rebind()

    def _rebind(self):
        views = []
        for p, o in self._flat_index:
            n = p.numel()
            p.data = self._flat_param[o:o + n].view(p.shape)
            p.grad = self._flat_grad[o:o + n].view(p.shape)
            views.append((p, p.grad))
        self._grad_views = views

    def _rebind_grads(self):
        """Re-attach only the gradient views something replaced (identity
        checks: the per-step zero_grad path, ~60 parameters)."""
        for p, v in self._grad_views:
            if p.grad is not v:
                p.grad = v

    def flat_view(self, first_param, numel, grad=False):
        """Contiguous view starting at `first_param` (e.g. an LSTM fwd+rev pair)."""
        for p, o in self._flat_index:
            if p is first_param:
                buf = self._flat_grad if grad else self._flat_param
                return buf[o:o + numel]
        raise KeyError('parameter not in the flat buffer')

    def _move(self, device):
        self._flat_param = self._flat_param.to(device)
        self._flat_grad = self._flat_grad.to(device)
        self._rebind()
        for name, buf in list(self.named_buffers()):
            mod = self
            *path, leaf = name.split('.')
            for pth in path:
                mod = getattr(mod, pth)
            mod._buffers[leaf] = buf.to(device)
        if hasattr(self, 'optimizer') and isinstance(self.optimizer, FlatOptimizer):
            self.optimizer._move(device)

    def cuda(self, device=None):
        self._move(torch.device('cuda', device) if isinstance(device, int) else
                   (device or torch.device('cuda', torch.cuda.current_device())))
        return self

    def cpu(self):
        self._move(torch.device('cpu'))
        return self

    def to(self, *args, **kwargs):
        device = torch._C._nn._parse_to(*args, **kwargs)[0]
        if device is not None:
            self._move(device)
        return self

    @property
    def device(self):
        return self._flat_param.device

    def zero_grad(self, set_to_none=False):
        self._flat_grad.zero_()
        self._rebind_grads()

    # ------------------------------------------------------------ properties
    @property
    def num_params_dict(self):
        if not hasattr(self, '_num_params_dict'):
            self._num_params_dict = {n: p.numel() for n, p in self.named_parameters()}
        return self._num_params_dict

    @property
    def total_parameters(self):
        return sum(p.numel() for p in self.parameters())

    @property
    def use_cuda(self):
        return torch.cuda.is_available()

    def set_cuda(self, deterministic=False, benchmark=True):
        """base.py:121-139.  The HIP kernels are deterministic by construction
        (no float atomics on any reduction that feeds a parameter update)."""
        if not self.use_cuda:
            raise N.NativeError('set_cuda: no GPU visible (this framework has no CPU path)')
        self.cuda()
        logger.info('GPU mode (MI355X HIP kernels)')

    def set_precision(self, precision):
        """'fp32' (parity mode) or 'bf16' (MFMA bf16, f32 accumulate / state)."""
        from ... import native_ops
        native_ops.set_compute_dtype(precision)

    # ------------------------------------------------------------ optimizer
    def set_optimizer(self, optimizer, learning_rate_init, weight_decay=0, clip_grad_norm=5,
                      lr_schedule=True, factor=0.1, patience_epoch=5):
        """base.py:141-213.  adam / sgd / momentum / nesterov run the fused HIP
        kernel over the flat buffers; adadelta / adagrad / rmsprop use torch.optim
        on the same parameter views (not on the training hot path)."""
        optimizer = optimizer.lower()
        if optimizer not in OPTIMIZER_KINDS and optimizer not in TORCH_ONLY:
            raise ValueError('Optimizer name should be one of [%s], you provided %s.' %
                             (', '.join(list(OPTIMIZER_KINDS) + list(TORCH_ONLY)), optimizer))
        if optimizer in OPTIMIZER_KINDS:
            self.optimizer = FlatOptimizer(self, optimizer, learning_rate_init, weight_decay)
        elif optimizer == 'adadelta':
            self.optimizer = torch.optim.Adadelta(self.parameters(), rho=0.95, eps=1e-8,
                                                  lr=learning_rate_init,
                                                  weight_decay=weight_decay)
        elif optimizer == 'adagrad':
            self.optimizer = torch.optim.Adagrad(self.parameters(), lr=learning_rate_init,
                                                 weight_decay=weight_decay)
        else:
            self.optimizer = torch.optim.RMSprop(self.parameters(), lr=learning_rate_init,
                                                 weight_decay=weight_decay)
        if lr_schedule:
            return torch.optim.lr_scheduler.ReduceLROnPlateau(
                self.optimizer, mode='min', factor=factor, patience=patience_epoch,
                threshold=0.0001, threshold_mode='rel', cooldown=0, min_lr=0, eps=1e-08)
        return None

    # ------------------------------------------------------------ checkpoints
    def set_save_path(self, save_path):
        """base.py:215-230."""
        model_index, tmp = 0, save_path
        while isfile(join(tmp, 'complete.txt')) or isfile(join(tmp, 'config.yml')):
            model_index += 1
            tmp = save_path + '_' + str(model_index)
        os.makedirs(tmp, exist_ok=True)
        self.save_path = tmp

    def save_checkpoint(self, save_path, epoch, step, lr, metric_dev_best,
                        remove_old_checkpoints=False):
        """base.py:232-264: same file name and dict keys (state_dict keys match
        the reference's, so checkpoints interchange)."""
        model_path = join(save_path, 'model.epoch-' + str(epoch))
        if remove_old_checkpoints:
            for path in glob(join(save_path, 'model.epoch-*')):
                os.remove(path)
        resolve_pending_losses(self)
        sd = {k: v.detach().cpu().clone() for k, v in self.state_dict().items()}
        checkpoint = {'state_dict': sd, 'optimizer': self.optimizer.state_dict(), 'epoch': epoch,
                      'step': step, 'lr': lr, 'metric_dev_best': metric_dev_best}
        torch.save(checkpoint, model_path)
        logger.info('=> Saved checkpoint (epoch:%d): %s' % (epoch, model_path))
        return model_path

    def load_checkpoint(self, save_path, epoch=-1, restart=False, load_pretrained_model=False):
        """base.py:266-341.  Loads with weights_only=True (no pickle code runs)."""
        if int(epoch) == -1:
            epochs = [(int(basename(x).split('-')[-1]), x) for x in glob(join(save_path, 'model.*'))]
            if len(epochs) == 0:
                raise ValueError
            epoch = sorted(epochs, key=lambda x: x[0])[-1][0]
        model_path = join(save_path, 'model.epoch-' + str(epoch))
        if not isfile(model_path):
            raise ValueError('No checkpoint found at %s' % model_path)
        checkpoint = torch.load(model_path, map_location='cpu', weights_only=True)
        if load_pretrained_model:
            own = self.state_dict()
            pre = {k: v for k, v in checkpoint['state_dict'].items()
                   if k in own and v.size() == own[k].size()}
            own.update(pre)
            self.load_state_dict(own)
        else:
            self.load_state_dict(checkpoint['state_dict'])
        if restart:
            if not hasattr(self, 'optimizer'):
                raise ValueError('Set optimizer.')
            self.optimizer.load_state_dict(checkpoint['optimizer'])
        return (checkpoint['epoch'] + 1, checkpoint['step'] + 1, checkpoint['lr'],
                checkpoint['metric_dev_best'])

    # ------------------------------------------------------------ host glue
    def np2var(self, array, dtype=None, cpu=False):
        """base.py:362-390: numpy -> tensor (pinned + async H2D when on GPU).
        A tensor already on the model's device (utils/dataset/device_batch.py)
        passes through without a copy."""
        if torch.is_tensor(array) and not cpu and array.device == self.device:
            if dtype == 'float' and array.dtype != torch.float32:
                return array.float()
            if dtype == 'int' and array.dtype != torch.int32:
                return array.int()
            if dtype == 'long' and array.dtype != torch.int64:
                return array.long()
            return array
        if isinstance(array, list):
            array = np.array(array)
        t = torch.from_numpy(np.ascontiguousarray(array))
        if dtype == 'float':
            t = t.float()
        elif dtype == 'long':
            t = t.long()
        elif dtype == 'int':
            t = t.int()
        if not cpu and self.device.type == 'cuda':
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t

    def var2np(self, var):
        return var.detach().cpu().numpy()

    def tensor2np(self, x):
        return x.cpu().numpy()


class FlatOptimizer(torch.optim.Optimizer):
    """Adam / SGD / momentum / nesterov over the model's flat buffers in one
    fused HIP kernel, with the global-norm gradient clip folded in (the clip
    coefficient never leaves the device)."""

    def __init__(self, model, kind, lr, weight_decay=0, betas=(0.9, 0.999), eps=1e-8,
                 momentum=0.9):
        super().__init__(model.parameters(), dict(lr=lr, weight_decay=weight_decay, betas=betas,
                                                  eps=eps, momentum=momentum))
        self.model = model
        self.kind = kind
        self._step = 0
        self._alloc(model._flat_param.device)

    def _alloc(self, device):
        n = self.model._flat_param.numel()
        self.m = torch.zeros(n, dtype=torch.float32, device=device)
        self.v = (torch.zeros(n, dtype=torch.float32, device=device) if self.kind == 'adam'
                  else None)
        self._sq = torch.zeros(1, dtype=torch.float32, device=device)

    def _move(self, device):
        self.m = self.m.to(device)
        if self.v is not None:
            self.v = self.v.to(device)
        self._sq = self._sq.to(device)

    def zero_grad(self, set_to_none=False):
        self.model.zero_grad()

    def grad_norm_sq(self):
        """Device scalar sum(g^2) over the flat gradient (no host sync)."""
        g = self.model._flat_grad
        nb = N.query('asr_grad_sqnorm_workspace_bytes')
        ws = torch.empty(nb, dtype=torch.uint8, device=g.device)
        N.call('asr_grad_sqnorm', N.ptr(g), g.numel(), N.ptr(self._sq), N.ptr(ws), nb,
               N.stream_handle(g.device))
        return self._sq

    @torch.no_grad()
    def step(self, closure=None, max_norm=0.0, guard=None):
        """guard: optional device int32[2] (asr_lstm_status_gather words, MAX
        over ranks); when nonzero the kernel leaves params and state alone."""
        loss = closure() if closure is not None else None
        self._step += 1
        g = self.param_groups[0]
        p, gr = self.model._flat_param, self.model._flat_grad
        sq = self.grad_norm_sq() if max_norm and max_norm > 0 else None
        N.require_device(p)
        b1, b2 = g['betas']
        # bf16 mode: the kernel also writes the bf16 shadow the next forward's
        # BLSTM layers stage W_ih from (native_ops.param_shadow)
        sh = ops.param_shadow(p)
        N.call('asr_optim_step_guarded', OPTIMIZER_KINDS[self.kind], N.ptr(p), N.ptr(gr),
               N.ptr(self.m), N.ptr(self.v), p.numel(), float(g['lr']), float(b1), float(b2),
               float(g['eps']), float(g['weight_decay']), self._step, float(g['momentum']), 0.0,
               N.ptr(sq), float(max_norm or 0.0), N.ptr(sh.buf) if sh is not None else None,
               N.ptr(guard), N.stream_handle(p.device))
        if sh is not None:
            ops.param_shadow_written(sh, p, self.model.parameters())
        return loss

    def clip_and_step(self, max_norm, guard=None):
        return self.step(max_norm=max_norm, guard=guard)

    def undo_step_count(self):
        """A guarded step that did not update (skipped batch) must not advance
        Adam's bias-correction count."""
        self._step -= 1

    # ------------------------------------------------------- checkpoints
    def _param_slices(self):
        """(index, param, offset) in model.parameters() order -- the order
        torch.optim numbers parameters in its state_dict."""
        offs = {id(p): o for p, o in self.model._flat_index}
        return [(i, p, offs[id(p)]) for i, p in enumerate(self.model.parameters())]

    def state_dict(self):
        """torch.optim.Adam / SGD state_dict format (what the reference's
        save_checkpoint stores, base.py:232-264): per-parameter 'step',
        'exp_avg', 'exp_avg_sq' (Adam) or 'momentum_buffer' (momentum /
        nesterov), views of the flat state buffers, and one param group."""
        resolve_pending_losses(self.model)   # a skipped last step undoes its count first
        g = self.param_groups[0]
        state = {}
        for i, p, o in self._param_slices():
            n = p.numel()
            if self.kind == 'adam':
                if self._step == 0:
                    continue
                state[i] = {'step': torch.tensor(float(self._step)),
                            'exp_avg': self.m[o:o + n].view(p.shape).detach().cpu().clone(),
                            'exp_avg_sq': self.v[o:o + n].view(p.shape).detach().cpu().clone()}
            elif self.kind in ('momentum', 'nesterov') and self._step > 0:
                state[i] = {'momentum_buffer':
                            self.m[o:o + n].view(p.shape).detach().cpu().clone()}
        group = {'lr': g['lr'], 'weight_decay': g['weight_decay'],
                 'params': [i for i, _, _ in self._param_slices()]}
        if self.kind == 'adam':
            group.update(betas=tuple(g['betas']), eps=g['eps'], amsgrad=False,
                         maximize=False, foreach=None, capturable=False, differentiable=False,
                         fused=None)
        else:
            group.update(momentum=g['momentum'] if self.kind != 'sgd' else 0, dampening=0,
                         nesterov=self.kind == 'nesterov', maximize=False, foreach=None,
                         differentiable=False, fused=None)
        return {'state': state, 'param_groups': [group], 'flat_kind': self.kind}

    def load_state_dict(self, sd):
        """Accepts torch.optim.Adam / SGD state_dicts (a reference checkpoint,
        torch 0.3 int steps or torch 2.x tensor steps) and this class's own."""
        if 'kind' in sd and 'm' in sd:            # round-1 flat format
            self._step = int(sd['step'])
            self.param_groups[0]['lr'] = sd['lr']
            self.m.copy_(sd['m'].to(self.m.device))
            if self.v is not None and sd.get('v') is not None:
                self.v.copy_(sd['v'].to(self.v.device))
            return
        grp = sd['param_groups'][0]
        for k in ('lr', 'weight_decay', 'eps', 'momentum'):
            if k in grp:
                self.param_groups[0][k] = grp[k]
        if 'betas' in grp:
            self.param_groups[0]['betas'] = tuple(grp['betas'])
        state = sd['state']
        steps = []
        with torch.no_grad():
            self.m.zero_()
            if self.v is not None:
                self.v.zero_()
            for i, p, o in self._param_slices():
                st = state.get(grp['params'][i] if i < len(grp['params']) else i)
                if st is None:
                    continue
                n = p.numel()
                if 'exp_avg' in st:
                    self.m[o:o + n].copy_(st['exp_avg'].reshape(-1).to(self.m.device))
                    self.v[o:o + n].copy_(st['exp_avg_sq'].reshape(-1).to(self.v.device))
                elif st.get('momentum_buffer') is not None:
                    self.m[o:o + n].copy_(st['momentum_buffer'].reshape(-1).to(self.m.device))
                if 'step' in st:
                    steps.append(int(float(st['step'])))
        self._step = max(steps) if steps else 0
