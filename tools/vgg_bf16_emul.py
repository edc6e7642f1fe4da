"""CPU emulation (float64 + explicit bf16 rounding points) of the VGG
front-end's backward at the bf16 parity pin's shape (tests/test_parity_pins_gpu
_vgg_bf16_case: [64, 64, 128, 128], BatchNorm, B = 8 x 101 frames x 40 bins):
which bf16 storage point puts the 0.08-0.13 relative L2 error on the gradients
below the BatchNorm layers (VERDICT r03 "What's weak" #2)?

Rounding points (each on / off):
  x    conv input operand (features, layer inputs) and the conv weights, bf16
  z    conv output stored bf16 (forward)
  dz   gradient of the conv output (the dgrad / wgrad GEMM operand), bf16
  dx   input gradient of a conv (the layer below's BN-backward input), bf16
  dout gradient arriving at the VGG output (upstream bf16 encoder), bf16

usage: python tools/vgg_bf16_emul.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

Fn = torch.nn.functional


def rb(t):
    return t.to(torch.bfloat16).to(t.dtype)


class Q(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, fwd, bwd):
        ctx.bwd = bwd
        return rb(x) if fwd else x.clone()

    @staticmethod
    def backward(ctx, g):
        return (rb(g) if ctx.bwd else g), None, None


def vgg(p, xs, flags, channels, poolings, dec=None, rec=None):
    """dec: the ReLU masks and pool argmax indices of another pass to replay
    (rec: where this pass records its own)."""
    x = xs.transpose(1, 2).unsqueeze(1)
    idx, first = 0, True
    for l, C in enumerate(channels):
        conv = 'encoder.conv.layers.%d.' % idx
        xq = Q.apply(x, 'x' in flags or 'x%d' % l in flags, 'dx' in flags and l > 0)
        wq = Q.apply(p[conv + 'weight'], 'x' in flags or 'w%d' % l in flags, False)
        z = Fn.conv2d(xq, wq, p.get(conv + 'bias'), stride=1, padding=1)
        z = Q.apply(z, 'z' in flags or 'z%d' % l in flags, 'dz' in flags)
        idx += 2
        mask = (z > 0) if dec is None else dec[('relu', l)]
        if rec is not None:
            rec[('relu', l)] = mask
        x = z * mask
        pl = poolings[l]
        if len(pl):
            _, ind = Fn.max_pool2d(x.detach(), kernel_size=tuple(pl), stride=tuple(pl),
                                   ceil_mode=not first, return_indices=True)
            if dec is not None:
                ind = dec[('pool', l)]
            if rec is not None:
                rec[('pool', l)] = ind
            Bq, Cq, Hq, Wq = x.shape
            x = x.flatten(2).gather(2, ind.flatten(2)).view(ind.shape)
            first = False
            idx += 1
        bn = 'encoder.conv.layers.%d.' % idx
        x = Fn.batch_norm(x, torch.zeros(C, dtype=x.dtype), torch.ones(C, dtype=x.dtype),
                          p[bn + 'weight'], p[bn + 'bias'], training=True)
        idx += 2
    B, C, Fo, To = x.shape
    return x.transpose(1, 3).reshape(B, To, Fo * C)


def main():
    from test_parity_pins_gpu import VGG_PROD, _ctc
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    kw = dict(VGG_PROD, input_size=40)
    model = _ctc(kw)
    sd = {k: v.detach().double() for k, v in model.state_dict().items()}
    rng = np.random.RandomState(21)
    B, T = 8, 101
    x_lens = np.sort(rng.randint(70, T + 1, B))[::-1].astype(np.int32)
    x_lens[0] = T
    xs = rng.randn(B, T, 40)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    xs = torch.from_numpy(xs)
    # the upstream gradient: a fixed random direction of the VGG output's shape
    # scaled like a CTC gradient (its structure is what the BN backward sees)
    ch, pools = kw['conv_channels'], kw['poolings']
    keys = [k for k in sd if k.startswith('encoder.conv') and 'running' not in k and
            'num_batches' not in k]

    replay = os.environ.get('EMUL_REPLAY') == '1'
    dec0 = {}
    vgg(sd, xs, (), ch, pools, rec=dec0)

    def grads(flags, dout):
        p = {k: (v.clone().requires_grad_(True) if k in keys else v) for k, v in sd.items()}
        out = vgg(p, xs, flags, ch, pools, dec=dec0 if replay else None)
        g = Q.apply(dout, 'dout' in flags, False)
        out.backward(g)
        return {k: p[k].grad.clone() for k in keys}

    out0 = vgg(sd, xs, (), ch, pools)
    g = torch.Generator().manual_seed(5)
    dout = torch.randn(out0.shape, generator=g, dtype=torch.float64) * 1e-3
    ref = grads((), dout)
    configs = [tuple(c.split('+')) for c in (sys.argv[1:] or [
        'x', 'z', 'dz', 'dx', 'dout', 'x+z', 'dz+dx', 'x+z+dz', 'x+z+dz+dx+dout'])]
    for flags in configs:
        got = grads(flags, dout)
        errs = {k: float((got[k] - ref[k]).norm() / ref[k].norm()) for k in keys}
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
        print('%-28s worst: %s' % ('+'.join(flags), ', '.join('%s %.2e' % (k.replace(
            'encoder.conv.layers.', ''), e) for k, e in worst)), flush=True)


if __name__ == '__main__':
    main()
