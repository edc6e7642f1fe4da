#!/usr/bin/env python
"""Training-throughput benchmark of the MI355X hybrid CTC/attention step.

Workload (BASELINE.json configs[1]): LibriSpeech-100h char CTC, 5-layer
bidirectional LSTM, 512 units per direction, no subsampling, dropout 0.2, Adam
lr 1e-3 wd 1e-6, clip 5.0; per GPU B = 32 synthetic utterances of 80-dim fbank,
x_lens ~ U[800, 1000] sorted descending (x_lens[0] = 1000), char labels
U[0, 27] (V = 28 + blank), y_lens ~ U[60, 125].  One step = the
reference's full train_step: H2D of the numpy batch, forward, CTC loss,
backward, RCCL gradient all-reduce (N > 1), fused global-norm clip + Adam, loss
read back.  Weak scaling: B = 32 per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints ONE JSON line (rank 0) with the metric, a live roofline of the dominant
kernel (per-launch HIP events on the kernel's own stream) and the CPU oracle
baseline timed on this host.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from pytorch_end2end_speech_recognition_amd import _native as N  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops  # noqa: E402
from pytorch_end2end_speech_recognition_amd.models.load_model import load  # noqa: E402
from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import (  # noqa: E402
    train_hierarchical_step, train_step)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
BF16_PEAK_TFLOPS = 2500.0    # dense bf16 MFMA (spec, no sparsity)

CONFIGS = {
    'ctc5x512': dict(
        workload='librispeech100h_char_ctc_blstm5x512', model_type='ctc',
        params=dict(input_freq=80, use_delta=False, use_double_delta=False, input_channel=1,
                    splice=1, num_stack=1, encoder_type='lstm', conv_channels=[],
                    conv_kernel_sizes=[], conv_strides=[], poolings=[], activation='relu',
                    batch_norm=False, encoder_bidirectional=True, encoder_residual=False,
                    encoder_dense_residual=False, encoder_num_units=512, encoder_num_proj=0,
                    encoder_num_layers=5, subsample_list=[], subsample_type='drop', fc_list=[],
                    optimizer='adam', learning_rate=1e-3, parameter_init_distribution='uniform',
                    parameter_init=0.1, recurrent_weight_orthogonal=False,
                    init_forget_gate_bias_with_one=True, char_init=False, clip_grad_norm=5.0,
                    dropout_input=0, dropout_encoder=0.2, weight_decay=1e-6,
                    logits_temperature=1, label_smoothing_prob=0, weight_noise_std=0,
                    num_classes=28)),
}


def _attention_params(ctc_weight):
    """configs[2] / configs[3]: the reference's LibriSpeech-100h location-attention
    recipe (examples/librispeech/s5/conf/attention/char_blstm_att_100h.yml, kept
    as the fixture tests/golden/char_blstm_att_100h.yml): 4x320 BLSTM with x4
    drop subsampling, location attention (128, 10 ch x 201), LSTM decoder 320,
    embedding 32, dropout 0.2 everywhere, scheduled sampling 0.2; hybrid adds
    lambda * CTC."""
    import yaml
    with open(os.path.join(ROOT, 'tests', 'golden', 'char_blstm_att_100h.yml')) as f:
        prm = yaml.safe_load(f)['param']
    prm.update(num_classes=28, ctc_loss_weight=ctc_weight)
    for k in ('learning_rate', 'weight_decay'):
        prm[k] = float(prm[k])
    return prm


CONFIGS['att4x320'] = dict(workload='librispeech100h_char_location_attention_blstm4x320',
                           model_type='attention', params=None, ctc_weight=0.0)
CONFIGS['hybrid4x320'] = dict(workload='librispeech_char_hybrid_ctc0.3_attention_blstm4x320',
                              model_type='attention', params=None, ctc_weight=0.3)


CONFIGS['vgg_hier'] = dict(
    workload='swbd_vgg_blstm4x320_hierarchical_word10k_char_ctc', model_type='hierarchical_ctc',
    params=dict(
        input_freq=80, use_delta=False, use_double_delta=False, input_channel=1, splice=1,
        num_stack=1, encoder_type='lstm', conv_channels=[64, 64, 128, 128],
        conv_kernel_sizes=[[3, 3]] * 4, conv_strides=[[1, 1]] * 4,
        poolings=[[], [2, 2], [], [2, 2]], activation='relu', batch_norm=True,
        encoder_bidirectional=True, encoder_residual=False, encoder_dense_residual=False,
        encoder_num_units=320, encoder_num_proj=0, encoder_num_layers=4,
        encoder_num_layers_sub=3, subsample_list=[], subsample_type='drop', fc_list=[],
        fc_list_sub=[], main_loss_weight=0.5, sub_loss_weight=0.5, optimizer='adam',
        learning_rate=1e-3, parameter_init_distribution='uniform', parameter_init=0.1,
        recurrent_weight_orthogonal=False, init_forget_gate_bias_with_one=True, char_init=False,
        clip_grad_norm=5.0, dropout_input=0, dropout_encoder=0.2, weight_decay=1e-6,
        logits_temperature=1, label_smoothing_prob=0, weight_noise_std=0,
        num_classes=10000, num_classes_sub=28))


def config_params(cfg):
    if cfg['params'] is None:
        cfg['params'] = _attention_params(cfg['ctc_weight'])
    return cfg['params']


def synthetic_batch(B, T, F, num_classes, seed):
    """SURVEY §8d synthetic inputs (numpy seed per rank)."""
    rng = np.random.RandomState(seed)
    x_lens = np.sort(rng.randint(800, T + 1, B))[::-1].astype(np.int32)
    x_lens[0] = T
    xs = rng.randn(B, T, F).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    y_lens = rng.randint(60, 126, B).astype(np.int32)
    ys = np.full((B, int(y_lens.max())), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, num_classes, y_lens[b])
    return dict(xs=xs, ys=ys, x_lens=x_lens, y_lens=y_lens)


def synthetic_hier_batch(B, T, F, num_words, num_chars, seed):
    """configs[4]: word targets (U[10, 25] words of a synthetic 10k vocabulary)
    for the main CTC, char targets (U[60, 125]) for the sub-task CTC."""
    batch = synthetic_batch(B, T, F, num_chars, seed)
    batch['ys_sub'], batch['y_lens_sub'] = batch.pop('ys'), batch.pop('y_lens')
    rng = np.random.RandomState(seed + 7919)
    y_lens = rng.randint(10, 26, B).astype(np.int32)
    ys = np.full((B, int(y_lens.max())), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, num_words, y_lens[b])
    batch['ys'], batch['y_lens'] = ys, y_lens
    return batch


def roofline_report(args, p, mean_us, launches, mean_work, workload):
    """Roofline of the dominant kernel (largest mean launch time x launches over
    the timed steps), from HIP-event timings taken on the kernels' own stream by
    the library's prof hooks (asr_prof_*).  Algorithmic work per launch:
      * lstm_{fwd,bwd}_pass (persistent, one launch = one layer pass, T steps x
        2 directions): HBM bytes that must move once -- gx / gate activations /
        y / c / dy read or written once per (b, t) cell plus W_hh once -- and
        the recurrent h @ W_hh^T flops;
      * lstm_{fwd,bwd}_step (per-step kernels): the same per time step, W_hh
        re-streamed every step;
      * gemm: 2*M*N*K summed over the launch's problems, reported by the library.
    """
    B, H = args.batch, p['encoder_num_units']
    # time steps of a layer pass, averaged over the layers (pyramidal drop
    # subsampling halves T after each flagged layer, rnn.py:413-439)
    t = args.frames
    for pool in p.get('poolings') or []:    # VGG front-end time pooling (ConvOutSize floor)
        if len(pool):
            t = (t - pool[1]) // pool[1] + 1
    T_l = []
    for flag in (p.get('subsample_list') or [False] * p['encoder_num_layers']):
        T_l.append(t)
        t = t // 2 if flag else t
    T = sum(T_l) / len(T_l)
    esz = 2 if args.precision == 'bf16' else 4
    cell = B * H                              # (utterance, unit) cells per direction
    w_hh = 2 * 4 * H * H * esz                # both directions
    flops_step = 2 * 2 * B * 4 * H * H        # h @ W_hh^T, 2 directions
    fwd_cell = 4 * 4 * 2 + 4 * 2              # gx read + act write (4 gates f32), y + c write
    bwd_cell = 4 * 4 * 2 + 4 * 3              # act read + dG write, dy + c_t + c_{t-1} read
    kinds = [
        ('lstm_fwd_step', 'hbm', 2 * cell * fwd_cell + w_hh, flops_step),
        ('lstm_bwd_step', 'hbm', 2 * cell * bwd_cell + w_hh, flops_step),
        ('lstm_fwd_pass', 'hbm', T * 2 * cell * fwd_cell + w_hh, T * flops_step),
        ('lstm_bwd_pass', 'hbm', T * 2 * cell * bwd_cell + w_hh, T * flops_step),
        ('gemm', 'mfma', 0, mean_work[4]),
        ('ctc_fwd', 'hbm', mean_work[5], 0.0),
        ('ctc_grad', 'hbm', mean_work[6], 0.0),
    ]
    rows = []
    for i, (name, bound, nbytes, flops) in enumerate(kinds):
        us = mean_us[i]
        if us <= 0 or launches[i] == 0:
            continue
        gbs = nbytes / (us * 1e-6) / 1e9
        tfs = flops / (us * 1e-6) / 1e12
        rows.append(dict(name=name, bound=bound, us=us, n=int(launches[i]), bytes=nbytes,
                         flops=flops, gbs=gbs, tfs=tfs, total=us * launches[i]))
    if not rows:
        return None
    dom = max(rows, key=lambda r: r['total'])

    def view(r):
        if r['bound'] == 'mfma':
            return {'achieved': round(r['tfs'], 2), 'peak': BF16_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                    'frac': round(r['tfs'] / BF16_PEAK_TFLOPS, 4)}
        return {'achieved': round(r['gbs'], 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(r['gbs'] / HBM_PEAK_GBS, 4)}

    out = {'bound': dom['bound']}
    out.update(view(dom))
    traffic, tsrc = pmc_traffic(dom['name'], workload)
    out.update({'traffic': traffic, 'kernel': dom['name'], 'mean_launch_us': round(dom['us'], 3),
                'launches_timed': dom['n'],
                'algorithmic_bytes_per_launch': int(dom['bytes']),
                'algorithmic_flops_per_launch': float(dom['flops']),
                'share_of_timed_kernel_time': round(dom['total'] / sum(r['total'] for r in rows),
                                                    3)})
    if tsrc:
        out['traffic_source'] = tsrc
    others = {}
    for r in rows:
        if r is dom:
            continue
        v = {'bound': r['bound'], 'mean_launch_us': round(r['us'], 3), 'launches': r['n']}
        v.update(view(r))
        if r['name'].startswith('lstm'):
            v['mfma_tflops'] = round(r['tfs'], 2)
            if r['name'].endswith('_pass'):
                v['us_per_time_step'] = round(r['us'] / T, 3)
        others[r['name']] = v
    out['other_kernels'] = others
    return out


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/rNN_pmc_traffic.json, written by tools/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench's
    own command; counters cannot be read inside the timed run).  (None, None)
    when no summary covers the kernel."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_pmc_traffic.json')))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get('_workload', 'librispeech100h_char_ctc_blstm5x512') != workload:
            continue
        if kernel in d:
            return d[kernel]['traffic_bytes_per_launch'], os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(cfg, batch, n_utts):
    """Oracle (torch-CPU restatement of the reference path) on a bounded sample:
    the first n_utts utterances of this rank's batch, one full training step
    (forward, backward, clip, Adam)."""
    from oracle import asr_ref
    cores = len(os.sched_getaffinity(0))
    threads = max(1, min(16, cores))
    torch.set_num_threads(threads)
    p = config_params(cfg)
    torch.manual_seed(0)
    model = load(cfg['model_type'], dict(p), 'pytorch')           # host-side init only
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    trainable = [v.requires_grad_(True) for k, v in sd.items()
                 if v.is_floating_point() and 'running' not in k]
    opt = torch.optim.Adam(trainable, lr=p['learning_rate'], weight_decay=p['weight_decay'])
    sub = {k: v[:n_utts] for k, v in batch.items()}
    sub['ys'] = sub['ys'][:, :int(sub['y_lens'].max())]
    if 'ys_sub' in sub:
        sub['ys_sub'] = sub['ys_sub'][:, :int(sub['y_lens_sub'].max())]
    t0 = time.perf_counter()
    opt.zero_grad()
    if cfg['model_type'] == 'hierarchical_ctc':
        ocfg = dict(num_layers=p['encoder_num_layers'], num_layers_sub=p['encoder_num_layers_sub'],
                    subsample_list=p['subsample_list'], conv_channels=p['conv_channels'],
                    poolings=p['poolings'], batch_norm=p['batch_norm'],
                    main_loss_weight=p['main_loss_weight'], sub_loss_weight=p['sub_loss_weight'])
        loss, _, _ = asr_ref.hierarchical_ctc_loss(sd, ocfg, sub['xs'], sub['ys'], sub['x_lens'],
                                                   sub['y_lens'], sub['ys_sub'],
                                                   sub['y_lens_sub'])
    elif cfg['model_type'] == 'attention':   # oracle decoder: teacher forcing, no dropout
        loss = asr_ref.attention_model_loss(sd, p, sub['xs'], sub['ys'], sub['x_lens'],
                                            sub['y_lens'])
    else:
        ocfg = dict(num_layers=p['encoder_num_layers'], subsample_list=p['subsample_list'],
                    fc_list=p['fc_list'])
        loss, _, _, _ = asr_ref.ctc_model_loss(sd, ocfg, sub['xs'], sub['ys'], sub['x_lens'],
                                               sub['y_lens'])
    loss.backward()
    torch.nn.utils.clip_grad_norm_(trainable, p['clip_grad_norm'])
    opt.step()
    dt = time.perf_counter() - t0
    frames = float(np.sum(sub['x_lens']))
    return {'value': frames / dt, 'unit': 'frames/s', 'cores': threads, 'kind': 'port',
            'sample': '%d utterances x %d max frames (%d frames), 1 full training step (fwd + '
                      'bwd + clip + Adam) of the fp32 torch-CPU oracle%s, %.1f s'
                      % (n_utts, int(sub['x_lens'].max()), int(frames),
                         ' (decoder without dropout / scheduled sampling)'
                         if cfg['model_type'] == 'attention' else '', dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', default='ctc5x512', choices=sorted(CONFIGS))
    ap.add_argument('--precision', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--frames', type=int, default=1000)
    ap.add_argument('--cpu-utts', type=int, default=2)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--prof-stride', type=int, default=8)
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local_rank)
    dev = torch.device('cuda', local_rank)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)

    cfg = CONFIGS[args.config]
    p = dict(config_params(cfg))
    torch.manual_seed(1623)
    native_ops.manual_seed(1623 + rank)
    model = load(cfg['model_type'], p, 'pytorch')
    if world > 1:   # identical initial weights on every rank
        model.set_cuda()
        dist.broadcast(model._flat_param, src=0)
    else:
        model.set_cuda()
    model.set_precision(args.precision)
    model.set_optimizer(p['optimizer'], p['learning_rate'], weight_decay=p['weight_decay'],
                        lr_schedule=False)
    if cfg['model_type'] == 'hierarchical_ctc':
        batch = synthetic_hier_batch(args.batch, args.frames, p['input_freq'], p['num_classes'],
                                     p['num_classes_sub'], seed=rank)

        def step(m, b):
            m, lv, _, _ = train_hierarchical_step(m, b, p['clip_grad_norm'])
            return m, lv
    else:
        batch = synthetic_batch(args.batch, args.frames, p['input_freq'], p['num_classes'],
                                seed=rank)

        def step(m, b):
            return train_step(m, b, p['clip_grad_norm'])
    frames_per_step = float(batch['x_lens'].sum())

    for _ in range(args.warmup):
        model, _ = step(model, batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    N.call('asr_prof_begin', args.prof_stride)
    t0 = time.perf_counter()
    losses = []
    for _ in range(args.steps):
        model, lv = step(model, batch)
        losses.append(lv)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    import ctypes
    NK = 7
    mean_us = (ctypes.c_double * NK)()
    launches = (ctypes.c_longlong * NK)()
    mean_work = (ctypes.c_double * NK)()
    N.call('asr_prof_end', ctypes.cast(mean_us, ctypes.c_void_p),
           ctypes.cast(launches, ctypes.c_void_p), ctypes.cast(mean_work, ctypes.c_void_p), NK)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        fr = torch.tensor([frames_per_step], dtype=torch.float64, device=dev)
        dist.all_reduce(fr, op=dist.ReduceOp.SUM)
        total_frames_per_step = float(fr.item())
    else:
        total_frames_per_step = frames_per_step

    if rank != 0:
        dist.destroy_process_group()
        return

    roofline = roofline_report(args, p, mean_us, launches, mean_work, cfg['workload'])

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, batch, args.cpu_utts)

    value = total_frames_per_step * args.steps / elapsed
    out = {
        'metric': 'training frames/sec', 'value': round(value, 1), 'unit': 'frames/s',
        'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(1000.0 * elapsed / args.steps, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': args.precision, 'data': 'synthetic',
        'config': {'workload': cfg['workload'], 'batch_per_gpu': args.batch,
                   'global_batch': args.batch * world, 'max_frames': args.frames,
                   'feat_dim': p['input_freq'], 'vocab': p['num_classes'] + 1,
                   'parallelism': 'dp%d' % world, 'frames_per_step': total_frames_per_step},
        'loss_last': losses[-1] if losses else None,
        'roofline': roofline,
        'cpu_baseline': cpu,
    }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
