"""Diagnostic (round 4): where and why do co-resident weight-gradient GEMMs
change the backward recurrence's results?

Runs the 5x512 encoder backward (contracting W_hh, so run-to-run differences
are not chaotic amplification) several times per VARIANT and compares every
layer's bf16 gate gradients dG (what the recurrence writes) and input
gradient dx against a mode-0 reference (weight gradients on the compute
stream; bitwise reproducible).  For each differing layer it reports where the
differing dG elements sit -- utterance row, direction, gate, 16-unit slice
(= the producing work-group), processing step of the first difference per
(row group, direction) -- plus the recurrences' give-up status words.

Variants (the side stream always waits for the next recurrence to be
resident, asr_lstm_wgrad_gate, exactly as ASR_OVERLAP_WGRAD=2):
  mode2        the real small-tile weight-gradient GEMMs (LDS-DMA staging)
  mode2_gen    the same GEMMs on the generic register-staged kernel (no LDS DMA)
  mode2_wt     mode2 with write-through hand-offs (ASR_XG_LOCAL=0)
  copy         side stream: large device copies (HBM / L2 traffic, few launches)
  tiny         side stream: many tiny kernels (kernel-boundary cache actions)
  lds          side stream: the LDS-only co-resident stand-in (asr_diag_lds_spin)

usage: python tools/cores_locate.py [variant ...]   (default: all)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import torch  # noqa: E402

from test_grad_buckets_gpu import _batch, _kw  # noqa: E402
from test_model_ctc import _build  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops as no  # noqa: E402
from pytorch_end2end_speech_recognition_amd import _native as N  # noqa: E402

H = int(os.environ.get('DIAG_H', 512))
L = int(os.environ.get('DIAG_L', 5))
T = int(os.environ.get('DIAG_T', 240))
REPS = int(os.environ.get('DIAG_REPS', 3))
WHH = float(os.environ.get('DIAG_WHH', 0.03))

_orig_wgrad = no._blstm_wgrad


def _side_workload(kind):
    dev = torch.device('cuda', 0)

    def copy(*a):
        src = torch.empty(64 << 20, dtype=torch.float32, device=dev).fill_(1.0)
        dst = torch.empty_like(src)
        for _ in range(6):
            dst.copy_(src)
            src.copy_(dst)

    def tiny(*a):
        x = torch.zeros(1024, device=dev)
        for _ in range(400):
            x.add_(1.0)

    def lds(*a):
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        N.call('asr_diag_lds_spin', 256, 2000, N.ptr(bad), N.stream_handle(dev))
        _lds_bad.append(bad)

    def generic(*a):
        old = os.environ.get('ASR_GEMM_FAST')
        os.environ['ASR_GEMM_FAST'] = '0'
        try:
            _orig_wgrad(*a)
        finally:
            if old is None:
                del os.environ['ASR_GEMM_FAST']
            else:
                os.environ['ASR_GEMM_FAST'] = old

    return {'copy': copy, 'tiny': tiny, 'lds': lds, 'mode2_gen': generic}.get(kind)


_lds_bad = []

VARIANTS = {
    'mode2': dict(env={'ASR_OVERLAP_WGRAD': '2'}),
    'mode2_gen': dict(env={'ASR_OVERLAP_WGRAD': '2'}, side='mode2_gen'),
    'mode2_wt': dict(env={'ASR_OVERLAP_WGRAD': '2', 'ASR_XG_LOCAL': '0'}),
    'copy': dict(env={'ASR_OVERLAP_WGRAD': '2'}, side='copy'),
    'tiny': dict(env={'ASR_OVERLAP_WGRAD': '2'}, side='tiny'),
    'lds': dict(env={'ASR_OVERLAP_WGRAD': '2'}, side='lds'),
}


DH = os.environ.get('DIAG_DH', '1') != '0'


def run_once(sd, batch, env, side=None):
    """One forward + backward; returns per layer-backward call (dG clone, dx)
    and, with DIAG_DH, (dh, spins) per call: every dh_t the backward
    recurrence's cell waves formed and each sweep's spin count."""
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    dgs, dxs, dhs = [], [], []
    orig_bwd = no.BLSTMLayerFn.backward
    work = _side_workload(side) if side else None
    dev = torch.device('cuda', 0)

    def wgrad(dg, *a):
        dgs.append(dg.detach().clone())          # stream-ordered after the recurrence
        cur = torch.cuda.current_stream()
        if work is not None and any(cur == e[0] for e in no._side_streams.values()):
            work(dg, *a)                          # side stream: the stand-in workload
        else:
            _orig_wgrad(dg, *a)

    def bwd(ctx, dy):
        if DH:
            Bb, Tt = dy.shape[0], dy.shape[1]
            Hh = dy.shape[2] // 2
            dh = torch.full((Bb, Tt, 2, Hh), float('nan'), device=dev)
            sp = torch.zeros(((Bb + 7) // 8, Tt, 2, Hh // 16), dtype=torch.int32, device=dev)
            N.call('asr_lstm_debug_dh', N.ptr(dh), N.ptr(sp), N.stream_handle(dev))
            dhs.append((dh, sp))
        out = orig_bwd(ctx, dy)
        if DH:
            N.call('asr_lstm_debug_dh', None, None, N.stream_handle(dev))
        dxs.append(out[0].detach().clone() if out[0] is not None else None)
        return out

    no._blstm_wgrad = wgrad
    no.BLSTMLayerFn.backward = staticmethod(bwd)
    try:
        m = _build(_kw(H, L))
        m.load_state_dict(sd)
        m.set_cuda()
        m.zero_grad()
        no.recurrence_status(torch.device('cuda', 0))
        loss = m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'])
        loss.backward()
        torch.cuda.synchronize()
        st = no.recurrence_status(torch.device('cuda', 0)).tolist()
    finally:
        no._blstm_wgrad = _orig_wgrad
        no.BLSTMLayerFn.backward = orig_bwd
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return dgs, dxs, st, dhs


def locate(ref, got, B, Tn):
    """Where do two dG tensors [B, T, 8H] differ?"""
    d = (ref.float() != got.float())
    n = int(d.sum())
    if n == 0:
        return 'equal'
    idx = d.nonzero()
    b, t, col = idx[:, 0], idx[:, 1], idx[:, 2]
    dirn = col // (4 * H)
    gate = (col % (4 * H)) // H
    unit = col % H
    sl = unit // 16
    # processing step of the backward: forward direction t = T-1-q, reverse t = q
    q = torch.where(dirn == 0, Tn - 1 - t, t)
    rg = b // 8
    first = {}
    for g in range(int(rg.max()) + 1):
        for dd in (0, 1):
            m = (rg == g) & (dirn == dd)
            if bool(m.any()):
                first['rg%d/dir%d' % (g, dd)] = int(q[m].min())
    qmin = int(q.min())
    mq = q == qmin
    rel = float((ref.float() - got.float()).abs().max() / ref.float().abs().max())
    return ('%d elems (%.2e of all), max rel %.2e; rows %s; dirs %s; gates %s; '
            'unit slices %d distinct; first step per (row group, dir) %s; '
            'at the earliest step %d: rows %s slices %s gates %s' % (
                n, n / d.numel(), rel, sorted(set(b.tolist()))[:12],
                torch.bincount(dirn, minlength=2).tolist(),
                torch.bincount(gate, minlength=4).tolist(),
                len(set(sl.tolist())), first, qmin,
                sorted(set(b[mq].tolist())), sorted(set(sl[mq].tolist()))[:16],
                sorted(set(gate[mq].tolist()))))


def first_diffs(ref, got, Tn, kind):
    """Per (row group, direction): the first processing step q whose values
    differ (dG [B, T, 8H] or dh [B, T, 2, H])."""
    if kind == 'dG':
        d = (ref.float() != got.float()).view(ref.shape[0], Tn, 2, 4, H).any(3)
    else:
        d = ~((ref == got) | (torch.isnan(ref) & torch.isnan(got)))
    out = {}
    idx = d.nonzero()
    if idx.numel() == 0:
        return out, idx
    b, t, dirn = idx[:, 0], idx[:, 1], idx[:, 2]
    q = torch.where(dirn == 0, Tn - 1 - t, t)
    for g in range(int(b.max()) // 8 + 1):
        for dd in (0, 1):
            m = (b // 8 == g) & (dirn == dd)
            if bool(m.any()):
                qq = int(q[m].min())
                mm = m & (q == qq)
                out[(g, dd)] = (qq, sorted(set(b[mm].tolist())), sorted(set((idx[mm, 3] // 16).tolist())))
    return out, idx


def report_dh(i, ref, got, Tn):
    (dref, sref), (dgot, sgot) = ref, got
    fd, _ = first_diffs(dref, dgot, Tn, 'dh')
    if not fd:
        print('   call %d dh: equal' % i, flush=True)
        return
    for (g, dd), (q, rows, sl) in sorted(fd.items()):
        t = Tn - 1 - q if dd == 0 else q
        r0 = rows[0]
        u = [s_ * 16 + k for s_ in sl[:1] for k in range(16)]
        a = dref[r0, t, dd, u]
        bq = dgot[r0, t, dd, u]
        print('   call %d dh first diff rg%d dir%d: step %d rows %s slices %s |diff| %.3e (|dh| %.3e) '
              'spins ref %s got %s' % (
                  i, g, dd, q, rows, sl[:8], float((a - bq).abs().max()), float(a.abs().max()),
                  sref[g, q, dd, sl[:4]].tolist(), sgot[g, q, dd, sl[:4]].tolist()), flush=True)


def main():
    names = sys.argv[1:] or list(VARIANTS)
    no.set_compute_dtype('bf16')
    batch = _batch(T=T)
    torch.manual_seed(1623)
    sd = {k: v.clone() for k, v in _build(_kw(H, L)).state_dict().items()}
    for k in sd:
        if 'weight_hh' in k:
            sd[k] = sd[k] * (WHH / 0.1)
    B = batch['xs'].shape[0]
    ref = run_once(sd, batch, {'ASR_OVERLAP_WGRAD': '0'})
    ref2 = run_once(sd, batch, {'ASR_OVERLAP_WGRAD': '0'})
    same = all(torch.equal(a, b) for a, b in zip(ref[0], ref2[0]))
    print('mode0 reproducible: %s  status %s %s' % (same, ref[2], ref2[2]), flush=True)
    for name in names:
        v = VARIANTS[name]
        for rep in range(REPS):
            del _lds_bad[:]
            dgs, dxs, st, dhs = run_once(sd, batch, v['env'], v.get('side'))
            print('== %s rep %d status %s%s' % (
                name, rep, st,
                (' lds-pattern-errors %d' % sum(int(x.item()) for x in _lds_bad)) if _lds_bad else ''),
                flush=True)
            for i, (r, g) in enumerate(zip(ref[0], dgs)):
                print('   call %d dG: %s' % (i, locate(r, g, B, T)), flush=True)
                if DH and i < len(dhs):
                    report_dh(i, ref[3][i], dhs[i], T)
                    fg, _ = first_diffs(r, g, T, 'dG')
                    fh, _ = first_diffs(ref[3][i][0], dhs[i][0], T, 'dh')
                    order = {k: ('dh first' if k in fh and fh[k][0] <= v[0] else 'dG first (dh equal so far)')
                             for k, v in fg.items()}
                    if order:
                        print('   call %d order: %s' % (i, order), flush=True)
            for i, (r, g) in enumerate(zip(ref[1], dxs)):
                if r is not None:
                    print('   call %d dx maxdiff %.3e (max %.3e)' % (
                        i, float((r - g).abs().max()), float(r.abs().max())), flush=True)


if __name__ == '__main__':
    main()
