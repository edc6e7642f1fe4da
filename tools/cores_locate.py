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
    'mode2_sc1': dict(env={'ASR_OVERLAP_WGRAD': '2', 'ASR_XG_CELL_SC1': '1'}),
    'mode3': dict(env={'ASR_OVERLAP_WGRAD': '3'}),
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
        if work is not None and any(cur == e for e in no._side_streams.values()):
            work(dg, *a)                          # side stream: the stand-in workload
        else:
            _orig_wgrad(dg, *a)

    def bwd(ctx, dy):
        if DH:
            Bb, Tt = dy.shape[0], dy.shape[1]
            Hh = dy.shape[2] // 2
            dh = torch.full((Bb, Tt, 2, Hh), float('nan'), device=dev)
            sp = torch.zeros(((Bb + 7) // 8, Tt, 2, Hh // 16), dtype=torch.int32, device=dev)
            cl = (torch.full((Bb, Tt, 2, Hh, 12), float('nan'), device=dev)
                  if os.environ.get('DIAG_CELL') == '1' else None)
            N.call('asr_lstm_debug_dh', N.ptr(dh), N.ptr(sp), N.ptr(cl), N.stream_handle(dev))
            if os.environ.get('DIAG_REPLAY', '0') == '1':
                # (the clones before the recurrence launch change its timing:
                # the perturbation then did not reproduce)
                saved = ctx.saved_tensors  # x_op, w_op, lens, w_hh, b_ih, b_hh, act, cst, y_op
                dhs.append((dh, sp, cl, saved[6].detach().clone(), saved[7].detach().clone(),
                            dy.detach().clone(), saved[2].detach().clone()))
            else:
                dhs.append((dh, sp, cl, None, None, None, None))
        out = orig_bwd(ctx, dy)
        if DH:
            N.call('asr_lstm_debug_dh', None, None, None, N.stream_handle(dev))
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


def report_cell(i, ref, got, dg_ref, dg_got, Tn):
    """The first step where the cell's recorded values differ: its computed
    gate gradients, the inputs it used, or only the stored bf16 dG."""
    cr, cg = ref[2], got[2]
    same = (cr == cg) | (torch.isnan(cr) & torch.isnan(cg))
    names = ['d_i', 'd_f', 'd_g', 'd_o', 'ig', 'fg', 'gg', 'og', 'c', 'cp', 'dy', 'dc']
    Bb = cr.shape[0]
    dgr = dg_ref.float().view(Bb, Tn, 2, 4, H).permute(0, 1, 2, 4, 3)
    dgg = dg_got.float().view(Bb, Tn, 2, 4, H).permute(0, 1, 2, 4, 3)
    stored = (dgr != dgg).any(-1)                                   # [B, T, 2, H]
    for dd in (0, 1):
        qs = []
        for what, m in (('cell record', ~same[:, :, dd].all(-1)), ('stored dG', stored[:, :, dd])):
            idx = m.nonzero()
            if idx.numel():
                q = torch.where(torch.tensor(dd == 0), Tn - 1 - idx[:, 1], idx[:, 1])
                qq = int(q.min())
                sel = idx[q == qq]
                qs.append('%s first at step %d (rows %s units %s)' % (
                    what, qq, sorted(set(sel[:, 0].tolist()))[:4], sorted(set(sel[:, 2].tolist()))[:6]))
                if what == 'cell record':
                    b0, t0, j0 = [int(v) for v in sel[0]]
                    fields = [names[k] for k in range(12)
                              if not bool(same[b0, t0, dd, j0, k])]
                    qs.append('   fields differing there: %s  ref %s  got %s' % (
                        fields, [round(float(v), 7) for v in cr[b0, t0, dd, j0]],
                        [round(float(v), 7) for v in cg[b0, t0, dd, j0]]))
        print('   call %d dir%d: %s' % (i, dd, ' | '.join(qs) if qs else 'equal'), flush=True)


def _dec_sig(e):
    neg = torch.signbit(e)
    return torch.where(neg, 1 + e, e), torch.where(neg, -e, 1 - e)


def _dec_tanh(e):
    a = e.abs()
    c = a / 16384.0
    cm = a >= 0.5
    return torch.where(cm, torch.copysign(1 - c, e), e), torch.where(cm, c * (2 - c), 1 - e * e)


def replay_cells(i, rec, dg_stored, Tn, tag):
    """Recompute every cell's gate gradients from the recorded dh_t (what the
    recurrence summed), the saved activations / c / dy and the dc carry, in
    f32 on the device, and compare with the stored bf16 dG: where the kernel's
    stored value departs from this recomputation while dh agrees, the cell
    math or its inputs went wrong.  For the first such cell, test which
    neighbouring inputs (other time steps / rows) explain the stored value."""
    dh, _, _, act, cst, dy, lens = rec
    Bb = dh.shape[0]
    Hh = dh.shape[3]
    a = act.float().view(Bb, Tn, 2, Hh, 4)
    ig, omi = _dec_sig(a[..., 0])
    fg, omf = _dec_sig(a[..., 1])
    gg, omg = _dec_tanh(a[..., 2])
    og, omo = _dec_sig(a[..., 3])
    c = cst.view(Bb, Tn, 2, Hh)
    dgs = dg_stored.float().view(Bb, Tn, 2, 4, Hh).permute(0, 1, 2, 4, 3)     # [B,T,2,H,4]
    L = lens.long().view(Bb, 1)
    worst = []
    for dd in (0, 1):
        dc = torch.zeros(Bb, Hh, device=dh.device)
        for q in range(Tn):
            t = Tn - 1 - q if dd == 0 else q
            tp = t - 1 if dd == 0 else t + 1
            act_m = (t < L).float()
            h = dh[:, t, dd]
            h = torch.nan_to_num(h)
            cc = c[:, t, dd]
            cp = c[:, tp, dd] if 0 <= tp < Tn else torch.zeros_like(cc)
            tc = torch.tanh(cc)
            dcell = dc + h * og[:, t, dd] * (1 - tc * tc)
            d = torch.stack([dcell * gg[:, t, dd] * ig[:, t, dd] * omi[:, t, dd],
                             dcell * cp * fg[:, t, dd] * omf[:, t, dd],
                             dcell * ig[:, t, dd] * omg[:, t, dd],
                             h * tc * og[:, t, dd] * omo[:, t, dd]], -1) * act_m.unsqueeze(-1)
            dc = dcell * fg[:, t, dd] * act_m
            st = dgs[:, t, dd]
            err = (st - d).abs() / (d.abs() + 1e-3 * d.abs().max() + 1e-30)
            m = float(err.max())
            if m > 0.05:
                k = int(err.argmax())
                b0, j0, g0 = k // (Hh * 4), (k // 4) % Hh, k % 4
                worst.append((q, dd, b0, j0, g0, m, float(st[b0, j0, g0]), float(d[b0, j0, g0])))
                # which substituted input explains the stored value?  (dc and
                # dh as recomputed / recorded; activations and c from another
                # frame or row)
                expl = []
                hh = float(h[b0, j0])
                dcv = float((dcell - h * og[:, t, dd] * (1 - tc * tc))[b0, j0])
                for tb in range(max(0, t - 3), min(Tn, t + 4)):
                    for bb in sorted(set([b0, b0 ^ 1, b0 ^ 2, b0 ^ 4, (b0 + 8) % Bb, (b0 - 8) % Bb])):
                        for jj in sorted(set([j0, j0 ^ 1, j0 ^ 8])):
                            for what in ('act', 'c', 'act+c'):
                                A = (bb, tb, dd, jj) if 'act' in what else (b0, t, dd, j0)
                                Cc = (bb, tb, dd, jj) if 'c' in what else (b0, t, dd, j0)
                                if A == (b0, t, dd, j0) and Cc == (b0, t, dd, j0):
                                    continue
                                i_, f_, g_, o_ = ig[A], fg[A], gg[A], og[A]
                                oi, of_, og2, oo = omi[A], omf[A], omg[A], omo[A]
                                cc_ = c[Cc]
                                tp_ = Cc[1] - 1 if dd == 0 else Cc[1] + 1
                                cp_ = c[Cc[0], tp_, dd, Cc[3]] if 0 <= tp_ < Tn else 0.0
                                tc_ = torch.tanh(cc_)
                                dcl = dcv + hh * o_ * (1 - tc_ * tc_)
                                dv = [dcl * g_ * i_ * oi, dcl * cp_ * f_ * of_, dcl * i_ * og2,
                                      hh * tc_ * o_ * oo]
                                e_ = max(abs(float(st[b0, j0, k_]) - float(dv[k_])) /
                                         (abs(float(dv[k_])) + 1e-8) for k_ in range(4))
                                if e_ < 1e-2:
                                    expl.append('%s from (row %d, t %d, unit %d)' % (what, bb, tb, jj))
                print('      stored %s recomputed %s dh %.6e dc %.6e; explained by: %s' % (
                    [round(float(v), 8) for v in st[b0, j0]], [round(float(v), 8) for v in d[b0, j0]],
                    hh, dcv, expl[:6] or 'nothing tried'), flush=True)
                break
    for w in worst:
        print('   call %d %s: first cell whose stored dG departs from the recomputation: step %d dir%d '
              'row %d unit %d gate %d rel %.2e stored %.6e recomputed %.6e' % ((i, tag) + w), flush=True)
    if not worst:
        print('   call %d %s: every stored dG matches the recomputation from the recorded dh' % (i, tag),
              flush=True)


def report_dh(i, ref, got, Tn):
    dref, sref = ref[0], ref[1]
    dgot, sgot = got[0], got[1]
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
                    if i == 1 and dhs[i][2] is not None:
                        report_cell(i, ref[3][i], dhs[i], r, g, T)
                    if i == 1 and dhs[i][3] is not None:
                        replay_cells(i, dhs[i], g, T, tag='got')
                        replay_cells(i, ref[3][i], r, T, tag='ref')
                    fg, _ = first_diffs(r, g, T, 'dG')
                    fh, _ = first_diffs(ref[3][i][0], dhs[i][0], T, 'dh')  # noqa
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
