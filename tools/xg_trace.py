"""Per-step phase timing of the tagged-granule recurrence (ASR_XG_TRACE=1):
one forward + backward layer pass at the bench shape, then the median
duration of each phase over steps 8..127 of work-groups 0..3."""
import ctypes
import os
import sys

os.environ['ASR_XG_TRACE'] = '1'
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_end2end_speech_recognition_amd import _native as N  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402

WG, STEPS, K = 64, 128, 12


def read():
    buf = (ctypes.c_ulonglong * (WG * STEPS * K))()
    N.query('asr_xg_trace_read', ctypes.cast(buf, ctypes.c_void_p))
    return np.frombuffer(buf, dtype=np.uint64).reshape(WG, STEPS, K).astype(np.int64)


def hop(name, tr, pub_k):
    """Per group (k=7 ids) and step: last producer publish (k=pub_k) -> each
    consumer's issue of its successful poll (k=6) and its success (k=1)."""
    ids = tr[:, 20, 7]
    grp = ids // 256
    lat_iss, lat_ok, late = [], [], []
    for g in np.unique(grp):
        mem = np.where(grp == g)[0]
        if len(mem) < 2:
            continue
        for s in range(8, STEPS - 1):
            last_pub = tr[mem, s, pub_k].max()
            for m in mem:
                lat_ok.append(tr[m, s + 1, 1] - last_pub)
                lat_iss.append(tr[m, s + 1, 6] - last_pub)
    lat_ok, lat_iss = np.array(lat_ok) / 100.0, np.array(lat_iss) / 100.0
    print('%s: last publish -> poll success median %.2f us (p10 %.2f, p90 %.2f); '
          '-> issue of the successful poll median %.2f us' % (
              name, np.median(lat_ok), np.percentile(lat_ok, 10), np.percentile(lat_ok, 90),
              np.median(lat_iss)))


def report(name, tr, names):
    print(name)
    for w in range(4):
        d = tr[w, 8:]
        step = np.diff(d[:, 0])
        parts = ['step %.2f us' % (np.median(step) / 100.0)]
        for a, b, nm in names:
            parts.append('%s %.2f' % (nm, np.median(d[:, b] - d[:, a]) / 100.0))
        parts.append('spins %.0f' % np.median(d[:, 5]))
        print('  wg%d ' % w + '  '.join(parts))


def main():
    B, T, H, Din = 32, 1000, 512, 1024
    ops.set_compute_dtype('bf16')
    dev = torch.device('cuda:0')
    rng = np.random.RandomState(0)
    x = torch.from_numpy(rng.randn(B, T, Din).astype(np.float32)).to(dev).requires_grad_(True)
    ws = [torch.from_numpy(rng.uniform(-0.1, 0.1, s).astype(np.float32)).to(dev).requires_grad_(True)
          for s in ((8 * H, Din), (8 * H, H), (8 * H,), (8 * H,))]
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    bwd = None
    for _ in range(2):
        y = ops.blstm_layer(x, lens, T, *ws)
        torch.cuda.synchronize()
        fwd = read()
        if bwd is not None and np.array_equal(fwd, bwd):
            # the fused forward (lstm_fwd_xgx) stamps only in a -DASR_XG_TRACE_FWD
            # build: what was read is the previous backward's trace
            print('WARNING: the forward pass wrote no stamps (build lstm_xg.hip with '
                  '-DASR_XG_TRACE_FWD, tools/build_variant.sh); its rows below repeat the '
                  'backward', flush=True)
        y.backward(torch.randn_like(y))
        torch.cuda.synchronize()
        bwd = read()
    hop('forward', fwd, 3)
    hop('backward', bwd, 4)
    report('forward (us): sweep = start->sweep ok, comb = sweep->barrier, cell = barrier->publish',
           fwd, [(0, 1, 'sweep'), (1, 4, 'mfma'), (4, 2, 'bar'), (2, 3, 'cell')])
    report('forward detail (us): prod = step start -> projection done; mm = sweep ok -> MFMA '
           'results; rd = barrier -> partial sums read; act = -> h; pub = -> published',
           fwd, [(0, 8, 'prod'), (1, 11, 'mm'), (11, 4, 'lds'), (2, 9, 'rd'), (9, 10, 'act'),
                 (10, 3, 'pub')])
    report('backward (us)', bwd, [(0, 1, 'sweep'), (1, 2, 'b1'), (2, 3, 'cell+b2'),
                                  (3, 4, 'mfma+pub')])
    report('backward detail (us): cell wave 0: pre = step start -> at B1, b1w = waits at B1, '
           'cell = B1 -> dg in LDS, b2w = -> past B2; mfma wave 0: b2m = B2 -> MFMA start, '
           'mp = -> published', bwd,
           [(0, 8, 'pre'), (8, 9, 'b1w'), (9, 10, 'cell'), (10, 3, 'b2w'), (3, 11, 'b2m'),
            (11, 4, 'mp')])


if __name__ == '__main__':
    main()
