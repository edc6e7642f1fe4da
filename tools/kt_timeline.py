"""Timeline of one training step from a rocprofv3 --kernel-trace CSV: every
kernel dispatch of the last step window (from the last optimizer kernel back to
the one before it) with start / end in µs relative to the window start, its
queue, and a short name -- to see what runs beside the persistent recurrences.

usage: python tools/kt_timeline.py <dir with *kernel_trace.csv> [filter substrings]
"""
import csv
import glob
import os
import sys


def short(name):
    n = name
    for pre in ('void ', 'asr::', '(anonymous namespace)::'):
        n = n.replace(pre, '')
    n = n.split('(')[0]
    return n[:60]


def main():
    d = sys.argv[1]
    filt = sys.argv[2:]
    files = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                             r.get('Queue_Id', r.get('Stream_Id', '?')), r['Kernel_Name']))
    rows.sort()
    opt = [i for i, r in enumerate(rows) if 'optim' in r[3]]
    if len(opt) < 2:
        print('fewer than two optimizer launches; %d kernels' % len(rows))
        return
    a, b = opt[-2] + 1, opt[-1] + 1
    t0 = rows[a][0]
    for s, e, q, n in rows[a:b]:
        nm = short(n)
        if filt and not any(f in nm for f in filt):
            continue
        print('%10.1f %10.1f %8.1f  q%-3s %s' % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, q,
                                                 nm))
    print('step window %.1f us' % ((rows[b - 1][1] - t0) / 1e3))


if __name__ == '__main__':
    main()
