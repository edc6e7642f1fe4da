"""Summarise a rocprofv3 kernel trace (rocpd SQLite db or kernel_trace.csv)
into per-kernel count / total / mean duration, sorted by total time."""
import csv
import sqlite3
import sys
from collections import defaultdict


def rows_from_db(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = 'kernel_name' if 'kernel_name' in cols else 'name'
    for n, s, e in c.execute('select %s, start, end from kernels' % name):
        yield n, e - s


def rows_from_csv(path):
    for r in csv.DictReader(open(path)):
        yield r['Kernel_Name'], int(r['End_Timestamp']) - int(r['Start_Timestamp'])


def main(path, top=40):
    agg = defaultdict(lambda: [0, 0])
    src = rows_from_db(path) if path.endswith('.db') else rows_from_csv(path)
    for n, d in src:
        a = agg[n]
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print('%-90s %8s %12s %10s %6s' % ('kernel', 'calls', 'total_us', 'mean_us', 'pct'))
    for n, (k, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print('%-90s %8d %12.1f %10.3f %6.2f' % (n[:90], k, d / 1e3, d / 1e3 / k, 100.0 * d / tot))
    print('total kernel time %.1f us' % (tot / 1e3))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
