"""Per-kernel mean of every counter in a rocprofv3 --pmc csv directory.

Usage: python tools/pmc_kernel.py <pmc-dir> [name-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    per = defaultdict(lambda: defaultdict(float))   # (file, dispatch) -> counter -> value
    names = {}
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            k = (f, r.get('Dispatch_Id') or r.get('Correlation_Id'))
            per[k][r['Counter_Name']] += float(r['Counter_Value'])
            names[k] = r.get('Kernel_Name', '')
    agg = defaultdict(lambda: defaultdict(list))
    for k, cs in per.items():
        nm = names[k]
        if keys and not any(s in nm for s in keys):
            continue
        short = nm.replace('(anonymous namespace)', '').split('(')[0][-60:]
        for c, v in cs.items():
            agg[short][c].append(v)
    for nm, cs in sorted(agg.items()):
        n = len(next(iter(cs.values())))
        print('%s  (%d dispatches)' % (nm, n))
        for c in sorted(cs):
            print('    %-28s %14.1f' % (c, sum(cs[c]) / len(cs[c])))


if __name__ == '__main__':
    main()
