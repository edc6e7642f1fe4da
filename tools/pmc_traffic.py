"""HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md §HBM).

Usage (on the GPU box, one pass per counter group, never combined with tracing):
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -- python3 bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write <workload> \
        > profiles/rNN_pmc_traffic.json

Corrections applied (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so it
is doubled; WRITE_SIZE is taken as is.  Both count Infinity-Cache-served
requests too (memory-side request counters), so the figure is an upper bound on
HBM bytes.  Output: per kernel-name family, mean bytes per launch."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

FAMILIES = [
    ('lstm_bwd_pass', ('lstm_bwd_xg', 'lstm_bwd_persist')),
    ('lstm_fwd_pass', ('lstm_fwd_xg', 'lstm_fwd_persist')),
    ('gemm', ('gemm_bf16_fast', 'gemm_kernel', 'gemm_bf16_big', 'gemm_bf16_8r', 'gemm_bf16_n64',
              'conv3x3_tr')),
    ('ctc_lattice', ('ctc_lattice',)),
    ('ctc_emit', ('ctc_emit',)),
    ('vgg_rows', ('rw_apply', 'rw_post_fwd', 'rw_bn_moments', 'rw_post_bwd')),
    ('ctc_grad', ('ctc_grad',)),
    ('optim_step', ('optim_step_kernel',)),
]


def family(name):
    for fam, keys in FAMILIES:
        if any(k in name for k in keys):
            return fam
    return None


def read_counter(d, counter):
    """{family: [per-dispatch value]} for one counter from a rocprofv3 csv dir."""
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    per = defaultdict(lambda: defaultdict(float))   # dispatch -> value (summed over dims)
    names = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get('Counter_Name') != counter:
                continue
            key = (f, r.get('Dispatch_Id') or r.get('Correlation_Id'))
            per[key]['v'] += float(r['Counter_Value'])
            names[key] = r.get('Kernel_Name', '')
    out = defaultdict(list)
    for key, v in per.items():
        fam = family(names[key])
        if fam:
            out[fam].append(v['v'])
    return out


def main(fetch_dir, write_dir, workload):
    fetch = read_counter(fetch_dir, 'FETCH_SIZE')
    write = read_counter(write_dir, 'WRITE_SIZE')
    res = {}
    for fam, _ in FAMILIES:
        f, w = fetch.get(fam, []), write.get(fam, [])
        if not f or not w:
            continue
        fb = 2.0 * 1024.0 * sum(f) / len(f)      # KiB -> B, x2 gfx950 read correction
        wb = 1024.0 * sum(w) / len(w)
        res[fam] = {'launches_fetch': len(f), 'launches_write': len(w),
                    'fetch_bytes_per_launch': int(fb), 'write_bytes_per_launch': int(wb),
                    'traffic_bytes_per_launch': int(fb + wb)}
    res['_workload'] = workload
    res['_method'] = ('rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), KiB '
                      'converted to bytes, FETCH_SIZE x2 (gfx950 correction, '
                      'MI355X_MICROARCH.md HBM section)')
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else
         'librispeech100h_char_ctc_blstm5x512')
