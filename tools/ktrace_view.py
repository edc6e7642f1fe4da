"""Timeline of the last N kernels of a rocprofv3 --kernel-trace CSV (start
offset, gap to the previous kernel's end, duration, queue, name)."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 140
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[0]['Start_Timestamp'])
prev = None
for r in rows[-n:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1000 if prev else 0.0
    print('%10.1f %7.1f %8.1f q%-3s %s' % ((s - t0) / 1000, gap, (e - s) / 1000, r['Queue_Id'],
                                         r['Kernel_Name'][:64]))
    prev = max(prev or 0, e)
