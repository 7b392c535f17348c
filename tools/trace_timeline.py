"""One solve's kernel timeline from a rocprofv3 --kernel-trace CSV: every launch with its start
offset, duration, stream (queue) and the idle gap before it on the device (tools/trace_gaps.py
gives the per-kernel totals).  The solve is the last complete one (r0 = b - A x0 SpMV to the next).

    python tools/trace_timeline.py trace.csv [max_rows]"""
import csv
import sys

from trace_gaps import R0, short

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 400
idx = [i for i, r in enumerate(rows) if any(k in r['Kernel_Name'] for k in R0)]
seg = rows[idx[-2]:idx[-1]]
t0 = int(seg[0]['Start_Timestamp'])
end = t0
print('%9s %8s %8s  %-5s %s' % ('start_us', 'dur_us', 'gap_us', 'queue', 'kernel'))
for r in seg[:lim]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - end) / 1e3
    print('%9.1f %8.1f %8.1f  %-5s %s' % ((s - t0) / 1e3, (e - s) / 1e3, gap if gap > 0 else 0.0,
                                          r.get('Queue_Id', r.get('Stream_Id', '?')), short(r['Kernel_Name'])))
    end = max(end, e)
print('solve wall %.1f us' % ((int(rows[idx[-1]]['Start_Timestamp']) - t0) / 1e3))
