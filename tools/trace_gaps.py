"""Per-solve kernel busy time and inter-kernel gaps from a rocprofv3 --kernel-trace CSV."""
import collections
import csv
import sys

KEYS = ['mgs_chain', 'spmv_pipe_kernel<2048, 4', 'spmv_pipe_kernel<2048, 3', 'spmv_pipe_kernel<2048, 1',
        'spmv_pipe_kernel<2048, 2', 'spmv_dual', 'mgs_step', 'spmv_rowblock_kernel<1>', 'spmv_rowblock_kernel<2>', 'spmv_rowblock_kernel<3>',
        'spmv_rowblock_kernel<0>', 'constraint_gram', 'gemv', 'normalize', 'transpose', 'gram_reduce',
        'copy_kernel', 'fillBuffer', 'copyBuffer', 'icwy_dot', 'cgs_update', 'cgs_finalize', 'finalize2', 'dot', 'finalize', 'gather']


def short(n):
    for k in KEYS:
        if k in n:
            return k
    return n[:30]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
R0 = ('spmv_rowblock_kernel<3>', 'spmv_pipe_kernel<2048, 3')  # r0 = b - A x0 opens every solve
idx = [i for i, r in enumerate(rows) if any(k in r['Kernel_Name'] for k in R0)]
s0, s1 = idx[-2], idx[-1]
seg = rows[s0:s1]
t0, t1 = int(seg[0]['Start_Timestamp']), int(rows[s1]['Start_Timestamp'])
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in seg)
print('solve wall %.1f us  busy %.1f us  launches %d' % ((t1 - t0) / 1e3, busy / 1e3, len(seg)))
kt = collections.defaultdict(float)
for r in seg:
    kt[short(r['Kernel_Name'])] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
print('busy by kernel:', {k: round(v, 1) for k, v in sorted(kt.items(), key=lambda kv: -kv[1])})
gaps = collections.defaultdict(list)
for a, b in zip(seg, seg[1:] + [rows[s1]]):
    gaps[(short(a['Kernel_Name']), short(b['Kernel_Name']))].append(int(b['Start_Timestamp']) - int(a['End_Timestamp']))
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:14]:
    print(f"{k[0]:26s}->{k[1]:26s} n={len(v):4d} mean={sum(v)/len(v)/1e3:7.2f}us max={max(v)/1e3:7.2f} total={sum(v)/1e3:8.1f}us")
