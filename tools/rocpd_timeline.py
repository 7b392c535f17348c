"""Timeline of one CGMRES solve from a rocprofv3 (rocpd SQLite) kernel trace: per-queue kernel
sequence with start offsets, durations and the idle time on the main queue.  Usage:
  python tools/rocpd_timeline.py run_results.db [solve_index_from_end] [--iters]"""
import collections
import re
import sqlite3
import sys

KEYS = ['mgs_chain_lag', 'mgs_chain_big', 'mgs_chain', 'constraint_gram', 'gemv', 'transpose',
        'gram_reduce', 'streamOpsWait', 'streamOpsWrite', 'copy_kernel', 'fillBuffer', 'copyBuffer', 'finalize']
SPMV = re.compile(r'spmv_(pipe|rowblock|dual)\w*<(\d+), (\d+)')
R0 = re.compile(r'spmv_(pipe_kernel<\d+, 3|rowblock_kernel<3>)')  # r0 = b - A x0 opens every solve


def short(n):
    m = SPMV.search(n)
    if m:
        return {'1': 'spmv x', '2': 'spmv res', '3': 'spmv r0', '4': 'spmv dual'}.get(m.group(3), 'spmv ' + m.group(3))
    for k in KEYS:
        if k in n:
            return k
    return n[:28]


def main():
    db = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith('-') else 2
    c = sqlite3.connect(db)
    rows = c.execute("select name, queue_id, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if R0.search(r[0])]
    s0, s1 = starts[-back], starts[-back + 1] if back > 1 else len(rows)
    seg = rows[s0:s1]
    t0 = seg[0][2]
    wall = (rows[s1][2] if s1 < len(rows) else seg[-1][3]) - t0
    print('solve wall %.1f us, %d launches' % (wall / 1e3, len(seg)))
    per_q = collections.defaultdict(float)
    per_k = collections.defaultdict(lambda: [0, 0.0])
    for n, q, a, b in seg:
        per_q[q] += (b - a) / 1e3
        per_k[short(n)][0] += 1
        per_k[short(n)][1] += (b - a) / 1e3
    print('busy per queue (us):', {q: round(v, 1) for q, v in per_q.items()})
    for k, (cnt, t) in sorted(per_k.items(), key=lambda kv: -kv[1][1]):
        print(f'  {k:28s} n={cnt:3d} total={t:8.1f} mean={t / cnt:7.2f}')
    # union of busy intervals over all queues -> GPU idle
    iv = sorted((a, b) for _, _, a, b in seg)
    busy, cur_a, cur_b = 0, None, None
    for a, b in iv:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    busy += cur_b - cur_a
    print('GPU busy (any queue) %.1f us, idle %.1f us' % (busy / 1e3, (wall - busy) / 1e3))
    if '--iters' in sys.argv:
        for n, q, a, b in seg:
            print(f'q{q} {(a - t0) / 1e3:9.1f} {(b - a) / 1e3:7.1f}  {short(n)}')


if __name__ == '__main__':
    main()
