"""Host KKT A/B: lsq_kkt_solve of two liblsq_host.so builds on dumped steps (tools/kkt_dump.py),
the tests/kkt_cases fixtures and 600 random problems: bitwise equality of y, message and
iterations, and the time per call.

    python tools/kkt_ab.py OLD.so [NEW.so] [dump.npz ...]
"""
import ctypes as C, glob, sys, time
import numpy as np
PD = C.POINTER(C.c_double)
def load(path):
    L = C.CDLL(path)
    L.lsq_kkt_solve.argtypes = [C.c_int, PD, C.c_double, C.c_int, PD, PD, PD, PD, PD, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    return L
old = load(sys.argv[1])
new = load(sys.argv[2] if len(sys.argv) > 2 else 'structurepreservingiterativesolvers_amd/liblsq_host.so')
def run(L, H, beta, t0, t1, t2, y0, reps=1):
    p = H.shape[1]; m = len(t0)
    Hc = np.ascontiguousarray(H.T)
    t0 = np.ascontiguousarray(t0, dtype=np.float64); t1 = np.ascontiguousarray(np.reshape(t1, (m, p))); t2 = np.ascontiguousarray(np.reshape(t2, (m, p * p)))
    y0 = np.ascontiguousarray(y0); y = np.zeros(p); msg, it = C.c_int(), C.c_int()
    a = (p, Hc.ctypes.data_as(PD), float(beta), m, t0.ctypes.data_as(PD), t1.ctypes.data_as(PD), t2.ctypes.data_as(PD), y0.ctypes.data_as(PD), y.ctypes.data_as(PD), C.byref(msg), C.byref(it))
    r = L.lsq_kkt_solve(*a)
    t = time.perf_counter()
    for _ in range(reps - 1): L.lsq_kkt_solve(*a)
    dt = (time.perf_counter() - t) / max(reps - 1, 1)
    return y.copy(), msg.value, it.value, r, dt
cases = []
for f in sys.argv[3:]:  # dumps of tools/kkt_dump.py
    z = np.load(f); cases.append((f.split('/')[-1], z['H'], z['beta'], z['term0'], z['term1'], z['term2'], z['y0'], 3000))
for f in sorted(glob.glob('tests/kkt_cases/*.npz')):
    z = np.load(f)
    if 'H' not in z.files: continue
    y0 = z['y0'] if 'y0' in z.files else np.zeros(z['H'].shape[1])
    g = lambda a, b: z[a] if a in z.files else z[b]
    cases.append((f.split('/')[-1], z['H'], z['beta'], g('term0', 't0'), g('term1', 't1'), g('term2', 't2'), y0, 300))
rng = np.random.default_rng(0)
for i in range(600):
    p = int(rng.integers(2, 33)); m = int(rng.integers(1, 4))
    H = np.triu(rng.standard_normal((p + 1, p)), -1)
    t2 = rng.standard_normal((m, p, p)) * 10.0 ** rng.uniform(-3, 1)
    if i % 3 == 0: t2 = t2 + np.transpose(t2, (0, 2, 1))
    cases.append(('rand%d' % i, H, abs(rng.standard_normal()) + 0.1, rng.standard_normal(m) * 0.1, rng.standard_normal((m, p)), t2,
                  rng.standard_normal(p) * (i % 2), 1))
bad = 0
for name, H, beta, t0, t1, t2, y0, reps in cases:
    a = run(old, H, beta, t0, t1, t2, y0, reps); b = run(new, H, beta, t0, t1, t2, y0, reps)
    same = np.array_equal(a[0], b[0]) and a[1:4] == b[1:4]
    if not same:
        bad += 1
        if bad < 10: print('DIFF', name, a[1:4], b[1:4], np.max(np.abs(a[0] - b[0])))
    if reps > 1: print('%-32s old %7.2f us  new %7.2f us  msg %d it %d' % (name, a[4] * 1e6, b[4] * 1e6, a[1], a[2]))
print('cases', len(cases), 'bitwise differences', bad)
