"""Where the drop-in call's "h2d" phase goes (C3, swe.LinearSolver.cgmresWrapper as bench.py's
wrapper_rate calls it): the b upload (scratch vector, staging copy, async DMA enqueue) and x0's zero
scan, each timed in place by wrapping the functions the call uses."""
import argparse
import ctypes as C
import sys
import time
from collections import defaultdict

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from structurepreservingiterativesolvers_amd import device, solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls  # noqa: E402

T = defaultdict(float)
N = defaultdict(int)


def timed(name, f):
    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[name] += time.perf_counter() - t
            N[name] += 1
    return g


ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--threads", type=int, default=None)
ap.add_argument("--copy-threads", type=int, default=None, help="override the b copy / x0 scan pool width only")
a = ap.parse_args()
args = argparse.Namespace(config="c3", M=None, cycles=1, k=30, tol=1e-19)
wl = bench.build_workload(args)
dic = wl["dic"]
x0 = np.zeros(dic["A"].shape[0])
if a.threads:
    device._HASH_THREADS = a.threads
from structurepreservingiterativesolvers_amd import _lib  # noqa: E402

L0 = _lib.load_library()
_r = C.c_int32()
_d = np.empty(len(x0))


def stage_us(label):
    """x0 scan + b copy into a pageable array, one thread, at points of the process's life"""
    t = time.perf_counter()
    for _ in range(100):
        L0.spis_host_nonzero(C.c_void_p(x0.ctypes.data), C.c_int64(len(x0)), 1, 1, C.byref(_r))
        L0.spis_host_copy(C.c_void_p(_d.ctypes.data), C.c_void_p(dic["b"].ctypes.data), C.c_int64(8 * len(x0)), 1)
    print(f"[{label}] scan+copy (1 thread): {(time.perf_counter() - t) / 100 * 1e6:.1f} us", flush=True)


stage_us("library loaded, no context")
device.get_context()
stage_us("context created")
for _ in range(3):
    ls.cgmresWrapper(dic, x0, 30, tol=1e-19)
ctx = device.get_context()
stage_us("after 3 calls")
L = ctx.L
for nm in ("spis_host_copy", "spis_memcpy_h2d_async", "spis_host_nonzero", "spis_memcpy_h2d"):
    setattr(L, nm, timed(nm, getattr(L, nm)))
if a.copy_threads:
    cp, nz = L.spis_host_copy, L.spis_host_nonzero
    L.spis_host_copy = lambda d, s, nb, t: cp(d, s, nb, a.copy_threads)
    L.spis_host_nonzero = lambda p, n, bw, t, out: nz(p, n, bw, a.copy_threads, out)
device._stage = timed("_stage", device._stage)
device.device_vector = timed("device_vector", device.device_vector)
solvers.device_vector = timed("solvers.device_vector(b)", solvers.device_vector)
solvers._host_x0 = timed("_host_x0", solvers._host_x0)
device.DeviceVector.scratch = classmethod(timed("scratch", device.DeviceVector.scratch.__func__))
solvers._PHASES = {}
t0 = time.perf_counter()
for _ in range(a.reps):
    ls.cgmresWrapper(dic, x0, 30, tol=1e-19)
el = time.perf_counter() - t0
ph, solvers._PHASES = solvers._PHASES, None
print(f"threads={device._HASH_THREADS} copy_threads={a.copy_threads} ms/call={1e3 * el / a.reps:.3f} phases_ms=" +
      str({k: round(1e3 * v / a.reps, 3) for k, v in ph.items()}))
for k in sorted(T):
    print(f"  {k:28s} calls/call={N[k] / a.reps:5.2f}  us/call={1e6 * T[k] / a.reps:8.1f}")

# after each call: copies of b (the same call's source) into a page-locked scratch and scans of x0,
# timed one after another (first after the solve, then again warm), and a context synchronize
pin = C.c_void_p()
L.spis_host_alloc(C.c_int64(8 * len(x0)), C.byref(pin))
b = dic["b"]
r = C.c_int32()
S = defaultdict(float)
for _ in range(a.reps):
    ls.cgmresWrapper(dic, x0, 30, tol=1e-19)
    t = [time.perf_counter()]
    ctx.synchronize()
    t.append(time.perf_counter())
    for _k in range(2):
        L.spis_host_copy(pin, C.c_void_p(b.ctypes.data), C.c_int64(b.nbytes), 16)
        t.append(time.perf_counter())
        L.spis_host_nonzero(C.c_void_p(x0.ctypes.data), C.c_int64(len(x0)), 1, 16, C.byref(r))
        t.append(time.perf_counter())
    for i, nm in enumerate(("sync", "copy1", "scan1", "copy2", "scan2")):
        S[nm] += t[i + 1] - t[i]
print("after a call: " + " ".join(f"{k}={1e6 * v / a.reps:.1f}us" for k, v in S.items()))

# the same copies and scans in this process with no solve in between (3 ms busy gap, as a solve)
S = defaultdict(float)
for _ in range(a.reps):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.003:
        pass
    t = [time.perf_counter()]
    for _k in range(2):
        L.spis_host_copy(pin, C.c_void_p(b.ctypes.data), C.c_int64(b.nbytes), 16)
        t.append(time.perf_counter())
        L.spis_host_nonzero(C.c_void_p(x0.ctypes.data), C.c_int64(len(x0)), 1, 16, C.byref(r))
        t.append(time.perf_counter())
    for i, nm in enumerate(("copy1", "scan1", "copy2", "scan2")):
        S[nm] += t[i + 1] - t[i]
print("no solve:     " + " ".join(f"{k}={1e6 * v / a.reps:.1f}us" for k, v in S.items()))
S = defaultdict(float)
for _ in range(a.reps):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.003:
        pass
    t = [time.perf_counter()]
    for _k in range(2):
        L.spis_host_copy(pin, C.c_void_p(b.ctypes.data), C.c_int64(b.nbytes), 1)
        t.append(time.perf_counter())
        L.spis_host_nonzero(C.c_void_p(x0.ctypes.data), C.c_int64(len(x0)), 1, 1, C.byref(r))
        t.append(time.perf_counter())
    for i, nm in enumerate(("copy1", "scan1", "copy2", "scan2")):
        S[nm] += t[i + 1] - t[i]
print("no solve, 1 thread: " + " ".join(f"{k}={1e6 * v / a.reps:.1f}us" for k, v in S.items()))
import os  # noqa: E402
print("affinity", len(os.sched_getaffinity(0)), "cpus; threads in process", len(os.listdir("/proc/self/task")))


def task_times():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                s = f.read()
            name = s[s.index("(") + 1:s.rindex(")")]
            fields = s[s.rindex(")") + 2:].split()
            out[tid] = (name, int(fields[11]) + int(fields[12]))  # utime + stime, clock ticks
        except (OSError, ValueError):
            pass
    return out


def cg_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return dict(line.split() for line in f)
    except OSError:
        return {}


c0, k0, w0 = cg_stat(), task_times(), time.perf_counter()
for _ in range(100):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.003:
        pass
    L.spis_host_nonzero(C.c_void_p(x0.ctypes.data), C.c_int64(len(x0)), 1, 1, C.byref(r))
c1, k1, w1 = cg_stat(), task_times(), time.perf_counter()
print(f"idle-gap loop {w1 - w0:.3f}s; cgroup delta:",
      {k: int(c1[k]) - int(c0.get(k, 0)) for k in c1 if k in ("usage_usec", "nr_throttled", "throttled_usec")})
busy = sorted(((k1[t][1] - k0.get(t, ("", 0))[1], k1[t][0], t) for t in k1), reverse=True)[:8]
print("busiest threads (ticks of 10 ms):", busy)


def cpu_now():
    with open("/proc/thread-self/stat") as f:
        s = f.read()
    return int(s[s.rindex(")") + 2:].split()[36])


def node_of_cpu(c):
    for e in os.listdir(f"/sys/devices/system/cpu/cpu{c}"):
        if e.startswith("node"):
            return int(e[4:])
    return -1


def pages_of(addr):
    with open("/proc/self/numa_maps") as f:
        for line in f:
            parts = line.split()
            start = int(parts[0], 16)
            if start <= addr < start + (64 << 20):
                return line.strip()[:200]
    return "?"


def scan_us(reps=100):
    t = time.perf_counter()
    for _ in range(reps):
        L.spis_host_nonzero(C.c_void_p(x0.ctypes.data), C.c_int64(len(x0)), 1, 1, C.byref(r))
        L.spis_host_copy(pin, C.c_void_p(b.ctypes.data), C.c_int64(b.nbytes), 1)
    return (time.perf_counter() - t) / reps * 1e6


nodes = sorted({node_of_cpu(c) for c in os.sched_getaffinity(0)})
print("cpu", cpu_now(), "node", node_of_cpu(cpu_now()), "nodes", nodes)
print("x0 pages:", pages_of(x0.ctypes.data))
print("b pages:", pages_of(b.ctypes.data))
print("scan+copy (1 thread) here:", round(scan_us(), 1), "us")
allc = os.sched_getaffinity(0)
for nd in nodes:
    cpus = {c for c in allc if node_of_cpu(c) == nd}
    os.sched_setaffinity(0, cpus)
    time.sleep(0.01)
    print(f"pinned to node {nd} (cpu {cpu_now()}): scan+copy (1 thread)", round(scan_us(), 1), "us")
os.sched_setaffinity(0, allc)


def pair_us(xz, xb, reps=100):
    t = time.perf_counter()
    for _ in range(reps):
        L.spis_host_nonzero(C.c_void_p(xz.ctypes.data), C.c_int64(len(xz)), 1, 1, C.byref(r))
        L.spis_host_copy(pin, C.c_void_p(xb.ctypes.data), C.c_int64(xb.nbytes), 1)
    return (time.perf_counter() - t) / reps * 1e6


fz, fb = np.zeros(len(x0)), np.random.default_rng(1).random(len(x0))
print("fresh zeros/random (1 thread):", round(pair_us(fz, fb), 1), "us; their pages:", pages_of(fz.ctypes.data)[:90])
cz, cb = x0.copy(), b.copy()
print("copies of x0/b (1 thread):", round(pair_us(cz, cb), 1), "us; their pages:", pages_of(cz.ctypes.data)[:90])
print("x0/b again (1 thread):", round(pair_us(x0, b), 1), "us")
dst = np.empty(len(x0))
t = time.perf_counter()
for _ in range(100):
    L.spis_host_copy(C.c_void_p(dst.ctypes.data), C.c_void_p(b.ctypes.data), C.c_int64(b.nbytes), 1)
print("b -> pageable numpy (1 thread):", round((time.perf_counter() - t) / 100 * 1e6, 1), "us")
t = time.perf_counter()
for _ in range(100):
    L.spis_host_nonzero(C.c_void_p(x0.ctypes.data), C.c_int64(len(x0)), 1, 1, C.byref(r))
print("x0 scan alone (1 thread):", round((time.perf_counter() - t) / 100 * 1e6, 1), "us")
import mmap  # noqa: E402

mz = np.frombuffer(mmap.mmap(-1, x0.nbytes), dtype=np.float64)
mz[:] = 0.0
mb = np.frombuffer(mmap.mmap(-1, b.nbytes), dtype=np.float64)
mb[:] = b
print("mmap'd zeros/b (1 thread):", round(pair_us(mz, mb), 1), "us; heap x0/b:", round(pair_us(x0, b), 1), "us")
t = time.perf_counter()
for _ in range(100):
    np.copyto(dst, b)
print("np.copyto b -> numpy:", round((time.perf_counter() - t) / 100 * 1e6, 1), "us")
