"""Host side of the drop-in upload (device_vector's staging, _host_x0's zero scan): time
spis_host_copy (pageable and page-locked destinations) and spis_host_nonzero on a C3-sized
vector (196,608 f64 = 1.5 MiB) for piece sizes 2^SHIFT (host-only builds of hash.cpp,
tools/r06_hostcopy.sh) and pool widths; "hot" reuses one source vector, "cold" rotates over
600 MiB of them (the wrapper's b and x0 arrive cold: the call's verifier digests read tens of MiB
between two calls)."""
import ctypes as C
import sys
import time

import numpy as np
import torch

n = 196608
a = np.random.default_rng(0).random(n)
z = np.zeros(n)
NCOLD = 400
cold_a = [np.random.default_rng(i).random(n) for i in range(NCOLD)]
cold_z = [np.zeros(n) + 0.0 for _ in range(NCOLD)]
pins = [torch.empty(n, dtype=torch.float64, pin_memory=torch.cuda.is_available()) for _ in range(2)]
it = [0]


def nxt():
    it[0] += 1
    return it[0] % NCOLD
pin = torch.empty(n, dtype=torch.float64, pin_memory=torch.cuda.is_available())  # pageable off the box
page = np.empty(n)
r = C.c_int32()


def t_us(f, reps=400):
    for _ in range(40):
        f()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    return (time.perf_counter() - t) / reps * 1e6


def t_gap(f, gap, reps=200):
    """f timed alone, after a 3 ms gap of each kind: "spin" (the caller busy), "sleep" (idle core)"""
    tot = 0.0
    for _ in range(reps):
        t = time.perf_counter()
        if gap == "sleep":
            time.sleep(0.003)
        else:
            while time.perf_counter() - t < 0.003:
                pass
        t = time.perf_counter()
        f()
        tot += time.perf_counter() - t
    return tot / reps * 1e6


for lib in sys.argv[1:]:
    L = C.CDLL(lib)
    for T in (1, 4, 8, 16):
        cp = t_us(lambda: L.spis_host_copy(C.c_void_p(pin.data_ptr()), C.c_void_p(a.ctypes.data), C.c_int64(a.nbytes), T))
        cq = t_us(lambda: L.spis_host_copy(C.c_void_p(page.ctypes.data), C.c_void_p(a.ctypes.data), C.c_int64(a.nbytes), T))
        sc = t_us(lambda: L.spis_host_nonzero(C.c_void_p(z.ctypes.data), C.c_int64(n), 1, T, C.byref(r)))
        kc = t_us(lambda: L.spis_host_copy(C.c_void_p(pins[it[0] & 1].data_ptr()),
                                           C.c_void_p(cold_a[nxt()].ctypes.data), C.c_int64(a.nbytes), T))
        ks = t_us(lambda: L.spis_host_nonzero(C.c_void_p(cold_z[nxt()].ctypes.data), C.c_int64(n), 1, T, C.byref(r)))
        print(f"{lib.split('/')[-1]} threads={T} hot: copy_pinned={cp:.1f}us copy_pageable={cq:.1f}us "
              f"zero_scan={sc:.1f}us  cold: copy_pinned={kc:.1f}us zero_scan={ks:.1f}us", flush=True)
        for gap in ("spin", "sleep"):
            gc = t_gap(lambda: L.spis_host_copy(C.c_void_p(pins[0].data_ptr()), C.c_void_p(a.ctypes.data),
                                                C.c_int64(a.nbytes), T), gap)
            gs = t_gap(lambda: L.spis_host_nonzero(C.c_void_p(z.ctypes.data), C.c_int64(n), 1, T, C.byref(r)), gap)
            print(f"    after a 3 ms {gap}: copy_pinned={gc:.1f}us zero_scan={gs:.1f}us", flush=True)
