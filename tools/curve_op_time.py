"""Single-call latency of halo_curve_op op 2 (lone GLV scalar multiplications, H' = xi_0 H and the
accumulator's combination in the prover) for n = 1, 2, 4.  usage: python tools/curve_op_time.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from halo_amd import _lib as H  # noqa: E402

H.ensure_device(0)
L = H.load()
H.check(L.halo_srs_synthesize(0, 8, 0x43555256))
G = np.zeros((8, 8), dtype=np.uint64)
H.check(L.halo_srs_read(0, 0, 8, H.ptr(G)))
rng = np.random.default_rng(5)
for n in (1, 2, 4):
    pts = np.ascontiguousarray(G[:n])
    ks = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
    ks[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    ks = np.ascontiguousarray(ks)
    out = np.zeros_like(pts)
    t = []
    for _ in range(12):
        a0 = time.perf_counter()
        H.check(L.halo_curve_op(0, 2, H.ptr(pts), None, H.ptr(ks), n, H.ptr(out)))
        t.append(time.perf_counter() - a0)
    print("curve_op smul n=%d: %.3f ms" % (n, 1e3 * min(t[2:])))
