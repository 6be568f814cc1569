"""Single-call MSM latency over the resident window-shifted SRS at small and medium n (the latency
floor of commits and of the IPA's per-round MSMs).  usage: python tools/msm_latency.py [lg ...]
Prints ms per synchronous halo_msm_dev call (device scalars, result to host) per size."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from halo_amd import _lib as H  # noqa: E402

lgs = [int(a) for a in sys.argv[1:]] or [2, 6, 10, 14, 16, 18]
H.ensure_device(0)
L = H.load()
N = 1 << max(max(lgs), 16)
H.check(L.halo_srs_synthesize(0, N, 0x4C415459))
H.check(L.halo_srs_precompute_windows(0))
g = torch.Generator(device="cuda")
g.manual_seed(7)
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
out = np.zeros(8, dtype=np.uint64)
for lg in lgs:
    n = 1 << lg
    sc = torch.randint(-(2**63), 2**63 - 1, (n, 4), dtype=torch.int64, device="cuda", generator=g)
    sc[:, 3] &= 0x0FFFFFFFFFFFFFFF
    for _ in range(3):
        H.check(L.halo_msm_dev(0, None, ctypes.c_void_p(sc.data_ptr()), n, H.ptr(out), sp))
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        H.check(L.halo_msm_dev(0, None, ctypes.c_void_p(sc.data_ptr()), n, H.ptr(out), sp))
    print(f"2^{lg}: {(time.perf_counter() - t0) * 1e3 / reps:.3f} ms", flush=True)
