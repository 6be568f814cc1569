"""Single-call latency of the variable-base MSM (caller bases in HBM, halo_msm_dev: GLV digits, window
sums, k_final's Horner) at a few sizes.  usage: python tools/varbase_time.py [lg ...]   (GPU box)"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from halo_amd import _lib as H  # noqa: E402

lgs = [int(a) for a in sys.argv[1:]] or [10, 16, 20]
H.ensure_device(0)
L = H.load()
N = 1 << max(lgs)
H.check(L.halo_srs_synthesize(0, N, 0x56415242))
G = np.zeros((N, 8), dtype=np.uint64)
H.check(L.halo_srs_read(0, 0, N, H.ptr(G)))
gd = torch.from_numpy(G.view(np.int64)).cuda()
g = torch.Generator(device="cuda")
g.manual_seed(11)
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
out = np.zeros(8, dtype=np.uint64)
for lg in lgs:
    n = 1 << lg
    sc = torch.randint(-(2**63), 2**63 - 1, (n, 4), dtype=torch.int64, device="cuda", generator=g)
    sc[:, 3] &= 0x0FFFFFFFFFFFFFFF
    for _ in range(3):
        H.check(L.halo_msm_dev(0, ctypes.c_void_p(gd.data_ptr()), ctypes.c_void_p(sc.data_ptr()), n, H.ptr(out), sp))
    t = []
    for _ in range(10):
        a0 = time.perf_counter()
        H.check(L.halo_msm_dev(0, ctypes.c_void_p(gd.data_ptr()), ctypes.c_void_p(sc.data_ptr()), n, H.ptr(out), sp))
        t.append(time.perf_counter() - a0)
    print("varbase 2^%d: %.3f ms" % (lg, 1e3 * min(t)))
