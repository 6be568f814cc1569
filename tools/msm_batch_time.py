"""A/B of batched commitments (halo_msm_batch_dev, fronts beside the previous accumulation) against
back-to-back halo_msm_dev_async calls, 2^logn points per MSM over the resident window-shifted
synthetic SRS.  Prints ms per MSM for each and whether every result agrees.
usage: python tools/msm_batch_time.py [logn] [k] [reps]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from halo_amd import _lib as H  # noqa: E402

logn = int(sys.argv[1]) if len(sys.argv) > 1 else 20
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
H.ensure_device(0)
L = H.load()
n = 1 << logn
H.check(L.halo_srs_synthesize(0, n, 0x48414C4F))
H.check(L.halo_srs_precompute_windows(0))
g = torch.Generator(device="cuda")
g.manual_seed(5)
sc = torch.randint(-(2**63), 2**63 - 1, (k, n, 4), dtype=torch.int64, device="cuda", generator=g)
sc[..., 3] &= 0x0FFFFFFFFFFFFFFF
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
ptrs = (ctypes.c_void_p * k)(*[sc[i].data_ptr() for i in range(k)])
lens = (ctypes.c_size_t * k)(*([n] * k))
out_a = torch.zeros((k, 8), dtype=torch.int64, device="cuda")
out_b = torch.zeros((k, 8), dtype=torch.int64, device="cuda")


def run_async():
    for i in range(k):
        H.check(L.halo_msm_dev_async(0, None, ctypes.c_void_p(sc[i].data_ptr()), n,
                                     ctypes.c_void_p(out_a[i].data_ptr()), sp))
    H.check(L.halo_msm_join(sp))


def run_batch():
    H.check(L.halo_msm_batch_dev(0, ptrs, lens, k, ctypes.c_void_p(out_b.data_ptr()), sp))
    H.check(L.halo_msm_join(sp))


def timeit(f):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / (reps * k)


ta = timeit(run_async)
tb = timeit(run_batch)
same = bool(torch.equal(out_a, out_b))
print(f"logn {logn} k {k}: async {ta:.3f} ms/MSM, batch {tb:.3f} ms/MSM, same={same}, "
      "")
