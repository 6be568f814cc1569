"""The 2^20 opening's time after a pipelined 2^20 MSM burst over S streams (the bench's headline then
its opening leg), optionally with halo_shutdown in between.  Usage (GPU box):
    python tools/ipa_after_msm.py S [reset]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from halo_amd import _lib as H  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reset = "reset" in sys.argv[2:]
H.ensure_device(0)
L = H.load()
HIP = ctypes.CDLL("libamdhip64.so")
HIP.hipStreamCreateWithFlags.restype = ctypes.c_int
n = 1 << 20
H.check(L.halo_srs_synthesize(0, n, 0x48414C4F))
H.check(L.halo_srs_precompute_windows(0))
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
streams = [sp]
for _ in range(S - 1):
    hs = ctypes.c_void_p()
    HIP.hipStreamCreateWithFlags(ctypes.byref(hs), 1)
    streams.append(hs)
nb, nmsm = (8, 23) if "bench" in sys.argv[2:] else (4, 32)  # "bench": the headline's batch and step counts
nb = int(os.environ.get("NB", nb))
nmsm = int(os.environ.get("NMSM", nmsm))
if os.environ.get("SMALL") == "1":
    sc = torch.randint(0, 2**62, (nb, n, 4), dtype=torch.int64, device="cuda")
else:
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234)
    sc = torch.randint(-(2**63), 2**63 - 1, (nb, n, 4), dtype=torch.int64, device="cuda", generator=gen)
    sc[..., 3] &= 0x0FFFFFFFFFFFFFFF
out = torch.zeros((nmsm, 8), dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(nmsm):
    H.check(L.halo_msm_dev_async(0, None, ctypes.c_void_p(sc[i % nb].data_ptr()), n,
                                 ctypes.c_void_p(out[i].data_ptr()), streams[i % S]))
for q in streams:
    H.check(L.halo_msm_join(q))
torch.cuda.synchronize()
print(f"S={S}: {(time.perf_counter() - t0) * 1e3 / nmsm:.3f} ms per MSM", flush=True)
if "sync" in sys.argv[2:]:  # the bench's standalone MSMs after its timed region
    o = np.zeros(8, dtype=np.uint64)
    for i in range(4):
        H.check(L.halo_msm_dev(0, None, ctypes.c_void_p(sc[i].data_ptr()), n, H.ptr(o), sp))
if reset:
    L.halo_shutdown()
R = 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001


def fe1(v):
    m = v * (1 << 256) % R
    return np.array([(m >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)


cs = np.random.default_rng(99).integers(0, 2**62, size=(n, 4), dtype=np.uint64)
hp = np.zeros(8, dtype=np.uint64)
H.check(L.halo_srs_read(0, 1, 1, H.ptr(hp)))
z = fe1(12345)
for rep in range(3):
    ses = ctypes.c_void_p()
    H.check(L.halo_ipa_begin(0, H.ptr(cs), n, H.ptr(z), H.ptr(hp), ctypes.byref(ses)))
    Lp = np.zeros(8, dtype=np.uint64)
    Rp = np.zeros(8, dtype=np.uint64)
    if "prof" in sys.argv[2:]:  # the bench's opening leg runs with the library's launch profiling on
        L.halo_profile_reset()
        L.halo_profile_enable(1)
    a0 = time.perf_counter()
    for r in range(20):
        H.check(L.halo_ipa_round_lr(ses, H.ptr(Lp), H.ptr(Rp)))
        xi = (int.from_bytes(Lp.tobytes()[:16], "little") ^ (r + 1)) % R or 1
        H.check(L.halo_ipa_fold(ses, H.ptr(fe1(xi)), H.ptr(fe1(pow(xi, -1, R)))))
    U = np.zeros(8, dtype=np.uint64)
    c0 = np.zeros(4, dtype=np.uint64)
    H.check(L.halo_ipa_end(ses, H.ptr(U), H.ptr(c0)))
    print(f"  open 2^20 rep {rep}: {(time.perf_counter() - a0) * 1e3:.2f} ms", flush=True)
