"""A/B of the prover's NTT onto the 8n domain (evaluate_over_domain_by_ref of a degree < n polynomial):
one zero-padded 2^(k+3) NTT vs 8 coset NTTs of size 2^k (twiddle omega_8n^(jk) on 8 copies, batched
2^k NTT, 8 x n transpose).  Checks equality and prints ms per transform."""
import ctypes, sys, time
sys.path.insert(0, '/root/repo')
import numpy as np
import torch
from halo_amd import _lib as H
H.ensure_device(0)
L = H.load()
F = H.FP
logn = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n, N = 1 << logn, 8 << logn
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())
g = torch.Generator(device='cuda').manual_seed(1)
a = torch.randint(0, 2**62, (n, 4), dtype=torch.int64, device='cuda', generator=g)


def padded():
    x = torch.zeros((N, 4), dtype=torch.int64, device='cuda')
    x[:n] = a
    H.check(L.halo_ntt_dev(F, P(x), logn + 3, 1, 0, s))
    return x


def coset():
    x = a.repeat(8, 1)
    H.check(L.halo_ntt_twiddle_dev(F, P(x), logn + 3, 8, n, 0, 0, 0, s))
    H.check(L.halo_ntt_dev(F, P(x), logn, 8, 0, s))
    y = torch.empty_like(x)
    H.check(L.halo_transpose_dev(P(x), P(y), 1, 8, n, 1, s))
    return y


r1, r2 = padded(), coset()
torch.cuda.synchronize()
print("equal:", bool(torch.equal(r1, r2)))
for name, f in (("padded", padded), ("coset", coset)):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per 2^{logn + 3} transform")
