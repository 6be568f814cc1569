"""Times k concurrent device openings (halo_ipa_round_lr_multi / fold_multi) vs one, at 2^logn."""
import sys, time
sys.path.insert(0, '/root/repo')
import numpy as np
from halo_amd import _lib as H
from halo_amd import prover
H.ensure_device(0)
L = H.load()
logn = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << logn
H.check(L.halo_srs_synthesize(0, n, 5))
H.check(L.halo_srs_precompute_windows(0))
B = prover.DeviceBackend("pallas")
rng = np.random.default_rng(2)
ps = [B.random_vec(n, rng) for _ in range(3)]
for rep in range(3):
    for k in (1, 2, 3):
        jobs = [(ps[i], n, 1234 + i, 77 + i) for i in range(k)]  # (p, n, z, xi_0): the prover's xi mode
        chals = [prover.Challenges(B.m, seed=i) for i in range(k)]
        B.sync()
        t = time.perf_counter()
        B.ipa_many_xi(jobs, chals)
        print(f"rep {rep} k={k}: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
t = time.perf_counter()
for i in range(2):
    B.ipa_many_xi([(ps[i], n, 1234 + i, 77 + i)], [prover.Challenges(B.m, seed=i)])
print(f"2 sequential: {1e3 * (time.perf_counter() - t):.1f} ms")
