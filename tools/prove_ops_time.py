"""Per-operation timing of the device prover backend at N8 = 2^23 (diagnostics)."""
import sys, time
sys.path.insert(0, '/root/repo')
import numpy as np
from halo_amd import _lib as H
from halo_amd import prover
H.ensure_device(0)
L = H.load()
n = 1 << 20
H.check(L.halo_srs_synthesize(0, n, 99))
H.check(L.halo_srs_precompute_windows(0))
B = prover.DeviceBackend("pallas")
rng = np.random.default_rng(1)
p = B.random_vec(n, rng)
big = B.random_vec(8 * n, rng)


def t(name, f, reps=5):
    f(); B.sync()
    a = time.perf_counter()
    for _ in range(reps):
        r = f()
    B.sync()
    print(f"{name:40s} {1e3 * (time.perf_counter() - a) / reps:9.3f} ms", flush=True)
    return r


e8 = t("ntt(p, 8n)", lambda: B.ntt(p, 8 * n))
t("intt(8n)", lambda: B.intt(e8))
t("evals mul 8n", lambda: e8 * e8)
t("evals add 8n", lambda: e8 + e8)
t("evals scale 8n", lambda: e8 * 12345)
t("sbox 8n", lambda: B.sbox(e8))
t("torch.zeros 8n", lambda: B.torch.zeros((8 * n, 4), dtype=B.torch.int64, device="cuda"))
t("roll 8n", lambda: B.shift_left(e8, 8))
t("poly_mul n x 8n", lambda: B.poly_mul(p, big))
t("poly_add", lambda: B.poly_add(p, big))
t("commit_many x16", lambda: B.commit_many([p] * 16), reps=2)
t("eval_many x16", lambda: B.eval_many([p] * 16, 12345), reps=2)
