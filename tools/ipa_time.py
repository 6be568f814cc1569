"""Times a full device-resident IPA opening (pcdl.rs:392-438 round loop): lg n rounds of L/R MSMs +
fold, with a stand-in transcript (fixed pseudo-random challenges).  MAT_N=<len>[,<len>...]: repeat
with the weighted rounds materialising G at each length (tuning ipa_mat_n)."""
import ctypes, os, random, sys, time
sys.path.insert(0, '/root/repo')
import numpy as np
from halo_amd import _lib as H
H.ensure_device(0)
for _kv in [x for x in os.environ.get('TUNE', '').split(',') if x]:  # tuning A/B: TUNE=key=value,...
    H.set_tuning(_kv.split('=')[0], int(_kv.split('=')[1]))
L = H.load()
R = 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001


def fe1(v):
    m = v * (1 << 256) % R
    return np.array([(m >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)


MATS = [int(x) for x in os.environ.get("MAT_N", "-1").split(",")]
for lg, mat in [(int(x), m) for x in (sys.argv[1:] or ['16', '20']) for m in MATS]:
    H.set_tuning("ipa_mat_n", mat)
    n = 1 << lg
    H.check(L.halo_srs_synthesize(0, n, 77))
    H.check(L.halo_srs_precompute_windows(0))  # as bench.py: round 1 L/R on the shifted SRS
    rnd = random.Random(lg)
    cs = np.array([[rnd.getrandbits(62) for _ in range(4)] for _ in range(n)], dtype=np.uint64)
    z = fe1(12345)
    Hp = np.zeros(8, dtype=np.uint64)
    H.check(L.halo_srs_read(0, 1, 1, H.ptr(Hp)))
    for rep in range(int(os.environ.get("REPS", "2"))):
        s = ctypes.c_void_p()
        if os.environ.get("NO_XI") == "1":  # H' given (the caller's scalar multiplication)
            H.check(L.halo_ipa_begin(0, H.ptr(cs), n, H.ptr(z), H.ptr(Hp), ctypes.byref(s)))
        else:  # H' = xi_0 H formed in the session (the prover's path)
            H.check(L.halo_ipa_begin_xi(0, H.ptr(cs), n, H.ptr(z), H.ptr(Hp), H.ptr(fe1(987654321)), ctypes.byref(s)))
        Lp = np.zeros(8, dtype=np.uint64); Rp = np.zeros(8, dtype=np.uint64)
        H.check(L.halo_profile_reset()); H.check(L.halo_profile_enable(1))
        t_lr = t_fold = 0.0
        per = []
        t0 = time.perf_counter()
        for r in range(lg):
            a = time.perf_counter()
            H.check(L.halo_ipa_round_lr(s, H.ptr(Lp), H.ptr(Rp)))
            b = time.perf_counter()
            xi = rnd.randrange(1, R)
            H.check(L.halo_ipa_fold(s, H.ptr(fe1(xi)), H.ptr(fe1(pow(xi, -1, R)))))
            c = time.perf_counter()
            t_lr += b - a; t_fold += c - b
            per.append((round(1e3 * (b - a), 2), round(1e3 * (c - b), 2)))
        U = np.zeros(8, dtype=np.uint64); c0 = np.zeros(4, dtype=np.uint64)
        H.check(L.halo_ipa_end(s, H.ptr(U), H.ptr(c0)))  # weighted rounds: U is one more MSM
        t1 = time.perf_counter()
        nl = ctypes.c_size_t(0); ms = ctypes.c_double(0)
        H.check(L.halo_profile_read(b"ipa_fold", ctypes.byref(nl), ctypes.byref(ms)))
        H.check(L.halo_profile_enable(0))
        print(f"open 2^{lg} (ipa_mat_n {H.get_tuning('ipa_mat_n')}): total {1e3*(t1-t0):.2f} ms (L/R rounds {1e3*t_lr:.2f} ms, folds {1e3*t_fold:.2f} ms; "
              f"fold kernels {ms.value:.2f} ms over {nl.value})", flush=True)
        print("  per round (lr ms, fold ms):", per, flush=True)
