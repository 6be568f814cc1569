"""Per-call host timing of the hiding pcdl::open (benches/pcdl.rs:35-57 shapes) through the C ABI:
evaluate, halo_pcdl_open_begin / _blind / _combine / _start, each round_lr + fold, end.
Usage: python tools/pcdl_open_time.py [lg ...]   (GPU box)"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from halo_amd import _lib as H  # noqa: E402
from halo_amd import pcdl  # noqa: E402


def main():
    lgs = [int(a) for a in sys.argv[1:]] or [2, 6, 10, 12, 16]
    H.ensure_device(0)
    for _kv in [x for x in os.environ.get('TUNE', '').split(',') if x]:  # tuning A/B: TUNE=key=value,...
        H.set_tuning(_kv.split('=')[0], int(_kv.split('=')[1]))
    L = H.load()
    N = 1 << max(lgs)
    H.check(L.halo_srs_synthesize(0, N, 0x50434C44))
    G = np.zeros((N, 8), dtype=np.uint64)
    H.check(L.halo_srs_read(0, 0, N, H.ptr(G)))
    H.check(L.halo_srs_upload(0, H.ptr(G), N, H.ptr(G[0]), H.ptr(G[1])))
    H.check(L.halo_srs_precompute_windows(0))
    rng = np.random.default_rng(3)

    def fes(k):
        a = rng.integers(0, 2**63, size=(k, 4), dtype=np.uint64)
        a[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
        return np.ascontiguousarray(a)

    for lg in lgs:
        n = 1 << lg
        p, w, z, q, wb = fes(n), fes(1), fes(1), fes(n - 1), fes(1)
        C = pcdl.commit(p, n - 1, w[0])
        rows = []
        for rep in range(12):
            t = {}
            tr = pcdl.StandInTranscript()
            s = ctypes.c_void_p()
            v = np.zeros(4, dtype=np.uint64)
            a = time.perf_counter()
            H.check(L.halo_pcdl_open_begin(0, H.ptr(p), n, n - 1, H.ptr(z), H.ptr(v), ctypes.byref(s)))
            t["begin+eval"] = time.perf_counter() - a
            Cb = np.zeros(8, dtype=np.uint64)
            a = time.perf_counter()
            H.check(L.halo_pcdl_open_blind(s, H.ptr(q), H.ptr(wb), H.ptr(Cb)))
            t["blind"] = time.perf_counter() - a
            tr.absorb_g([C, Cb])
            tr.absorb_fr([z[0], v])
            al = tr.challenge()
            wp = np.zeros(4, dtype=np.uint64)
            Cp = np.zeros(8, dtype=np.uint64)
            a = time.perf_counter()
            H.check(L.halo_pcdl_open_combine(s, H.ptr(al), H.ptr(C), H.ptr(w), H.ptr(wp), H.ptr(Cp)))
            t["combine"] = time.perf_counter() - a
            tr.absorb_g([Cp])
            xi = tr.challenge()
            a = time.perf_counter()
            H.check(L.halo_pcdl_open_start(s, None, H.ptr(xi)))
            t["start"] = time.perf_counter() - a
            Lp = np.zeros(8, dtype=np.uint64)
            Rp = np.zeros(8, dtype=np.uint64)
            t["rounds"] = 0.0
            t["folds"] = 0.0
            t["host_transcript"] = 0.0
            for _ in range(lg):
                a = time.perf_counter()
                H.check(L.halo_ipa_round_lr(s, H.ptr(Lp), H.ptr(Rp)))
                b = time.perf_counter()
                tr.absorb_g([Lp, Rp])
                xi = tr.challenge()
                c = time.perf_counter()
                H.check(L.halo_ipa_fold(s, H.ptr(xi), None))  # xi^-1 formed by the library, as pcdl.open
                d = time.perf_counter()
                t["rounds"] += b - a
                t["host_transcript"] += c - b
                t["folds"] += d - c
            U = np.zeros(8, dtype=np.uint64)
            c0 = np.zeros(4, dtype=np.uint64)
            a = time.perf_counter()
            H.check(L.halo_ipa_end(s, H.ptr(U), H.ptr(c0)))
            t["end"] = time.perf_counter() - a
            t["total"] = sum(t.values())
            if rep >= 2:
                rows.append(t)
        med = {k: float(np.median([r[k] for r in rows])) * 1e3 for k in rows[0]}
        print(f"2^{lg}: " + " ".join(f"{k}={v:.3f}" for k, v in med.items()) + f"  per_round={med['rounds'] / lg:.3f}",
              flush=True)


if __name__ == "__main__":
    main()
