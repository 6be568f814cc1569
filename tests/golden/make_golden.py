#!/usr/bin/env python3
"""Regenerate tests/golden/golden.npz (committed).  Run in the build container, where the reference
checkout is mounted read-only at /root/reference:

    python3 tests/golden/make_golden.py

Two kinds of arrays are written (uint64, and uint8 for raw wire bytes; loaded with numpy's default
allow_pickle=False):

1. Data copied from the reference's own committed artefacts (the reference is Rust and cannot be
   built or run here -- SURVEY §8c -- so these are the only reference-produced values available):
   * ref_srs_<curve>_*   : decoded points of crates/group/.precompute/<curve>/gs-XX.bin
                           (bincode Vec<WrappedPoint>, pp.rs:36-53) -- first 64 of block 0, first 8 of
                           block 1 and the last 8 of block 63;
   * ref_sh_<curve>      : (S, H) from sh.bin;
   * ref_gs_<curve>_b00_head_bytes / ref_sh_<curve>_bytes : raw bytes (length prefix + first 64
                           records of gs-00.bin; all of sh.bin) for the device bincode loader;
   * ref_omega_fp16 / ref_omega_fq16 : IVC_FP_CIRCUIT.omega / IVC_FQ_CIRCUIT.omega
                           (crates/plonk/src/frontend/ivc/mod.rs:55,112), Montgomery limbs.
2. Golden vectors computed by the pure-Python oracle (oracle/pasta.py) from seeded inputs on top of
   that reference data: MSMs over the reference SRS, NTTs, one IPA round, the test_u_check fold
   (pcdl.rs:627-687), h(X) coefficients (pcdl.rs:735-758) and Horner evaluations.
"""
from __future__ import annotations

import os
import random
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pasta as P  # noqa: E402

REF = "/root/reference/crates"


def fe(vals, m):
    return np.array([P.int_to_limbs(P.to_mont(v % m, m)) for v in vals], dtype=np.uint64).reshape(-1, 4)


def pts(c, points):
    return np.array([P.point_to_wrapped(c, q) for q in points], dtype=np.uint64).reshape(-1, 8)


def main():
    out = {}
    rng = random.Random(0x48414C4F)
    # ---- 1. reference data
    for cname in ("pallas", "vesta"):
        d = f"{REF}/group/.precompute/{cname}/"
        _, b0 = P.decode_wrapped_points(open(d + "gs-00.bin", "rb").read(), 64)
        _, b1 = P.decode_wrapped_points(open(d + "gs-01.bin", "rb").read(), 8)
        n63, b63 = P.decode_wrapped_points(open(d + "gs-63.bin", "rb").read(), None)
        out[f"ref_srs_{cname}_b00_first64"] = np.array(b0, dtype=np.uint64)
        out[f"ref_srs_{cname}_b01_first8"] = np.array(b1, dtype=np.uint64)
        out[f"ref_srs_{cname}_b63_last8"] = np.array(b63[n63 - 8:], dtype=np.uint64)
        out[f"ref_sh_{cname}"] = np.array(P.decode_sh(open(d + "sh.bin", "rb").read()), dtype=np.uint64)
        # raw wire bytes (uint8) for the bincode loader test: the varint length prefix and the first
        # 64 records of gs-00.bin verbatim, and the whole sh.bin
        raw = open(d + "gs-00.bin", "rb").read()
        _, off = P.bincode_varint(raw, 0)
        out[f"ref_gs_{cname}_b00_head_bytes"] = np.frombuffer(raw[: off + 64 * 72], dtype=np.uint8).copy()
        out[f"ref_sh_{cname}_bytes"] = np.frombuffer(open(d + "sh.bin", "rb").read(), dtype=np.uint8).copy()
    ivc = open(f"{REF}/plonk/src/frontend/ivc/mod.rs").read()
    for tag, name in (("fp", "IVC_FP_CIRCUIT"), ("fq", "IVC_FQ_CIRCUIT")):
        block = ivc[ivc.index(f"pub const {name}"):]
        mo = re.search(r"omega:\s*const_f[pq]\(\[([0-9,\s]+)\]\)", block)
        out[f"ref_omega_{tag}16"] = np.array([int(x) for x in mo.group(1).split(",")], dtype=np.uint64)

    # ---- 2. oracle golden vectors over the reference data
    for cname in ("pallas", "vesta"):
        c = P.CURVES[cname]
        r = c.scalar
        G = [P.wrapped_to_point(c, list(x)) for x in out[f"ref_srs_{cname}_b00_first64"]]
        for n in (1, 2, 5, 16, 64):
            sc = [rng.randrange(r) for _ in range(n)]
            if n >= 5:
                sc[0], sc[1], sc[2] = 0, r - 1, 1
            out[f"msm_{cname}_n{n}_scalars"] = fe(sc, r)
            out[f"msm_{cname}_n{n}_result"] = pts(c, [P.msm(c, G[:n], sc)])
        # one IPA round over 16 points (pcdl.rs:404-438), plus the H'-free L/R and the dots
        gs, cs, zs = G[:16], [rng.randrange(r) for _ in range(16)], P.construct_powers(rng.randrange(r), 16, r)
        xi = rng.randrange(1, r)
        L, R, dl, dr, g2, c2, z2 = P.ipa_round(c, gs, cs, zs, xi)
        out[f"ipa_{cname}_cs"] = fe(cs, r)
        out[f"ipa_{cname}_zs"] = fe(zs, r)
        out[f"ipa_{cname}_xi"] = fe([xi, P.inv(xi, r)], r)
        out[f"ipa_{cname}_LR_noH"] = pts(c, [L, R])
        out[f"ipa_{cname}_dots"] = fe([dl, dr], r)
        out[f"ipa_{cname}_gs1"] = pts(c, g2)
        out[f"ipa_{cname}_cs1"] = fe(c2, r)
        out[f"ipa_{cname}_zs1"] = fe(z2, r)
        # test_u_check (pcdl.rs:627-687): xis = [0, 1, 2, 3], three folds of G[0..8] == <h, G>
        xis = [0, 1, 2, 3]
        cur = G[:8]
        for i in range(3):
            half = len(cur) // 2
            cur = [P.add(c, cur[j], P.mul_fast(c, xis[i + 1], cur[j + half])) for j in range(half)]
        hc = P.h_coeffs(xis, r)
        out[f"ucheck_{cname}_U"] = pts(c, cur)
        out[f"ucheck_{cname}_hcoeffs"] = fe(hc, r)
        assert cur[0] == P.msm(c, G[:8], hc)
    for tag, m in (("fp", P.FP_MODULUS), ("fq", P.FQ_MODULUS)):
        for logn in range(0, 9):
            n = 1 << logn
            a = [rng.randrange(m) for _ in range(n)]
            out[f"ntt_{tag}_log{logn}_in"] = fe(a, m)
            out[f"ntt_{tag}_log{logn}_out"] = fe(P.ntt(a, n, m), m)
        # evaluate_over_domain of a longer polynomial (mod X^N - 1) and Horner evaluations
        a = [rng.randrange(m) for _ in range(40)]
        out[f"fold_{tag}_in40"] = fe(a, m)
        out[f"fold_{tag}_out16"] = fe(P.ntt(a, 16, m), m)
        zs = [rng.randrange(m) for _ in range(3)] + [0, 1]
        out[f"eval_{tag}_z"] = fe(zs, m)
        out[f"eval_{tag}_poly"] = fe(a, m)
        out[f"eval_{tag}_out"] = fe([P.horner(a, z, m) for z in zs], m)
        # h(X) = prod (1 + xi_{lg n - i} X^{2^i}) for n = 8 (test_construct_h_with_degree_7)
        xis = [rng.randrange(m) for _ in range(4)]
        out[f"hpoly_{tag}_xis"] = fe(xis, m)
        out[f"hpoly_{tag}_coeffs"] = fe(P.h_coeffs(xis, m), m)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    print(f"wrote {len(out)} arrays")


if __name__ == "__main__":
    main()
