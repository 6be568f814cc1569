#!/usr/bin/env python3
"""Regenerate tests/golden/transcript.npz (committed).  Run in the build container, where the
reference checkout is mounted read-only at /root/reference:

    python3 tests/golden/make_transcript.py

Arrays (uint64 limbs; loaded with numpy's default allow_pickle=False):
1. Data taken from the reference's files:
   * poseidon_{fq,fp}_mds / _rc : FQ_MDS / FQ_ROUND_CONSTANTS and FP_* of
     crates/group/src/poseidon_consts.rs (Montgomery limbs, as written there);
   * kimchi_{i}_in / kimchi_{i}_out : crates/poseidon/test-vectors/kimchi-vecs.json (Fq, canonical
     limbs; the hex strings are little-endian field encodings, inner_sponge.rs:278-281);
   * mina_fq_* / mina_fp_* : the manual_mina_fq (Vesta sponge over Fp) / manual_mina_fp (Pallas sponge
     over Fq) vectors of inner_sponge.rs:323-368.
2. pcdl::open EvalProofs computed by the CPU restatement (oracle/pcdl_ref.py: open_without_eval with
   the Poseidon PCDL transcript, oracle/poseidon.py) over the reference-recipe SRS and the
   reference's (S, H) (crates/group/.precompute/*/sh.bin): case open_<curve>_n<N>_<plain|hiding>_*.
"""
from __future__ import annotations

import json
import os
import random
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pasta as P  # noqa: E402

REF = "/root/reference/crates"


def limbs_of_hex(h: str) -> list[int]:
    return P.int_to_limbs(int.from_bytes(bytes.fromhex(h), "little"))


def parse_consts(src: str, name: str, rows: int) -> np.ndarray:
    body = src[src.index(f"const {name}"):]
    body = body[: body.index("];\n") + 2]
    vals = [[int(x) for x in m.split(",")] for m in re.findall(r"f[pq]\(\[([0-9, ]+)\]\)", body)]
    assert len(vals) == rows * 3, (name, len(vals))
    return np.array(vals, dtype=np.uint64)


def main():
    out = {}
    src = open(f"{REF}/group/src/poseidon_consts.rs").read()
    out["poseidon_fq_mds"] = parse_consts(src, "FQ_MDS", 3)
    out["poseidon_fq_rc"] = parse_consts(src, "FQ_ROUND_CONSTANTS", 55)
    out["poseidon_fp_mds"] = parse_consts(src, "FP_MDS", 3)
    out["poseidon_fp_rc"] = parse_consts(src, "FP_ROUND_CONSTANTS", 55)
    vecs = json.load(open(f"{REF}/poseidon/test-vectors/kimchi-vecs.json"))["test_vectors"]
    for i, v in enumerate(vecs):
        out[f"kimchi_{i}_in"] = np.array([limbs_of_hex(h) for h in v["input"]], dtype=np.uint64).reshape(-1, 4)
        out[f"kimchi_{i}_out"] = np.array(limbs_of_hex(v["output"]), dtype=np.uint64)
    isrc = open(f"{REF}/poseidon/src/inner_sponge.rs").read()
    for test, tag in (("manual_mina_fq", "mina_fq"), ("manual_mina_fp", "mina_fp")):
        body = isrc[isrc.index(f"fn {test}"):]
        body = body[: body.index("assert_eq!")]
        exp = re.search(r'expected_out_hex = "([0-9a-f]+)"', body).group(1)
        ins = re.findall(r'"([0-9a-f]{64})"', body[body.index("inputs_hex"):])
        out[f"{tag}_in"] = np.array([limbs_of_hex(h) for h in ins], dtype=np.uint64)
        out[f"{tag}_out"] = np.array(limbs_of_hex(exp), dtype=np.uint64)

    # the Poseidon constants first: oracle/poseidon.py reads them from this file
    np.savez_compressed(os.path.join(HERE, "transcript.npz"), **out)
    import corc
    import pcdl_ref
    corc.build()
    rng = random.Random(0x50434C44)
    for cname, n, hiding in (("pallas", 16, False), ("pallas", 64, True), ("pallas", 256, False),
                             ("pallas", 1024, True), ("vesta", 16, True), ("vesta", 64, False)):
        c = P.CURVES[cname]
        r = c.scalar
        d = n - 1
        gs = corc.srs_generate(cname, n)
        S, H = [P.wrapped_to_point(c, [int(x) for x in row]) for row in
                P.decode_sh(open(f"{REF}/group/.precompute/{cname}/sh.bin", "rb").read())]
        plen = n - rng.randrange(0, 3)  # degree <= d, sometimes lower
        p = [rng.randrange(r) for _ in range(plen)]
        z = rng.randrange(r)
        v = P.horner(p, z, r)
        w = rng.randrange(r) if hiding else None
        q = [rng.randrange(r) for _ in range(d)] if hiding else None
        w_bar = rng.randrange(r) if hiding else None
        C = pcdl_ref.commit(cname, gs, p, w, S)
        pi = pcdl_ref.open_without_eval(cname, p, C, d, z, v, gs, S, H, w=w, q=q, w_bar=w_bar)
        key = f"open_{cname}_n{n}_{'hiding' if hiding else 'plain'}"
        fe = lambda xs: np.array([P.int_to_limbs(P.to_mont(x % r, r)) for x in xs], dtype=np.uint64).reshape(-1, 4)  # noqa: E731
        pw = lambda pts: np.array([P.point_to_wrapped(c, x) for x in pts], dtype=np.uint64).reshape(-1, 8)  # noqa: E731
        out[key + "_p"] = fe(p)
        out[key + "_zv"] = fe([z, v])
        out[key + "_C"] = pw([C])
        out[key + "_Ls"] = pw(pi["Ls"])
        out[key + "_Rs"] = pw(pi["Rs"])
        out[key + "_U"] = pw([pi["U"]])
        out[key + "_c"] = fe([pi["c"]])
        out[key + "_xis"] = fe(pi["xis"])
        if hiding:
            out[key + "_w"] = fe([w, w_bar])
            out[key + "_q"] = fe(q)
            out[key + "_Cbar"] = pw([pi["C_bar"]])
            out[key + "_wprime_alpha"] = fe([pi["w_prime"], pi["alpha"]])
        print(key, "done", flush=True)
    # round 3: openings long enough for the device's weighted -> materialised ->
    # tail rounds (n > 2048) under the reference's transcript order (pcdl.rs:387-425).  Their inputs
    # p, q, z, w, w_bar are not stored: det_scalars(seed, k) (shared with tests/test_gpu_transcript.py)
    # regenerates them from the stored seed, so only the outputs take space.
    for seed, (cname, n, hiding) in enumerate((("pallas", 4096, True), ("pallas", 16384, False),
                                                ("vesta", 4096, False), ("vesta", 16384, True),
                                                ("pallas", 4096, False), ("vesta", 4096, True)), start=100):
        c = P.CURVES[cname]
        r = c.scalar
        d = n - 1
        gs = corc.srs_generate(cname, n)
        S, H = [P.wrapped_to_point(c, [int(x) for x in row]) for row in
                P.decode_sh(open(f"{REF}/group/.precompute/{cname}/sh.bin", "rb").read())]
        ins = det_scalars(seed, 2 * n + 4)  # p (n - 1: degree d - 1), q (d), z, w, w_bar
        val = [P.from_mont(limbs_int(x), r) for x in ins]
        p = val[: n - 1]
        q = val[n: n + d] if hiding else None
        z = val[2 * n]
        w = val[2 * n + 1] if hiding else None
        w_bar = val[2 * n + 2] if hiding else None
        v = P.horner(p, z, r)
        C = pcdl_ref.commit(cname, gs, p, w, S)
        pi = pcdl_ref.open_without_eval(cname, p, C, d, z, v, gs, S, H, w=w, q=q, w_bar=w_bar)
        key = f"big_{cname}_n{n}_{'hiding' if hiding else 'plain'}"
        fe = lambda xs: np.array([P.int_to_limbs(P.to_mont(x % r, r)) for x in xs], dtype=np.uint64).reshape(-1, 4)  # noqa: E731
        pw = lambda pts: np.array([P.point_to_wrapped(c, x) for x in pts], dtype=np.uint64).reshape(-1, 8)  # noqa: E731
        out[key + "_seed"] = np.array([seed], dtype=np.uint64)
        out[key + "_zv"] = fe([z, v])
        out[key + "_C"] = pw([C])
        out[key + "_Ls"] = pw(pi["Ls"])
        out[key + "_Rs"] = pw(pi["Rs"])
        out[key + "_U"] = pw([pi["U"]])
        out[key + "_c"] = fe([pi["c"]])
        if hiding:
            out[key + "_Cbar"] = pw([pi["C_bar"]])
            out[key + "_wprime_alpha"] = fe([pi["w_prime"], pi["alpha"]])
        print(key, "done", flush=True)
    np.savez_compressed(os.path.join(HERE, "transcript.npz"), **out)


def det_scalars(seed: int, k: int) -> np.ndarray:
    """k Montgomery-form scalars (valid in Fp and Fq: every value is < 2^254 < r) from seed."""
    a = np.random.default_rng(seed).integers(0, 2**64 - 1, size=(k, 4), dtype=np.uint64, endpoint=True)
    a[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    return np.ascontiguousarray(a)


def limbs_int(x) -> int:
    return int(x[0]) | int(x[1]) << 64 | int(x[2]) << 128 | int(x[3]) << 192


if __name__ == "__main__":
    main()
