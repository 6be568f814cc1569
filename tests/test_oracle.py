"""CPU tests: the oracle itself, pinned to the reference's committed data.

The reference (Rust) cannot be built here, so the oracle is pinned by (1) the SRS points / S / H the
reference ships in crates/group/.precompute (decoded into tests/golden/golden.npz), which fix the
curve, generator, Montgomery convention and the SRS recipe of crates/group/src/main.rs:55-67;
(2) IVC_FP/FQ_CIRCUIT.omega (crates/plonk/src/frontend/ivc/mod.rs:55,112), which fix the NTT domain
generator; (3) the reference's own algebraic tests re-expressed (pedersen.rs:38-79 homomorphism,
pcdl.rs:627-687 test_u_check, pcdl.rs:735-758 h(X) coefficients, protocol.rs:1037-1118 evals_*).
"""
import random

import numpy as np
import pytest

import pasta as P

CURVES = ["pallas", "vesta"]


def fe(vals, m):
    return np.array([P.int_to_limbs(P.to_mont(v % m, m)) for v in vals], dtype=np.uint64).reshape(-1, 4)


def unfe(a, m):
    return [P.from_mont(P.limbs_to_int(r), m) for r in np.asarray(a).reshape(-1, 4)]


@pytest.mark.parametrize("cname", CURVES)
def test_srs_recipe_matches_reference_files(golden, cname):
    c = P.CURVES[cname]
    b0 = golden[f"ref_srs_{cname}_b00_first64"]
    for k in (0, 1, 2, 17, 63):
        assert P.wrapped_to_point(c, list(b0[k])) == P.srs_hash_point(c, P.srs_index(k))
    b1 = golden[f"ref_srs_{cname}_b01_first8"]
    for k in range(8):
        assert P.wrapped_to_point(c, list(b1[k])) == P.srs_hash_point(c, P.srs_index(16384 + k))
    b63 = golden[f"ref_srs_{cname}_b63_last8"]
    j = 64 * 16384 - 1
    assert P.wrapped_to_point(c, list(b63[-1])) == P.srs_hash_point(c, P.srs_index(j))
    S, Hh = golden[f"ref_sh_{cname}"]
    assert P.wrapped_to_point(c, list(S)) == P.srs_hash_point(c, 0)
    assert P.wrapped_to_point(c, list(Hh)) == P.srs_hash_point(c, 1)


@pytest.mark.parametrize("cname", CURVES)
def test_c_srs_generator_matches_reference_files(golden, corc, cname):
    g = corc.srs_generate(cname, 16384 + 8)
    assert np.array_equal(g[:64], golden[f"ref_srs_{cname}_b00_first64"])
    assert np.array_equal(g[16384:16392], golden[f"ref_srs_{cname}_b01_first8"])


def test_omega_matches_reference(golden):
    for tag, m in (("fp", P.FP_MODULUS), ("fq", P.FQ_MODULUS)):
        w = P.from_mont(P.limbs_to_int(golden[f"ref_omega_{tag}16"]), m)
        assert w == P.root_of_unity(m, 1 << 16)
        assert pow(w, 1 << 15, m) == m - 1  # exact order 2^16


@pytest.mark.parametrize("cname", CURVES)
def test_c_msm_golden(golden, corc, cname):
    bases = golden[f"ref_srs_{cname}_b00_first64"]
    for n in (1, 2, 5, 16, 64):
        got = corc.msm(cname, bases[:n], golden[f"msm_{cname}_n{n}_scalars"])
        assert np.array_equal(got, golden[f"msm_{cname}_n{n}_result"][0])


@pytest.mark.parametrize("cname", CURVES)
def test_c_msm_known_discrete_logs(corc, cname):
    """MSM over SRS points with known logs h_j equals (sum s_j h_j) * G (size-independent check)."""
    c = P.CURVES[cname]
    n = 300
    g = corc.srs_generate(cname, n)
    rng = random.Random(3)
    sc = [rng.randrange(c.scalar) for _ in range(n)]
    k = sum(s * P.srs_hash_scalar(c, P.srs_index(j)) for j, s in enumerate(sc)) % c.scalar
    got = corc.msm(cname, g, fe(sc, c.scalar))
    assert list(got) == P.point_to_wrapped(c, P.mul_fast(c, k, c.generator))


@pytest.mark.parametrize("cname", CURVES)
def test_homomorphism(corc, cname):
    """pedersen.rs:38-79: commit(m1 + m2) = commit(m1) + commit(m2)."""
    c = P.CURVES[cname]
    r = c.scalar
    n = 257
    g = corc.srs_generate(cname, n)
    rng = random.Random(11)
    m1 = [rng.randrange(r) for _ in range(n)]
    m2 = [rng.randrange(r) for _ in range(n)]
    a = P.wrapped_to_point(c, list(corc.msm(cname, g, fe(m1, r))))
    b = P.wrapped_to_point(c, list(corc.msm(cname, g, fe(m2, r))))
    s = P.wrapped_to_point(c, list(corc.msm(cname, g, fe([x + y for x, y in zip(m1, m2)], r))))
    assert P.add(c, a, b) == s


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_c_ntt_golden(golden, corc, tag):
    for logn in range(0, 9):
        x = golden[f"ntt_{tag}_log{logn}_in"]
        assert np.array_equal(corc.ntt(tag, x), golden[f"ntt_{tag}_log{logn}_out"])
        assert np.array_equal(corc.ntt(tag, golden[f"ntt_{tag}_log{logn}_out"], inverse=True), x)


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_ntt_convolution_theorem(corc, tag):
    """protocol.rs:1037-1118 evals_mul: NTT(a) * NTT(b) interpolates to a * b (2n domain)."""
    m = P.FIELDS[tag]
    rng = random.Random(5)
    for n in (32, 256, 1024):
        a = [rng.randrange(m) for _ in range(n)]
        b = [rng.randrange(m) for _ in range(n)]
        A = unfe(corc.ntt(tag, fe(a + [0] * n, m)), m)
        B = unfe(corc.ntt(tag, fe(b + [0] * n, m)), m)
        prod = unfe(corc.ntt(tag, fe([x * y for x, y in zip(A, B)], m), inverse=True), m)
        if n <= 256:
            assert P.trim(prod) == P.poly_mul(a, b, m)
        else:  # spot-check coefficients of a*b
            for k in (0, 1, n - 1, 2 * n - 2):
                assert prod[k] == sum(a[i] * b[k - i] for i in range(max(0, k - n + 1), min(k, n - 1) + 1)) % m


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_fold_and_eval_golden(golden, corc, tag):
    m = P.FIELDS[tag]
    a = unfe(golden[f"fold_{tag}_in40"], m)
    assert P.ntt(a, 16, m) == unfe(golden[f"fold_{tag}_out16"], m)
    poly = golden[f"eval_{tag}_poly"]
    for z, v in zip(golden[f"eval_{tag}_z"], golden[f"eval_{tag}_out"]):
        assert np.array_equal(corc.poly_eval(tag, poly, z), v)


@pytest.mark.parametrize("cname", CURVES)
def test_c_ipa_round_golden(golden, corc, cname):
    bases = golden[f"ref_srs_{cname}_b00_first64"][:16]
    xi, xinv = golden[f"ipa_{cname}_xi"]
    gs, cs, zs = corc.ipa_fold(cname, bases, golden[f"ipa_{cname}_cs"], golden[f"ipa_{cname}_zs"], xi, xinv)
    assert np.array_equal(gs, golden[f"ipa_{cname}_gs1"])
    assert np.array_equal(cs, golden[f"ipa_{cname}_cs1"])
    assert np.array_equal(zs, golden[f"ipa_{cname}_zs1"])
    cs0 = golden[f"ipa_{cname}_cs"]
    zs0 = golden[f"ipa_{cname}_zs"]
    L = corc.msm(cname, bases[:8], cs0[8:])
    R = corc.msm(cname, bases[8:], cs0[:8])
    assert np.array_equal(np.stack([L, R]), golden[f"ipa_{cname}_LR_noH"])
    tag = "fp" if cname == "pallas" else "fq"
    assert np.array_equal(corc.scalar_dot(tag, cs0[8:], zs0[:8]), golden[f"ipa_{cname}_dots"][0])
    assert np.array_equal(corc.scalar_dot(tag, cs0[:8], zs0[8:]), golden[f"ipa_{cname}_dots"][1])


@pytest.mark.parametrize("cname", CURVES)
def test_u_check(golden, corc, cname):
    """pcdl.rs:627-687: three folds with xis = [0,1,2,3] equal the MSM with h(X)'s coefficients."""
    c = P.CURVES[cname]
    r = c.scalar
    bases = np.ascontiguousarray(golden[f"ref_srs_{cname}_b00_first64"][:8])
    gs = bases.copy()
    zeros = np.zeros((8, 4), dtype=np.uint64)
    for xi in (1, 2, 3):
        half = len(gs) // 2
        x = fe([xi], r)[0]
        gs, _, _ = corc.ipa_fold(cname, gs, zeros[: 2 * half], zeros[: 2 * half], x, fe([P.inv(xi, r)], r)[0])
    assert np.array_equal(gs, golden[f"ucheck_{cname}_U"])
    assert np.array_equal(corc.msm(cname, bases, golden[f"ucheck_{cname}_hcoeffs"]), golden[f"ucheck_{cname}_U"][0])


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_h_coeffs(golden, tag):
    """pcdl.rs:735-758 test_construct_h_with_degree_7: coefficient k = product of xi's by bit."""
    m = P.FIELDS[tag]
    xis = unfe(golden[f"hpoly_{tag}_xis"], m)
    exp = [1, xis[3], xis[2], xis[2] * xis[3], xis[1], xis[1] * xis[3], xis[1] * xis[2], xis[1] * xis[2] * xis[3]]
    assert P.h_coeffs(xis, m) == [e % m for e in exp] == unfe(golden[f"hpoly_{tag}_coeffs"], m)
    # and the product form (pcdl.rs:198-219)
    h = [1]
    for i in range(3):
        term = [0] * ((1 << i) + 1)
        term[0], term[1 << i] = 1, xis[3 - i]
        h = P.poly_mul(h, term, m)
    assert h == P.h_coeffs(xis, m)


def test_prover_pipeline_runs_on_cpu_restatement():
    """The generic naive_prover pipeline (halo_amd.prover) on the CPU restatement backend at n = 8:
    the checker side of tests/test_gpu_prover.py must itself run (no GPU needed)."""
    import pasta as P
    import prover_ref

    from halo_amd import prover

    c = P.PALLAS
    n = 8
    srs = np.array([P.point_to_wrapped(c, P.mul_fast(c, 1000 + i, c.generator)) for i in range(n)], dtype=np.uint64)
    B = prover_ref.RefBackend("pallas", srs, srs[1])
    out = prover.naive_prover(B, prover.synthetic_witness(B, n, seed=3), n, prover.Challenges(B.m))
    assert len(out["C_ws"]) == 16 and len(out["C_ts"]) == 16 and len(out["vs"]) == 91
    assert len(out["q_r"]["Ls"]) == 3 and len(out["acc"]["Rs"]) == 3
    # the opened polynomial's evaluation is the one the instance reports
    assert out["q_r"]["v"] == out["q_r"]["v"] % B.m


def test_succinct_check_and_decider_on_cpu_restatement(corc):
    """oracle/pcdl_check.py (pcdl.rs:483-583) accepts the three openings the naive_prover pipeline
    produces on the CPU restatement backend (q_r, q_r_omega, acc::prover's open of h), the decider
    identity U == commit(h) holds for each, and a tampered L, c or v is rejected."""
    import pcdl_check
    import prover_ref

    from halo_amd import prover

    c = P.PALLAS
    n = 16
    srs = np.array([P.point_to_wrapped(c, P.mul_fast(c, 5000 + 7 * i, c.generator)) for i in range(n)], dtype=np.uint64)
    H = srs[1]
    B = prover_ref.RefBackend("pallas", srs, H)
    out = prover.naive_prover(B, prover.synthetic_witness(B, n, seed=11), n, prover.Challenges(B.m))
    for key in ("q_r", "q_r_omega", "acc"):
        q = out[key]
        pcdl_check.succinct_check("pallas", q["C"], n - 1, q["z"], q["v"], q["Ls"], q["Rs"], q["U"], q["c"], q["xis"], H)
        assert pcdl_check.decider_commit_matches("pallas", q["U"], q["xis"], srs, corc.msm), key
    q = out["q_r"]
    with pytest.raises(AssertionError, match="C_\\(log_n\\)"):
        pcdl_check.succinct_check("pallas", q["C"], n - 1, q["z"], (q["v"] + 1) % B.m, q["Ls"], q["Rs"], q["U"],
                                  q["c"], q["xis"], H)
    with pytest.raises(AssertionError, match="C_\\(log_n\\)"):
        pcdl_check.succinct_check("pallas", q["C"], n - 1, q["z"], q["v"], [q["Rs"][0]] + q["Ls"][1:], q["Rs"],
                                  q["U"], q["c"], q["xis"], H)
    with pytest.raises(AssertionError, match="C_\\(log_n\\)"):
        pcdl_check.succinct_check("pallas", q["C"], n - 1, q["z"], q["v"], q["Ls"], q["Rs"], q["U"], q["c"] + 1,
                                  q["xis"], H)
    m = B.m
    xis = q["xis"]
    z = 0x1234
    assert pcdl_check.h_eval(xis, z, m) == P.horner(pcdl_check.h_coeffs(xis, m), z, m)
    assert pcdl_check.h_coeffs(xis, m) == P.h_coeffs(xis, m)


@pytest.mark.parametrize("cname", CURVES)
def test_known_log_msm_identity(corc, cname):
    """corc.known_log_msm (the 2^22 / 2^24 MSM checker) equals the oracle MSM over bases G_j = k_j G
    built from the same synthetic logs (corc.synth_scalars restates halo_synth_scalar)."""
    c = P.CURVES[cname]
    n = 300
    k = corc.synth_scalars(77, n)
    assert all(P.limbs_to_int(k[j]) < c.scalar for j in range(n))
    bases = np.stack([corc.generator_mul(cname, k[j]) for j in range(n)])
    rng = np.random.default_rng(1)
    sc = rng.integers(0, 2**62, size=(n, 4), dtype=np.uint64)
    assert np.array_equal(corc.known_log_msm(cname, sc, k), corc.msm(cname, bases, sc))


def test_poseidon_sponge_reference_vectors():
    """oracle/poseidon.py against the reference's own Poseidon vectors: the six Kimchi vectors
    (kimchi-vecs.json, inner_sponge.rs:315-321, Pallas sponge over Fq) and the two Mina vectors
    (inner_sponge.rs:323-368: Vesta sponge over Fp, Pallas sponge over Fq)."""
    import os

    import poseidon
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "transcript.npz"))
    i = 0
    while f"kimchi_{i}_in" in g:
        s = poseidon.InnerSponge("fq")
        s.absorb([P.limbs_to_int(x) for x in g[f"kimchi_{i}_in"]])
        assert s.squeeze() == P.limbs_to_int(g[f"kimchi_{i}_out"]), i
        i += 1
    assert i == 6
    for tag, field in (("mina_fq", "fp"), ("mina_fp", "fq")):
        s = poseidon.InnerSponge(field)
        s.absorb([P.limbs_to_int(x) for x in g[f"{tag}_in"]])
        assert s.squeeze() == P.limbs_to_int(g[f"{tag}_out"]), tag


def test_transcript_pcdl_open_fixtures_verify(golden, corc):
    """The committed pcdl::open fixtures (tests/golden/make_transcript.py: oracle/pcdl_ref.py with the
    Poseidon transcript) pass the transcript-driven succinct_check (pcdl.rs:483-554, challenges
    re-derived) and the decider U == commit(h) (pcdl.rs:579-581), hiding and plain."""
    import os

    import pcdl_check
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "transcript.npz"))
    keys = sorted({k[:-2] for k in g.files if k.startswith("open_") and k.endswith("_p")})
    assert len(keys) == 6
    for key in keys:
        cname = key.split("_")[1]
        c = P.CURVES[cname]
        n = int(key.split("_")[2][1:])
        r = c.scalar
        S, Hh = golden[f"ref_sh_{cname}"]
        z, v = unfe(g[key + "_zv"], r)
        hiding = key.endswith("hiding")
        wp = unfe(g[key + "_wprime_alpha"], r)[0] if hiding else None
        xis = pcdl_check.succinct_check_transcript(
            cname, g[key + "_C"][0], n - 1, z, v, list(g[key + "_Ls"]), list(g[key + "_Rs"]), g[key + "_U"][0],
            unfe(g[key + "_c"], r)[0], Hh, S=S, C_bar=g[key + "_Cbar"][0] if hiding else None, w_prime=wp)
        assert xis == unfe(g[key + "_xis"], r), key
        if n <= 256:
            srs = corc.srs_generate(cname, n)
            assert pcdl_check.decider_commit_matches(cname, g[key + "_U"][0], xis, srs, corc.msm), key
