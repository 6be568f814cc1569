"""GPU parity: MSM, pedersen::commit, pcdl::commit, SRS provider.

Bit-exact against the committed golden vectors over the reference SRS, against the C oracle
(ark-ec msm_bigint_wnaf restatement) up to 2^16, and at BASELINE sizes (2^20 reference-recipe SRS,
2^22 synthetic SRS) against the size-independent identity MSM(G, s) = (sum_j s_j k_j) * G where
k_j are the known discrete logs of the bases.
"""
import random

import numpy as np
import pytest

import pasta as P
from halo_amd import group, pcdl, pedersen

pytestmark = pytest.mark.gpu
CURVES = [("pallas", 0), ("vesta", 1)]


def fe(vals, m):
    return np.array([P.int_to_limbs(P.to_mont(v % m, m)) for v in vals], dtype=np.uint64).reshape(-1, 4)


def rand_sc(n, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * 2 + rng.integers(0, 2, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    return np.ascontiguousarray(a)


def limbs_canon(x) -> int:
    return int(x[0]) | int(x[1]) << 64 | int(x[2]) << 128 | int(x[3]) << 192


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_golden_reference_srs(hal, golden, cname, cid):
    bases = golden[f"ref_srs_{cname}_b00_first64"]
    for n in (1, 2, 5, 16, 64):
        got = group.point_dot_affine(golden[f"msm_{cname}_n{n}_scalars"], bases[:n], cname)
        assert np.array_equal(got, golden[f"msm_{cname}_n{n}_result"][0]), n


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_vs_c_oracle(hal, corc, cname, cid):
    c = P.CURVES[cname]
    g = corc.srs_generate(cname, 1 << 16)
    for n in (0, 1, 3, 31, 32, 33, 100, 1000, 4096, 5000, 1 << 16):
        sc = rand_sc(n, n)
        if n >= 8:
            sc[0] = 0                                           # zero scalar
            sc[1] = fe([c.scalar - 1], c.scalar)[0]             # r - 1
            sc[2] = sc[3]                                       # repeated scalar
            sc[4] = fe([1 << 15], c.scalar)[0]                  # digit on a window boundary
            sc[5] = fe([(c.scalar - 1) // 2], c.scalar)[0]      # largest scalar kept as is
            sc[6] = fe([(c.scalar + 1) // 2], c.scalar)[0]      # smallest scalar folded to p - s
            sc[7] = fe([1], c.scalar)[0]
        exp = corc.msm(cname, g[:n], sc) if n else np.zeros(8, dtype=np.uint64)
        assert np.array_equal(group.point_dot_affine(sc, g[:n], cname), exp), n


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_length_is_min_of_inputs(hal, corc, cname, cid):
    """msm_unchecked uses min(#bases, #scalars) (trimmed coefficient vectors, trace.rs:196)."""
    g = corc.srs_generate(cname, 300)
    sc = rand_sc(200, 1)
    assert np.array_equal(group.point_dot_affine(sc, g, cname), corc.msm(cname, g[:200], sc))
    assert np.array_equal(group.point_dot_affine(rand_sc(300, 2), g[:50], cname), corc.msm(cname, g[:50], rand_sc(300, 2)))


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_skewed_scalars(hal, corc, cname, cid):
    """All-equal scalars put every point in one bucket per window (task splitting path)."""
    g = corc.srs_generate(cname, 1 << 14)
    sc = np.ascontiguousarray(np.repeat(rand_sc(1, 5), 1 << 14, axis=0))
    assert np.array_equal(group.point_dot_affine(sc, g, cname), corc.msm(cname, g, sc))
    small = np.zeros((1 << 12, 4), dtype=np.uint64)
    small[:, 0] = np.arange(1 << 12) % 3  # tiny scalars: most windows empty
    assert np.array_equal(group.point_dot_affine(small, g[: 1 << 12], cname), corc.msm(cname, g[: 1 << 12], small))


@pytest.mark.parametrize("cname,cid", CURVES)
def test_pedersen_homomorphism_and_hiding(hal, golden, corc, cname, cid):
    """pedersen.rs:38-79 (homomorphism) with hiding S * w; S, H from the reference's sh.bin."""
    c = P.CURVES[cname]
    r = c.scalar
    g = corc.srs_generate(cname, 4096)
    S, Hh = golden[f"ref_sh_{cname}"]
    group.PublicParams.upload(cname, g, S, Hh, precompute_windows=False)
    rng = random.Random(17)
    for n in (2, 100, 4096):
        m1 = [rng.randrange(r) for _ in range(n)]
        m2 = [rng.randrange(r) for _ in range(n)]
        w1, w2 = rng.randrange(r), rng.randrange(r)
        inner = pedersen.commit(fe([w1 + w2], r), g[:n], fe([a + b for a, b in zip(m1, m2)], r), cname)
        outer = P.add(c, P.wrapped_to_point(c, list(pedersen.commit(fe([w1], r), g[:n], fe(m1, r), cname))),
                      P.wrapped_to_point(c, list(pedersen.commit(fe([w2], r), g[:n], fe(m2, r), cname))))
        assert list(inner) == P.point_to_wrapped(c, outer)
        exp = P.add(c, P.wrapped_to_point(c, list(corc.msm(cname, g[:n], fe(m1, r)))),
                    P.mul_fast(c, w1, P.wrapped_to_point(c, list(S))))
        assert list(pedersen.commit(fe([w1], r), g[:n], fe(m1, r), cname)) == P.point_to_wrapped(c, exp)


def test_pedersen_length_assert(hal, corc):
    g = corc.srs_generate("pallas", 8)
    with pytest.raises(AssertionError, match="ms must be larger than Gs"):
        pedersen.commit(None, g[:4], rand_sc(8, 1), "pallas")


@pytest.mark.parametrize("cname,cid", CURVES)
def test_small_srs_msm_table_path(hal, golden, corc, cname, cid):
    """SRS MSMs of n <= 1024 points (the multiples-table path, msm_srs_small): n = 1, an SRS shorter
    than the table (n0 = SRS length), all-zero scalars, the 1024 / 1025 boundary with the bucket
    pipeline, hiding, and a re-uploaded SRS with a different prefix (the table must be rebuilt)."""
    c = P.CURVES[cname]
    r = c.scalar
    S, Hh = golden[f"ref_sh_{cname}"]
    base = corc.srs_generate(cname, 2048)
    for g in (np.ascontiguousarray(base[:300]), np.ascontiguousarray(base[::-1]), base):
        group.PublicParams.upload(cname, g, S, Hh, precompute_windows=len(g) == 2048)
        N = len(g)
        for d in (0, 3, 255, 1023, 2047):
            if d > N - 1:
                continue
            coeffs = rand_sc(d + 1, d + 11)
            if d >= 7:
                coeffs[:6] = fe([(r - 1) // 2, (r + 1) // 2, 0, 1, r - 1, 1 << 254], r)
            assert np.array_equal(pcdl.commit(coeffs, d, None, cname), corc.msm(cname, g[: d + 1], coeffs)), (N, d)
        zero = np.zeros((16, 4), dtype=np.uint64)
        assert np.array_equal(pcdl.commit(zero, 15, None, cname), corc.msm(cname, g[:16], zero))
        w = rand_sc(1, 5)
        coeffs = rand_sc(64, 6)
        exp = P.add(c, P.wrapped_to_point(c, list(corc.msm(cname, g[:64], coeffs))),
                    P.mul_fast(c, P.from_mont(limbs_canon(w[0]), r), P.wrapped_to_point(c, list(S))))
        assert list(pcdl.commit(coeffs, 63, w, cname)) == P.point_to_wrapped(c, exp)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_pcdl_commit_reference_srs(hal, golden, corc, cname, cid):
    """pcdl.rs:275-287 over the resident reference-recipe SRS (2^16 here), both MSM paths (windowed,
    and window-shifted precomputed bases), with and without hiding; and its assertion messages."""
    c = P.CURVES[cname]
    r = c.scalar
    n = 1 << 16
    g = corc.srs_generate(cname, n)
    S, Hh = golden[f"ref_sh_{cname}"]
    for pre in (False, True):
        group.PublicParams.upload(cname, g, S, Hh, precompute_windows=pre)
        for d in (0, 1, 255, 4095, n - 1):
            coeffs = rand_sc(d + 1, d)
            if d >= 7:  # scalars around p / 2 (k_digits folds s > p / 2 to p - s), 0, 1, p - 1
                coeffs[:8] = fe([(r - 1) // 2, (r + 1) // 2, 0, 1, r - 1, r - 2, (r - 1) // 2 + 2, 1 << 254], r)
            exp = corc.msm(cname, g[: d + 1], coeffs)
            assert np.array_equal(pcdl.commit(coeffs, d, None, cname), exp), (pre, d)
        w = rand_sc(1, 9)
        coeffs = rand_sc(1000, 3)
        exp = P.add(c, P.wrapped_to_point(c, list(corc.msm(cname, g[:1000], coeffs))),
                    P.mul_fast(c, P.from_mont(limbs_canon(w[0]), r), P.wrapped_to_point(c, list(S))))
        assert list(pcdl.commit(coeffs, 1023, w, cname)) == P.point_to_wrapped(c, exp)
    with pytest.raises(AssertionError, match=r"n \(11\) is not a power of two"):
        pcdl.commit(rand_sc(4, 1), 10, None, cname)
    with pytest.raises(AssertionError, match=r"p_deg \(7\) <= d \(3\)"):
        pcdl.commit(rand_sc(8, 1), 3, None, cname)
    with pytest.raises(AssertionError, match=r"d \(131071\) <= D \(65535\)"):
        pcdl.commit(rand_sc(4, 1), (1 << 17) - 1, None, cname)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_2p20_reference_srs_known_logs(hal, corc, cname, cid):
    """BASELINE configs[1]: 2^20-point MSM over the reference SRS recipe, bit-exact via the known
    discrete logs h(j) of the reference's own SRS (crates/group/src/main.rs:55-67)."""
    c = P.CURVES[cname]
    r = c.scalar
    n = 1 << 20
    g = corc.srs_generate(cname, n)
    group.PublicParams.upload(cname, g, precompute_windows=True)
    sc = rand_sc(n, 2024)
    got = pcdl.commit(sc, n - 1, None, cname)
    # sum_j s_j h(srs_index(j)): only 16447 distinct hash indices
    logs = {}
    acc = 0
    sb = sc.tobytes()
    for j in range(n):
        t = P.srs_index(j)
        if t not in logs:
            logs[t] = P.srs_hash_scalar(c, t)
        acc += int.from_bytes(sb[32 * j:32 * j + 32], "little") * logs[t]
    acc = acc * pow(1 << 256, -1, r) % r
    exp = P.mul_fast(c, acc, c.generator)
    assert list(got) == P.point_to_wrapped(c, exp)


def test_msm_2p22_synthetic_srs_known_logs(hal):
    """2^22 points (beyond the reference N = 2^20): synthetic SRS G_j = k_j G, checked as
    (sum_j s_j k_j) G with k_j from halo_synth_scalar."""
    c = P.PALLAS
    r = c.scalar
    n = 1 << 22
    seed = 99
    group.PublicParams.synthesize("pallas", n, seed, precompute_windows=True)
    sc = rand_sc(n, 7)
    got = pcdl.commit(sc, n - 1, None, "pallas")
    k = synth_scalars_np(seed, n)
    from halo_amd.group import synth_scalar
    assert [limbs_canon(k[j]) for j in (0, 1, n - 1)] == [synth_scalar(seed, j) for j in (0, 1, n - 1)]
    sb = sc.tobytes()
    kb = k.tobytes()
    acc = 0
    for j in range(n):
        acc += int.from_bytes(sb[32 * j:32 * j + 32], "little") * int.from_bytes(kb[32 * j:32 * j + 32], "little")
    acc = acc * pow(1 << 256, -1, r) % r  # scalars are Montgomery: s = S / 2^256
    assert list(got) == P.point_to_wrapped(c, P.mul_fast(c, acc, c.generator))


def test_msm_2p20_all_equal_scalars_shifted(hal):
    """Worst-case bucket skew on the window-shifted path: every scalar equal, so each window's digit
    puts all 2^20 points in one bucket (exercises the chunk-group merge, k_group_sums).  Expected:
    (s * sum_j k_j) G over the synthetic SRS; also a half-skewed mix (two distinct scalars)."""
    c = P.PALLAS
    r = c.scalar
    n = 1 << 20
    seed = 5
    group.PublicParams.synthesize("pallas", n, seed, precompute_windows=True)
    k = synth_scalars_np(seed, n)
    kb = k.tobytes()
    ks = [int.from_bytes(kb[32 * j:32 * j + 32], "little") for j in range(n)]
    s1 = fe([r - 12345], r)[0]
    s2 = fe([(1 << 200) + 7], r)[0]
    sc = np.ascontiguousarray(np.repeat(s1[None, :], n, axis=0))
    got = pcdl.commit(sc, n - 1, None, "pallas")
    assert list(got) == P.point_to_wrapped(c, P.mul_fast(c, (r - 12345) * sum(ks) % r, c.generator))
    sc[n // 3:] = s2
    got = pcdl.commit(sc, n - 1, None, "pallas")
    acc = ((r - 12345) * sum(ks[: n // 3]) + ((1 << 200) + 7) * sum(ks[n // 3:])) % r
    assert list(got) == P.point_to_wrapped(c, P.mul_fast(c, acc, c.generator))


@pytest.mark.gpu
def test_msm_small_chunks_shifted_skew(hal):
    """Latency-bound MSMs over the 2^20 window-shifted SRS take short accumulation chunks (K =
    ceil(sqrt(entries / buckets)), msm.hip msm_chunk_len): random, all-equal, two-valued and mostly
    zero scalars at n = 2^4 .. 2^16, checked against (sum_j s_j k_j) G."""
    c = P.PALLAS
    r = c.scalar
    N = 1 << 20
    seed = 11
    group.PublicParams.synthesize("pallas", N, seed, precompute_windows=True)
    k = synth_scalars_np(seed, 1 << 16)
    kb = k.tobytes()
    ks = [int.from_bytes(kb[32 * j:32 * j + 32], "little") for j in range(1 << 16)]
    inv_r = pow(1 << 256, -1, r)
    rng = np.random.default_rng(4)
    for lg in (4, 9, 12, 16):
        n = 1 << lg
        cases = {"random": rand_sc(n, lg)}
        cases["equal"] = np.ascontiguousarray(np.repeat(fe([r - 99], r)[0][None, :], n, axis=0))
        two = cases["equal"].copy()
        two[n // 2:] = fe([(1 << 201) + 3], r)[0]
        cases["two"] = two
        sparse = np.zeros((n, 4), dtype=np.uint64)
        idx = rng.choice(n, size=max(1, n // 64), replace=False)
        sparse[idx] = rand_sc(len(idx), lg + 100)
        cases["sparse"] = sparse
        for name, sc in cases.items():
            got = pcdl.commit(sc, n - 1, None, "pallas")
            sb = sc.tobytes()
            acc = sum(int.from_bytes(sb[32 * j:32 * j + 32], "little") * ks[j] for j in range(n)) * inv_r % r
            assert list(got) == P.point_to_wrapped(c, P.mul_fast(c, acc, c.generator)), (lg, name)


def test_small_table_follows_synthesize(hal, golden, corc):
    """the small-MSM multiples table must be rebuilt when halo_srs_synthesize
    replaces the points (same length, so the same table size): upload A, a small commit over A,
    synthesize B, a small commit over B checked by B's known logs; then an IPA opening's tail over B."""
    c = P.PALLAS
    r = c.scalar
    n = 4096
    S, Hh = golden["ref_sh_pallas"]
    group.PublicParams.upload("pallas", corc.srs_generate("pallas", n), S, Hh, precompute_windows=True)
    sc = rand_sc(300, 77)
    assert np.array_equal(pcdl.commit(sc, 511, None, "pallas"),
                          corc.msm("pallas", corc.srs_generate("pallas", 300), sc))
    seed = 1234
    group.PublicParams.synthesize("pallas", n, seed, precompute_windows=True)
    ks = [limbs_canon(k) for k in synth_scalars_np(seed, 300)]
    sb = sc.tobytes()
    acc = sum(int.from_bytes(sb[32 * j:32 * j + 32], "little") * ks[j] for j in range(300)) * pow(1 << 256, -1, r) % r
    assert list(pcdl.commit(sc, 511, None, "pallas")) == P.point_to_wrapped(c, P.mul_fast(c, acc, c.generator))
    for d in (0, 1023, 2047):  # the table's full range, and both sides of the old 1024 threshold
        sc2 = rand_sc(d + 1, d)
        sb2 = sc2.tobytes()
        ks2 = [limbs_canon(k) for k in synth_scalars_np(seed, d + 1)]
        acc = sum(int.from_bytes(sb2[32 * j:32 * j + 32], "little") * ks2[j] for j in range(d + 1)) * pow(1 << 256, -1, r) % r
        assert list(pcdl.commit(sc2, d, None, "pallas")) == P.point_to_wrapped(c, P.mul_fast(c, acc, c.generator)), d


def synth_scalars_np(seed: int, n: int) -> np.ndarray:
    """numpy restatement of halo_synth_scalar (splitmix64 stream per index; top word masked)."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    j = np.arange(n, dtype=np.uint64)
    st = np.uint64(seed) ^ (j * np.uint64(0xD1B54A32D192ED03))
    out = np.zeros((n, 4), dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in range(4):
            st = st + np.uint64(0x9E3779B97F4A7C15)
            z = st.copy()
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out[:, i] = z ^ (z >> np.uint64(31))
    out[:, 3] &= np.uint64(0x1FFFFFFFFFFFFFFF)
    zero = (out == 0).all(axis=1)
    out[zero, 0] = 1
    del M
    return out


def test_point_sum(hal, corc):
    c = P.PALLAS
    g = corc.srs_generate("pallas", 40)
    exp = None
    for x in g[:37]:
        exp = P.add(c, exp, P.wrapped_to_point(c, list(x)))
    assert list(group.point_sum(g[:37], "pallas")) == P.point_to_wrapped(c, exp)
    assert list(group.point_sum(g[:0], "pallas")) == [0] * 8


@pytest.mark.parametrize("rows,k", [(20, 8), (3, 1), (5, 300)])
def test_point_sum_rows_dev(hal, corc, rows, k):
    """halo_point_sum_rows_dev (the N-rank combine of several steps in one launch): row b of the result
    is the oracle sum of its k points; a row of identities sums to the identity."""
    import ctypes

    import torch

    c = P.PALLAS
    g = corc.srs_generate("pallas", rows * k)
    g[:k] = 0  # row 0: identities only
    d_pts = torch.from_numpy(g.view(np.int64).copy()).cuda()
    d_out = torch.zeros((rows, 8), dtype=torch.int64, device="cuda")
    hal.check(hal.load().halo_point_sum_rows_dev(0, ctypes.c_void_p(d_pts.data_ptr()), rows, k,
                                                 ctypes.c_void_p(d_out.data_ptr()), None))
    got = d_out.cpu().numpy().view(np.uint64)
    for b in range(rows):
        exp = None
        for x in g[b * k:(b + 1) * k]:
            if int(x.any()):
                exp = P.add(c, exp, P.wrapped_to_point(c, list(x)))
        assert list(got[b]) == (P.point_to_wrapped(c, exp) if exp is not None else [0] * 8), b


def test_srs_read_roundtrip(hal, corc):
    g = corc.srs_generate("vesta", 1000)
    group.PublicParams.upload("vesta", g, precompute_windows=False)
    assert group.PublicParams.len("vesta") == 1000
    assert np.array_equal(group.PublicParams.read("vesta", 100, 50), g[100:150])


@pytest.mark.parametrize("cname,cid", CURVES)
def test_trace_commit_batch(hal, corc, cname, cid):
    """SURVEY f2 (trace.rs:165-192): batched from_vec_and_domain -> interpolate -> pcdl::commit,
    against the per-polynomial path (poly.Evals + pcdl.commit) and the oracle MSM; includes an
    all-zero row, a row of low degree, and the degree assertion."""
    from halo_amd import poly
    c = P.CURVES[cname]
    r = c.scalar
    n = 1 << 10
    g = corc.srs_generate(cname, n)
    for pre in (False, True):
        group.PublicParams.upload(cname, g, precompute_windows=pre)
        ev = np.stack([rand_sc(n, 100 + i) for i in range(5)])
        ev[1] = 0
        # row 2: evaluations of a constant polynomial (degree 0 after interpolation)
        ev[2] = fe([7], r)[0]
        commits, coeffs = pcdl.trace_commit_batch(ev, n - 1, cname, want_coeffs=True)
        dom = poly.Domain(n, "fp" if cname == "pallas" else "fq")
        for i in range(5):
            p = poly.Evals.from_vec_and_domain(ev[i], dom).interpolate_by_ref()
            assert np.array_equal(coeffs[i], p), i
            assert np.array_equal(commits[i], pcdl.commit(p, n - 1, None, cname)), i
            exp = corc.msm(cname, g[: len(p)], p) if len(p) else np.zeros(8, dtype=np.uint64)
            assert np.array_equal(commits[i], exp), i
        assert len(coeffs[1]) == 0 and len(coeffs[2]) == 1
    with pytest.raises(AssertionError, match=r"p_deg \(1023\) <= d \(511\)"):
        pcdl.trace_commit_batch(ev, 511, cname)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_srs_load_bincode(hal, golden, corc, cname, cid):
    """SURVEY f3 (pp.rs:26-61): the reference's own gs-00.bin bytes (length prefix + first 64
    records, verbatim) and sh.bin decode on the device to the golden points / (S, H); general
    varints take the host path and an off-curve point is rejected like wrappers.rs:606."""
    c = P.CURVES[cname]
    head = golden[f"ref_gs_{cname}_b00_head_bytes"].tobytes()
    sh = golden[f"ref_sh_{cname}_bytes"].tobytes()
    group.PublicParams.load_bincode(cname, [head], sh, n=64, precompute_windows=False)
    assert np.array_equal(group.PublicParams.read(cname, 0, 64), golden[f"ref_srs_{cname}_b00_first64"])
    # (S, H) installed: the hiding term of pcdl::commit uses S (compare with the upload path)
    w = rand_sc(1, 3)
    coeffs = rand_sc(64, 4)
    got = pcdl.commit(coeffs, 63, w, cname)
    S, Hh = golden[f"ref_sh_{cname}"]
    group.PublicParams.upload(cname, golden[f"ref_srs_{cname}_b00_first64"], S, Hh, precompute_windows=False)
    assert np.array_equal(got, pcdl.commit(coeffs, 63, w, cname))
    # two blocks re-encoded by a bincode varint encoder (32 + 32 points)

    def enc_varint(v):
        if v < 251:
            return bytes([v])
        for tag, width in ((251, 2), (252, 4), (253, 8)):
            if v < 1 << (8 * width):
                return bytes([tag]) + v.to_bytes(width, "little")
        raise ValueError

    pts = golden[f"ref_srs_{cname}_b00_first64"]

    def block(points):
        return enc_varint(len(points)) + b"".join(enc_varint(int(l)) for p in points for l in p)
    group.PublicParams.load_bincode(cname, [block(pts[:32]), block(pts[32:])], sh, n=64,
                                    precompute_windows=False)
    assert np.array_equal(group.PublicParams.read(cname, 0, 64), pts)
    bad = pts[:4].copy()
    bad[2] = [1, 0, 0, 0, 2, 0, 0, 0]  # small limbs (1-byte varints), not on the curve
    with pytest.raises(Exception, match="is_on_curve"):
        group.PublicParams.load_bincode(cname, [block(bad)], sh, n=4, precompute_windows=False)
    with pytest.raises(Exception, match="is_power_of_two"):
        group.PublicParams.load_bincode(cname, [head], sh, n=48, precompute_windows=False)
    with pytest.raises(Exception, match="n <= N"):
        group.PublicParams.load_bincode(cname, [block(pts[:16])], sh, n=32, precompute_windows=False)


def test_async_msm_caller_bases_concurrent_streams(hal, corc):
    """halo_msm_dev_async over caller-supplied (ark) bases from three torch streams at once, several
    MSMs per stream back to back: every result equals the synchronous halo_msm of the same inputs
    (the conversion buffer of a scratch set is claimed together with the set, after its last tail)."""
    import ctypes

    import torch
    L = hal.load()
    g = corc.srs_generate("pallas", (1 << 14) + 128)
    streams = [torch.cuda.Stream() for _ in range(3)]
    jobs = []
    for k in range(9):
        n = [1 << 14, 5000, 1 << 12][k % 3]
        bases = torch.from_numpy(np.ascontiguousarray(g[(k * 37) % 100:][:n]).view(np.int64)).cuda()
        sc = rand_sc(n, 500 + k)
        jobs.append((bases, torch.from_numpy(sc.view(np.int64)).cuda(), n, sc))
    outs = torch.zeros((len(jobs), 8), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for k, (bases, sc_d, n, _) in enumerate(jobs):
        st = streams[k % 3]
        hal.check(L.halo_msm_dev_async(0, ctypes.c_void_p(bases.data_ptr()), ctypes.c_void_p(sc_d.data_ptr()), n,
                                       ctypes.c_void_p(outs[k].data_ptr()), ctypes.c_void_p(st.cuda_stream)))
    for st in streams:
        hal.check(L.halo_msm_join(ctypes.c_void_p(st.cuda_stream)))
    torch.cuda.synchronize()
    got = outs.cpu().numpy().view(np.uint64)
    for k, (bases, _, n, sc) in enumerate(jobs):
        exp = np.zeros(8, dtype=np.uint64)
        b = bases.cpu().numpy().view(np.uint64)
        hal.check(L.halo_msm(0, hal.ptr(np.ascontiguousarray(b)), n, hal.ptr(sc), n, hal.ptr(exp)))
        assert np.array_equal(got[k], exp), k


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_batch_dev_one_msm_path(hal, corc, cname, cid):
    """halo_msm_batch_dev (the commitment batches of protocol.rs:114,263 / trace.rs:188-192): k
    polynomials of ragged lengths (including empty and length 1) over the resident window-shifted
    SRS as one MSM with (polynomial, bucket) keys, each result bit-exact vs the oracle MSM; and the
    same batch on the per-MSM pipelined path (tuning msm_multi_max = 0)."""
    import ctypes

    import torch
    L = hal.load()
    n = 1 << 12
    g = corc.srs_generate(cname, n)
    group.PublicParams.upload(cname, g, precompute_windows=True)
    lens = [n, 0, 1, 777, n - 1, n, 2048, 5]
    scs = [rand_sc(max(m, 1), 40 + i)[:m] for i, m in enumerate(lens)]
    scs[0][:3] = scs[0][3]  # repeated scalars
    dev = [torch.from_numpy(np.ascontiguousarray(sc).view(np.int64)).cuda() if len(sc) else torch.zeros((1, 4), dtype=torch.int64, device="cuda") for sc in scs]
    ptrs = (ctypes.c_void_p * len(lens))(*[d.data_ptr() for d in dev])
    lns = (ctypes.c_size_t * len(lens))(*lens)
    out = torch.zeros((len(lens), 8), dtype=torch.int64, device="cuda")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    exps = [corc.msm(cname, g[:m], scs[i]) if m else np.zeros(8, dtype=np.uint64) for i, m in enumerate(lens)]
    for multi_max in (-1, 0):  # the default one-MSM batch, then one pipelined MSM per polynomial
        out.zero_()
        with hal.tuning(msm_multi_max=multi_max):
            hal.check(L.halo_msm_batch_dev(cid, ptrs, lns, len(lens), ctypes.c_void_p(out.data_ptr()), sp))
            hal.check(L.halo_msm_join(sp))
        got = out.cpu().numpy().view(np.uint64)
        for i, m in enumerate(lens):
            assert np.array_equal(got[i], exps[i]), (multi_max, i, m)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_point_dot_projective(hal, corc, cname, cid):
    """group.rs:53-56 point_dot over ark Projective bases: random Jacobian representatives
    (lambda^2 x, lambda^3 y, lambda) of the SRS points, one identity (Z = 0), against the oracle MSM
    of the affine points."""
    c = P.CURVES[cname]
    q = c.base
    n = 3000
    g = corc.srs_generate(cname, n)
    rng = random.Random(7)
    jac = np.zeros((n, 12), dtype=np.uint64)
    aff = g.copy()
    for i in range(n):
        pt = P.wrapped_to_point(c, [int(x) for x in g[i]])
        if i == 17:
            jac[i] = P.int_to_limbs(P.to_mont(1, q)) + P.int_to_limbs(P.to_mont(1, q)) + [0, 0, 0, 0]
            aff[i] = 0
            continue
        lam = rng.randrange(1, q)
        X, Y = pt[0] * lam * lam % q, pt[1] * pow(lam, 3, q) % q
        jac[i] = P.int_to_limbs(P.to_mont(X, q)) + P.int_to_limbs(P.to_mont(Y, q)) + P.int_to_limbs(P.to_mont(lam, q))
    sc = rand_sc(n, 77)
    assert np.array_equal(group.point_dot(sc, jac, cname), corc.msm(cname, aff, sc))
    assert np.array_equal(group.point_dot(sc[:100], jac, cname), corc.msm(cname, aff[:100], sc[:100]))


def test_window_partitioned_msm_virtual_ranks(hal, corc):
    """BASELINE configs[4] on one GPU with P virtual ranks: halo_msm_srs_windows_dev over each rank's
    window range, partials summed (halo_point_sum) == the whole MSM; one rank's partial equals the
    oracle MSM of its window share of the scalars (corc.window_scalars restates the digit recoding)."""
    import ctypes

    import torch
    from halo_amd.dist import window_range
    L = hal.load()
    n = 1 << 14
    g = corc.srs_generate("pallas", n)
    group.PublicParams.upload("pallas", g, precompute_windows=True)
    c = L.halo_srs_window_bits(0)
    W = L.halo_srs_windows(0)
    assert W == -(-255 // c)
    sc = rand_sc(n, 91)
    sc[0] = fe([P.PALLAS.scalar - 1], P.PALLAS.scalar)[0]
    d_sc = torch.from_numpy(sc.view(np.int64)).cuda()
    full = pcdl.commit(sc, n - 1, None, "pallas")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for world in (2, 3, 8):
        outs = torch.zeros((world, 8), dtype=torch.int64, device="cuda")
        for r in range(world):
            lo, hi = window_range(W, r, world)
            hal.check(L.halo_msm_srs_windows_dev(0, ctypes.c_void_p(d_sc.data_ptr()), n, lo, hi,
                                                 ctypes.c_void_p(outs[r].data_ptr()), sp))
        hal.check(L.halo_msm_join(sp))
        parts = outs.cpu().numpy().view(np.uint64)
        assert np.array_equal(group.point_sum(parts, "pallas"), full), world
        if world == 3:
            lo, hi = window_range(W, 1, 3)
            assert np.array_equal(parts[1], corc.msm("pallas", g, corc.window_scalars("pallas", sc, c, lo, hi)))


@pytest.mark.parametrize("cname,cid", CURVES)
def test_shifted_srs_with_identity_points(hal, corc, cname, cid):
    """k_acc skips the bases' identity test only when the window precompute found no identity point in
    the SRS; an SRS holding identities (WrappedPoint (0, 0)) must keep the test: the window-shifted
    MSM against the C oracle, with identity points among the bases (and an identity-free SRS after)."""
    n = 1 << 14  # above the small-table path (n <= 8192): the bucket MSM over the shifted SRS
    g = corc.srs_generate(cname, n).copy()
    g[[0, 5, 1000, n - 1]] = 0
    group.PublicParams.upload(cname, g, precompute_windows=True)
    for seed in (31, 32):
        sc = rand_sc(n, seed)
        assert np.array_equal(pcdl.commit(sc, n - 1, None, cname), corc.msm(cname, g, sc)), seed
    g2 = corc.srs_generate(cname, n)
    group.PublicParams.upload(cname, g2, precompute_windows=True)
    sc = rand_sc(n, 33)
    assert np.array_equal(pcdl.commit(sc, n - 1, None, cname), corc.msm(cname, g2, sc))


@pytest.mark.parametrize("cname,cid", CURVES)
def test_msm_caller_bases_sparse_windows(hal, corc, cname, cid):
    """k_final's Horner over the window sums (caller bases, GLV windows): window sums that are the
    identity at the top, in the middle and at the bottom of the chain (scalars built from a few set
    bits), and a single term, against the C oracle."""
    c = P.CURVES[cname]
    g = corc.srs_generate(cname, 64)
    cases = [
        [1] * 64,                                           # only window 0
        [1 << 200] * 64,                                     # only a high window (GLV: both halves)
        [(1 << 250) + 1] * 32 + [1 << 100] * 32,             # top and bottom, empty middle
        [(c.scalar - 1)] + [0] * 63,                         # one term, r - 1
        list(range(64)),                                     # small scalars: empty upper windows
    ]
    for k, vals in enumerate(cases):
        sc = fe(vals, c.scalar)
        exp = corc.msm(cname, g, sc)
        assert np.array_equal(group.point_dot_affine(sc, g, cname), exp), k
