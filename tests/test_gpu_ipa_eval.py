"""GPU parity: IPA folding, polynomial evaluation / dots / powers (a8).

The IPA round loop is driven exactly like pcdl::open_without_eval (pcdl.rs:392-450): device-resident
(G, c, z), L/R per round, a host transcript supplying xi, fold.  The transcript here is a
deterministic stand-in (SHA3 of the round's L, R); the same stand-in drives the pure-Python oracle
loop, so every L, R, the final U and c compare bit-exactly.  test_u_check (pcdl.rs:627-687) pins
the fold against the h(X)-coefficient MSM.
"""
import hashlib
import random

import numpy as np
import pytest

import pasta as P
from halo_amd import group, pcdl, poly

pytestmark = pytest.mark.gpu
CURVES = [("pallas", 0), ("vesta", 1)]


def fe(vals, m):
    return np.array([P.int_to_limbs(P.to_mont(v % m, m)) for v in vals], dtype=np.uint64).reshape(-1, 4)


def unfe(a, m):
    return [P.from_mont(P.limbs_to_int(r), m) for r in np.asarray(a).reshape(-1, 4)]


@pytest.mark.parametrize("cname,cid", CURVES)
def test_fold_host_golden(hal, golden, cname, cid):
    L = hal.load()
    gs = np.ascontiguousarray(golden[f"ref_srs_{cname}_b00_first64"][:16].copy())
    cs = np.ascontiguousarray(golden[f"ipa_{cname}_cs"].copy())
    zs = np.ascontiguousarray(golden[f"ipa_{cname}_zs"].copy())
    xi, xinv = golden[f"ipa_{cname}_xi"]
    hal.check(L.halo_ipa_fold_host(cid, hal.ptr(gs), hal.ptr(cs), hal.ptr(zs), 8, hal.ptr(np.ascontiguousarray(xi)),
                                   hal.ptr(np.ascontiguousarray(xinv))))
    assert np.array_equal(gs[:8], golden[f"ipa_{cname}_gs1"])
    assert np.array_equal(cs[:8], golden[f"ipa_{cname}_cs1"])
    assert np.array_equal(zs[:8], golden[f"ipa_{cname}_zs1"])


@pytest.mark.parametrize("cname,cid", CURVES)
def test_u_check(hal, golden, corc, cname, cid):
    """pcdl.rs:627-687: folding G[0..8] with xis = [0,1,2,3] gives <h, G>."""
    c = P.CURVES[cname]
    r = c.scalar
    g = corc.srs_generate(cname, 8)
    group.PublicParams.upload(cname, g, precompute_windows=False)
    ses = pcdl.IpaSession(np.zeros((8, 4), dtype=np.uint64), fe([5], r), g[0], cname)
    for xi in (1, 2, 3):
        ses.fold(fe([xi], r), fe([P.inv(xi, r)], r))
    U, _ = ses.end()
    assert np.array_equal(U, golden[f"ucheck_{cname}_U"][0])
    assert np.array_equal(U, group.point_dot_affine(golden[f"ucheck_{cname}_hcoeffs"], g, cname))


def transcript(cname):
    c = P.CURVES[cname]

    def challenge(xi_prev, L, R):
        h = hashlib.sha3_256((b"" if xi_prev is None else np.asarray(xi_prev).tobytes()) + L.tobytes() + R.tobytes())
        v = int.from_bytes(h.digest(), "little") % c.scalar or 1
        return fe([v], c.scalar)[0]

    def inverse(x):
        return fe([P.inv(P.from_mont(P.limbs_to_int(x), c.scalar), c.scalar)], c.scalar)[0]

    return challenge, inverse


@pytest.mark.parametrize("cname,cid", CURVES)
@pytest.mark.parametrize("n", [2, 16, 64])
def test_ipa_rounds_vs_oracle(hal, corc, cname, cid, n):
    """The whole round loop of pcdl.rs:404-438 against a pure-Python restatement."""
    c = P.CURVES[cname]
    r = c.scalar
    g = corc.srs_generate(cname, 64)
    group.PublicParams.upload(cname, g, precompute_windows=False)
    rng = random.Random(n)
    cs = [rng.randrange(r) for _ in range(n)]
    z = rng.randrange(r)
    Hp = P.mul_fast(c, rng.randrange(r), c.generator)
    challenge, inverse = transcript(cname)
    Ls, Rs, U, cfin = pcdl.ipa_rounds(fe(cs, r), fe([z], r), np.array(P.point_to_wrapped(c, Hp), dtype=np.uint64),
                                      challenge, inverse, cname)
    # oracle loop
    G = [P.wrapped_to_point(c, list(x)) for x in g[:n]]
    C, Z = cs[:], P.construct_powers(z, n, r)
    xi = None
    for k in range(n.bit_length() - 1):
        m = len(G) // 2
        L = P.add(c, P.msm(c, G[:m], C[m:]), P.mul_fast(c, P.scalar_dot(C[m:], Z[:m], r), Hp))
        R = P.add(c, P.msm(c, G[m:], C[:m]), P.mul_fast(c, P.scalar_dot(C[:m], Z[m:], r), Hp))
        assert list(Ls[k]) == P.point_to_wrapped(c, L), k
        assert list(Rs[k]) == P.point_to_wrapped(c, R), k
        xi = challenge(xi, np.array(P.point_to_wrapped(c, L), dtype=np.uint64),
                       np.array(P.point_to_wrapped(c, R), dtype=np.uint64))
        x = P.from_mont(P.limbs_to_int(xi), r)
        _, _, _, _, G, C, Z = P.ipa_round(c, G, C, Z, x)
    assert list(U) == P.point_to_wrapped(c, G[0])
    assert unfe(cfin, r) == [C[0]]


@pytest.mark.parametrize("cname,cid", CURVES)
@pytest.mark.parametrize("n", [2, 16, 2048, 8192])
def test_ipa_xi_mode_equals_h_prime(hal, corc, cname, cid, n):
    """halo_ipa_begin_xi (H' = xi_0 H formed on the device, hiding terms from the shared 2^i H table
    scaled by xi_0) gives the same L, R, U, c as a session handed H' = xi_0 H, across the weighted
    rounds, the materialisation at 1024 and the tail rounds; two different H in a row rebuild the
    table."""
    c = P.CURVES[cname]
    r = c.scalar
    g = corc.srs_generate(cname, n)
    group.PublicParams.upload(cname, g, precompute_windows=False)
    rng = random.Random(n + cid)
    cs = fe([rng.randrange(r) for _ in range(n)], r)
    zz = fe([rng.randrange(r)], r)
    for trial in range(2):
        Hpt = P.mul_fast(c, rng.randrange(1, r), c.generator)
        Hw = np.array(P.point_to_wrapped(c, Hpt), dtype=np.uint64)
        x0v = rng.randrange(1, r)
        x0 = fe([x0v], r)
        Hp = np.array(P.point_to_wrapped(c, P.mul_fast(c, x0v, Hpt)), dtype=np.uint64)
        a = pcdl.IpaSession(cs, zz, Hp, cname)
        b = pcdl.IpaSession.with_xi(cs, zz, Hw, x0, cname)
        challenge, inverse = transcript(cname)
        xi = None
        for k in range(n.bit_length() - 1):
            La, Ra = a.round_lr()
            Lb, Rb = b.round_lr()
            assert np.array_equal(La, Lb) and np.array_equal(Ra, Rb), (trial, k)
            xi = challenge(xi, La, Ra)
            a.fold(xi, inverse(xi))
            b.fold(xi, inverse(xi))
        Ua, ca = a.end()
        Ub, cb = b.end()
        assert np.array_equal(Ua, Ub) and np.array_equal(ca, cb), trial


@pytest.mark.parametrize("c_s", [18, 20])
def test_ipa_wide_shifted_windows(hal, corc, c_s):
    """A full window-shifted set of width 18 / 20 (halo_srs_precompute_window_range over every window)
    drives the weighted rounds and the switch round's shared-scalar batch, whose sub-digits then need
    three windows (2^(c_s / 2) > 256 buckets): the opening's L, R, U, c equal the same
    opening over the SRS's default-width copies."""
    c = P.PALLAS
    r = c.scalar
    n = 1 << 14
    L = hal.load()
    g = corc.srs_generate("pallas", n)
    rng = random.Random(c_s)
    cs = fe([rng.randrange(r) for _ in range(n)], r)
    zz = fe([rng.randrange(r)], r)
    Hw = np.array(P.point_to_wrapped(c, P.mul_fast(c, rng.randrange(1, r), c.generator)), dtype=np.uint64)
    x0 = fe([rng.randrange(1, r)], r)
    chal = [fe([rng.randrange(1, r)], r)[0] for _ in range(14)]
    inv = [fe([P.inv(P.from_mont(P.limbs_to_int(x), r), r)], r)[0] for x in chal]

    def opening():
        s_ = pcdl.IpaSession.with_xi(cs, zz, Hw, x0, "pallas")
        lr = []
        for rd in range(14):
            lr += [a.copy() for a in s_.round_lr()]
            s_.fold(chal[rd], inv[rd])
        return lr + list(s_.end())

    group.PublicParams.upload("pallas", g, precompute_windows=True)
    assert L.halo_srs_window_bits(0) < 18
    ref = opening()
    hal.check(L.halo_srs_precompute_window_range(0, c_s, 0, 0))
    assert L.halo_srs_window_bits(0) == c_s
    got = opening()
    for a, b in zip(ref, got):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("k", [2, 3, 5])
def test_ipa_lockstep_sessions_equal_single(hal, corc, k):
    """halo_ipa_round_lr_multi over k sessions in lockstep (their weighted rounds share one L/R MSM,
    up to 4 sessions per MSM) and halo_ipa_end_multi give every session's L, R, U, c exactly as that
    session run alone with halo_ipa_end."""
    import ctypes
    c = P.PALLAS
    r = c.scalar
    n = 1 << 13
    L = hal.load()
    g = corc.srs_generate("pallas", n)
    group.PublicParams.upload("pallas", g, precompute_windows=True)
    rng = random.Random(k)
    Hw = np.array(P.point_to_wrapped(c, P.mul_fast(c, rng.randrange(1, r), c.generator)), dtype=np.uint64)
    jobs = [(fe([rng.randrange(r) for _ in range(n)], r), fe([rng.randrange(r)], r), fe([rng.randrange(1, r)], r))
            for _ in range(k)]
    chal = [[fe([rng.randrange(1, r)], r)[0] for _ in range(13)] for _ in range(k)]
    inv = [[fe([P.inv(P.from_mont(P.limbs_to_int(x), r), r)], r)[0] for x in row] for row in chal]

    def run(idx):
        sess = [pcdl.IpaSession.with_xi(jobs[i][0], jobs[i][1], Hw, jobs[i][2], "pallas") for i in idx]
        arr = (ctypes.c_void_p * len(sess))(*[s_._s.value for s_ in sess])
        out = [([], []) for _ in idx]
        for rd in range(13):
            Lb = np.zeros((len(idx), 8), dtype=np.uint64)
            Rb = np.zeros((len(idx), 8), dtype=np.uint64)
            hal.check(L.halo_ipa_round_lr_multi(arr, len(idx), hal.ptr(Lb), hal.ptr(Rb)))
            xa = np.ascontiguousarray(np.stack([chal[i][rd] for i in idx]))
            xia = np.ascontiguousarray(np.stack([inv[i][rd] for i in idx]))
            hal.check(L.halo_ipa_fold_multi(arr, len(idx), hal.ptr(xa), hal.ptr(xia)))
            for q in range(len(idx)):
                out[q][0].append(Lb[q].copy())
                out[q][1].append(Rb[q].copy())
        ends = pcdl.IpaSession.end_many(sess) if len(sess) > 1 else [s_.end() for s_ in sess]
        return [(o[0], o[1], e[0], e[1]) for o, e in zip(out, ends)]

    together = run(list(range(k)))
    for i in range(k):
        alone = run([i])[0]
        for a, b in zip(together[i][0] + together[i][1], alone[0] + alone[1]):
            assert np.array_equal(a, b), i
        assert np.array_equal(together[i][2], alone[2]) and np.array_equal(together[i][3], alone[3]), i
    # and the lockstep session 0 against the C oracle's round loop itself (not only the lone session)
    to_int = lambda x: P.from_mont(P.limbs_to_int(x), r)
    zv = to_int(jobs[0][1][0])
    Hp = np.array(P.point_to_wrapped(c, P.mul_fast(c, to_int(jobs[0][2][0]), P.wrapped_to_point(c, Hw))),
                  dtype=np.uint64)
    Ls, Rs, U, c0 = oracle_ipa_loop(corc, "pallas", g, jobs[0][0], fe(P.construct_powers(zv, n, r), r), Hp, chal[0],
                                    inv[0])
    for a, b in zip(together[0][0] + together[0][1], Ls + Rs):
        assert np.array_equal(a, b)
    assert np.array_equal(together[0][2], U) and np.array_equal(together[0][3], c0)


def test_ipa_fold_large_vs_c_oracle(hal, corc):
    """One fold at m = 2^14 (per-element scalar multiplication + affine normalisation)."""
    c = P.PALLAS
    r = c.scalar
    m = 1 << 14
    g = corc.srs_generate("pallas", 2 * m)
    rng = np.random.default_rng(3)
    cs = rng.integers(0, 2**62, size=(2 * m, 4), dtype=np.uint64)
    zs = rng.integers(0, 2**62, size=(2 * m, 4), dtype=np.uint64)
    xi = fe([12345678901234567890123456789], r)[0]
    xinv = fe([P.inv(12345678901234567890123456789, r)], r)[0]
    eg, ec, ez = corc.ipa_fold("pallas", g, cs, zs, xi, xinv)
    G, C, Z = g.copy(), cs.copy(), zs.copy()
    hal.check(hal.load().halo_ipa_fold_host(0, hal.ptr(G), hal.ptr(C), hal.ptr(Z), m, hal.ptr(np.ascontiguousarray(xi)),
                                            hal.ptr(np.ascontiguousarray(xinv))))
    assert np.array_equal(G[:m], eg) and np.array_equal(C[:m], ec) and np.array_equal(Z[:m], ez)


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_poly_eval_golden_and_batch(hal, golden, corc, tag):
    m = P.FIELDS[tag]
    p40 = golden[f"eval_{tag}_poly"]
    for z, v in zip(golden[f"eval_{tag}_z"], golden[f"eval_{tag}_out"]):
        assert np.array_equal(poly.evaluate_batch([p40], z, tag)[0], v)
    rng = np.random.default_rng(1)
    polys = [np.ascontiguousarray(rng.integers(0, 2**62, size=(k, 4), dtype=np.uint64)) for k in (0, 1, 7, 8191, 100000)]
    z = fe([987654321987654321], m)[0]
    got = poly.evaluate_batch(polys, z, tag)
    for p, v in zip(polys, got):
        exp = corc.poly_eval(tag, p, z) if len(p) else np.zeros(4, dtype=np.uint64)
        assert np.array_equal(v, exp)


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_scalar_dot_and_powers(hal, corc, tag):
    m = P.FIELDS[tag]
    rng = np.random.default_rng(2)
    for n in (0, 1, 1000, 100003):
        x = np.ascontiguousarray(rng.integers(0, 2**62, size=(n, 4), dtype=np.uint64))
        y = np.ascontiguousarray(rng.integers(0, 2**62, size=(n, 4), dtype=np.uint64))
        assert np.array_equal(group.scalar_dot(x, y, tag), corc.scalar_dot(tag, x, y) if n else np.zeros(4, np.uint64))
    z = 31337
    pw = group.construct_powers(fe([z], m), 1000, tag)
    assert unfe(pw, m) == P.construct_powers(z, 1000, m)


# ---- h(X) coefficients (HPoly::get_poly) and the decider commitment --------
@pytest.mark.parametrize("tag,cname", [("fp", "pallas"), ("fq", "vesta")])
def test_hpoly_golden(hal, golden, tag, cname):
    """pcdl.rs:735-758 test_construct_h_with_degree_7 on the device."""
    got = pcdl.HPoly(golden[f"hpoly_{tag}_xis"], cname).get_poly()
    assert np.array_equal(got, golden[f"hpoly_{tag}_coeffs"])


@pytest.mark.parametrize("cname", ["pallas", "vesta"])
def test_hpoly_random_and_combine(hal, cname):
    c = P.CURVES[cname]
    r = c.scalar
    rnd = random.Random(17)
    for lg in (1, 2, 5, 11, 14):
        xis = [rnd.randrange(1, r) for _ in range(lg + 1)]
        assert unfe(pcdl.HPoly(fe(xis, r), cname).get_poly(), r) == P.h_coeffs(xis, r), lg
    lg = 9
    hs_x = [[rnd.randrange(1, r) for _ in range(lg + 1)] for _ in range(3)]
    alphas = [rnd.randrange(r) for _ in range(3)]
    got = pcdl.HPoly.combine([pcdl.HPoly(fe(x, r), cname) for x in hs_x], fe(alphas, r))
    exp = [sum(a * h for a, h in zip(alphas, col)) % r for col in zip(*[P.h_coeffs(x, r) for x in hs_x])]
    while exp and exp[-1] == 0:
        exp.pop()
    assert unfe(got, r) == exp


@pytest.mark.parametrize("cname,cid", CURVES)
def test_decider_commit_equals_folded_U(hal, golden, corc, cname, cid):
    """pcdl::check step 5 (pcdl.rs:579): U == pedersen::commit(Gs[0..d+1], h.get_poly().coeffs) for
    the U that the IPA fold produces from the same challenges (the identity test_u_check pins)."""
    c = P.CURVES[cname]
    r = c.scalar
    # the reference's own u-check case: xis = [0, 1, 2, 3] over G[0..8]
    g = corc.srs_generate(cname, 1 << 12)
    group.PublicParams.upload(cname, g, precompute_windows=False)
    assert np.array_equal(pcdl.decider_commit(fe([0, 1, 2, 3], r), 7, cname), golden[f"ucheck_{cname}_U"][0])
    # random challenges over 2^12 bases: fold on the device, then the decider MSM
    rnd = random.Random(5)
    lg = 12
    xis = [rnd.randrange(1, r) for _ in range(lg + 1)]
    ses = pcdl.IpaSession(np.zeros((1 << lg, 4), dtype=np.uint64), fe([5], r), g[0], cname)
    for xi in xis[1:]:
        ses.fold(fe([xi], r), fe([P.inv(xi, r)], r))
    U, _ = ses.end()
    assert np.array_equal(pcdl.decider_commit(fe(xis, r), (1 << lg) - 1, cname), U)
    with pytest.raises(AssertionError, match=r"ms must be larger than Gs: \(Gs: 8\), \(ms: 4096\)"):
        pcdl.decider_commit(fe(xis, r), 7, cname)


# ---------------------------------------------------------------------------------------------
# distributed opening and evaluation, P virtual ranks on one GPU (the gather is the
# identity over the P local sessions; tests/test_dist.py runs the same code over gloo ranks)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("cname,cid", CURVES)
@pytest.mark.parametrize("n,world", [(64, 4), (1024, 8), (16, 2)])
def test_sharded_ipa_virtual_ranks(hal, corc, cname, cid, n, world):
    """Strided shards + per-round point sums + collapsed final rounds == the single session."""
    from halo_amd.dist import GpuIpaOps, ipa_shard, sharded_ipa_rounds

    c = P.CURVES[cname]
    r = c.scalar
    g = corc.srs_generate(cname, n)
    group.PublicParams.upload(cname, g, precompute_windows=False)
    rng = random.Random(n + world)
    cs = fe([rng.randrange(r) for _ in range(n)], r)
    z = rng.randrange(r)
    zs = fe(P.construct_powers(z, n, r), r)
    Hp = np.array(P.point_to_wrapped(c, P.mul_fast(c, rng.randrange(r), c.generator)), dtype=np.uint64)
    challenge, inverse = transcript(cname)
    Ls, Rs, U, cfin = pcdl.ipa_rounds(cs, fe([z], r), Hp, challenge, inverse, cname)
    shards = [(ipa_shard(g[:n], k, world), ipa_shard(cs, k, world), ipa_shard(zs, k, world)) for k in range(world)]
    Ls2, Rs2, U2, c2 = sharded_ipa_rounds(shards, Hp, challenge, inverse, GpuIpaOps(cname), world, lambda o: o)
    assert len(Ls2) == len(Ls)
    for a, b in zip(Ls + Rs, Ls2 + Rs2):
        assert np.array_equal(a, b)
    assert np.array_equal(U, U2)
    assert np.array_equal(cfin, c2)


@pytest.mark.parametrize("logn,world", [(20, 8), (14, 4), (12, 2)])
def test_sharded_ipa_weighted_virtual_ranks(hal, logn, world):
    """The distributed opening on the weighted-round path: rank r's resident SRS
    is its shard G[r::P] with window-shifted copies, its session the single-GPU weighted one over
    c[r::P] with z^P and H'_r = z^r H' (halo_amd.dist.GpuWeightedIpaOps).  The virtual ranks run one
    after another against a fixed challenge sequence (each needs its own resident shard on the one
    GPU); every L, R, U and c equals the single-GPU opening over the whole SRS with the same
    challenges -- 2^20 over 8 ranks is the BASELINE size."""
    from halo_amd.dist import GpuIpaOps, GpuWeightedIpaOps, sharded_ipa_fixed_challenges, xyzz_pair_reducer

    c = P.PALLAS
    r = c.scalar
    n = 1 << logn
    L = hal.load()
    hal.check(L.halo_srs_synthesize(0, n, 4242 + logn))
    G = np.zeros((n, 8), dtype=np.uint64)
    hal.check(L.halo_srs_read(0, 0, n, hal.ptr(G)))
    hal.check(L.halo_srs_precompute_windows(0))
    rng = np.random.default_rng(logn)
    cs = np.ascontiguousarray(rng.integers(0, 2**62, size=(n, 4), dtype=np.uint64))
    pr = random.Random(logn)
    z = fe([pr.randrange(1, r)], r)[0]
    Hp = G[3].copy()
    xis = [fe([pr.randrange(1, r)], r)[0] for _ in range(logn)]
    xinv = [fe([P.inv(P.from_mont(P.limbs_to_int(x), r), r)], r)[0] for x in xis]
    # the single-GPU opening over the whole resident SRS (weighted rounds too)
    ses = pcdl.IpaSession(cs, z, Hp, "pallas")
    Ls, Rs = [], []
    for k in range(logn):
        Lk, Rk = ses.round_lr()
        Ls.append(Lk.copy())
        Rs.append(Rk.copy())
        ses.fold(xis[k], xinv[k])
    U, cfin = ses.end()

    def ops_for_rank(k):
        group.PublicParams.upload("pallas", np.ascontiguousarray(G[k::world]), precompute_windows=True)
        return GpuWeightedIpaOps("pallas", k, world)

    def shard_for_rank(k):
        return (np.ascontiguousarray(cs[k::world]), z)

    # the shard sessions must be weighted ones: their G is never materialised
    probe = ops_for_rank(1)
    s1 = probe.begin(shard_for_rank(1), Hp)
    with pytest.raises(hal.HaloError):
        s1.state()
    hal.check(L.halo_ipa_end(s1._s, None, None))  # (released without U: not every round ran)
    s1._s = None
    Ls2, Rs2, U2, c2 = sharded_ipa_fixed_challenges(ops_for_rank, shard_for_rank, Hp, xis, xinv, world,
                                                    lambda pts: group.point_sum(pts, "pallas"), GpuIpaOps("pallas"))
    assert len(Ls2) == logn
    for k, (a, b) in enumerate(zip(Ls + Rs, Ls2 + Rs2)):
        assert np.array_equal(a, b), k
    assert np.array_equal(U, U2)
    assert np.array_equal(cfin, c2)
    # the device-resident per-round reduce: L_r, R_r left on the device as packed
    # XYZZ (halo_ipa_round_lr_dev), summed there (halo_point_sum_xyzz_dev), one D2H per round
    Ls3, Rs3, U3, c3 = sharded_ipa_fixed_challenges(ops_for_rank, shard_for_rank, Hp, xis, xinv, world, None,
                                                    GpuIpaOps("pallas"),
                                                    reduce_pairs=xyzz_pair_reducer("pallas", "cuda"))
    for k, (a, b) in enumerate(zip(Ls + Rs, Ls3 + Rs3)):
        assert np.array_equal(a, b), k
    assert np.array_equal(U, U3)
    assert np.array_equal(cfin, c3)


def oracle_ipa_loop(corc, cname, G, cs, zs, Hp, xis, xinvs):
    """pcdl.rs:404-438 on the C oracle: per round L = <c_r, G_l> + <c_r, z_l> H' and R likewise (one
    oracle MSM each, H' as an extra base), then the oracle fold (pcdl.rs:427-435)."""
    field = "fp" if cname == "pallas" else "fq"
    G, C, Z = (np.ascontiguousarray(a) for a in (G, cs, zs))
    Ls, Rs = [], []
    for k in range(len(G).bit_length() - 1):
        m = len(G) // 2
        dl = corc.scalar_dot(field, C[m:], Z[:m])
        dr = corc.scalar_dot(field, C[:m], Z[m:])
        Ls.append(corc.msm(cname, np.ascontiguousarray(np.vstack([G[:m], Hp[None]])),
                           np.ascontiguousarray(np.vstack([C[m:], dl[None]]))))
        Rs.append(corc.msm(cname, np.ascontiguousarray(np.vstack([G[m:], Hp[None]])),
                           np.ascontiguousarray(np.vstack([C[:m], dr[None]]))))
        G, C, Z = corc.ipa_fold(cname, G, C, Z, xis[k], xinvs[k])
    return Ls, Rs, G[0], C[0]


@pytest.mark.parametrize("logn,world", [(15, 2), (15, 4)])
def test_sharded_ipa_weighted_vs_oracle(hal, corc, logn, world):
    """The distributed opening on the weighted-round path checked against the C oracle's round loop
    directly (the 2^20 virtual-rank test compares with the one-GPU opening only).  At
    2^15 over 2 / 4 ranks each shard runs weighted rounds (2^14 / 2^13 per rank), the switch and tail
    rounds; both per-round reduces (host pairs and the device-resident XYZZ sums) must give the
    oracle's L, R, U, c."""
    from halo_amd.dist import GpuIpaOps, GpuWeightedIpaOps, sharded_ipa_fixed_challenges, xyzz_pair_reducer

    c = P.PALLAS
    r = c.scalar
    n = 1 << logn
    L = hal.load()
    hal.check(L.halo_srs_synthesize(0, n, 777 + logn))
    G = np.zeros((n, 8), dtype=np.uint64)
    hal.check(L.halo_srs_read(0, 0, n, hal.ptr(G)))
    pr = random.Random(logn * world)
    cs = fe([pr.randrange(r) for _ in range(n)], r)
    zv = pr.randrange(1, r)
    z = fe([zv], r)[0]
    zs = fe(P.construct_powers(zv, n, r), r)
    Hp = G[5].copy()
    xis = [fe([pr.randrange(1, r)], r)[0] for _ in range(logn)]
    xinv = [fe([P.inv(P.from_mont(P.limbs_to_int(x), r), r)], r)[0] for x in xis]
    Ls, Rs, U, cfin = oracle_ipa_loop(corc, "pallas", G, cs, zs, Hp, xis, xinv)

    def ops_for_rank(k):
        group.PublicParams.upload("pallas", np.ascontiguousarray(G[k::world]), precompute_windows=True)
        return GpuWeightedIpaOps("pallas", k, world)

    def shard_for_rank(k):
        return (np.ascontiguousarray(cs[k::world]), z)

    for reduce_pairs in (None, xyzz_pair_reducer("pallas", "cuda")):
        Ls2, Rs2, U2, c2 = sharded_ipa_fixed_challenges(ops_for_rank, shard_for_rank, Hp, xis, xinv, world,
                                                        lambda pts: group.point_sum(pts, "pallas"),
                                                        GpuIpaOps("pallas"), reduce_pairs=reduce_pairs)
        assert len(Ls2) == logn
        for k, (a, b) in enumerate(zip(Ls + Rs, Ls2 + Rs2)):
            assert np.array_equal(a, b), k
        assert np.array_equal(U, U2)
        assert np.array_equal(cfin, c2)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_ipa_weighted_one_element_per_rank(hal, world):
    """n == P on the weighted path: no shard rounds run, each rank contributes its one
    element (G_r = element 0 of its resident shard, c_r, z^r) through GpuWeightedIpaOps.trivial_final,
    and the lg P collapsed rounds reproduce the single-GPU opening of the same instance.  Virtual
    ranks: rank r's shard is uploaded before its element is read; gather hands the collected elements
    to sharded_ipa_rounds."""
    from halo_amd.dist import GpuWeightedIpaOps, sharded_ipa_rounds

    c = P.PALLAS
    r = c.scalar
    n = world
    L = hal.load()
    hal.check(L.halo_srs_synthesize(0, 64, 5150 + world))
    G = np.zeros((n, 8), dtype=np.uint64)
    hal.check(L.halo_srs_read(0, 0, n, hal.ptr(G)))
    pr = random.Random(world)
    cs = fe([pr.randrange(r) for _ in range(n)], r)
    z = fe([pr.randrange(1, r)], r)[0]
    Hp = np.array(P.point_to_wrapped(c, P.mul_fast(c, pr.randrange(1, r), c.generator)), dtype=np.uint64)
    challenge, inverse = transcript("pallas")
    group.PublicParams.upload("pallas", np.ascontiguousarray(G), precompute_windows=False)
    Ls, Rs, U, cfin = pcdl.ipa_rounds(cs, z, Hp, challenge, inverse, "pallas")
    finals = []
    for k in range(world):
        group.PublicParams.upload("pallas", np.ascontiguousarray(G[k::world]), precompute_windows=False)
        fin = GpuWeightedIpaOps("pallas", k, world).trivial_final((np.ascontiguousarray(cs[k::world]), z))
        assert np.array_equal(fin[0][0], G[k]) and np.array_equal(fin[1][0], cs[k])
        assert unfe(fin[2], r) == [pow(unfe([z], r)[0], k, r)]
        finals.append(fin)
    ops0 = GpuWeightedIpaOps("pallas", 0, world)
    Ls2, Rs2, U2, c2 = sharded_ipa_rounds([(np.ascontiguousarray(cs[0::world]), z)], Hp, challenge, inverse, ops0,
                                          world, lambda objs: finals)
    assert len(Ls2) == len(Ls)
    for a, b in zip(Ls + Rs, Ls2 + Rs2):
        assert np.array_equal(a, b)
    assert np.array_equal(U, U2)
    assert np.array_equal(cfin, c2)


@pytest.mark.parametrize("n,world", [(1000, 3), (1 << 16, 8), (5, 8)])
def test_sharded_poly_eval_virtual_ranks(hal, n, world):
    from halo_amd.dist import PolyOps, poly_eval_combine, poly_eval_partial, shard_range

    rng = np.random.default_rng(n)
    m = P.FIELDS["fp"]
    coeffs = fe([int(x) for x in rng.integers(0, 2**62, size=n)], m)
    z = fe([int(rng.integers(1, 2**62))], m)[0]
    ops = PolyOps("fp")
    parts = [poly_eval_partial(coeffs[slice(*shard_range(n, k, world))], z, ops) for k in range(world)]
    got = poly_eval_combine(parts, n, z, ops)
    exp = poly.evaluate_batch([coeffs], z, "fp")[0]
    assert np.array_equal(got, exp)
    assert unfe(exp, m) == [P.horner(unfe(coeffs, m), unfe(z, m)[0], m)]


@pytest.mark.parametrize("world", [2, 5])
def test_torch_reduce_lr_device_sum(hal, corc, world):
    """dist.torch_reduce_lr (the distributed opening's per-round L/R reduction in bench.py --gpus N):
    every rank's (L_r, R_r) gathered as 16-word rows, then the L column and the R column summed on
    the device by halo_point_sum_dev == the oracle's point sums.  The collective is a stub that plays
    the other ranks' rows (gloo / RCCL gather semantics: one flat tensor of world x 16 words)."""
    import torch

    from halo_amd.dist import torch_reduce_lr
    c = P.PALLAS
    g = corc.srs_generate("pallas", 2 * world)
    rows = [np.concatenate([g[2 * r], g[2 * r + 1]]).astype(np.uint64) for r in range(world)]

    class StubDist:
        def get_world_size(self):
            return world

        def get_backend(self):
            return "gloo"

        def all_gather_into_tensor(self, out, t):
            assert out.shape == (world * 16,) and t.shape == (16,)
            for r in range(world):
                out[16 * r:16 * (r + 1)] = t if r == 0 else torch.from_numpy(rows[r].view(np.int64))

    L, R = torch_reduce_lr(StubDist(), "pallas", "cuda")([(rows[0][:8], rows[0][8:])])
    expL = expR = None
    for r in range(world):
        expL = P.add(c, expL, P.wrapped_to_point(c, [int(x) for x in rows[r][:8]]))
        expR = P.add(c, expR, P.wrapped_to_point(c, [int(x) for x in rows[r][8:]]))
    assert L.tolist() == P.point_to_wrapped(c, expL) and R.tolist() == P.point_to_wrapped(c, expR)


@pytest.mark.parametrize("cname,cid", CURVES)
def test_ipa_fold_forms_xi_inverse(hal, corc, cname, cid):
    """halo_ipa_fold with xi_inv = NULL forms xi^-1 on the host (pcdl.rs:430): the same opening as
    with the caller's inverse, and xi = 0 is refused (HALO_EINVAL)."""
    c = P.CURVES[cname]
    r = c.scalar
    n = 64
    g = corc.srs_generate(cname, n)
    group.PublicParams.upload(cname, g, precompute_windows=False)
    rng = random.Random(7)
    cs = fe([rng.randrange(r) for _ in range(n)], r)
    z = fe([rng.randrange(r)], r)
    Hp = np.array(P.point_to_wrapped(c, P.mul_fast(c, 5, c.generator)), dtype=np.uint64)
    challenge, inverse = transcript(cname)
    exp = pcdl.ipa_rounds(cs, z, Hp, challenge, inverse, cname)
    challenge, _ = transcript(cname)
    got = pcdl.ipa_rounds(cs, z, Hp, challenge, lambda x: None, cname)
    for a, b in zip(exp, got):
        assert np.array_equal(np.asarray(a, dtype=np.uint64), np.asarray(b, dtype=np.uint64))
    ses = pcdl.IpaSession.from_vectors(g[:n], cs, fe(P.construct_powers(P.from_mont(P.limbs_to_int(z[0]), r), n, r), r),
                                       Hp, cname)
    ses.round_lr()
    with pytest.raises(hal.HaloError):
        ses.fold(np.zeros(4, dtype=np.uint64))
    s, ses._s = ses._s, None  # release without the remaining rounds
    hal.check(hal.load().halo_ipa_end(s, None, None))


@pytest.mark.gpu
def test_ipa_end_multi_arguments(hal, corc):
    """halo_ipa_end_multi refuses a repeated or closed session without releasing anything (HALO_EINVAL),
    and releases every listed session otherwise (U, c NULL: no final sum)."""
    import ctypes
    c = P.PALLAS
    r = c.scalar
    n = 64
    g = corc.srs_generate("pallas", n)
    group.PublicParams.upload("pallas", g, precompute_windows=False)
    rng = random.Random(11)
    Hp = np.array(P.point_to_wrapped(c, P.mul_fast(c, 3, c.generator)), dtype=np.uint64)
    L = hal.load()
    sess = []
    for _ in range(2):
        cs = fe([rng.randrange(r) for _ in range(n)], r)
        z = rng.randrange(r)
        sess.append(pcdl.IpaSession.from_vectors(g[:n], cs, fe(P.construct_powers(z, n, r), r), Hp, "pallas"))
    h = [s_._s.value for s_ in sess]
    dup = (ctypes.c_void_p * 2)(h[0], h[0])
    assert L.halo_ipa_end_multi(dup, 2, None, None) == 1  # HALO_EINVAL
    both = (ctypes.c_void_p * 2)(h[0], h[1])
    for s_ in sess:
        s_._s = None
    hal.check(L.halo_ipa_end_multi(both, 2, None, None))
    assert L.halo_ipa_end_multi(both, 2, None, None) == 1  # HALO_EINVAL  # both closed now
