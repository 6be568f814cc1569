"""GPU parity at the north-star sizes (BASELINE.json north_star: "2^24-point MSM and 2^24-element
NTT bit-exact"; configs[3]: the full prove at n = 2^20).

* 2^24-point MSM over a synthetic SRS G_j = k_j G (beyond the reference's N = 2^20): bit-exact through
  the known-log identity MSM(G, s) = (sum_j s_j k_j) G, the dot product and the generator
  multiplication done by the C oracle (corc.known_log_msm).
* 2^24-element NTT and iNTT over Fp (and the forward NTT over Fq) against the C oracle's
  ark-poly radix-2 restatement, element by element.
* naive_prover at n = 2^20 on the device: its three openings (the two Instance::open of round 5 and
  acc::prover's open of h) pass the CPU restatement of pcdl::succinct_check (oracle/pcdl_check.py,
  pcdl.rs:483-554) and the decider identity U == commit(h) (pcdl.rs:563-583) against the oracle MSM.
"""
import numpy as np
import pytest

import pasta as P
from halo_amd import group, pcdl

pytestmark = pytest.mark.gpu


def rand_words(n, seed, top_mask=0x0FFFFFFFFFFFFFFF):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * np.uint64(2)
    a |= rng.integers(0, 2, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64(top_mask)  # < 2^252 < r: valid Montgomery words
    return np.ascontiguousarray(a)


def test_msm_2p24_synthetic_srs_known_logs(hal, corc):
    n = 1 << 24
    seed = 0x2424
    group.PublicParams.synthesize("pallas", n, seed, precompute_windows=True)
    k = corc.synth_scalars(seed, n)
    from halo_amd.group import synth_scalar
    assert [P.limbs_to_int(k[j]) for j in (0, 1, n - 1)] == [synth_scalar(seed, j) for j in (0, 1, n - 1)]
    sc = rand_words(n, 24)
    sc[0] = 0                                                                  # zero scalar
    sc[1] = P.int_to_limbs(P.to_mont(P.FP_MODULUS - 1, P.FP_MODULUS))         # r - 1
    sc[2:1026] = sc[3000]                                                      # a skewed bucket
    got = pcdl.commit(sc, n - 1, None, "pallas")
    assert np.array_equal(got, corc.known_log_msm("pallas", sc, k))
    # a ragged prefix (n_scalars < n_bases: the MSM length is the shorter one, pedersen.rs:21)
    m = (1 << 23) + 12345
    got = pcdl.commit(sc[:m], n - 1, None, "pallas")
    assert np.array_equal(got, corc.known_log_msm("pallas", sc[:m], k[:m]))


def test_msm_2p24_window_partitioned_virtual_ranks_known_logs(hal, corc):
    """BASELINE configs[4] at its size on one GPU: the 2^24-point MSM split by windows over 8 virtual
    ranks as bench.py --gpus 8 splits it -- 16 windows of 16 bits (halo_amd.dist.partition_window_bits),
    2 per rank, and each rank precomputing ONLY its own windows' shifted copies
    (halo_srs_precompute_window_range) before its partial (halo_msm_srs_windows_dev); the partials
    summed on the device (halo_point_sum_dev, the RCCL leg's combine) and checked against the
    known-log identity (an independent oracle).  Then the 3-rank partition (15 windows of 17 bits,
    5 each) over the full set of copies."""
    import ctypes

    import torch
    from halo_amd.dist import partition_window_bits, window_range

    L = hal.load()
    n = 1 << 24
    seed = 0x57494E44
    cid = hal.CURVES["pallas"]
    hal.check(L.halo_srs_synthesize(cid, n, seed))
    k = corc.synth_scalars(seed, n)
    sc = rand_words(n, 4242)
    sc[0] = P.int_to_limbs(P.to_mont(P.FP_MODULUS - 1, P.FP_MODULUS))
    sc[1:2049] = sc[7]  # one bucket per window takes 2^11 extra points
    exp = corc.known_log_msm("pallas", sc, k)
    d_sc = torch.from_numpy(sc.view(np.int64)).cuda()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def combine(outs, world):
        total = torch.zeros(8, dtype=torch.int64, device="cuda")
        hal.check(L.halo_point_sum_dev(cid, ctypes.c_void_p(outs.data_ptr()), world, 64,
                                       ctypes.c_void_p(total.data_ptr()), sp))
        torch.cuda.synchronize()
        return total.cpu().numpy().view(np.uint64)

    world = 8
    c = partition_window_bits(world)
    W = -(-255 // c)
    assert (c, W) == (16, 16)
    outs = torch.zeros((world, 8), dtype=torch.int64, device="cuda")
    for r in range(world):
        lo, hi = window_range(W, r, world)
        assert hi - lo == W // world  # balanced: no rank carries an extra window
        hal.check(L.halo_srs_precompute_window_range(cid, c, lo, hi))  # this rank's copies only
        assert L.halo_srs_windows(cid) == W and L.halo_srs_window_bits(cid) == c
        if r:  # a window outside the resident range is refused
            assert L.halo_msm_srs_windows_dev(cid, ctypes.c_void_p(d_sc.data_ptr()), n, 0, hi,
                                              ctypes.c_void_p(outs[r].data_ptr()), sp) != 0
        hal.check(L.halo_msm_srs_windows_dev(cid, ctypes.c_void_p(d_sc.data_ptr()), n, lo, hi,
                                             ctypes.c_void_p(outs[r].data_ptr()), sp))
        hal.check(L.halo_msm_join(sp))
    assert np.array_equal(combine(outs, world), exp)

    group.PublicParams.synthesize("pallas", n, seed, precompute_windows=True)
    W = L.halo_srs_windows(cid)
    world = 3
    outs = torch.zeros((world, 8), dtype=torch.int64, device="cuda")
    for r in range(world):
        lo, hi = window_range(W, r, world)
        assert hi - lo == 5
        hal.check(L.halo_msm_srs_windows_dev(cid, ctypes.c_void_p(d_sc.data_ptr()), n, lo, hi,
                                             ctypes.c_void_p(outs[r].data_ptr()), sp))
    hal.check(L.halo_msm_join(sp))
    assert np.array_equal(combine(outs, world), exp)
    del d_sc


@pytest.mark.parametrize("tag,fid,inverse", [("fp", 0, True), ("fq", 1, False)])
def test_ntt_2p24_vs_c_oracle(hal, corc, tag, fid, inverse):
    L = hal.load()
    logn = 24
    x = rand_words(1 << logn, 240 + fid)
    exp = corc.ntt(tag, x)
    got = x.copy()
    hal.check(L.halo_ntt(fid, hal.ptr(got), logn, 0))
    assert np.array_equal(got, exp)
    if inverse:
        back = exp.copy()
        hal.check(L.halo_ntt(fid, hal.ptr(back), logn, 1))
        assert np.array_equal(back, x)
        assert np.array_equal(corc.ntt(tag, exp, inverse=True), x)


@pytest.fixture(scope="module")
def prove_2p20(hal):
    """One run of naive_prover at n = 2^20 (BASELINE configs[3]) over the synthetic SRS G_j = k_j G,
    with the intermediate polynomials kept for the checks below."""
    from halo_amd import prover

    L = hal.load()
    n = 1 << 20
    seed = 0x505256 + 20
    cid = hal.CURVES["pallas"]
    hal.check(L.halo_srs_synthesize(cid, n, seed))
    hal.check(L.halo_srs_precompute_windows(cid))
    B = prover.DeviceBackend("pallas")
    wit = prover.synthetic_witness(B, n, seed=1)
    keep = {}
    out = prover.naive_prover(B, wit, n, prover.Challenges(B.m), keep=keep)
    B.sync()
    return {"n": n, "seed": seed, "B": B, "wit": wit, "keep": keep, "out": out}


def test_prove_2p20_openings_pass_succinct_check_and_decider(hal, corc, prove_2p20):
    import pcdl_check

    L = hal.load()
    n, B, out = prove_2p20["n"], prove_2p20["B"], prove_2p20["out"]
    srs = np.zeros((n, 8), dtype=np.uint64)
    hal.check(L.halo_srs_read(hal.CURVES["pallas"], 0, n, hal.ptr(srs)))
    for key in ("q_r", "q_r_omega", "acc"):
        q = out[key]
        assert len(q["Ls"]) == 20
        pcdl_check.succinct_check("pallas", q["C"], n - 1, q["z"], q["v"], q["Ls"], q["Rs"], q["U"], q["c"],
                                  q["xis"], B.H_point)
        assert pcdl_check.decider_commit_matches("pallas", q["U"], q["xis"], srs, corc.msm), key


def _host(t):
    return np.ascontiguousarray(t.cpu().numpy().view(np.uint64))


class _Fr:
    """A scalar-field element for the scalar restatement of the constraint formulas below."""

    __slots__ = ("v",)
    m = P.FP_MODULUS

    def __init__(self, v):
        self.v = v.v if isinstance(v, _Fr) else v % self.m

    def __add__(self, o):
        return _Fr(self.v + _Fr(o).v)

    __radd__ = __add__

    def __sub__(self, o):
        return _Fr(self.v - _Fr(o).v)

    def __rsub__(self, o):
        return _Fr(_Fr(o).v - self.v)

    def __mul__(self, o):
        return _Fr(self.v * _Fr(o).v)

    __rmul__ = __mul__


def test_prove_2p20_commitments_quotient_and_evaluations(hal, corc, prove_2p20):
    """configs[3] at its own size, beyond the openings (VERDICT r03 missing #1), every check by the CPU
    oracle on the device's downloaded polynomials:

    * the 33 commitments (16 C_ws, C_z, 16 C_ts; protocol.rs:114,161,263) by the known-log identity
      commit(p) = (sum_j p_j k_j) G over the synthetic SRS;
    * the permutation accumulator z (protocol.rs:143-154): NTT_n(z) shifted is z_vals with
      z_vals[0] = 1 and z_vals[i] g[i] = z_vals[i-1] f[i], f and g formed by the oracle from its own
      NTTs of w, id, sigma;
    * f (protocol.rs:193-199) at a random point: f(x) = f_gc(x) + alpha l_1(x)(z(x) - 1)
      + alpha^2 (z(x) f'(x) - z(omega x) g'(x)), with f_gc(x) the reference's constraint formulas
      (protocol.rs:170-191) over the witness polynomials' oracle Horner values (every constraint has
      degree < 8n, so the 8n-domain interpolation is exact) and the Lagrange values in closed form;
    * the quotient (protocol.rs:255-260, the reference's own commented-out check made exact):
      f(x) = t(x) Z_H(x) + (f mod Z_H)(x), t(x) = sum_k x^(k n) t_k(x), the remainder folded by the oracle;
    * the 91 evaluations of the proof (protocol.rs:315-323) by oracle Horner (w_omega_i(xi) as
      w_i(omega xi), z(omega xi));
    * the two openings' C and v as the zeta-combinations of those commitments and values
      (protocol.rs:273-280)."""
    from concurrent.futures import ThreadPoolExecutor

    from halo_amd import prover

    n, B, wit, keep, out = (prove_2p20[k] for k in ("n", "B", "wit", "keep", "out"))
    m = B.m
    assert m == P.FP_MODULUS
    tag = "fp"
    k_logs = corc.synth_scalars(prove_2p20["seed"], n)
    pool = ThreadPoolExecutor(16)

    def fe(x):
        return B.fe(x)

    def to_int(a):
        return B.to_int(a)

    hw = {key: [_host(p) for p in wit[key]] for key in ("qs", "ws", "rs", "ids", "sigmas")}
    z = _host(keep["z"])
    f = _host(keep["f"])
    ts = [_host(t) for t in keep["ts"]]
    assert len(ts) == prover.T_POLYS and all(len(t) == n for t in ts) and len(z) == n

    # -- commitments by known logs
    def commit(p):
        return corc.known_log_msm("pallas", p, k_logs[:len(p)])

    exp_ws = list(pool.map(commit, hw["ws"]))
    exp_ts = list(pool.map(commit, ts))
    for i, (a, b) in enumerate(zip(out["C_ws"], exp_ws)):
        assert np.array_equal(a, b), ("C_ws", i)
    assert np.array_equal(out["C_z"], commit(z)), "C_z"
    for i, (a, b) in enumerate(zip(out["C_ts"], exp_ts)):
        assert np.array_equal(a, b), ("C_ts", i)

    # -- z: the accumulator's recurrence over the oracle's own NTTs
    beta, gamma, alpha = keep["beta"], keep["gamma"], keep["alpha"]
    ntt_n = list(pool.map(lambda p: corc.ntt(tag, p, threads=2), hw["ws"][:8] + hw["ids"] + hw["sigmas"] + [z]))
    w_ev, id_ev, sg_ev, z_ev = ntt_n[:8], ntt_n[8:16], ntt_n[16:24], ntt_n[24]
    bb, gg = fe(beta), fe(gamma)

    def factor(w, o):
        return corc.evals_op(tag, 4, corc.evals_op(tag, 0, w, corc.evals_op(tag, 3, o, s=bb)), s=gg)

    fe_v = ge_v = None
    for i in range(8):
        a, b = factor(w_ev[i], id_ev[i]), factor(w_ev[i], sg_ev[i])
        fe_v = a if fe_v is None else corc.evals_op(tag, 2, fe_v, a)
        ge_v = b if ge_v is None else corc.evals_op(tag, 2, ge_v, b)
    z_vals = np.ascontiguousarray(np.roll(z_ev, -1, axis=0))   # z_evals = shift_right(z_vals, 1)
    assert to_int(z_vals[0]) == 1
    lhs = corc.evals_op(tag, 2, np.ascontiguousarray(z_vals[1:]), np.ascontiguousarray(ge_v[1:]))
    rhs = corc.evals_op(tag, 2, np.ascontiguousarray(z_vals[:-1]), np.ascontiguousarray(fe_v[1:]))
    bad = np.nonzero((lhs != rhs).any(axis=1))[0]
    assert len(bad) == 0, f"z recurrence fails at {bad[:5] + 1}"

    # -- f at a random point from the constraint formulas
    omega = B.omega(n)
    x = 0x7A3B9C1D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F7 % m

    def evals_at(polys, pt):
        zf = fe(pt)
        return list(pool.map(lambda p: _Fr(to_int(corc.poly_eval(tag, p, zf))), polys))

    q, w, r = evals_at(hw["qs"], x), evals_at(hw["ws"], x), evals_at(hw["rs"], x)
    ids, sig = evals_at(hw["ids"], x), evals_at(hw["sigmas"], x)
    nw = evals_at(hw["ws"][:3], omega * x % m)
    zx, zwx = evals_at([z], x)[0], evals_at([z], omega * x % m)[0]
    one = _Fr(1)
    zh = _Fr(pow(x, n, m) - 1)

    def lagrange(j):  # L_j(x) = omega^j (x^n - 1) / (n (x - omega^j))
        wj = pow(omega, j, m)
        return _Fr(wj * zh.v * pow(n * (x - wj), -1, m))

    pi_x = _Fr(0)
    for i, v in enumerate(wit["public_inputs"]):  # pi = from_vec_and_domain(-public inputs)
        pi_x = pi_x + _Fr(-v) * lagrange(i + 1)
    mds = wit["mds"]
    f_gc = (w[0] * q[0] + q[1] * w[1] + q[2] * w[2] + q[3] * w[0] * w[1] + q[4]
            + q[5] * prover.poseidon_constraints(mds, r, w, nw, lambda s: s * s * s * s * s * s * s)
            + q[6] * prover.affine_add_constraints(w, one)
            + q[7] * prover.affine_mul_constraints(w, nw, r[0], one)
            + q[8] * prover.eq_constraints(w)
            + q[9] * prover.range_check_constraints(w, nw, r) + pi_x)
    fp_x = gp_x = one
    for i in range(8):
        fp_x = fp_x * (w[i] + ids[i] * beta + gamma)
        gp_x = gp_x * (w[i] + sig[i] * beta + gamma)
    f_exp = f_gc + lagrange(1) * (zx - 1) * alpha + (zx * fp_x - zwx * gp_x) * (alpha * alpha)
    f_x = evals_at([f], x)[0]
    assert f_x.v == f_exp.v, "f(x) differs from the constraint formulas"

    # -- quotient: f = t Z_H + (f mod Z_H)
    rem = np.ascontiguousarray(f[:n].copy())
    for s in range(n, len(f), n):
        k = min(n, len(f) - s)
        rem[:k] = corc.evals_op(tag, 0, np.ascontiguousarray(rem[:k]), np.ascontiguousarray(f[s:s + k]))
    t_vals = evals_at(ts, x)
    t_x, xn = _Fr(0), _Fr(pow(x, n, m))
    for tv in reversed(t_vals):
        t_x = t_x * xn + tv
    assert f_x.v == (t_x * zh + evals_at([rem], x)[0]).v, "f != t Z_H + remainder"

    # -- the 91 evaluations at xi
    xi = keep["xi"]
    at_xi = hw["ws"] + hw["rs"] + hw["qs"] + ts + hw["ids"] + hw["sigmas"] + [z]
    exp_vs = [e.v for e in evals_at(at_xi, xi)]
    exp_vs += [e.v for e in evals_at(hw["ws"], omega * xi % m)]  # w_omega_i(xi) = w_i(omega xi)
    exp_vs.append(evals_at([z], omega * xi % m)[0].v)
    assert len(out["vs"]) == len(exp_vs) == 91
    for i, (a, b) in enumerate(zip(out["vs"], exp_vs)):
        assert a == b, ("vs", i)

    # -- the openings' C and v are the zeta-combinations (protocol.rs:273-280)
    zeta = keep["zeta"]
    exp_qs = list(pool.map(commit, hw["qs"]))
    r_pts = exp_qs + exp_ws + exp_ts + [commit(z)]
    r_vals = [e.v for e in evals_at(hw["qs"], xi)] + exp_vs[:16] + exp_vs[41:57] + [exp_vs[73]]
    ro_pts = exp_ws[:3] + [commit(z)]
    ro_vals = exp_vs[74:77] + [exp_vs[90]]
    for key, pts, vals in (("q_r", r_pts, r_vals), ("q_r_omega", ro_pts, ro_vals)):
        zs = [pow(zeta, i, m) for i in range(len(pts))]
        C = corc.msm("pallas", np.ascontiguousarray(np.stack(pts)), np.ascontiguousarray(np.stack([fe(s) for s in zs])))
        assert np.array_equal(out[key]["C"], C), key
        assert out[key]["v"] == sum(a * b for a, b in zip(zs, vals)) % m, key
    pool.shutdown()
