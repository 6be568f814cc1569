"""Device-resident hot path of ``PlonkProof::naive_prover`` (BASELINE.json
configs[3]).

``naive_prover`` (crates/plonk/src/plonk/protocol.rs:64-330) is transcribed round by round onto a
backend ``B``; with ``DeviceBackend`` every data-parallel step runs in libhalo_gpu on the MI355X:

* round 0: 17 iNTTs of size n and 42 NTTs of size 8n (protocol.rs:76-106),
* round 1: 16 commitments (pcdl::commit = resident-SRS MSM, protocol.rs:114),
* round 3: f' and g' (on the CPU backends the reference's 14 growing FFT products; on the device
  the same polynomials through the 8n domain: 16 NTT(8n), pointwise products, 2 iNTT(8n), and their
  n-domain evaluations as strided reads), the permutation accumulator z as prefix/suffix product
  scans (no per-element inversion), 2 iNTTs, 1 commitment (protocol.rs:126-161),
* round 4: the gate-constraint evaluation over the 8n domain (protocol.rs:591-1011: on the device
  three fused passes, halo_gate_constraints_dev; on the CPU backends the ``*_generic`` forms
  transcribed below over ``Evals`` algebra), iNTT(8n), f_cc1 / f_cc2 products (on the device f_cc2 on
  one evaluation domain, z_omega's evaluations as a rotation of z's), the vanishing division, t_split
  and 16 commitments (protocol.rs:170-265),
* round 5: the geometric combinations, two ``Instance::open`` (commit + evaluation + IPA opening),
  ``acc::prover`` (h(X) of three instances, one more IPA opening; acc.rs:178-204) and the 91
  polynomial evaluations of the proof (protocol.rs:273-323).

Out of scope (SURVEY §8 "out of scope"): circuit construction and witness generation (the witness
polynomials here are synthetic), the Poseidon Fiat-Shamir transcript (challenges come from a seeded
stand-in, ``Challenges``), the succinct checks of acc::prover (verifier arithmetic over lg n
elements) and the hiding terms (``naive_prover`` opens with w = None).  The generic pipeline also
runs on the CPU restatement backend (oracle/prover_ref.py) at small n: tests/test_gpu_prover.py
checks every commitment, evaluation and opening bit-exact against it.
"""
from __future__ import annotations

import ctypes

import numpy as np

W_POLYS, R_POLYS, Q_POLYS, S_POLYS, T_POLYS = 16, 15, 10, 8, 16  # crates/plonk/src/utils.rs:16-24
SCALAR_MODULUS = {  # ark_pallas::Fr (Pallas scalars) and ark_pallas::Fq (Vesta scalars)
    "pallas": 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001,
    "vesta": 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001,
}
CONSTRAINT_DEGREE_MULTIPLIER = 8                                 # utils.rs:25


class Challenges:
    """Stand-in for the Poseidon sponge: the k-th challenge is a fixed function of (seed, k)."""

    def __init__(self, modulus: int, seed: int = 0x48414C4F):
        self.m, self.seed, self.k = modulus, seed, 0

    def __call__(self) -> int:
        self.k += 1
        x = (self.seed * 0x9E3779B97F4A7C15 + self.k * 0xD1B54A32D192ED03) & ((1 << 256) - 1)
        x = pow(x | 1, 3, self.m)  # spread over the field; nonzero w.h.p.
        return x or 1


# ---------------------------------------------------------------------------------------------
# gate constraints: the *_generic forms of protocol.rs, over any value type with + - * (Evals here)
# ---------------------------------------------------------------------------------------------
def poseidon_constraints(M, r, w, nw, sbox):
    """protocol.rs:623-648 (poseidon_constraints_generic); sbox = x^7."""
    def rnd(w0, w1, w2, w3, w4, w5, r0, r1, r2):
        s0, s1, s2 = sbox(w0), sbox(w1), sbox(w2)
        return (w3 - (r0 + s0 * M[0][0] + s1 * M[0][1] + s2 * M[0][2])
                + w4 - (r1 + s0 * M[1][0] + s1 * M[1][1] + s2 * M[1][2])
                + w5 - (r2 + s0 * M[2][0] + s1 * M[2][1] + s2 * M[2][2]))
    return (rnd(w[0], w[1], w[2], w[3], w[4], w[5], r[0], r[1], r[2])
            + rnd(w[3], w[4], w[5], w[6], w[7], w[8], r[3], r[4], r[5])
            + rnd(w[6], w[7], w[8], w[9], w[10], w[11], r[6], r[7], r[8])
            + rnd(w[9], w[10], w[11], w[12], w[13], w[14], r[9], r[10], r[11])
            + rnd(w[12], w[13], w[14], nw[0], nw[1], nw[2], r[12], r[13], r[14]))


def affine_add_constraints(w, one):
    """protocol.rs:705-761 (affine_add_constraints_generic)."""
    xp, yp, xq, yq, xr, yr, al, be, ga, de, lam = w[:11]
    xq_xp = xq - xp
    yq_yp = yq - yp
    result = xq_xp * (xq_xp * lam - yq_yp)
    yp2 = yp + yp
    xpxp = xp * xp
    xpxp3 = xpxp + xpxp + xpxp
    result = result + (one - xq_xp * al) * (yp2 * lam - xpxp3)
    xpxq = xp * xq
    xpxq_d = xpxq * (xq - xp)
    ll = lam * lam
    ll_x = ll - xp - xq - xr
    result = result + xpxq_d * ll_x
    l_y = lam * (xp - xr) - yp - yr
    result = result + xpxq_d * l_y
    xpxq_s = xpxq * (yq + yp)
    result = result + xpxq_s * ll_x
    result = result + xpxq_s * l_y
    l_xpb = one - xp * be
    result = result + l_xpb * (xr - xq)
    result = result + l_xpb * (yr - yq)
    l_xqg = one - xq * ga
    result = result + l_xqg * (xr - xp)
    result = result + l_xqg * (yr - yp)
    l_ad = one - (xq - xp) * al - (yq + yp) * de
    result = result + l_ad * xr
    return result + l_ad * yr


def affine_mul_constraints(w, nw, two_pow_i, one):
    """protocol.rs:851-937 (affine_mul_constraints_generic)."""
    xp, yp, a, xg, yg, b, xq, yq, xr, yr, bq, lq, ar, gr, dr, lr = w
    xpxp = xp * xp
    xp2 = xp + xp
    ll = lq * lq
    xpxp3 = xpxp + xpxp + xpxp
    yp2 = yp + yp
    result = (one - xp * bq) * xq
    result = result + (one - xp * bq) * yq
    result = result + (yp2 * lq - xpxp3)
    result = result + (ll - xp2 - xq)
    result = result + (lq * (xp - xq) - yp - yq)
    xg_xq = xg - xq
    yg_yq = yg - yq
    result = result + xg_xq * (xg_xq * lr - yg_yq)
    yq2 = yq + yq
    xqxq = xq * xq
    xqxq3 = xqxq + xqxq + xqxq
    result = result + (one - xg_xq * ar) * (yq2 * lr - xqxq3)
    xqxg = xq * xg
    xqxg_d = xqxg * (xg - xq)
    ll = lr * lr
    ll_x = ll - xq - xg - xr
    result = result + xqxg_d * ll_x
    l_y = lr * (xq - xr) - yq - yr
    result = result + xqxg_d * l_y
    xqxg_s = xqxg * (yg + yq)
    result = result + xqxg_s * ll_x
    result = result + xqxg_s * l_y
    l_xpb = one - xp * bq
    result = result + l_xpb * (xr - xg)
    result = result + l_xpb * (yr - yg)
    l_xgg = one - xg * gr
    result = result + l_xgg * (xr - xq)
    result = result + l_xgg * (yr - yq)
    l_ad = one - (xg - xq) * ar - (yg + yq) * dr
    result = result + l_ad * xr
    result = result + l_ad * yr
    result = result + b * (b - one)
    xs, ys = nw[0], nw[1]
    result = result + (xs - (b * xr + (one - b) * xq))
    result = result + (ys - (b * yr + (one - b) * yq))
    return result + nw[2] - (a + b * two_pow_i)


def range_check_constraints(w, nw, r):
    """protocol.rs:966-990 (range_check_generic)."""
    result = nw[0] - w[0]
    for i in range(15):
        result = result - w[1 + i] * r[i]
    return result


def eq_constraints(w):
    """protocol.rs:1001-1011 (eq_generic)."""
    a, b, one, eq, inv = w[:5]
    return (a - b) * eq + ((a - b) * inv + eq - one)


# ---------------------------------------------------------------------------------------------
# the prover
# ---------------------------------------------------------------------------------------------
def synthetic_witness(B, n: int, seed: int = 1):
    """Random witness polynomials of degree < n (qs, ws, rs, ids, sigmas), w_evals = NTT_n(ws), and
    4 public inputs (circuit construction is out of scope)."""
    rng = np.random.default_rng(seed)

    def poly():
        return B.random_vec(n, rng)

    wit = {k: [poly() for _ in range(c)] for k, c in
           (("qs", Q_POLYS), ("ws", W_POLYS), ("rs", R_POLYS), ("ids", S_POLYS), ("sigmas", S_POLYS))}
    wit["w_evals"] = [B.ntt(w, n) for w in wit["ws"]]
    wit["public_inputs"] = [int(x) for x in rng.integers(1, 2**62, size=4)]
    wit["mds"] = [[int(x) for x in rng.integers(1, 2**62, size=3)] for _ in range(3)]
    return wit


def geometric_polys(B, zeta: int, polys):
    """protocol.rs:542-548: sum_i zeta^i p_i (the device backend: one fused launch, halo_poly_lincomb_dev)."""
    if hasattr(B, "lincomb"):
        return B.lincomb(polys, zeta)
    result = None
    zi = 1
    for p in polys:
        t = B.poly_scale(p, zi)
        result = t if result is None else B.poly_add(result, t)
        zi = zi * zeta % B.m
    return result


def naive_prover(B, wit, n: int, chal: Challenges, acc_prev=None, keep=None):
    """protocol.rs:64-330 on backend B.  Returns the proof's commitments, evaluations, the three IPA
    openings and per-round wall times (seconds; B.sync() before each stamp).  ``keep``: an optional
    dict that receives the intermediate polynomials and challenges (z, f, t's pieces, beta, gamma,
    alpha, zeta, xi, ...) so a test can check them at full size against the oracle."""
    import time

    m = B.m
    d = n - 1
    N8 = n * CONSTRAINT_DEGREE_MULTIPLIER
    times = {}
    t0 = time.perf_counter()

    # ---- round 0 (protocol.rs:76-106)
    pi = B.sparse_vec(n, {i: (-x) % m for i, x in enumerate(wit["public_inputs"])})
    pi_poly = B.intt(B.shift_right(pi, 1))                      # from_vec_and_domain + interpolate
    w_omegas = [B.intt(B.shift_left(e, 1)) for e in wit["w_evals"]]
    q_evals = [B.ntt(p, N8) for p in wit["qs"]]
    w_evals = [B.ntt(p, N8) for p in wit["ws"]]
    r_evals = [B.ntt(p, N8) for p in wit["rs"]]
    fused_gates = hasattr(B, "gate_constraints")  # the device reads w_omega as w shifted in place
    w_omega_evals = None if fused_gates else [B.shift_left(w_evals[i], CONSTRAINT_DEGREE_MULTIPLIER)
                                              for i in range(3)]
    pi_evals = B.ntt(pi_poly, N8)
    B.sync()
    times["round0"] = time.perf_counter() - t0

    # ---- round 1 (protocol.rs:114)
    t1 = time.perf_counter()
    C_ws = B.commit_many(wit["ws"])
    B.sync()
    times["round1"] = time.perf_counter() - t1

    # ---- round 3 (protocol.rs:126-161)
    t3 = time.perf_counter()
    beta, gamma = chal(), chal()

    def perm_factor(other, i):
        return B.poly_add_const(B.poly_add(wit["ws"][i], B.poly_scale(other[i], beta)), gamma)

    if hasattr(B, "perm_products"):  # the same f', g' via the 8n evaluations (see DeviceBackend.perm_products)
        f_prime, g_prime, f_ev, g_ev = B.perm_products(w_evals, wit["ws"], wit["ids"], wit["sigmas"], beta, gamma, n)
    else:
        f_prime = perm_factor(wit["ids"], 0)
        g_prime = perm_factor(wit["sigmas"], 0)
        for i in range(1, S_POLYS):
            f_prime = B.poly_mul(f_prime, perm_factor(wit["ids"], i))
            g_prime = B.poly_mul(g_prime, perm_factor(wit["sigmas"], i))
        f_ev = B.ntt(f_prime, n)
        g_ev = B.ntt(g_prime, n)
    z_vals = B.permutation_accumulator(f_ev, g_ev)              # z[0] = 1, z[i] = z[i-1] f[i] / g[i]
    z_evals = B.shift_right(z_vals, 1)                          # from_vec_and_domain
    z_omega = B.intt(B.shift_left(z_evals, 1))
    z = B.intt(z_evals)
    C_z = B.commit_many([z])[0]
    B.sync()
    times["round3"] = time.perf_counter() - t3

    # ---- round 4 (protocol.rs:170-265)
    t4 = time.perf_counter()
    alpha = chal()
    if fused_gates:
        f_gc_evals = B.gate_constraints(w_evals, r_evals, q_evals, pi_evals, wit["mds"], CONSTRAINT_DEGREE_MULTIPLIER)
    else:
        one = B.ones(N8)
        poseidon = poseidon_constraints(wit["mds"], r_evals, w_evals, w_omega_evals, B.sbox)
        affine_add = affine_add_constraints(w_evals, one)
        affine_mul = affine_mul_constraints(w_evals, w_omega_evals, r_evals[0], one)
        eq = eq_constraints(w_evals)
        range_check = range_check_constraints(w_evals, w_omega_evals, r_evals)
        q, w = q_evals, w_evals
        f_gc_evals = (w[0] * q[0] + q[1] * w[1] + q[2] * w[2] + q[3] * w[0] * w[1] + q[4] + q[5] * poseidon
                      + q[6] * affine_add + q[7] * affine_mul + q[8] * eq + q[9] * range_check + pi_evals)
        del poseidon, affine_add, affine_mul, eq, range_check, one
    f_gc = B.intt(f_gc_evals)
    del f_gc_evals
    e1 = B.sparse_vec(n, {0: 1})
    l1 = B.intt(B.shift_right(e1, 1))                           # lagrange_basis_poly(1, domain)
    f_cc1 = B.poly_mul(l1, B.poly_add_const(z, m - 1))
    if hasattr(B, "perm_cc2"):  # the same polynomial through one evaluation domain (DeviceBackend.perm_cc2)
        f_cc2 = B.perm_cc2(z, z_omega, f_prime, g_prime, n)
    else:
        f_cc2 = B.poly_sub(B.poly_mul(z, f_prime), B.poly_mul(z_omega, g_prime))
    f = B.poly_add(B.poly_add(f_gc, B.poly_scale(f_cc1, alpha)), B.poly_scale(f_cc2, alpha * alpha % m))
    if keep is not None:
        keep.update(pi_poly=pi_poly, z=z, f=f, beta=beta, gamma=gamma, alpha=alpha, w_omegas=w_omegas)
    t = B.divide_by_vanishing(f, n)
    assert B.length(t) <= T_POLYS * n, f"{B.length(t)} < {T_POLYS * n}"
    ts = B.split(B.resize(t, T_POLYS * n), n)                  # t_split (protocol.rs:509-517)
    C_ts = B.commit_many(ts)
    B.sync()
    times["round4"] = time.perf_counter() - t4

    # ---- round 5 (protocol.rs:273-323)
    t5 = time.perf_counter()
    zeta = chal()
    r = geometric_polys(B, zeta, wit["qs"] + wit["ws"] + ts + [z])
    r_omega = geometric_polys(B, zeta, wit["ws"][0:3] + [z])
    xi = chal()
    omega = B.omega(n)
    if keep is not None:
        keep.update(ts=ts, zeta=zeta, xi=xi)
    if acc_prev is None:
        acc_prev = synthetic_accumulator(B, n, chal)
    B.sync()
    t5a = time.perf_counter()
    q_r, q_r_omega = instances_open(B, [(r, xi), (r_omega, xi * omega % m)], d)
    B.sync()
    t5b = time.perf_counter()
    acc_next = acc_prover(B, [acc_prev, q_r, q_r_omega], d, chal)
    B.sync()
    t5c = time.perf_counter()
    at_xi = wit["ws"] + wit["rs"] + wit["qs"] + ts + wit["ids"] + wit["sigmas"] + [z] + w_omegas
    vs = B.eval_many(at_xi, xi)
    vs.append(B.eval_many([z], xi * omega % m)[0])
    B.sync()
    times["round5"] = time.perf_counter() - t5
    times["r5_open"] = t5b - t5a    # two Instance::open (concurrent openings)
    times["r5_acc"] = t5c - t5b     # acc::prover (h(X), one opening)
    times["r5_other"] = times["round5"] - times["r5_open"] - times["r5_acc"]
    times["total"] = time.perf_counter() - t0
    return {
        "C_ws": C_ws, "C_z": C_z, "C_ts": C_ts, "vs": vs,
        "q_r": q_r, "q_r_omega": q_r_omega, "acc": acc_next, "times": times,
    }


def open_seed(z: int, v: int) -> int:
    """Stand-in for the opening's own transcript (open_without_eval starts a fresh PCDL sponge that
    absorbs C', z, v; pcdl.rs:336,387-389): its challenge stream is seeded by (z, v)."""
    return (z * 0x9E3779B97F4A7C15 + v) & ((1 << 64) - 1)


def ipa_open_many(B, items, d: int):
    """pcdl::open_without_eval with w = None (pcdl.rs:326-453) for independent openings
    items = [(p, z, v)]: per opening xi_0 from its own transcript, H' = xi_0 H, lg n rounds of
    (L, R, xi, fold).  The device backend advances all openings in lockstep on their own streams.
    Returns [(Ls, Rs, U, c, [xi_0] + xis)]."""
    chals = [Challenges(B.m, seed=open_seed(z, v)) for (_, z, v) in items]
    xi0s = [ch() for ch in chals]
    if hasattr(B, "ipa_many_xi"):  # H' = xi_0 H formed inside the device sessions
        outs = B.ipa_many_xi([(p, d + 1, z, x0) for (p, z, _), x0 in zip(items, xi0s)], chals)
    else:
        hps = B.h_mul_many(xi0s) if hasattr(B, "h_mul_many") else [B.h_mul(x0) for x0 in xi0s]
        outs = B.ipa_many([(p, d + 1, z, hp) for (p, z, _), hp in zip(items, hps)], chals)
    return [(Ls, Rs, U, c, [x0] + xis) for (Ls, Rs, U, c, xis), x0 in zip(outs, xi0s)]


def instances_open(B, polys_points, d: int):
    """Instance::open (pcdl.rs:41-51) for independent (p, z): C = commit(p), v = p(z), pi = open."""
    Cs = B.commit_many([p for p, _ in polys_points])
    vs = [B.eval_many([p], z)[0] for p, z in polys_points]
    opens = ipa_open_many(B, [(p, z, v) for (p, z), v in zip(polys_points, vs)], d)
    return [{"C": C, "z": z, "v": v, "Ls": o[0], "Rs": o[1], "U": o[2], "c": o[3], "xis": o[4]}
            for C, (_, z), v, o in zip(Cs, polys_points, vs, opens)]


def synthetic_accumulator(B, n: int, chal: Challenges):
    """The previous accumulator's instance (its h(X) challenges and U = commit(h)), synthetic."""
    xis = [chal() for _ in range(n.bit_length())]
    h = B.hpoly([xis], [1])
    return {"xis": xis, "U": B.commit_many([h])[0]}


def acc_prover(B, qs, d: int, chal: Challenges):
    """acc::prover (acc.rs:178-204) without the succinct checks: h(X) = sum alpha^i h_i(X),
    C = sum alpha^i U_i, z, v = h(z), pi = pcdl::open(h, C, d, z)."""
    m = B.m
    alpha = chal()
    alphas = [pow(alpha, i, m) for i in range(len(qs))]
    C = B.point_combine([q["U"] for q in qs], alphas)
    z = chal()
    h = B.hpoly([q["xis"] for q in qs], alphas)
    v = B.eval_many([h], z)[0]
    Ls, Rs, U, c, xis = ipa_open_many(B, [(h, z, v)], d)[0]
    return {"C": C, "z": z, "v": v, "Ls": Ls, "Rs": Rs, "U": U, "c": c, "xis": xis}


# ---------------------------------------------------------------------------------------------
# device backend (libhalo_gpu over torch device buffers)
# ---------------------------------------------------------------------------------------------
class DeviceBackend:
    """Values are torch int64 (len, 4) device tensors of ark words; scalars are canonical ints."""

    def __init__(self, curve: str = "pallas"):
        import torch

        from . import _lib as H

        H.ensure_device()
        self.torch, self.H, self.L = torch, H, H.load()
        self.curve = H.CURVES[curve]
        self.field = H.SCALAR_FIELD[self.curve]
        self.m = SCALAR_MODULUS[curve]
        self.r_inv = pow(1 << 256, -1, self.m)  # ark Montgomery words -> canonical (once, not per value)
        self.stream = torch.cuda.current_stream().cuda_stream
        self.sp = ctypes.c_void_p(self.stream)
        hp = np.zeros(8, dtype=np.uint64)
        H.check(self.L.halo_srs_read(self.curve, 1, 1, H.ptr(hp)))  # H = Gs[1] of the resident SRS
        self.H_point = hp

    # -- conversions
    def fe(self, x: int) -> np.ndarray:
        v = (x % self.m) * (1 << 256) % self.m
        return np.array([(v >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)

    def to_int(self, a: np.ndarray) -> int:
        v = int(a[0]) | int(a[1]) << 64 | int(a[2]) << 128 | int(a[3]) << 192
        return v * self.r_inv % self.m

    def _p(self, t):
        return ctypes.c_void_p(t.data_ptr())

    def _empty(self, n):
        return self.torch.empty((n, 4), dtype=self.torch.int64, device="cuda")

    def sync(self):
        self.torch.cuda.synchronize()

    def random_vec(self, n, rng):
        a = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
        a[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)  # < 2^252 < r: valid ark words
        return self.torch.from_numpy(a.view(np.int64)).cuda()

    def from_ints(self, xs):
        return self.torch.from_numpy(np.stack([self.fe(x) for x in xs]).view(np.int64)).cuda()

    def sparse_vec(self, n, entries):
        # zeroed on the device; only the nonzero entries cross PCIe (a host-built 2^20 x 32 B vector cost
        # 2-4 ms of host time and a pageable copy per call)
        out = self.torch.zeros((n, 4), dtype=self.torch.int64, device="cuda")
        if entries:
            idx = self.torch.tensor(list(entries.keys()), dtype=self.torch.int64, device="cuda")
            vals = np.stack([self.fe(x) for x in entries.values()]).view(np.int64)
            out[idx] = self.torch.from_numpy(vals).cuda()
        return out

    def ones(self, n):
        return DevEvals(self, self.torch.from_numpy(self.fe(1).view(np.int64)).cuda().repeat(n, 1))

    def length(self, p):
        return p.shape[0]

    def omega(self, n: int) -> int:
        return pow(5, (self.m - 1) // n, self.m)  # the radix-2 domain generator

    # -- NTT (ark words in and out)
    def ntt(self, p, N: int):
        """evaluate_over_domain_by_ref: fold mod X^N - 1 when longer, zero-pad, forward NTT."""
        p = p.t if isinstance(p, DevEvals) else p
        L = p.shape[0]
        # a zero tail is cleared (only as far as it is read) by halo_ntt_dev_zero_tail itself
        x = (self.torch.empty if L < N else self.torch.zeros)((N, 4), dtype=self.torch.int64, device="cuda")
        x[:min(L, N)] = p[:min(L, N)]
        for s in range(N, L, N):
            k = min(N, L - s)
            self._op(0, x[:k], p[s:s + k], None, 0, x[:k])
        if L < N:  # zero tail: the first pass skips the stages that only replicate values
            self.H.check(self.L.halo_ntt_dev_zero_tail(self.field, self._p(x), N.bit_length() - 1, 1, L, self.sp))
        else:
            self.H.check(self.L.halo_ntt_dev(self.field, self._p(x), N.bit_length() - 1, 1, 0, self.sp))
        return DevEvals(self, x)

    def intt(self, e):
        x = (e.t if isinstance(e, DevEvals) else e).clone()
        N = x.shape[0]
        self.H.check(self.L.halo_ntt_dev(self.field, self._p(x), N.bit_length() - 1, 1, 1, self.sp))
        return x

    def shift_left(self, e, k):
        t = e.t if isinstance(e, DevEvals) else e
        r = self.torch.roll(t, -k, 0)
        return DevEvals(self, r) if isinstance(e, DevEvals) else r

    def shift_right(self, e, k):
        t = e.t if isinstance(e, DevEvals) else e
        r = self.torch.roll(t, k, 0)
        return DevEvals(self, r) if isinstance(e, DevEvals) else r

    # -- elementwise (Evals ops, halo_evals_op_dev)
    def _op(self, op, a, b, s, e, out):
        self.H.check(self.L.halo_evals_op_dev(self.field, op, self._p(a), self._p(b) if b is not None else None,
                                              self.H.ptr(self.fe(s)) if s is not None else None, e, self._p(out),
                                              a.shape[0], self.sp))
        return out

    def sbox(self, x):
        return DevEvals(self, self._op(6, x.t, None, None, 7, self._empty(x.t.shape[0])))

    def gate_constraints(self, w, r, q, pi, mds, shift):
        """protocol.rs:170-191 fused on the device (halo_gate_constraints_dev): one pass per group of
        constraint polynomials instead of ~250 Evals kernels; w_omega = w[0..3] shifted by `shift`."""
        N = w[0].t.shape[0]
        vp = ctypes.c_void_p
        dw = (vp * 16)(*[e.t.data_ptr() for e in w])
        dr = (vp * 15)(*[e.t.data_ptr() for e in r])
        dq = (vp * 10)(*[e.t.data_ptr() for e in q])
        m9 = np.ascontiguousarray(np.stack([self.fe(x) for row in mds for x in row]))
        out = self._empty(N)
        self.H.check(self.L.halo_gate_constraints_dev(self.field, dw, dr, dq, self._p(pi.t), self.H.ptr(m9), N, shift,
                                                      self._p(out), self.sp))
        return DevEvals(self, out)

    # -- polynomials (coefficient tensors; lengths may differ)
    def poly_add(self, a, b, sub=False):
        if a.shape[0] < b.shape[0] and not sub:
            a, b = b, a
        out = self.torch.zeros((max(a.shape[0], b.shape[0]), 4), dtype=self.torch.int64, device="cuda")
        out[:a.shape[0]] = a
        k = b.shape[0]
        if sub:
            self._op(1, out[:k].contiguous(), b, None, 0, out[:k])
        else:
            self._op(0, out[:k].contiguous(), b, None, 0, out[:k])
        return out

    def poly_sub(self, a, b):
        return self.poly_add(a, b, sub=True)

    def lincomb(self, polys, zeta: int):
        """sum_i zeta^i polys[i] in one device pass (halo_poly_lincomb_dev); length = the longest."""
        k = len(polys)
        n_out = max(p.shape[0] for p in polys)
        out = self._empty(n_out)
        ptrs = (ctypes.c_void_p * k)(*[p.data_ptr() for p in polys])
        lens = (ctypes.c_size_t * k)(*[p.shape[0] for p in polys])
        self.H.check(self.L.halo_poly_lincomb_dev(self.field, ptrs, lens, k, self.H.ptr(self.fe(zeta)), self._p(out),
                                                  n_out, self.sp))
        return out

    def poly_scale(self, a, s):
        return self._op(3, a, None, s, 0, self._empty(a.shape[0]))

    def poly_add_const(self, a, s):
        out = a.clone()
        self._op(4, out[:1].contiguous(), None, s, 0, out[:1])
        return out

    def poly_mul(self, a, b):
        la, lb = a.shape[0], b.shape[0]
        rl = la + lb - 1
        N = 1 << (rl - 1).bit_length()
        fa, fb = self.ntt(a, N), self.ntt(b, N)
        prod = self._op(2, fa.t, fb.t, None, 0, fa.t)
        return self.intt(prod)[:rl].contiguous()

    def perm_products(self, w_evals, ws, ids, sigmas, beta, gamma, n):
        """protocol.rs:132-141 computed through the 8n domain: f' = prod_i (w_i + beta id_i + gamma) (and
        g' with sigma_i) has degree < 8n, so its 8n evaluations are the pointwise product of the factors'
        8n evaluations (w_i's are round 0's w_evals; one NTT(8n) per id_i / sigma_i), one iNTT(8n) gives
        the coefficients (the same polynomial the reference's 7 growing FFT products give), and
        f'(omega_n^j) = F[8 j], so f_ev / g_ev are strided reads instead of two more NTTs."""
        N8 = CONSTRAINT_DEGREE_MULTIPLIER * n
        assert S_POLYS <= CONSTRAINT_DEGREE_MULTIPLIER
        outs = []
        wg = [w_evals[i] + gamma for i in range(S_POLYS)]  # shared by both products
        for other in (ids, sigmas):
            acc = None
            deg = 0
            for i in range(S_POLYS):
                t = self.ntt(other[i], N8) * beta + wg[i]
                deg += max(ws[i].shape[0], other[i].shape[0]) - 1
                acc = t if acc is None else acc * t
            assert deg < N8
            outs.append((acc, deg + 1))
        (F, lf), (G, lg) = outs
        f_prime = self.intt(F)[:lf].contiguous()
        g_prime = self.intt(G)[:lg].contiguous()
        f_ev = DevEvals(self, F.t[::CONSTRAINT_DEGREE_MULTIPLIER].contiguous())
        g_ev = DevEvals(self, G.t[::CONSTRAINT_DEGREE_MULTIPLIER].contiguous())
        return f_prime, g_prime, f_ev, g_ev

    def perm_cc2(self, z, z_omega, f_prime, g_prime, n):
        """z f' - z_omega g' (protocol.rs:198-199) on one N-point domain covering both products: NTT z,
        f', g', pointwise Z F - Z_omega G, one iNTT (4 transforms instead of the reference's two FFT
        products, 6).  z_omega(X) = z(omega_n X) (round 3 interpolates z's evaluations shifted by one),
        so its N-point evaluations are z's rotated by N / n."""
        rl = max(z.shape[0] + f_prime.shape[0] - 1, z_omega.shape[0] + g_prime.shape[0] - 1)
        N = 1 << (rl - 1).bit_length()
        assert N % n == 0 and z.shape[0] <= n and z_omega.shape[0] <= n
        Z = self.ntt(z, N)
        Zw = DevEvals(self, self.torch.roll(Z.t, -(N // n), 0))
        P = Z * self.ntt(f_prime, N) - Zw * self.ntt(g_prime, N)
        return self.intt(P)[:rl].contiguous()

    def divide_by_vanishing(self, f, n):
        L = f.shape[0]
        q = self._empty(max(L - n, 1))
        r = self._empty(n)
        self.H.check(self.L.halo_divide_by_vanishing_dev(self.field, self._p(f), L, n, self._p(q), self._p(r),
                                                         self.sp))
        return q[:L - n]

    def resize(self, p, N):
        out = self.torch.zeros((N, 4), dtype=self.torch.int64, device="cuda")
        out[:min(N, p.shape[0])] = p[:min(N, p.shape[0])]
        return out

    def split(self, p, n):
        return [p[i:i + n].contiguous() for i in range(0, p.shape[0], n)]

    def permutation_accumulator(self, f_ev, g_ev):
        """z[0] = 1, z[i] = prod_{j=1..i} f[j] / g[j] (protocol.rs:143-154) without per-element
        inversion: z[i] = F[i] * Sg[i+1] / G, F = prefix product of f (f[0] := 1), Sg = suffix
        product of g (g[0] := 1), G = Sg[0]; one inversion in total."""
        one = self.from_ints([1])
        f = f_ev.t.clone()
        g = g_ev.t.clone()
        f[0:1] = one
        g[0:1] = one
        F = self._empty(f.shape[0])
        Sg = self._empty(g.shape[0])
        self.H.check(self.L.halo_evals_scan_dev(self.field, 0, self._p(f), self._p(F), f.shape[0], self.sp))
        self.H.check(self.L.halo_evals_scan_dev(self.field, 1, self._p(g), self._p(Sg), g.shape[0], self.sp))
        total = self.to_int(Sg[0].cpu().numpy().view(np.uint64))
        sh = self.torch.roll(Sg, -1, 0)
        sh[-1:] = one
        z = self._op(2, F, sh, None, 0, F)
        return DevEvals(self, self._op(3, z, None, pow(total, -1, self.m), 0, z))

    # -- commitments, evaluations, openings
    def commit_many(self, polys):
        """pcdl::commit of every polynomial (protocol.rs:114,263): one halo_msm_batch_dev call (small
        polynomials as one MSM with (polynomial, bucket) keys, larger ones pipelined)."""
        k = len(polys)
        outs = self.torch.zeros((k, 8), dtype=self.torch.int64, device="cuda")
        ptrs = (ctypes.c_void_p * k)(*[p.data_ptr() for p in polys])
        lens = (ctypes.c_size_t * k)(*[p.shape[0] for p in polys])
        self.H.check(self.L.halo_msm_batch_dev(self.curve, ptrs, lens, k, ctypes.c_void_p(outs.data_ptr()), self.sp))
        self.H.check(self.L.halo_msm_join(self.sp))
        return [o.view(np.uint64) for o in outs.cpu().numpy()]

    def eval_many(self, polys, z: int):
        ptrs = (ctypes.c_void_p * len(polys))(*[p.data_ptr() for p in polys])
        lens = (ctypes.c_size_t * len(polys))(*[p.shape[0] for p in polys])
        out = self._empty(len(polys))
        self.H.check(self.L.halo_poly_eval_batch_dev(self.field, ptrs, lens, len(polys), self.H.ptr(self.fe(z)),
                                                     self._p(out), self.sp))
        return [self.to_int(r.view(np.uint64)) for r in out.cpu().numpy()]

    def h_mul(self, k: int):
        out = np.zeros(8, dtype=np.uint64)
        self.H.check(self.L.halo_curve_op(self.curve, 2, self.H.ptr(self.H_point), None, self.H.ptr(self.fe(k)), 1,
                                          self.H.ptr(out)))
        return out

    def h_mul_many(self, ks):
        """[k H for k in ks] in one device call (the lanes run concurrently)."""
        pts = np.ascontiguousarray(np.stack([self.H_point] * len(ks)))
        kk = np.ascontiguousarray(np.stack([self.fe(k) for k in ks]))
        out = np.zeros_like(pts)
        self.H.check(self.L.halo_curve_op(self.curve, 2, self.H.ptr(pts), None, self.H.ptr(kk), len(ks),
                                          self.H.ptr(out)))
        return list(out)

    def point_combine(self, points, scalars):
        """sum_i scalars[i] points[i] (acc.rs:166 point_dot over the U_i): one small MSM over the
        caller's points (halo_msm) instead of per-point scalar multiplications and a point sum."""
        pts = np.ascontiguousarray(np.stack(points))
        ks = np.ascontiguousarray(np.stack([self.fe(s) for s in scalars]))
        out = np.zeros(8, dtype=np.uint64)
        self.H.check(self.L.halo_msm(self.curve, self.H.ptr(pts), len(pts), self.H.ptr(ks), len(ks), self.H.ptr(out)))
        return out

    def hpoly(self, xis_rows, alphas):
        """sum_i alphas[i] h_i(X) (acc.rs:89) generated on the device (halo_hpoly_combine_dev): h never
        crosses PCIe before its commitment and opening."""
        k, nx = len(xis_rows), len(xis_rows[0])
        xs = np.ascontiguousarray(np.stack([self.fe(x) for row in xis_rows for x in row]))
        al = np.ascontiguousarray(np.stack([self.fe(a) for a in alphas]))
        out = self._empty(1 << (nx - 1))
        self.H.check(self.L.halo_hpoly_combine_dev(self.field, self.H.ptr(xs), k, nx, self.H.ptr(al), self._p(out),
                                                   self.sp))
        return out

    def ipa_many(self, jobs, chals, xi_mode=False):
        """jobs = [(p, n, z, H')] with one challenge stream each; all sessions advance in lockstep
        (halo_ipa_round_lr_multi / halo_ipa_fold_multi: one host round trip per round for all).
        xi_mode: jobs = [(p, n, z, xi_0)] and the sessions form H' = xi_0 H themselves
        (halo_ipa_begin_dev_xi with this backend's H)."""
        k = len(jobs)
        n = jobs[0][1]
        assert all(j[1] == n for j in jobs)
        css = [self.resize(p, n) for (p, _, _, _) in jobs]
        self.sync()  # the coefficients were produced on the caller's stream
        sess = (ctypes.c_void_p * k)()
        for i, ((_, _, z, hx), cs) in enumerate(zip(jobs, css)):
            s = ctypes.c_void_p()
            if xi_mode:
                self.H.check(self.L.halo_ipa_begin_dev_xi(self.curve, self._p(cs), n, self.H.ptr(self.fe(z)),
                                                          self.H.ptr(self.H_point), self.H.ptr(self.fe(hx)),
                                                          ctypes.byref(s)))
            else:
                self.H.check(self.L.halo_ipa_begin_dev(self.curve, self._p(cs), n, self.H.ptr(self.fe(z)),
                                                       self.H.ptr(np.ascontiguousarray(hx)), ctypes.byref(s)))
            sess[i] = s.value
        Ls = [[] for _ in range(k)]
        Rs = [[] for _ in range(k)]
        xis = [[] for _ in range(k)]
        Lb = np.zeros((k, 8), dtype=np.uint64)
        Rb = np.zeros((k, 8), dtype=np.uint64)
        for _ in range(n.bit_length() - 1):
            self.H.check(self.L.halo_ipa_round_lr_multi(sess, k, self.H.ptr(Lb), self.H.ptr(Rb)))
            xs = [ch() for ch in chals]
            xa = np.ascontiguousarray(np.stack([self.fe(x) for x in xs]))
            # xi^-1 formed by the library (halo_ipa_fold_multi with a NULL xi_inv, pcdl.rs:430)
            self.H.check(self.L.halo_ipa_fold_multi(sess, k, self.H.ptr(xa), None))
            for i in range(k):
                Ls[i].append(Lb[i].copy())
                Rs[i].append(Rb[i].copy())
                xis[i].append(xs[i])
        Us = np.zeros((k, 8), dtype=np.uint64)
        c0s = np.zeros((k, 4), dtype=np.uint64)
        self.H.check(self.L.halo_ipa_end_multi(sess, k, self.H.ptr(Us), self.H.ptr(c0s)))
        return [(Ls[i], Rs[i], Us[i].copy(), self.to_int(c0s[i]), xis[i]) for i in range(k)]

    def ipa_many_xi(self, jobs, chals):
        return self.ipa_many(jobs, chals, xi_mode=True)

    def ipa(self, p, n: int, z: int, h_prime, chal):
        return self.ipa_many([(p, n, z, h_prime)], [chal])[0]


class DevEvals:
    """Evals on the device (poly.rs:90-327): + - * between vectors, * / + - with a scalar."""

    __slots__ = ("B", "t")

    def __init__(self, B: DeviceBackend, t):
        self.B, self.t = B, t

    def _bin(self, other, op_vec, op_scalar, swap=False):
        B = self.B
        out = B._empty(self.t.shape[0])
        if isinstance(other, DevEvals):
            a, b = (other.t, self.t) if swap else (self.t, other.t)
            return DevEvals(B, B._op(op_vec, a, b, None, 0, out))
        return DevEvals(B, B._op(op_scalar, self.t, None, int(other), 0, out))

    def __add__(self, o):
        return self._bin(o, 0, 4)

    __radd__ = __add__

    def __sub__(self, o):
        return self._bin(o, 1, 5)

    def __mul__(self, o):
        return self._bin(o, 2, 3)

    __rmul__ = __mul__
