"""Mirror of crates/accumulation/src/pcdl.rs (commit + the IPA round loop) on the MI355X backend.

The Fiat-Shamir transcript (Poseidon sponge, crates/poseidon) stays with the caller: the round loop
of ``open_without_eval`` (pcdl.rs:404-438) asks a ``challenge(xi_prev, L, R) -> xi`` callable for
each round's challenge, exactly where the reference calls ``transcript.challenge()``.
"""
from __future__ import annotations

import ctypes
from typing import Callable

import numpy as np

from . import _lib as H
from .group import _curve


def commit(p, d: int, w=None, curve="pallas") -> np.ndarray:
    """pcdl.rs:275-287: n = d + 1 must be a power of two, deg(p) <= d <= D, then
    pedersen::commit(w, Gs[0..n], p.coeffs) over the resident SRS."""
    H.ensure_device()
    c = H.fe_array(p) if len(p) else np.zeros((0, 4), dtype=np.uint64)
    wa = H.fe_array(w, 1) if w is not None else None
    out = np.zeros(8, dtype=np.uint64)
    H.check(H.load().halo_pcdl_commit(_curve(curve), H.ptr(c) if len(c) else None, len(c), d, H.ptr(wa), H.ptr(out)))
    return out


class IpaSession:
    """Device-resident (G, c, z) of one opening; mirrors the loop state of pcdl.rs:392-438."""

    def __init__(self, cs, z, H_prime, curve="pallas"):
        H.ensure_device()
        self.curve = _curve(curve)
        cs = H.fe_array(cs)
        self.n = len(cs)
        zz = H.fe_array(z, 1)
        hp = H.point_array(H_prime)
        s = ctypes.c_void_p()
        H.check(H.load().halo_ipa_begin(self.curve, H.ptr(cs), self.n, H.ptr(zz), H.ptr(hp), ctypes.byref(s)))
        self._s = s

    @classmethod
    def with_xi(cls, cs, z, H_point, xi0, curve="pallas") -> "IpaSession":
        """Session whose H' = xi_0 H (pcdl.rs:390-391) is formed on the device (halo_ipa_begin_xi):
        no host scalar multiplication, and the 2^i H table is shared by every opening under H."""
        H.ensure_device()
        self = cls.__new__(cls)
        self.curve = _curve(curve)
        c = H.fe_array(cs)
        self.n = len(c)
        zz = H.fe_array(z, 1)
        hp = H.point_array(H_point)
        x0 = H.fe_array(xi0, 1)
        s = ctypes.c_void_p()
        H.check(H.load().halo_ipa_begin_xi(self.curve, H.ptr(c), self.n, H.ptr(zz), H.ptr(hp), H.ptr(x0),
                                           ctypes.byref(s)))
        self._s = s
        return self

    @classmethod
    def from_vectors(cls, gs, cs, zs, H_prime, curve="pallas") -> "IpaSession":
        """Session over explicit (G, c, z) of length n (a shard of a distributed opening,
        halo_amd.dist.sharded_ipa_rounds)."""
        H.ensure_device()
        self = cls.__new__(cls)
        self.curve = _curve(curve)
        g = H.point_array(gs)
        c = H.fe_array(cs)
        z = H.fe_array(zs)
        if not (len(g) == len(c) == len(z)):
            raise ValueError("G, c and z must have the same length")
        self.n = len(c)
        hp = H.point_array(H_prime)
        s = ctypes.c_void_p()
        H.check(H.load().halo_ipa_begin_vectors(self.curve, H.ptr(g), H.ptr(c), H.ptr(z), self.n, H.ptr(hp),
                                                ctypes.byref(s)))
        self._s = s
        return self

    def _stage(self):
        """Per-session staging arrays with their addresses taken once: a round's ctypes call then
        passes plain integers (numpy's per-call ctypes pointer objects cost a few us each, on a
        ~100 us round of the small openings)."""
        st = getattr(self, "_st", None)
        if st is None:
            lr, xi = np.zeros((2, 8), dtype=np.uint64), np.zeros(4, dtype=np.uint64)
            st = self._st = (lr, lr.ctypes.data, lr.ctypes.data + 64, xi, xi.ctypes.data, H.load())
        return st

    def round_lr(self):
        lr, pl, pr, _, _, lib = self._stage()
        H.check(lib.halo_ipa_round_lr(self._s, pl, pr))
        return lr[0].copy(), lr[1].copy()

    def round_lr_dev(self, d_lr: int, stream: int) -> None:
        """halo_ipa_round_lr_dev: the round's L and R land in the 256 device bytes at d_lr as packed XYZZ,
        ordered before later work on `stream`; no host wait."""
        _, _, _, _, _, lib = self._stage()
        H.check(lib.halo_ipa_round_lr_dev(self._s, ctypes.c_void_p(d_lr), ctypes.c_void_p(stream)))

    def fold(self, xi, xi_inv=None):
        """xi_inv None: the library forms xi^-1 itself (halo_ipa_fold with a NULL xi_inv)."""
        _, _, _, xb, px, lib = self._stage()
        if xi_inv is not None:
            H.check(lib.halo_ipa_fold(self._s, H.ptr(H.fe_array(xi, 1)), H.ptr(H.fe_array(xi_inv, 1))))
            return
        np.copyto(xb, np.asarray(xi, dtype=np.uint64).reshape(4))
        H.check(lib.halo_ipa_fold(self._s, px, None))

    def state(self, with_gs: bool = True):
        """(m, gs, cs, zs): the folded vectors (length 2m).  Sessions over the resident SRS do not
        materialise G in their weighted / tail rounds: with_gs=False there (gs is None)."""
        m = ctypes.c_size_t(0)
        H.check(H.load().halo_ipa_state(self._s, ctypes.byref(m), None, None, None))
        k = max(2 * m.value, 1)
        gs = np.zeros((k, 8), dtype=np.uint64) if with_gs else None
        cs = np.zeros((k, 4), dtype=np.uint64)
        zs = np.zeros((k, 4), dtype=np.uint64)
        H.check(H.load().halo_ipa_state(self._s, ctypes.byref(m), H.ptr(gs) if with_gs else None, H.ptr(cs),
                                        H.ptr(zs)))
        return m.value, gs, cs, zs

    def end(self):
        U = np.zeros(8, dtype=np.uint64)
        c = np.zeros(4, dtype=np.uint64)
        # halo_ipa_end returns the session to the pool even when it reports an error, so the handle
        # is dropped first: no caller path can end (release) it a second time
        s, self._s = self._s, None
        H.check(H.load().halo_ipa_end(s, H.ptr(U), H.ptr(c)))
        return U, c

    @staticmethod
    def end_many(sessions):
        """end() of lockstep sessions in one halo_ipa_end_multi call (their final U sums overlap on the
        device); [(U, c)] in order."""
        k = len(sessions)
        U = np.zeros((k, 8), dtype=np.uint64)
        c = np.zeros((k, 4), dtype=np.uint64)
        handles = [s_._s for s_ in sessions]
        # the library's argument checks first, here: they release nothing, so the handles must stay
        if any(h is None for h in handles):
            raise ValueError("end_many: a session was already ended")
        if len({h.value for h in handles}) != k:
            raise ValueError("end_many: a session is listed twice")
        arr = (ctypes.c_void_p * k)(*[h.value for h in handles])
        rc = H.load().halo_ipa_end_multi(arr, k, H.ptr(U), H.ptr(c))
        # past its argument checks the call releases every session, also on an error (halo_gpu.h); an
        # argument error (its own "halo_ipa_end_multi:" messages) releases none, and the handles stay
        # with their wrappers so that end() can still release them
        if rc == H.HALO_OK or not H.last_error().startswith("halo_ipa_end_multi:"):
            for s_ in sessions:
                s_._s = None
        H.check(rc)
        return [(U[i].copy(), c[i].copy()) for i in range(k)]


def ipa_rounds(cs, z, H_prime, challenge: Callable, inverse: Callable, curve="pallas"):
    """The round loop of open_without_eval (pcdl.rs:392-450) given p'.coeffs resized to n, z, H' and
    the caller's transcript.  ``challenge(xi_prev, L, R)`` returns the next xi (ark limbs, shape (4,));
    ``inverse(xi)`` returns xi^-1.  Returns (Ls, Rs, U, c)."""
    ses = IpaSession(cs, z, H_prime, curve)
    n = ses.n
    lg_n = n.bit_length() - 1
    Ls, Rs = [], []
    xi = None
    for _ in range(lg_n):
        L, R = ses.round_lr()
        Ls.append(L)
        Rs.append(R)
        xi = challenge(xi, L, R)
        ses.fold(xi, inverse(xi))
    U, c = ses.end()
    return Ls, Rs, U, c


_SCALAR = {0: 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001,   # Pallas: Fp
           1: 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001}   # Vesta: Fq


def _ark_inverse(x: np.ndarray, cid: int) -> np.ndarray:
    """x^-1 for an ark Montgomery scalar (x R -> x^-1 R), host big integers."""
    r = _SCALAR[cid]
    v = int(x[0]) | int(x[1]) << 64 | int(x[2]) << 128 | int(x[3]) << 192
    inv = pow(v, -1, r) * pow(2, 512, r) % r  # (x R)^-1 R^2 = x^-1 R: one modular inverse
    return np.array([(inv >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)


def open_without_eval(p, C, d: int, z, v, w=None, transcript=None, q=None, w_bar=None, curve="pallas") -> dict:
    """pcdl::open_without_eval (pcdl.rs:326-453) on the device, hiding branch included.

    p: coefficients (ark scalars, degree <= d); C its commitment; z, v ark scalars; w the commitment
    randomness (None: non-hiding).  ``transcript`` is the caller's Fiat-Shamir sponge with the
    reference's interface (outer_sponge.rs: absorb_g(points), absorb_fr(scalars), challenge()) over
    WrappedPoints / ark scalars -- a fresh PCDL sponge, as pcdl.rs:336 creates; it is required (the
    sponge is host logic outside this backend).  q (d coefficients) and w_bar are the random draws the
    reference takes from its rng (pcdl.rs:347,352).  p, p_bar and p' stay in the session's device
    buffers from the blind to the rounds (halo_pcdl_open_begin / _blind / _combine / _start).
    Returns the EvalProof: dict(Ls, Rs, U, c, C_bar, w_prime)."""
    if transcript is None:
        raise ValueError("open_without_eval needs the caller's PCDL transcript (pcdl.rs:336 Sponge::new(PCDL))")
    H.ensure_device()
    L = H.load()
    cid = _curve(curve)
    n = d + 1
    p = H.fe_array(p) if len(p) else np.zeros((0, 4), dtype=np.uint64)
    zz = H.fe_array(z, 1)[0]
    vv = H.fe_array(v, 1)[0] if v is not None else None
    C = H.point_array(C).reshape(8)
    s = ctypes.c_void_p()
    # asserts n > 1, n a power of two, p.degree() <= d, d <= D (pcdl.rs:338-341)
    v_out = np.zeros(4, dtype=np.uint64) if v is None else None  # pcdl::open: v = p(z) on the device
    H.check(L.halo_pcdl_open_begin(cid, H.ptr(p) if len(p) else None, len(p), d, H.ptr(zz), H.ptr(v_out),
                                   ctypes.byref(s)))
    if v is None:
        vv = v_out
    ses = IpaSession.__new__(IpaSession)
    ses.curve, ses.n, ses._s = cid, n, s
    try:
        C_bar = w_prime = None
        if w is not None:
            C_bar = np.zeros(8, dtype=np.uint64)
            H.check(L.halo_pcdl_open_blind(s, H.ptr(H.fe_array(q, d)), H.ptr(H.fe_array(w_bar, 1)), H.ptr(C_bar)))
            transcript.absorb_g([C, C_bar])
            transcript.absorb_fr([zz, vv])
            alpha = np.ascontiguousarray(transcript.challenge(), dtype=np.uint64)
            w_prime = np.zeros(4, dtype=np.uint64)
            C_prime = np.zeros(8, dtype=np.uint64)
            H.check(L.halo_pcdl_open_combine(s, H.ptr(alpha), H.ptr(C), H.ptr(H.fe_array(w, 1)), H.ptr(w_prime),
                                             H.ptr(C_prime)))
        else:
            C_prime = C
        transcript.absorb_g([C_prime])
        transcript.absorb_fr([zz, vv])
        xi = np.ascontiguousarray(transcript.challenge(), dtype=np.uint64)
        H.check(L.halo_pcdl_open_start(s, None, H.ptr(xi)))  # H' = xi_0 pp.H (pcdl.rs:390)
        Ls, Rs = [], []
        for _ in range(n.bit_length() - 1):
            Lp, Rp = ses.round_lr()
            Ls.append(Lp)
            Rs.append(Rp)
            transcript.absorb_fr([xi])
            transcript.absorb_g([Lp, Rp])
            xi = np.ascontiguousarray(transcript.challenge(), dtype=np.uint64)
            ses.fold(xi)  # xi^-1 formed by the library (pcdl.rs:430)
        U, c = ses.end()
    finally:
        if ses._s is not None:  # an assertion or error above: return the session to the pool
            L.halo_ipa_end(ses._s, None, None)
            ses._s = None
    return {"Ls": Ls, "Rs": Rs, "U": U, "c": c, "C_bar": C_bar, "w_prime": w_prime, "v": vv}


class StandInTranscript:
    """A stand-in for the reference's Poseidon PCDL sponge (outer_sponge.rs) with its interface, for
    timing runs only: challenges are SHA-256 of everything absorbed, reduced mod r.  (The Fiat-Shamir
    transcript is host logic outside the device path; tests drive the device with the restated
    Poseidon sponge, tests/test_gpu_transcript.py.)"""

    def __init__(self, curve="pallas"):
        import hashlib
        self._h = hashlib.sha256(b"PCDL")
        self._r = _SCALAR[_curve(curve)]

    def absorb_g(self, pts):
        for q in pts:
            self._h.update(np.ascontiguousarray(q, dtype=np.uint64).tobytes())

    def absorb_fr(self, xs):
        for x in xs:
            self._h.update(np.ascontiguousarray(x, dtype=np.uint64).tobytes())

    def challenge(self) -> np.ndarray:
        d = self._h.digest()
        self._h.update(d)
        v = (int.from_bytes(d, "little") % self._r) or 1
        m = v * (1 << 256) % self._r
        return np.array([(m >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)


def evaluate(p, z, curve="pallas") -> np.ndarray:
    """DensePolynomial::evaluate (pcdl.rs:49,471) on the device (halo_poly_eval_batch)."""
    import ctypes as _ct
    H.ensure_device()
    c = H.fe_array(p)
    out = np.zeros((1, 4), dtype=np.uint64)
    ptrs = (_ct.c_void_p * 1)(c.ctypes.data)
    lens = (_ct.c_size_t * 1)(len(c))
    field = H.FP if _curve(curve) == 0 else H.FQ
    H.check(H.load().halo_poly_eval_batch(field, ptrs, lens, 1, H.ptr(H.fe_array(z, 1)), H.ptr(out)))
    return out[0]


def open(p, C, d: int, z, w=None, transcript=None, q=None, w_bar=None, curve="pallas") -> dict:  # noqa: A001
    """pcdl::open (pcdl.rs:463-473): v = p(z) (evaluated on the device inside the session start,
    halo_pcdl_open_begin), then open_without_eval.  The EvalProof dict carries v."""
    return open_without_eval(p, C, d, z, None, w=w, transcript=transcript, q=q, w_bar=w_bar, curve=curve)


class HPoly:
    """pcdl.rs:184-229 HPoly: h(X) = prod_{i < lg n} (1 + xi_{lg n - i} X^(2^i)) from the round
    challenges xis (ark Montgomery scalars, xis[0] unused by h as in the reference)."""

    def __init__(self, xis, curve="pallas"):
        self.curve = _curve(curve)
        self.field = H.FP if self.curve == 0 else H.FQ
        self.xis = H.fe_array(xis)

    def get_poly(self) -> np.ndarray:
        """Coefficients (2^(len(xis) - 1) of them), generated on the device (halo_hpoly_coeffs)."""
        H.ensure_device()
        n = 1 << (len(self.xis) - 1)
        out = np.zeros((n, 4), dtype=np.uint64)
        H.check(H.load().halo_hpoly_coeffs(self.field, H.ptr(self.xis), len(self.xis), H.ptr(out)))
        return out

    @staticmethod
    def combine(hs: list["HPoly"], alphas) -> np.ndarray:
        """sum_i alphas[i] * h_i(X) (acc.rs:89), trimmed like DensePolynomial."""
        H.ensure_device()
        k = len(hs)
        xis = np.ascontiguousarray(np.concatenate([h.xis for h in hs]))
        a = H.fe_array(alphas, k)
        n = 1 << (len(hs[0].xis) - 1)
        out = np.zeros((n, 4), dtype=np.uint64)
        m = ctypes.c_size_t(0)
        H.check(H.load().halo_hpoly_combine(hs[0].field, H.ptr(xis), k, len(hs[0].xis), H.ptr(a), H.ptr(out),
                                            ctypes.byref(m)))
        return out[: m.value]


def decider_commit(xis, d: int, curve="pallas") -> np.ndarray:
    """pcdl.rs:579 (check step 5): pedersen::commit(None, &pp.Gs[0..d+1], &h.get_poly().coeffs)."""
    H.ensure_device()
    x = H.fe_array(xis)
    out = np.zeros(8, dtype=np.uint64)
    H.check(H.load().halo_pcdl_decider_commit(_curve(curve), H.ptr(x), len(x), d, H.ptr(out)))
    return out


def trace_commit_batch(evals, d: int, curve="pallas", want_coeffs: bool = False):
    """Trace::new's interpolate + commit (crates/plonk/src/circuit/trace.rs:165-192) for k evaluation
    vectors at once: Evals::from_vec_and_domain -> interpolate_by_ref -> pcdl::commit(poly, d, None).
    evals: (k, n, 4) ark scalars.  Returns the k commitments (k, 8) and, if asked, the trimmed
    coefficient vectors."""
    H.ensure_device()
    e = np.ascontiguousarray(np.asarray(evals, dtype=np.uint64))
    k, n = e.shape[0], e.shape[1]
    log_n = n.bit_length() - 1
    if 1 << log_n != n:
        raise ValueError("domain size must be a power of two")
    commits = np.zeros((k, 8), dtype=np.uint64)
    coeffs = np.zeros((k, n, 4), dtype=np.uint64) if want_coeffs else None
    lens = (ctypes.c_size_t * k)()
    H.check(H.load().halo_trace_commit_batch(_curve(curve), H.ptr(e), k, log_n, d,
                                             H.ptr(coeffs) if want_coeffs else None, lens, H.ptr(commits)))
    if want_coeffs:
        return commits, [coeffs[i, : lens[i]] for i in range(k)]
    return commits
