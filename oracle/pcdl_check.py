"""CPU restatement of the PCDL verifier side: ``succinct_check`` and the decider of ``check``.
TEST INFRASTRUCTURE ONLY (the checker): only ``tests/`` and ``bench.py``'s CPU leg import it.

Follows crates/accumulation/src/pcdl.rs:
  * ``succinct_check`` (pcdl.rs:483-554): C' = C (+ alpha C_bar - w' S when hiding), H' = xi_0 H,
    C_0 = C' + v H', C_(i+1) = C_i + xi_(i+1)^-1 L_i + xi_(i+1) R_i, h(X) = prod_i (1 + xi_(lg n - i)
    X^(2^i)), v' = c h(z), accept iff C_(lg n) == c U + v' H';
  * ``HPoly::eval`` (pcdl.rs:222-235) and ``HPoly::get_poly``'s coefficients (pcdl.rs:198-219,
    coef[k] = product of xi_(lg n - b) over the set bits b of k);
  * ``check``'s decider (pcdl.rs:563-583): U == commit(h coefficients) over Gs[0..n).
The challenges are passed in (the xi the prover used): the pipeline's transcript is a seeded stand-in
(halo_amd/prover.py), so what this pins is the algebra of the opening -- every L_i, R_i, U and c
against C and v -- not the Fiat-Shamir derivation of the xi.
"""
from __future__ import annotations

import pasta as P


def _pt(c, wrapped):
    return P.wrapped_to_point(c, [int(x) for x in wrapped])


def h_eval(xis, z: int, m: int) -> int:
    """HPoly::eval (pcdl.rs:222-235); xis = [xi_0, xi_1, ..., xi_lg_n]."""
    lg_n = len(xis) - 1
    v = (1 + xis[lg_n] * z) % m
    zi = z
    for i in range(1, lg_n):
        zi = zi * zi % m
        v = v * (1 + xis[lg_n - i] * zi) % m
    return v


def h_coeffs(xis, m: int):
    """Coefficients of h(X) by doubling: after bit b the first 2^(b+1) entries are final."""
    lg_n = len(xis) - 1
    out = [1]
    for b in range(lg_n):
        x = xis[lg_n - b]
        out = out + [v * x % m for v in out]
    return out


def succinct_check(curve: str, C, d: int, z: int, v: int, Ls, Rs, U, c: int, xis, H, S=None,
                   C_bar=None, w_prime=None, alpha=None):
    """pcdl::succinct_check with the given challenges.  Points are ark WrappedPoints (8 u64 limbs,
    Montgomery) or None; scalars canonical ints.  Returns U (as a point) on success, raises
    AssertionError with the reference's message otherwise."""
    cv = P.CURVES[curve]
    m = cv.scalar
    n = d + 1
    lg_n = n.bit_length() - 1
    assert n & (n - 1) == 0, f"n ({n}) is not a power of two"
    assert len(Ls) == lg_n and len(Rs) == lg_n and len(xis) == lg_n + 1
    Cp = _pt(cv, C)
    if C_bar is not None:  # hiding: C' = C + alpha C_bar - w' S (pcdl.rs:503-511)
        Cp = P.add(cv, P.add(cv, Cp, P.mul_fast(cv, alpha, _pt(cv, C_bar))),
                   P.neg(cv, P.mul_fast(cv, w_prime % m, _pt(cv, S))))
    Hp = P.mul_fast(cv, xis[0], _pt(cv, H))
    Ci = P.add(cv, Cp, P.mul_fast(cv, v % m, Hp))
    for i in range(lg_n):
        x = xis[i + 1]
        Ci = P.add(cv, Ci, P.add(cv, P.mul_fast(cv, pow(x, -1, m), _pt(cv, Ls[i])), P.mul_fast(cv, x, _pt(cv, Rs[i]))))
    v_prime = c * h_eval(xis, z, m) % m
    Up = _pt(cv, U)
    rhs = P.add(cv, P.mul_fast(cv, c % m, Up), P.mul_fast(cv, v_prime, Hp))
    assert Ci == rhs, "C_(log_n) != CM.Commit_Sigma(c || v')"
    return Up


def decider_commit_matches(curve: str, U, xis, gs, msm) -> bool:
    """check()'s second step (pcdl.rs:579-581): U == commit(Gs[0..n), h coefficients).  `msm` is
    the C oracle's MSM (corc.msm), called with Montgomery scalars."""
    import numpy as np
    cv = P.CURVES[curve]
    m = cv.scalar
    hc = h_coeffs(xis, m)
    sc = np.array([P.int_to_limbs(P.to_mont(x, m)) for x in hc], dtype=np.uint64).reshape(-1, 4)
    got = msm(curve, np.ascontiguousarray(gs[: len(hc)]), np.ascontiguousarray(sc))
    return [int(x) for x in got] == [int(x) for x in U]


def succinct_check_transcript(curve: str, C, d: int, z: int, v: int, Ls, Rs, U, c: int, H, S=None, C_bar=None,
                              w_prime=None):
    """pcdl::succinct_check exactly as pcdl.rs:483-554: the challenges are re-derived from the
    Poseidon PCDL transcript (oracle/poseidon.py), alpha included in the hiding case.  Returns the
    xis (for the decider)."""
    import poseidon
    cv = P.CURVES[curve]
    m = cv.scalar
    n = d + 1
    lg_n = n.bit_length() - 1
    t = poseidon.Sponge(curve, poseidon.PCDL)
    Cp = _pt(cv, C)
    alpha = None
    if C_bar is not None:
        t.absorb_g([Cp, _pt(cv, C_bar)])
        t.absorb_fr([z, v])
        alpha = t.challenge()
    t.absorb_g([_cprime(cv, Cp, C_bar, alpha, w_prime, S)])
    t.absorb_fr([z, v])
    xis = [t.challenge()]
    for i in range(lg_n):
        t.absorb_fr([xis[i]])
        t.absorb_g([_pt(cv, Ls[i]), _pt(cv, Rs[i])])
        xis.append(t.challenge())
    succinct_check(curve, C, d, z, v, Ls, Rs, U, c, xis, H, S=S, C_bar=C_bar, w_prime=w_prime, alpha=alpha)
    return xis


def _cprime(cv, Cp, C_bar, alpha, w_prime, S):
    if C_bar is None:
        return Cp
    return P.add(cv, P.add(cv, Cp, P.mul_fast(cv, alpha, _pt(cv, C_bar))),
                 P.neg(cv, P.mul_fast(cv, w_prime % cv.scalar, _pt(cv, S))))
