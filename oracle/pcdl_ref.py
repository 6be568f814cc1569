"""CPU restatement of pcdl::open_without_eval with the reference's transcript.
TEST INFRASTRUCTURE ONLY (fixture generator / checker; never imported by halo_amd).

Follows crates/accumulation/src/pcdl.rs:326-453 step by step, including the hiding branch
(pcdl.rs:344-371: p_bar = (X - z) q, C_bar = commit(p_bar, d, w_bar), alpha = rho(C, C_bar, z, v),
p' = p + alpha p_bar, w' = w_bar alpha + w, C' = C + alpha C_bar - w' S) and the PCDL transcript
(oracle/poseidon.py).  The random draws of the reference (q, w_bar) are inputs here.  MSMs and the
folds of G run on the C oracle (oracle.c via corc); everything else with Python integers.
"""
from __future__ import annotations

import numpy as np

import corc
import pasta as P
import poseidon


def _w(c, pt):
    return np.array(P.point_to_wrapped(c, pt), dtype=np.uint64)


def _pt(c, w):
    return P.wrapped_to_point(c, [int(x) for x in w])


def _fe(xs, m):
    return np.array([P.int_to_limbs(P.to_mont(x % m, m)) for x in xs], dtype=np.uint64).reshape(-1, 4)


def commit(curve, gs_wrapped, coeffs, w=None, S=None):
    """pcdl::commit over Gs[0..len(coeffs)) (+ w S)."""
    c = P.CURVES[curve]
    acc = _pt(c, corc.msm(curve, np.ascontiguousarray(gs_wrapped[: len(coeffs)]), _fe(coeffs, c.scalar))) \
        if len(coeffs) else None
    if w is not None:
        acc = P.add(c, acc, P.mul_fast(c, w % c.scalar, S))
    return acc


def open_without_eval(curve, p, C, d, z, v, gs_wrapped, S, H, w=None, q=None, w_bar=None):
    """p: coefficient ints; C, S, H: affine points; gs_wrapped: SRS WrappedPoints (>= d + 1).
    Returns dict(Ls, Rs (affine), U (affine), c, C_bar, w_prime, xis, alpha)."""
    c = P.CURVES[curve]
    r = c.scalar
    n = d + 1
    lg_n = n.bit_length() - 1
    assert n > 1 and n & (n - 1) == 0
    t = poseidon.Sponge(curve, poseidon.PCDL)
    C_bar = w_prime = alpha = None
    if w is not None:
        p_bar = P.poly_mul(list(q), [(-z) % r, 1], r)
        C_bar = commit(curve, gs_wrapped, p_bar, w_bar, S)
        t.absorb_g([C, C_bar])
        t.absorb_fr([z, v])
        alpha = t.challenge()
        pp = [0] * max(len(p), len(p_bar))
        for i, x in enumerate(p):
            pp[i] = x
        for i, x in enumerate(p_bar):
            pp[i] = (pp[i] + alpha * x) % r
        w_prime = (w_bar * alpha + w) % r
        C_prime = P.add(c, P.add(c, C, P.mul_fast(c, alpha, C_bar)), P.neg(c, P.mul_fast(c, w_prime, S)))
        p = pp
    else:
        C_prime = C
    t.absorb_g([C_prime])
    t.absorb_fr([z, v])
    xi = t.challenge()
    xis = [xi]
    Hp = P.mul_fast(c, xi, H)
    cs = [x % r for x in p] + [0] * (n - len(p))
    gs = np.ascontiguousarray(gs_wrapped[:n].copy())
    zs = [pow(z, i, r) for i in range(n)]
    Ls, Rs = [], []
    m = n // 2
    for _ in range(lg_n):
        cl, cr, zl, zr = cs[:m], cs[m:2 * m], zs[:m], zs[m:2 * m]
        dot_l = sum(a * b for a, b in zip(cr, zl)) % r
        dot_r = sum(a * b for a, b in zip(cl, zr)) % r
        L = P.add(c, _pt(c, corc.msm(curve, gs[:m], _fe(cr, r))), P.mul_fast(c, dot_l, Hp))
        R = P.add(c, _pt(c, corc.msm(curve, gs[m:2 * m], _fe(cl, r))), P.mul_fast(c, dot_r, Hp))
        Ls.append(L)
        Rs.append(R)
        t.absorb_fr([xi])
        t.absorb_g([L, R])
        xi = t.challenge()
        xis.append(xi)
        xinv = pow(xi, -1, r)
        g2, _, _ = corc.ipa_fold(curve, gs[:2 * m], _fe(cs[:2 * m], r), _fe(zs[:2 * m], r), _fe([xi], r)[0],
                                 _fe([xinv], r)[0])
        gs = np.ascontiguousarray(g2)
        cs = [(cl[j] + cr[j] * xinv) % r for j in range(m)]
        zs = [(zl[j] + zr[j] * xi) % r for j in range(m)]
        m //= 2
    return {"Ls": Ls, "Rs": Rs, "U": _pt(c, gs[0]), "c": cs[0], "C_bar": C_bar, "w_prime": w_prime,
            "xis": xis, "alpha": alpha}
