"""CPU oracle (pure-Python big-int) for the halo hot path.  TEST INFRASTRUCTURE ONLY.

This module is the parity *checker*.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path (``halo_amd``) never does.

It restates, with Python integers, the algorithms the reference runs on the hot path
(all citations relative to the reference root, rasmus-kirk/halo):

* Pasta fields: ``Fp = ark_pallas::Fr`` and ``Fq = ark_pallas::Fq``
  (``crates/group/src/lib.rs:8-9``; moduli consts ``crates/group/src/wrappers.rs:524-525,585-586``),
  Montgomery form with R = 2^256 (arkworks ``Fp256`` / ``BigInt<4>`` limbs).
* Pallas / Vesta short-Weierstrass curves y^2 = x^3 + 5, generator (-1, 2)
  (``crates/group/src/group.rs:28-29``).
* MSM  = sum_i s_i * G_i over i < min(#G, #s)  (``crates/accumulation/src/pedersen.rs:7-27``,
  ``crates/group/src/group.rs:48-56``).  The result is a unique group element, so a naive sum
  is bit-exact once both sides are normalised to canonical affine.
* Radix-2 NTT over the 2^k domain with omega = 5^((r-1)/N) (ark-poly 0.5.0
  ``Radix2EvaluationDomain``, called from ``crates/group/src/poly.rs:56-64,133-139``),
  inputs longer than N reduced mod X^N - 1 first; interpolate trims trailing zeros.
* Horner evaluation (``DensePolynomial::evaluate``; ``crates/accumulation/src/pcdl.rs:49,471``),
  ``scalar_dot`` / ``construct_powers`` (``crates/group/src/group.rs:43-45,58-66``).
* One IPA folding round (``crates/accumulation/src/pcdl.rs:404-438``).
* The SRS recipe G[i*16384+k] = H(i+k+2), S = H(0), H = H(1) with
  H(j) = [from_le_bytes_mod_order(SHA3-256(u64le(j) || GENESIS))] * (-1, 2)
  (``crates/group/src/main.rs:55-67,97-121``) and the bincode-v2 ``Vec<WrappedPoint>`` decoder
  (``crates/group/src/pp.rs:36-53``, ``crates/group/src/wrappers.rs:592-597``).

Parity pinning: this restatement is checked (tests/test_oracle.py) against the reference's own
committed data -- SRS points / S / H decoded from ``crates/group/.precompute/*`` (fixtures in
``tests/golden/``) and the 2^16 domain generators ``IVC_FP_CIRCUIT.omega`` /
``IVC_FQ_CIRCUIT.omega`` (``crates/plonk/src/frontend/ivc/mod.rs:55,112``).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass

# --------------------------------------------------------------------------------------
# Fields
# --------------------------------------------------------------------------------------

FP_MODULUS = 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001  # ark_pallas::Fr
FQ_MODULUS = 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001  # ark_pallas::Fq
R_MONT = 1 << 256
TWO_ADICITY = 32
GENERATOR = 5  # multiplicative generator used by ark for both Pasta fields

FIELDS = {"fp": FP_MODULUS, "fq": FQ_MODULUS}


def to_mont(x: int, m: int) -> int:
    return (x * R_MONT) % m


def from_mont(x: int, m: int) -> int:
    return (x * pow(R_MONT, -1, m)) % m


def int_to_limbs(x: int, n: int = 4) -> list[int]:
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)]


def limbs_to_int(limbs) -> int:
    return sum(int(l) << (64 * i) for i, l in enumerate(limbs))


def inv(x: int, m: int) -> int:
    return pow(x, -1, m)


def root_of_unity(m: int, n: int) -> int:
    """omega_N = g^((m-1)/N), g = 5: ark ``get_root_of_unity`` for a 2-adic domain."""
    assert n & (n - 1) == 0 and n.bit_length() - 1 <= TWO_ADICITY
    return pow(GENERATOR, (m - 1) // n, m)


# --------------------------------------------------------------------------------------
# Curves
# --------------------------------------------------------------------------------------


@dataclass(frozen=True)
class Curve:
    name: str
    base: int   # modulus of the coordinate field
    scalar: int  # group order
    b: int = 5

    @property
    def generator(self):
        return (self.base - 1, 2)


PALLAS = Curve("pallas", base=FQ_MODULUS, scalar=FP_MODULUS)
VESTA = Curve("vesta", base=FP_MODULUS, scalar=FQ_MODULUS)
CURVES = {"pallas": PALLAS, "vesta": VESTA}

INF = None  # point at infinity in affine form


def on_curve(c: Curve, P) -> bool:
    if P is INF:
        return True
    x, y = P
    return (y * y - x * x * x - c.b) % c.base == 0


def add(c: Curve, P, Q):
    p = c.base
    if P is INF:
        return Q
    if Q is INF:
        return P
    x1, y1 = P
    x2, y2 = Q
    if x1 == x2:
        if (y1 + y2) % p == 0:
            return INF
        lam = 3 * x1 * x1 * inv(2 * y1, p) % p
    else:
        lam = (y2 - y1) * inv(x2 - x1, p) % p
    x3 = (lam * lam - x1 - x2) % p
    y3 = (lam * (x1 - x3) - y1) % p
    return (x3, y3)


def neg(c: Curve, P):
    if P is INF:
        return INF
    return (P[0], (-P[1]) % c.base)


def mul(c: Curve, k: int, P):
    k %= c.scalar
    R = INF
    Q = P
    while k:
        if k & 1:
            R = add(c, R, Q)
        Q = add(c, Q, Q)
        k >>= 1
    return R


# Jacobian arithmetic for fast fixed-base generation in the oracle (no per-step inversion)
def _jdbl(p, X, Y, Z):
    if Z == 0 or Y == 0:
        return (1, 1, 0)
    A = X * X % p
    B = Y * Y % p
    C = B * B % p
    D = 2 * ((X + B) ** 2 - A - C) % p
    E = 3 * A % p
    X3 = (E * E - 2 * D) % p
    Y3 = (E * (D - X3) - 8 * C) % p
    Z3 = 2 * Y * Z % p
    return (X3, Y3, Z3)


def _jadd_affine(p, X1, Y1, Z1, x2, y2):
    if Z1 == 0:
        return (x2, y2, 1)
    Z1Z1 = Z1 * Z1 % p
    U2 = x2 * Z1Z1 % p
    S2 = y2 * Z1 * Z1Z1 % p
    H = (U2 - X1) % p
    r = (S2 - Y1) % p
    if H == 0:
        if r == 0:
            return _jdbl(p, X1, Y1, Z1)
        return (1, 1, 0)
    HH = H * H % p
    HHH = H * HH % p
    V = X1 * HH % p
    X3 = (r * r - HHH - 2 * V) % p
    Y3 = (r * (V - X3) - Y1 * HHH) % p
    Z3 = Z1 * H % p
    return (X3, Y3, Z3)


def _to_affine(p, J):
    X, Y, Z = J
    if Z == 0:
        return INF
    zi = inv(Z, p)
    zi2 = zi * zi % p
    return (X * zi2 % p, Y * zi2 * zi % p)


def mul_fast(c: Curve, k: int, P):
    """k*P with Jacobian intermediates (same result as ``mul``)."""
    k %= c.scalar
    if P is INF or k == 0:
        return INF
    p = c.base
    J = (1, 1, 0)
    for bit in bin(k)[2:]:
        J = _jdbl(p, *J)
        if bit == "1":
            J = _jadd_affine(p, *J, P[0], P[1])
    return _to_affine(p, J)


def msm(c: Curve, bases, scalars):
    """sum_i s_i * G_i over i < min(len) (pedersen.rs:21 ``msm_unchecked`` semantics)."""
    acc = INF
    for G, s in zip(bases, scalars):
        acc = add(c, acc, mul_fast(c, s, G))
    return acc


# --------------------------------------------------------------------------------------
# Wire formats
# --------------------------------------------------------------------------------------


def point_to_wrapped(c: Curve, P) -> list[int]:
    """Affine point -> WrappedPoint limbs (x[4], y[4]) in Montgomery form; identity = (0, 0)
    (``PastaAffine::identity`` convention, wrappers.rs:91-93)."""
    if P is INF:
        return [0] * 8
    return int_to_limbs(to_mont(P[0], c.base)) + int_to_limbs(to_mont(P[1], c.base))


def wrapped_to_point(c: Curve, limbs):
    x = limbs_to_int(limbs[0:4])
    y = limbs_to_int(limbs[4:8])
    if x == 0 and y == 0:
        return INF
    P = (from_mont(x, c.base), from_mont(y, c.base))
    assert on_curve(c, P), "WrappedPoint not on curve (wrappers.rs:606)"
    return P


def bincode_varint(buf: bytes, off: int):
    """bincode-v2 ``standard()`` unsigned varint."""
    b = buf[off]
    if b < 251:
        return b, off + 1
    width = {251: 2, 252: 4, 253: 8, 254: 16}[b]
    return int.from_bytes(buf[off + 1: off + 1 + width], "little"), off + 1 + width


def decode_wrapped_points(buf: bytes, max_points: int | None = None):
    """Decode a bincode ``Vec<WrappedPoint>`` (pp.rs:37) -> list of 8-limb lists."""
    n, off = bincode_varint(buf, 0)
    if max_points is not None:
        n_take = min(n, max_points)
    else:
        n_take = n
    out = []
    for _ in range(n_take):
        limbs = []
        for _ in range(8):
            v, off = bincode_varint(buf, off)
            limbs.append(v)
        out.append(limbs)
    return n, out


def decode_sh(buf: bytes):
    """Decode ``(WrappedPoint, WrappedPoint)`` = (S, H) (pp.rs:53-55)."""
    off = 0
    pts = []
    for _ in range(2):
        limbs = []
        for _ in range(8):
            v, off = bincode_varint(buf, off)
            limbs.append(v)
        pts.append(limbs)
    return pts


# --------------------------------------------------------------------------------------
# SRS recipe (crates/group/src/main.rs:55-67, 97-121)
# --------------------------------------------------------------------------------------

GENESIS = b"To understand recursion, one must first understand recursion"


def srs_hash_scalar(c: Curve, i: int) -> int:
    h = hashlib.sha3_256(i.to_bytes(8, "little") + GENESIS).digest()
    return int.from_bytes(h, "little") % c.scalar


def srs_hash_point(c: Curve, i: int):
    return mul_fast(c, srs_hash_scalar(c, i), c.generator)


def srs_index(j: int) -> int:
    """Hash index of SRS entry j: block i = j >> 14, k = j & 16383, point = H(i + k + 2)."""
    return (j >> 14) + (j & 16383) + 2


# --------------------------------------------------------------------------------------
# Polynomials / NTT (ark-poly semantics)
# --------------------------------------------------------------------------------------


def fold_mod_xn_minus_1(coeffs, n: int, m: int):
    out = [0] * n
    for i, c in enumerate(coeffs):
        out[i % n] = (out[i % n] + c) % m
    return out


def ntt(coeffs, n: int, m: int, inverse: bool = False):
    """evals[i] = p(omega^i) (forward); inverse: coeffs = N^-1 sum evals omega^-ij.
    Iterative radix-2 DIT, natural order in and out."""
    a = fold_mod_xn_minus_1(coeffs, n, m)
    logn = n.bit_length() - 1
    # bit-reverse permutation
    for i in range(n):
        j = int(format(i, f"0{logn}b")[::-1], 2) if logn else 0
        if i < j:
            a[i], a[j] = a[j], a[i]
    w_n = root_of_unity(m, n)
    if inverse:
        w_n = inv(w_n, m)
    length = 2
    while length <= n:
        w_len = pow(w_n, n // length, m)
        half = length // 2
        tw = [1] * half
        for k in range(1, half):
            tw[k] = tw[k - 1] * w_len % m
        for start in range(0, n, length):
            for k in range(half):
                u = a[start + k]
                v = a[start + k + half] * tw[k] % m
                a[start + k] = (u + v) % m
                a[start + k + half] = (u - v) % m
        length <<= 1
    if inverse:
        ninv = inv(n, m)
        a = [x * ninv % m for x in a]
    return a


def trim(coeffs):
    """``DensePolynomial::from_coefficients_vec`` trims trailing zeros."""
    c = list(coeffs)
    while c and c[-1] == 0:
        c.pop()
    return c


def horner(coeffs, z: int, m: int) -> int:
    v = 0
    for c in reversed(coeffs):
        v = (v * z + c) % m
    return v


def scalar_dot(xs, ys, m: int) -> int:
    return sum(x * y for x, y in zip(xs, ys)) % m


def construct_powers(z: int, n: int, m: int):
    out = []
    cur = 1
    for _ in range(n):
        out.append(cur)
        cur = cur * z % m
    return out


def poly_mul(a, b, m: int):
    if not a or not b:
        return []
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x == 0:
            continue
        for j, y in enumerate(b):
            out[i + j] = (out[i + j] + x * y) % m
    return trim(out)


# --------------------------------------------------------------------------------------
# IPA fold (crates/accumulation/src/pcdl.rs:404-438)
# --------------------------------------------------------------------------------------


def ipa_round(c: Curve, gs, cs, zs, xi: int):
    """One round over vectors of length 2m.  Returns (L_noH, R_noH, dot_l, dot_r, gs', cs', zs').

    L = <c_r, G_l> + H'*<c_r, z_l>,  R = <c_l, G_r> + H'*<c_l, z_r>; the H' term is added by the
    caller.  Fold: G' = G_l + xi*G_r, c' = c_l + xi^-1 c_r, z' = z_l + xi z_r.
    """
    r = c.scalar
    m = len(gs) // 2
    gl, gr = gs[:m], gs[m:]
    cl, cr = cs[:m], cs[m:]
    zl, zr = zs[:m], zs[m:]
    dot_l = scalar_dot(cr, zl, r)
    dot_r = scalar_dot(cl, zr, r)
    L = msm(c, gl, cr)
    R = msm(c, gr, cl)
    xinv = inv(xi, r)
    g2 = [add(c, gl[j], mul_fast(c, xi, gr[j])) for j in range(m)]
    c2 = [(cl[j] + xinv * cr[j]) % r for j in range(m)]
    z2 = [(zl[j] + xi * zr[j]) % r for j in range(m)]
    return L, R, dot_l, dot_r, g2, c2, z2


def h_coeffs(xis, m: int):
    """Coefficients of h(X) = prod_{i=0}^{lg n - 1} (1 + xi_{lg n - i} X^{2^i})  (pcdl.rs:198-219):
    coef[k] = prod over set bits b of k of xi_{lg n - b}."""
    lg_n = len(xis) - 1
    n = 1 << lg_n
    out = []
    for k in range(n):
        v = 1
        for b in range(lg_n):
            if (k >> b) & 1:
                v = v * xis[lg_n - b] % m
        out.append(v)
    return out
