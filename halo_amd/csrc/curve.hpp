// Device group arithmetic for Pallas / Vesta (y^2 = x^3 + 5) on gfx950.
//
// Replaces ark-ec 0.5.0 short-Weierstrass `Projective`/`Affine` arithmetic used on the hot path
// (reference: crates/group/src/group.rs:28-29,48-56; crates/accumulation/src/pedersen.rs:21-26;
// crates/accumulation/src/pcdl.rs:413-429).
//
// Accumulators use XYZZ coordinates (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): mixed addition costs
// 8M + 2S with no inversion, which is the cheapest complete-enough formula for bucket
// accumulation.  Affine points are (x, y) in internal Montgomery form; the identity is encoded as
// (0, 0) (not on the curve, matching `PastaAffine::identity`, crates/group/src/wrappers.rs:91-93).
#pragma once
#include "fields.hpp"

HALO_ARITH_BEGIN

struct PallasCurve {
    using Base = FqCfg;
    using Scalar = FpCfg;
    using K = PallasCurveCfg;
};
struct VestaCurve {
    using Base = FpCfg;
    using Scalar = FqCfg;
    using K = VestaCurveCfg;
};

template <class F>
struct Affine {
    Fe<F> x, y;
};

template <class F>
struct XYZZ {
    Fe<F> X, Y, ZZ, ZZZ;
};

template <class F>
HALO_DEV bool aff_is_id(const Affine<F>& a) {
    return fe_is_zero(a.x) && fe_is_zero(a.y);
}

template <class F>
HALO_DEV XYZZ<F> xyzz_id() {
    XYZZ<F> r;
    r.X = fe_one<F>();
    r.Y = fe_one<F>();
    r.ZZ = fe_zero<F>();
    r.ZZZ = fe_zero<F>();
    return r;
}

template <class F>
HALO_DEV bool xyzz_is_id(const XYZZ<F>& p) {
    return fe_is_zero(p.ZZ);
}

template <class F>
HALO_DEV XYZZ<F> xyzz_from_aff(const Affine<F>& a) {
    if (aff_is_id(a)) return xyzz_id<F>();
    XYZZ<F> r;
    r.X = a.x;
    r.Y = a.y;
    r.ZZ = fe_one<F>();
    r.ZZZ = fe_one<F>();
    return r;
}

template <class F>
HALO_DEV Affine<F> aff_neg(const Affine<F>& a) {
    Affine<F> r;
    r.x = a.x;
    r.y = fe_neg(a.y);
    return r;
}

// dbl-2008-s-1 (a = 0): U = 2Y, V = U^2, W = U V, S = X V, M = 3 X^2,
// X3 = M^2 - 2S, Y3 = M (S - X3) - W Y, ZZ3 = V ZZ, ZZZ3 = W ZZZ.
// Intermediates that only feed multiplications are left lazily reduced (fields.hpp).
template <class F>
HALO_DEV XYZZ<F> xyzz_dbl(const XYZZ<F>& p) {
    if (xyzz_is_id(p)) return p;
    const Fe<F> U = fe_norm(fe_add_nc(p.Y, p.Y));  // normalized: squared below (fields.hpp bounds)
    const Fe<F> V = fe_sqr(U);
    const Fe<F> W = fe_mul(U, V);
    const Fe<F> S = fe_mul(p.X, V);
    const Fe<F> X2 = fe_sqr(p.X);
    const Fe<F> M = fe_norm(fe_add_nc(X2, fe_add_nc(X2, X2)));  // < 6p
    XYZZ<F> r;
    r.X = fe_reduce_8p(fe_sub_k<4>(fe_sqr(M), fe_add_nc(S, S)));
    r.Y = fe_sub(fe_mul(M, fe_sub_k<2>(S, r.X)), fe_mul(W, p.Y));
    r.ZZ = fe_mul(V, p.ZZ);
    r.ZZZ = fe_mul(W, p.ZZZ);
    return r;
}

// Doubling of an affine point into XYZZ (mdbl-2008-s-1)
template <class F>
HALO_DEV XYZZ<F> xyzz_mdbl(const Affine<F>& a) {
    const Fe<F> U = fe_norm(fe_add_nc(a.y, a.y));  // normalized: squared below
    const Fe<F> V = fe_sqr(U);
    const Fe<F> W = fe_mul(U, V);
    const Fe<F> S = fe_mul(a.x, V);
    const Fe<F> X2 = fe_sqr(a.x);
    const Fe<F> M = fe_norm(fe_add_nc(X2, fe_add_nc(X2, X2)));
    XYZZ<F> r;
    r.X = fe_reduce_8p(fe_sub_k<4>(fe_sqr(M), fe_add_nc(S, S)));
    r.Y = fe_sub(fe_mul(M, fe_sub_k<2>(S, r.X)), fe_mul(W, a.y));
    r.ZZ = V;
    r.ZZZ = W;
    return r;
}

// Mixed addition p + q (madd-2008-s), handles identity and the doubling / inverse cases.
// P = U2 - X1 == 0 is detected through ZZ3 = ZZ1 P^2 == 0 (ZZ1 != 0 here), off the common path.
template <class F>
HALO_DEV XYZZ<F> xyzz_madd(const XYZZ<F>& p, const Affine<F>& q) {
    if (aff_is_id(q)) return p;
    if (xyzz_is_id(p)) return xyzz_from_aff(q);
    const Fe<F> U2 = fe_mul(q.x, p.ZZ);
    const Fe<F> S2 = fe_mul(q.y, p.ZZZ);
    const Fe<F> P = fe_sub_k<2>(U2, p.X);  // < 4p
    const Fe<F> R = fe_sub_k<2>(S2, p.Y);  // < 4p
    const Fe<F> PP = fe_sqr(P);
    const Fe<F> ZZ3 = fe_mul(p.ZZ, PP);
    if (fe_is_zero(ZZ3)) {
        if (fe_is_zero_4p(R)) return xyzz_mdbl(q);
        return xyzz_id<F>();
    }
    const Fe<F> PPP = fe_mul(P, PP);
    const Fe<F> Q = fe_mul(p.X, PP);
    XYZZ<F> r;
    r.X = fe_reduce_8p(fe_sub_k<6>(fe_sqr(R), fe_add_nc(PPP, fe_add_nc(Q, Q))));
    r.Y = fe_sub(fe_mul(R, fe_sub_k<2>(Q, r.X)), fe_mul(p.Y, PPP));
    r.ZZ = ZZ3;
    r.ZZZ = fe_mul(p.ZZZ, PPP);
    return r;
}

// Bucket-accumulation form of madd-2008-s (k_acc's inner loop), same result as
// xyzz_madd(p, negmask ? -q : q) but ~14 % fewer instructions:
//   * the sign of q is folded into R = +-S2 - Y1 + 4p (no separate negation of y);
//   * X is carried lazily in [0, 8p) between additions (no reduction of X3; callers reduce with
//     xyzz_settle before storing or handing the point to the general formulas);
//   * Y3 = R (Q - X3) + PPP (2p - Y1) is one product sum with a single Montgomery reduction.
// Bounds: P < 10p, R < 6p, T = Q - X3 + 8p < 10p; P^2 < 100p^2 and R T + PPP (2p - Y1) < 64p^2 stay
// below p 2^261 (~127p^2), so every product is < 2p.  (Measured: an instantiation without the
// identity test of q was 15-25 % SLOWER -- worse schedule -- so the test stays.)
template <class F>
HALO_DEV XYZZ<F> xyzz_madd_acc(const XYZZ<F>& p, const Affine<F>& q, uint32_t negmask) {
    if (aff_is_id(q)) return p;
    if (xyzz_is_id(p)) {
        XYZZ<F> r = xyzz_from_aff(q);
        if (negmask) r.Y = fe_neg(q.y);
        return r;
    }
    const Fe<F> U2 = fe_mul(q.x, p.ZZ);
    const Fe<F> S2 = fe_mul(q.y, p.ZZZ);
    const Fe<F> P = fe_sub_k<8>(U2, p.X);              // < 10p
    const Fe<F> R = fe_sub_k_sgn<4>(S2, p.Y, negmask);  // < 6p
    // no branch until the end: independent products stay in one basic block, where the scheduler
    // interleaves their dependent multiply-add chains (PP | R^2, then ZZ3 | PPP | Q, then Y3 | ZZZ3)
    const Fe<F> PP = fe_sqr(P);
    const Fe<F> R2 = fe_sqr(R);
    const Fe<F> ZZ3 = fe_mul(p.ZZ, PP);
    const Fe<F> PPP = fe_mul(P, PP);
    const Fe<F> Q = fe_mul(p.X, PP);
    XYZZ<F> r;
    r.X = fe_sub_k<6>(R2, fe_add_nc(PPP, fe_add_nc(Q, Q)));  // < 8p
    const Fe<F> T = fe_sub_k<8>(Q, r.X);                       // < 10p
    r.Y = fe_mul2(R, T, PPP, fe_sub_k<2>(fe_zero<F>(), p.Y));
    r.ZZ = ZZ3;
    r.ZZZ = fe_mul(p.ZZZ, PPP);
    if (fe_is_zero(ZZ3)) {  // U2 == X1: q = +-p (ZZ1 != 0), off the common path
        if (fe_is_zero(fe_reduce_8p(R))) {
            Affine<F> qs = q;
            if (negmask) qs.y = fe_neg(q.y);
            return xyzz_mdbl(qs);
        }
        return xyzz_id<F>();
    }
    return r;
}

// xyzz_madd_acc for k_acc's running bucket sums, with fewer identity tests per addition: the caller
// tracks whether the accumulator is the identity (`fresh`) instead of testing ZZ, the base point's
// identity test runs only when the bases may hold one (check_q), and the exceptional case q = +-acc
// (P = U2 - X1 = 0 mod p) is screened by P's low limb: P < 10p with normalized limbs is a multiple of
// p only if that limb is < 10 (p = 1 mod 2^29), so the full ZZ3 test runs (almost) never.  Same
// formula and results as xyzz_madd_acc.
template <class F>
HALO_DEV XYZZ<F> xyzz_madd_run(const XYZZ<F>& p, bool& fresh, const Affine<F>& q, uint32_t negmask, bool check_q) {
    if (check_q && aff_is_id(q)) return p;
    if (fresh) {
        fresh = false;
        XYZZ<F> r;
        r.X = q.x;
        r.Y = negmask ? fe_neg(q.y) : q.y;
        r.ZZ = fe_one<F>();
        r.ZZZ = fe_one<F>();
        return r;
    }
    const Fe<F> U2 = fe_mul(q.x, p.ZZ);
    const Fe<F> S2 = fe_mul(q.y, p.ZZZ);
    const Fe<F> P = fe_sub_k<8>(U2, p.X);              // < 10p
    const Fe<F> R = fe_sub_k_sgn<4>(S2, p.Y, negmask);  // < 6p
    const Fe<F> PP = fe_sqr(P);
    const Fe<F> R2 = fe_sqr(R);
    const Fe<F> ZZ3 = fe_mul(p.ZZ, PP);
    const Fe<F> PPP = fe_mul(P, PP);
    const Fe<F> Q = fe_mul(p.X, PP);
    XYZZ<F> r;
    r.X = fe_sub_k<6>(R2, fe_add_nc(PPP, fe_add_nc(Q, Q)));  // < 8p
    const Fe<F> T = fe_sub_k<8>(Q, r.X);                       // < 10p
    r.Y = fe_mul2(R, T, PPP, fe_sub_k<2>(fe_zero<F>(), p.Y));
    r.ZZ = ZZ3;
    r.ZZZ = fe_mul(p.ZZZ, PPP);
    if (P.v[0] < 10u && fe_is_zero(ZZ3)) {  // U2 == X1: q = +-p, off the common path
        if (fe_is_zero(fe_reduce_8p(R))) {
            Affine<F> qs = q;
            if (negmask) qs.y = fe_neg(q.y);
            return xyzz_mdbl(qs);
        }
        fresh = true;
        return xyzz_id<F>();
    }
    return r;
}

// X of an xyzz_madd_acc accumulator back below 2p (storage needs < 2^256; the general formulas < 2p)
template <class F>
HALO_DEV XYZZ<F> xyzz_settle(const XYZZ<F>& p) {
    XYZZ<F> r = p;
    r.X = fe_reduce_8p(p.X);
    return r;
}

// General addition (add-2008-s), handles identity and the doubling / inverse cases.
template <class F>
HALO_DEV XYZZ<F> xyzz_add(const XYZZ<F>& p, const XYZZ<F>& q) {
    if (xyzz_is_id(q)) return p;
    if (xyzz_is_id(p)) return q;
    const Fe<F> U1 = fe_mul(p.X, q.ZZ);
    const Fe<F> U2 = fe_mul(q.X, p.ZZ);
    const Fe<F> S1 = fe_mul(p.Y, q.ZZZ);
    const Fe<F> S2 = fe_mul(q.Y, p.ZZZ);
    const Fe<F> P = fe_sub_k<2>(U2, U1);
    const Fe<F> R = fe_sub_k<2>(S2, S1);
    const Fe<F> PP = fe_sqr(P);
    const Fe<F> ZZ3 = fe_mul(fe_mul(p.ZZ, q.ZZ), PP);
    if (fe_is_zero(ZZ3)) {
        if (fe_is_zero_4p(R)) return xyzz_dbl(p);
        return xyzz_id<F>();
    }
    const Fe<F> PPP = fe_mul(P, PP);
    const Fe<F> Q = fe_mul(U1, PP);
    XYZZ<F> r;
    r.X = fe_reduce_8p(fe_sub_k<6>(fe_sqr(R), fe_add_nc(PPP, fe_add_nc(Q, Q))));
    r.Y = fe_sub(fe_mul(R, fe_sub_k<2>(Q, r.X)), fe_mul(S1, PPP));
    r.ZZ = ZZ3;
    r.ZZZ = fe_mul(fe_mul(p.ZZZ, q.ZZZ), PPP);
    return r;
}

template <class F>
HALO_DEV XYZZ<F> xyzz_neg(const XYZZ<F>& p) {
    XYZZ<F> r = p;
    r.Y = fe_neg(p.Y);
    return r;
}

// XYZZ -> affine (one inversion); identity -> (0, 0)
template <class F>
HALO_DEV Affine<F> xyzz_to_aff(const XYZZ<F>& p) {
    Affine<F> r;
    if (xyzz_is_id(p)) {
        r.x = fe_zero<F>();
        r.y = fe_zero<F>();
        return r;
    }
    const Fe<F> t = fe_inv(fe_mul(p.ZZ, p.ZZZ));  // 1 / (ZZ * ZZZ)
    r.x = fe_mul(p.X, fe_mul(t, p.ZZZ));          // X / ZZ
    r.y = fe_mul(p.Y, fe_mul(t, p.ZZ));           // Y / ZZZ
    return r;
}

// ---------------------------------------------------------------------------------------------
// Storage: packed points.  Affine internal = 2 x 32 B (x, y); XYZZ internal = 4 x 32 B.
// ---------------------------------------------------------------------------------------------
template <class F>
HALO_DEV Affine<F> aff_load(const uint4* p) {
    Affine<F> a;
    a.x = fe_load<F>(p);
    a.y = fe_load<F>(p + 2);
    return a;
}
template <class F>
HALO_DEV void aff_store(uint4* p, const Affine<F>& a) {
    fe_store(p, a.x);
    fe_store(p + 2, a.y);
}
template <class F>
HALO_DEV XYZZ<F> xyzz_load(const uint4* p) {
    XYZZ<F> a;
    a.X = fe_load<F>(p);
    a.Y = fe_load<F>(p + 2);
    a.ZZ = fe_load<F>(p + 4);
    a.ZZZ = fe_load<F>(p + 6);
    return a;
}
template <class F>
HALO_DEV void xyzz_store(uint4* p, const XYZZ<F>& a) {
    fe_store(p, a.X);
    fe_store(p + 2, a.Y);
    fe_store(p + 4, a.ZZ);
    fe_store(p + 6, a.ZZZ);
}

// Chunk partials (k_acc -> k_group_sums -> k_merge): XYZZ as 4 x 9 raw limbs, 36 dwords = 9 uint4
// (144 B), with X as k_acc's running sum leaves it (normalized limbs, < 8p).  k_acc then stores
// without settling X or packing limbs; its bucket-boundary stores are divergent (at 2^20 about a
// quarter of its steps have a lane at a boundary), so they cost the whole wave.  The loader settles X.
constexpr int PARTIAL_U4 = 9;
template <class F>
HALO_DEV void partial_store(uint4* p, const XYZZ<F>& a) {
    const Fe<F>* c[4] = {&a.X, &a.Y, &a.ZZ, &a.ZZZ};
    uint32_t w[4 * NLIMB];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int i = 0; i < NLIMB; i++) w[k * NLIMB + i] = c[k]->v[i];
#pragma unroll
    for (int q = 0; q < PARTIAL_U4; q++) p[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
template <class F>
HALO_DEV XYZZ<F> partial_load(const uint4* p) {
    uint32_t w[4 * NLIMB];
#pragma unroll
    for (int q = 0; q < PARTIAL_U4; q++) {
        const uint4 v = p[q];
        w[4 * q] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
    XYZZ<F> a;
    Fe<F>* c[4] = {&a.X, &a.Y, &a.ZZ, &a.ZZZ};
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int i = 0; i < NLIMB; i++) c[k]->v[i] = w[k * NLIMB + i];
    a.X = fe_reduce_8p(a.X);
    return a;
}

// WrappedPoint (ark Montgomery x, y; (0,0) = identity) -> internal affine
template <class F>
HALO_DEV Affine<F> aff_from_wrapped(const uint4* p) {
    Affine<F> a;
    a.x = fe_from_ark<F>(p);
    a.y = fe_from_ark<F>(p + 2);
    return a;
}
template <class F>
HALO_DEV void aff_to_wrapped(uint4* p, const Affine<F>& a) {
    fe_to_ark(p, a.x);
    fe_to_ark(p + 2, a.y);
}

// Jacobian (x = X/Z^2, y = Y/Z^3): used for long doubling chains (Horner), where dbl-2009-l
// (1M + 5S) is ~30 % cheaper than the XYZZ doubling (6M + 3S).
template <class F>
struct Jac {
    Fe<F> X, Y, Z;
};

// XYZZ -> Jacobian without inversion: Z = ZZZ, X = X ZZ^2, Y = Y ZZZ^2 (uses ZZ^3 = ZZZ^2)
template <class F>
HALO_DEV Jac<F> jac_from_xyzz(const XYZZ<F>& p) {
    Jac<F> r;
    if (xyzz_is_id(p)) {
        r.X = fe_one<F>();
        r.Y = fe_one<F>();
        r.Z = fe_zero<F>();
        return r;
    }
    r.X = fe_mul(p.X, fe_sqr(p.ZZ));
    r.Y = fe_mul(p.Y, fe_sqr(p.ZZZ));
    r.Z = p.ZZZ;
    return r;
}

template <class F>
HALO_DEV XYZZ<F> jac_to_xyzz(const Jac<F>& j) {
    XYZZ<F> r;
    r.X = j.X;
    r.Y = j.Y;
    r.ZZ = fe_sqr(j.Z);
    r.ZZZ = fe_mul(r.ZZ, j.Z);
    return r;
}

// dbl-2009-l (a = 0): A = X^2, B = Y^2, C = B^2, D = 2((X + B)^2 - A - C), E = 3A, F = E^2,
// X3 = F - 2D, Y3 = E (D - X3) - 8C, Z3 = 2 Y Z.  The identity (Z = 0) maps to itself.
template <class F>
HALO_DEV Jac<F> jac_dbl(const Jac<F>& p) {
    const Fe<F> A = fe_sqr(p.X);
    const Fe<F> B = fe_sqr(p.Y);
    const Fe<F> C = fe_sqr(B);
    const Fe<F> D = fe_dbl(fe_sub(fe_sub(fe_sqr(fe_add(p.X, B)), A), C));
    const Fe<F> E = fe_add(A, fe_dbl(A));
    const Fe<F> Fv = fe_sqr(E);
    Jac<F> r;
    r.X = fe_sub(Fv, fe_dbl(D));
    const Fe<F> C8 = fe_dbl(fe_dbl(fe_dbl(C)));
    r.Y = fe_sub(fe_mul(E, fe_sub(D, r.X)), C8);
    r.Z = fe_dbl(fe_mul(p.Y, p.Z));
    return r;
}

// Variable-base scalar multiplication k * P (k canonical, 8 x u32 words), left-to-right binary.
template <class F>
HALO_DEV XYZZ<F> xyzz_scalar_mul(const Affine<F>& P, const uint32_t (&k)[8]) {
    XYZZ<F> acc = xyzz_id<F>();
    for (int i = 255; i >= 0; i--) {
        acc = xyzz_dbl(acc);
        if ((k[i >> 5] >> (i & 31)) & 1u) acc = xyzz_madd(acc, P);
    }
    return acc;
}

HALO_ARITH_END  // namespace halo
