// Tree sums of XYZZ points across the lanes of a block (the MSM reduction tail, msm_tail.hip, and
// the IPA's tail rounds, ipa.hip), in the arithmetic namespace of the including unit (fields.hpp).
#pragma once
#include "curve.hpp"

HALO_ARITH_BEGIN

// ---------------------------------------------------------------------------------------------
// Tree sums of XYZZ points across lanes.  Inside a wave the partner's point comes over the lane
// crossbar (__shfl_xor: 36 dwords, no LDS round trip, no barrier), so each level costs one addition;
// only the wave sums of a group wider than a wave meet in LDS.  Every lane of the wave must call
// these (idle lanes pass the identity).
// ---------------------------------------------------------------------------------------------
template <class F>
HALO_DEV XYZZ<F> xyzz_shfl_xor(const XYZZ<F>& p, int m) {
    XYZZ<F> r;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) {
        r.X.v[l] = __shfl_xor(p.X.v[l], m);
        r.Y.v[l] = __shfl_xor(p.Y.v[l], m);
        r.ZZ.v[l] = __shfl_xor(p.ZZ.v[l], m);
        r.ZZZ.v[l] = __shfl_xor(p.ZZZ.v[l], m);
    }
    return r;
}

// ---------------------------------------------------------------------------------------------
// Quad-cooperative additions.  A tree level inside one wave is issue-bound, not latency-bound: the
// wave's SIMD spends the same cycles on an addition whether 32 lanes or 1 lane need it, and a level
// with one addition per lane costs the full 12M + 2S of xyzz_add.  Here four lanes (a quad) share
// one addition: its multiplications form four dependent rounds (U1 U2 S1 S2 | PP RR ZZ1ZZ2 ZZZ1ZZZ2 |
// ZZ3 PPP Q | Y3a Y3b ZZZ3), each lane computes one product per round (operands picked by its role)
// and the quad exchanges the products with DPP quad broadcasts, so a level costs four multiplication
// issues per 16 additions instead of fourteen.  Same formula and operations as xyzz_add (curve.hpp),
// so the results are bit-identical; the exceptional case (P == +-Q) falls back to xyzz_dbl / the
// identity, wave-uniformly skipped when no lane hits it.
// ---------------------------------------------------------------------------------------------
// v_mov_b32 with a DPP quad permutation: lane i of each quad reads lane (CTRL >> 2 i) & 3
template <int CTRL, class F>
HALO_DEV Fe<F> qperm(const Fe<F>& a) {
    Fe<F> r;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) r.v[l] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[l], CTRL, 0xF, 0xF, false);
    return r;
}
constexpr int qp(int l0, int l1, int l2, int l3) { return l0 | (l1 << 2) | (l2 << 4) | (l3 << 6); }
// branch-free per-lane pick: m all ones -> a, zero -> b (v_bfi_b32)
template <class F>
HALO_DEV Fe<F> pick(uint32_t m, const Fe<F>& a, const Fe<F>& b) {
    Fe<F> r;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) r.v[l] = (a.v[l] & m) | (b.v[l] & ~m);
    return r;
}
template <class F>
HALO_DEV XYZZ<F> xyzz_shfl(const XYZZ<F>& p, int src) {
    XYZZ<F> r;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) {
        r.X.v[l] = __shfl(p.X.v[l], src);
        r.Y.v[l] = __shfl(p.Y.v[l], src);
        r.ZZ.v[l] = __shfl(p.ZZ.v[l], src);
        r.ZZZ.v[l] = __shfl(p.ZZZ.v[l], src);
    }
    return r;
}
// p + q (the points of lanes s1 and s2 of v) by the quad: role = lane & 3 computes one product per
// round and the quad trades products by DPP quad permutations:
//   round 1  U1 = X1 ZZ2 | U2 = X2 ZZ1 | S1 = Y1 ZZZ2 | S2 = Y2 ZZZ1    (operands fetched by lane)
//            pairs swap: lanes 0, 1 form P = U2 - U1, lanes 2, 3 R = S2 - S1
//   round 2  PP = P P | A = ZZ1 ZZ2 | RR = R R | B = ZZZ1 ZZZ2          (ZZ / ZZZ from the pair swap)
//   round 3  Q = U1 PP | PPP = P PP | ZZ3 = A PP | -
//   round 4  - | ZZZ3 = B PPP | Y3a = R (Q - X3) | Y3b = S1 PPP         (X3 = RR - PPP - 2 Q)
// The sum is assembled in the quad's lane 2.  Trivial additions (an identity operand, idp / idq) are
// left to the caller, which takes the other operand instead.
template <class F>
HALO_DEV XYZZ<F> xyzz_add_quad(const XYZZ<F>& v, uint32_t s1, uint32_t s2, bool idp, bool idq) {
    const uint32_t role = threadIdx.x & 3u;
    const uint32_t odd = (role & 1u) ? ~0u : 0u, lo = role < 2 ? ~0u : 0u, r2 = role == 2 ? ~0u : 0u;
    const uint32_t sa = (role & 1u) ? s2 : s1, sb = (role & 1u) ? s1 : s2;
    Fe<F> a, b;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) {  // role 0: p.X q.ZZ, 1: q.X p.ZZ, 2: p.Y q.ZZZ, 3: q.Y p.ZZZ
        const uint32_t x = __shfl(v.X.v[l], (int)sa), y = __shfl(v.Y.v[l], (int)sa);
        const uint32_t zz = __shfl(v.ZZ.v[l], (int)sb), zzz = __shfl(v.ZZZ.v[l], (int)sb);
        a.v[l] = (x & lo) | (y & ~lo);
        b.v[l] = (zz & lo) | (zzz & ~lo);
    }
    const Fe<F> t1 = fe_mul(a, b);
    constexpr int SWAP = qp(1, 0, 3, 2);
    const Fe<F> t1s = qperm<SWAP>(t1), bs = qperm<SWAP>(b);
    const Fe<F> d = fe_sub_k<2>(pick(odd, t1, t1s), pick(odd, t1s, t1));  // P (lanes 0, 1), R (2, 3)
    const Fe<F> t2 = fe_mul(pick(odd, b, d), pick(odd, bs, d));
    const Fe<F> PPb = qperm<qp(0, 0, 0, 0)>(t2), Ab = qperm<qp(0, 1, 1, 3)>(t2);
    const Fe<F> t3 = fe_mul(pick(lo, pick(odd, d, t1), Ab), PPb);
    const Fe<F> Bb = qperm<qp(0, 3, 2, 3)>(t2), Qb = qperm<qp(0, 1, 0, 3)>(t3), PPPb = qperm<qp(1, 1, 1, 1)>(t3);
    XYZZ<F> r;
    r.X = fe_reduce_8p(fe_sub_k<6>(t2, fe_add_nc(PPPb, fe_add_nc(Qb, Qb))));  // (lane 2: t2 = RR)
    const Fe<F> t4 = fe_mul(pick(lo, Bb, pick(odd, t1s, d)), pick(r2, fe_sub_k<2>(Qb, r.X), PPPb));
    r.Y = fe_sub(t4, qperm<qp(0, 1, 3, 3)>(t4));
    r.ZZ = t3;
    r.ZZZ = qperm<qp(0, 1, 1, 3)>(t4);
    const bool exc = role == 2 && !idp && !idq && fe_is_zero(t3);
    if (__any(exc)) {  // P == +-Q: doubling or the identity (rare)
        const XYZZ<F> p = xyzz_shfl(v, (int)s1);
        if (exc) r = fe_is_zero_4p(d) ? xyzz_dbl(p) : xyzz_id<F>();
    }
    return r;
}
// 2p by the quad (every lane of an aligned quad holds p; every lane gets 2p): xyzz_dbl's nine products
// in three dependent rounds (V = U^2, X^2 | W = U V, S = X V, M^2, ZZ V | M (S - X3), W Y, W ZZZ),
// one product per lane per round, exchanged by DPP quad broadcasts.  The identity doubles to a point
// with ZZ = 0, i.e. the identity again.
template <class F>
HALO_DEV XYZZ<F> xyzz_dbl_quad(const XYZZ<F>& p) {
    const uint32_t role = threadIdx.x & 3u;
    const uint32_t odd = (role & 1u) ? ~0u : 0u, lo = role < 2 ? ~0u : 0u, r0 = role == 0 ? ~0u : 0u;
    const Fe<F> U = fe_norm(fe_add_nc(p.Y, p.Y));  // normalized: squared below (fields.hpp bounds)
    const Fe<F> t1 = fe_sqr(pick(odd, p.X, U));  // lanes 0, 2: V = U^2; 1, 3: X^2
    const Fe<F> V = qperm<qp(0, 0, 0, 0)>(t1), X2 = qperm<qp(1, 1, 1, 1)>(t1);
    const Fe<F> M = fe_norm(fe_add_nc(X2, fe_add_nc(X2, X2)));  // < 6p
    // lane 0: W = U V; 1: S = X V; 2: M^2; 3: ZZ3 = V ZZ
    const Fe<F> t2 = fe_mul(pick(lo, pick(odd, p.X, U), pick(odd, V, M)), pick(lo, V, pick(odd, p.ZZ, M)));
    const Fe<F> W = qperm<qp(0, 0, 0, 0)>(t2), S = qperm<qp(1, 1, 1, 1)>(t2), MM = qperm<qp(2, 2, 2, 2)>(t2);
    XYZZ<F> r;
    r.ZZ = qperm<qp(3, 3, 3, 3)>(t2);
    r.X = fe_reduce_8p(fe_sub_k<4>(MM, fe_add_nc(S, S)));
    // lane 0: M (S - X3); 1: W Y; 2 (and 3): ZZZ3 = W ZZZ
    const Fe<F> t3 = fe_mul(pick(r0, M, W), pick(r0, fe_sub_k<2>(S, r.X), pick(odd, p.Y, p.ZZZ)));
    r.Y = fe_sub(qperm<qp(0, 0, 0, 0)>(t3), qperm<qp(1, 1, 1, 1)>(t3));
    r.ZZZ = qperm<qp(2, 2, 2, 2)>(t3);
    return r;
}
// p + q as xyzz_add_quad, valid in the quad's lane 2 only, for the tree levels below:
//  * an identity operand (idp / idq, quad-uniform) yields the other operand, reassembled in lane 2 by
//    DPP quad broadcasts from the coordinates the quad fetched anyway (role 0: p.X, q.ZZ; 1: q.X, p.ZZ;
//    2: p.Y, q.ZZZ; 3: q.Y, p.ZZZ) -- no lane gathers, so a level can leave its sums in place; two
//    identities give q, the identity;
//  * lazy coordinates: X3 = RR - PPP - 2Q + 6p stays in (0, 8p) and Y3 in (0, 4p) (normalized limbs,
//    valid multiplication operands: the products here stay below 40 p^2 < p 2^261), so the two
//    conditional-subtraction chains per addition go; wave_group_sum reduces its result once.
// Operands may be lazy the same way (the previous level's sums).
// live: the quad's addition exists (a tree level's last batch may have idle quads; their r is left
// undefined, and they neither force the multiplications nor the identity path).
template <class F>
HALO_DEV XYZZ<F> xyzz_add_quad_lane2(const XYZZ<F>& v, uint32_t s1, uint32_t s2, bool idp, bool idq, bool live) {
    const uint32_t role = threadIdx.x & 3u;
    const uint32_t odd = (role & 1u) ? ~0u : 0u, lo = role < 2 ? ~0u : 0u, r2 = role == 2 ? ~0u : 0u;
    const uint32_t sa = (role & 1u) ? s2 : s1, sb = (role & 1u) ? s1 : s2;
    Fe<F> a, b;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) {
        const uint32_t x = __shfl(v.X.v[l], (int)sa), y = __shfl(v.Y.v[l], (int)sa);
        const uint32_t zz = __shfl(v.ZZ.v[l], (int)sb), zzz = __shfl(v.ZZZ.v[l], (int)sb);
        a.v[l] = (x & lo) | (y & ~lo);
        b.v[l] = (zz & lo) | (zzz & ~lo);
    }
    XYZZ<F> r;
    if (!__all(!live || idp || idq)) {
        const Fe<F> t1 = fe_mul(a, b);
        constexpr int SWAP = qp(1, 0, 3, 2);
        const Fe<F> t1s = qperm<SWAP>(t1), bs = qperm<SWAP>(b);
        const Fe<F> d = fe_sub_k<2>(pick(odd, t1, t1s), pick(odd, t1s, t1));
        const Fe<F> t2 = fe_mul(pick(odd, b, d), pick(odd, bs, d));
        const Fe<F> PPb = qperm<qp(0, 0, 0, 0)>(t2), Ab = qperm<qp(0, 1, 1, 3)>(t2);
        const Fe<F> t3 = fe_mul(pick(lo, pick(odd, d, t1), Ab), PPb);
        const Fe<F> Bb = qperm<qp(0, 3, 2, 3)>(t2), Qb = qperm<qp(0, 1, 0, 3)>(t3), PPPb = qperm<qp(1, 1, 1, 1)>(t3);
        r.X = fe_sub_k<6>(t2, fe_add_nc(PPPb, fe_add_nc(Qb, Qb)));  // (lane 2: t2 = RR) in (0, 8p)
        const Fe<F> t4 = fe_mul(pick(lo, Bb, pick(odd, t1s, d)), pick(r2, fe_sub_k<8>(Qb, r.X), PPPb));
        r.Y = fe_sub_k<2>(t4, qperm<qp(0, 1, 3, 3)>(t4));  // in (0, 4p)
        r.ZZ = t3;
        r.ZZZ = qperm<qp(0, 1, 1, 3)>(t4);
        const bool exc = live && role == 2 && !idp && !idq && fe_is_zero(t3);
        if (__any(exc)) {  // P == +-Q: doubling or the identity (rare)
            XYZZ<F> p;
            p.X = qperm<qp(0, 0, 0, 0)>(a);
            p.Y = qperm<qp(2, 2, 2, 2)>(a);
            p.ZZ = qperm<qp(1, 1, 1, 1)>(b);
            p.ZZZ = qperm<qp(3, 3, 3, 3)>(b);
            if (exc) r = fe_is_zero_4p(d) ? xyzz_dbl(p) : xyzz_id<F>();
        }
    }
    if (__any(live && (idp || idq))) {  // an identity operand: the other one (wave-uniform branch: every lane
                              // takes part in the broadcasts, the choice is a per-lane pick)
        const uint32_t mq = idp ? ~0u : 0u;
        XYZZ<F> o;
        o.X = pick(mq, qperm<qp(1, 1, 1, 1)>(a), qperm<qp(0, 0, 0, 0)>(a));
        o.Y = pick(mq, qperm<qp(3, 3, 3, 3)>(a), qperm<qp(2, 2, 2, 2)>(a));
        o.ZZ = pick(mq, qperm<qp(0, 0, 0, 0)>(b), qperm<qp(1, 1, 1, 1)>(b));
        o.ZZZ = pick(mq, qperm<qp(2, 2, 2, 2)>(b), qperm<qp(3, 3, 3, 3)>(b));
        if (idp || idq) r = o;
    }
    return r;
}

// sum over aligned groups of G lanes (G a power of two <= 64), valid in the group's first lane.  The
// points form a flat list (group g's elements [g G, g G + G)); a level turns the list of groups of
// size gs into one of size gs / 2 by 64 / G * gs / 2 quad additions (16 per batch, at most two
// batches), and each sum stays where its quad formed it: element a of the new list at lane
// 4 (a mod 16) + 2 (batch 0) or 4 (a mod 16) (batch 1, moved inside the quad by a DPP broadcast).
// The next level gathers its operands from there, so no level moves its sums across lanes.
template <class F>
HALO_DEV XYZZ<F> wave_group_sum(XYZZ<F> v, uint32_t G) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t r0m = (lane & 3u) == 0u ? ~0u : 0u;
    bool placed = false;  // false: element e at lane e
    auto where = [&](uint32_t e) { return placed ? ((4u * (e & 15u) + (e < 16u ? 2u : 0u)) & 63u) : (e & 63u); };
    for (uint32_t gs = G; gs > 1; gs >>= 1) {
        const uint32_t m = gs >> 1, nadd = (64u / G) * m;  // 64 / G groups x m additions
        const uint32_t idv = xyzz_is_id(v) ? 1u : 0u;
        XYZZ<F> nxt;
        for (uint32_t b = 0; b * 16 < nadd; b++) {
            const uint32_t a = b * 16 + (lane >> 2);
            const uint32_t e1 = (a / m) * gs + a % m, e2 = e1 + m;
            const uint32_t s1 = where(e1), s2 = where(e2);
            const uint32_t fp = __shfl(idv, (int)s1), fq = __shfl(idv, (int)s2);
            const XYZZ<F> r = xyzz_add_quad_lane2(v, s1, s2, fp != 0u, fq != 0u, a < nadd);
            if (b == 0) {
                nxt = r;
            } else {  // batch 1's sums to lane 0 of their quads
                nxt.X = pick(r0m, qperm<qp(2, 2, 2, 2)>(r.X), nxt.X);
                nxt.Y = pick(r0m, qperm<qp(2, 2, 2, 2)>(r.Y), nxt.Y);
                nxt.ZZ = pick(r0m, qperm<qp(2, 2, 2, 2)>(r.ZZ), nxt.ZZ);
                nxt.ZZZ = pick(r0m, qperm<qp(2, 2, 2, 2)>(r.ZZZ), nxt.ZZZ);
            }
        }
        v = nxt;
        placed = true;
    }
    if (!placed) return v;
    v.X = fe_reduce_8p(v.X);  // the lazy coordinates of xyzz_add_quad_lane2, reduced once
    v.Y = fe_reduce_2p(v.Y);
    if (G == 64) {  // element 0 (lane 2) to its quad
        XYZZ<F> r;
        r.X = qperm<qp(2, 2, 2, 2)>(v.X);
        r.Y = qperm<qp(2, 2, 2, 2)>(v.Y);
        r.ZZ = qperm<qp(2, 2, 2, 2)>(v.ZZ);
        r.ZZZ = qperm<qp(2, 2, 2, 2)>(v.ZZZ);
        return r;
    }
    // group g's sum is element g; every lane of the group gets it
    return xyzz_shfl(v, (int)where(lane / G));
}

// sum over aligned groups of G threads (G a power of two <= blockDim): valid in the group's first
// thread.  Every wave sums its lanes (G <= 64: its groups) cooperatively; for G > 64 the first wave
// of the block sums the waves' sums of every group and hands each group's sum back to its first
// thread through LDS.  red: LDS scratch for blockDim / 64 points (>= 1).  Every thread of the block must
// call it.
template <class F>
HALO_DEV XYZZ<F> block_group_sum(XYZZ<F> v, uint32_t G, uint4* red) {
    if (G <= 64) return wave_group_sum<F>(v, G);
    v = wave_group_sum<F>(v, 64u);
    const uint32_t wv = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = threadIdx.x & 63u;
    if (lane == 0) xyzz_store(red + 8 * wv, v);
    __syncthreads();
    XYZZ<F> w = xyzz_id<F>();
    if (wv == 0 && lane < nw) w = xyzz_load<F>(red + 8 * lane);
    __syncthreads();
    if (wv == 0) {  // (wave-uniform)
        w = wave_group_sum<F>(w, G >> 6);
        if (lane < nw && (lane & ((G >> 6) - 1)) == 0) xyzz_store(red + 8 * (lane / (G >> 6)), w);
    }
    __syncthreads();
    const uint32_t gpos = threadIdx.x & (G - 1);
    if (gpos == 0) v = xyzz_load<F>(red + 8 * (threadIdx.x / G));
    return v;
}

HALO_ARITH_END
