// Device field arithmetic for the Pasta fields on gfx950 (CDNA4).
//
// Replaces the arkworks 0.5.0 `Fp256` Montgomery arithmetic behind `halo_group::{Fp, Fq}`
// (reference: crates/group/src/lib.rs:8-9; used on the hot path in crates/group/src/group.rs:43-66,
// crates/accumulation/src/pcdl.rs:404-438 and inside every MSM / NTT).
//
// Representation (MI355X-first, see DESIGN.md "Field representation"):
//   * 9 limbs of 29 bits held in 32-bit VGPRs (radix 2^29, 261 bits of headroom over the 255-bit
//     moduli), Montgomery form with R' = 2^261, values weakly reduced to [0, 2p).
//   * Multiplication is product-scanning (FIPS) Montgomery: every partial product is a single
//     `v_mad_u64_u32` accumulating straight into a 64-bit column accumulator.  29-bit limbs leave
//     6 bits of headroom, so a whole column (<= 9 products + <= 5 reduction products + carry) never
//     overflows and no add-with-carry chains are needed.  Measured on MI355X this is 1.9x faster
//     than 32-bit CIOS (tools/micro/modmul_bench.hip), because `v_mad_u64_u32` issues at the same
//     rate as a 64-bit add while carry-propagating adds cost as much as a mad.
//   * Both Pasta moduli are 2^254 + c with c < 2^126 and p = 1 mod 2^32, so -p^-1 = -1 mod 2^29 and
//     the 29-bit limbs of p are nonzero only at indices 0..4 and 8: Montgomery reduction needs 5
//     mads per limb and the per-limb quotient is just (-acc) & mask.
//   * Storage format for device-internal buffers: the internal value packed into 8 x u32 (it is
//     < 2p < 2^256).  ABI buffers use ark's format (4 x u64, Montgomery R = 2^256, canonical); the
//     conversion is one Montgomery multiplication by a constant (ARK2INT / INT2ARK).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "consts.hpp"

// Default build: every column of a product is ONE inline-asm v_mad_u64_u32 chain (mad_chain.hpp,
// HALO_MAD_COL).  HALO_MAD_ILP (latency-bound tail kernels) and HALO_MAD_C: the plain C expression,
// which the compiler splits into parallel partial sums.
#if !defined(HALO_MAD_ILP) && !defined(HALO_MAD_C) && !defined(HALO_MAD_PER_PRODUCT)
#define HALO_MAD_COL 1
#include "mad_chain.hpp"
#endif

// Arithmetic namespace: translation units compiled with HALO_MAD_ILP (latency-bound kernels, see
// msm_tail.hip) get the same code in the inline namespace halo::ilp with split column sums.
#ifdef HALO_MAD_ILP
#define HALO_ARITH_BEGIN namespace halo { inline namespace ilp {
#define HALO_ARITH_END } }
#else
#define HALO_ARITH_BEGIN namespace halo {
#define HALO_ARITH_END }
#endif

#define HALO_DEV __device__ __forceinline__

HALO_ARITH_BEGIN

// Column accumulation acc + a * b as ONE v_mad_u64_u32 per product.  Written as inline asm so that
// the compiler keeps each column as a single dependent chain instead of splitting it into partial
// sums joined by 64-bit adds (it does that to shorten the critical path): at >= 2 waves per SIMD the
// chain form issues ~12% fewer VALU instructions per multiplication and is ~10% faster
// (tools/micro/fe_mul_bench.hip); latency-bound single-wave code loses a little.
HALO_DEV uint64_t mad_acc(uint32_t a, uint32_t b, uint64_t c) {
#if defined(HALO_MAD_ILP) || defined(HALO_MAD_C)
    return (uint64_t)a * b + c;
#else
    uint64_t d, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cc) : "v"(a), "v"(b), "v"(c));
    return d;
#endif
}
// acc + a * K for a compile-time constant K (SGPR operand)
template <uint32_t K>
HALO_DEV uint64_t mad_acc_k(uint32_t a, uint64_t c) {
#if defined(HALO_MAD_ILP) || defined(HALO_MAD_C)
    return (uint64_t)a * K + c;
#else
    uint64_t d, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cc) : "v"(a), "s"(K), "v"(c));
    return d;
#endif
}

template <class C>
struct Fe {
    uint32_t v[NLIMB];
};

template <class C>
HALO_DEV Fe<C> fe_from_const(const uint32_t (&k)[NLIMB]) {
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = k[i];
    return r;
}

template <class C>
HALO_DEV Fe<C> fe_zero() {
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = 0;
    return r;
}

template <class C>
HALO_DEV Fe<C> fe_one() {
    return fe_from_const<C>(C::ONE);
}

// ----------------------------------------------------------------------------------------------
// Packing: 8 x u32 (256-bit little endian) <-> 9 x 29-bit limbs.  Value must be < 2^256.
// ----------------------------------------------------------------------------------------------
template <class C>
HALO_DEV Fe<C> fe_unpack(const uint32_t (&w)[8]) {
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        const int bit = i * LIMB_BITS;
        const int j = bit >> 5, s = bit & 31;
        uint32_t lo = w[j];
        uint32_t hi = (j + 1 < 8) ? w[j + 1] : 0u;
        uint32_t x = (s == 0) ? lo : __builtin_amdgcn_alignbit(hi, lo, s);
        r.v[i] = (i == NLIMB - 1) ? (x & 0xffffffu) : (x & LIMB_MASK);
    }
    return r;
}

template <class C>
HALO_DEV void fe_pack(const Fe<C>& a, uint32_t (&w)[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int bit = j * 32;
        const int i = bit / LIMB_BITS, s = bit % LIMB_BITS;
        uint32_t x = a.v[i] >> s;
        if (i + 1 < NLIMB) x |= a.v[i + 1] << (LIMB_BITS - s);
        if (i + 2 < NLIMB && (LIMB_BITS - s) + LIMB_BITS < 32) x |= a.v[i + 2] << (2 * LIMB_BITS - s);
        w[j] = x;
    }
}

template <class C>
HALO_DEV Fe<C> fe_load(const uint4* p) {
    uint4 a = p[0], b = p[1];
    uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    return fe_unpack<C>(w);
}

template <class C>
HALO_DEV void fe_store(uint4* p, const Fe<C>& x) {
    uint32_t w[8];
    fe_pack(x, w);
    p[0] = make_uint4(w[0], w[1], w[2], w[3]);
    p[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// ----------------------------------------------------------------------------------------------
// Montgomery multiplication (product scanning, R' = 2^261).  Inputs < 8p (normalized limbs),
// output < 2p.
// ----------------------------------------------------------------------------------------------
// Montgomery reduction products of column k: sum_{i<k, 1<=j=k-i<NLIMB} m_i p_j
template <class C, int J>
HALO_DEV uint64_t fe_red_term(const uint32_t (&m)[NLIMB], int k, uint64_t acc) {
    if constexpr (J < NLIMB) {
        if constexpr (C::P[J] != 0) {
            const int i = k - J;
            if (i >= 0 && i < NLIMB) acc = mad_acc_k<C::P[J]>(m[i], acc);
        }
        return fe_red_term<C, J + 1>(m, k, acc);
    } else {
        return acc;
    }
}
template <class C>
HALO_DEV uint64_t fe_reduce_col(const uint32_t (&m)[NLIMB], int k, uint64_t acc) {
    return fe_red_term<C, 1>(m, k, acc);
}

#ifdef HALO_MAD_COL
// ---- column form (HALO_MAD_COL): per column one asm chain of the products, one of the reduction terms
namespace colmul {
// products a_i b_j, i + j = K (or, SQR, the doubled cross products a2_i a_j, i < j, and a_(K/2)^2)
template <int K, bool SQR>
constexpr int n_prod() {
    int c = 0;
    for (int i = 0; i < NLIMB; i++) {
        const int j = K - i;
        if (j < 0 || j >= NLIMB) continue;
        if (!SQR || i < j || i == j) c++;
    }
    return c;
}
template <class C, int K>
constexpr int n_red() {
    int c = 0;
    for (int j = 1; j < NLIMB; j++)
        if (C::P[j] != 0 && K - j >= 0 && K - j < NLIMB) c++;
    return c;
}
// acc (+)= the column-K products of a and b (SQR: a2 = 2a limb-wise, b unused)
template <int K, bool SQR, bool ZERO>
HALO_DEV void prod(uint64_t& acc, const uint32_t (&a)[NLIMB], const uint32_t (&a2)[NLIMB], const uint32_t (&b)[NLIMB]) {
    constexpr int N = n_prod<K, SQR>();
    uint32_t x[N > 0 ? N : 1], y[N > 0 ? N : 1];
    int t = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        const int j = K - i;
        if (j < 0 || j >= NLIMB) continue;
        if (!SQR) {
            x[t] = a[i];
            y[t] = b[j];
            t++;
        } else if (i < j) {
            x[t] = a2[i];
            y[t] = a[j];
            t++;
        } else if (i == j) {
            x[t] = a[i];
            y[t] = a[i];
            t++;
        }
    }
    if constexpr (ZERO)
        MadCol<N>::vv_z(acc, x, y);
    else
        MadCol<N>::vv(acc, x, y);
}
template <class C, int K>
HALO_DEV void red(uint64_t& acc, const uint32_t (&m)[NLIMB]) {
    constexpr int R = n_red<C, K>();
    uint32_t x[R > 0 ? R : 1], y[R > 0 ? R : 1];
    int t = 0;
#pragma unroll
    for (int j = 1; j < NLIMB; j++)
        if (C::P[j] != 0 && K - j >= 0 && K - j < NLIMB) {
            x[t] = m[K - j];
            y[t] = C::P[j];
            t++;
        }
    MadCol<R>::vs(acc, x, y);
}
template <class C, int K>
HALO_DEV void finish(uint64_t& acc, uint32_t (&m)[NLIMB], uint32_t (&r)[NLIMB]) {
    if constexpr (K < NLIMB) {
        const uint32_t mk = (0u - (uint32_t)acc) & LIMB_MASK;
        m[K] = mk;
        acc += mk;  // p[0] == 1: clears the low 29 bits
        acc >>= LIMB_BITS;
    } else {
        r[K - NLIMB] = (uint32_t)acc & LIMB_MASK;
        acc >>= LIMB_BITS;
    }
}
// one product (SQR: a^2), columns K..2 NLIMB - 2
template <class C, int K, bool SQR>
HALO_DEV void mul_cols(uint64_t& acc, const uint32_t (&a)[NLIMB], const uint32_t (&a2)[NLIMB], const uint32_t (&b)[NLIMB],
                       uint32_t (&m)[NLIMB], uint32_t (&r)[NLIMB]) {
    if constexpr (K < 2 * NLIMB - 1) {
        prod<K, SQR, K == 0>(acc, a, a2, b);
        red<C, K>(acc, m);
        finish<C, K>(acc, m, r);
        mul_cols<C, K + 1, SQR>(acc, a, a2, b, m, r);
    }
}
// a b + c d with one reduction: the two products as two chains per column, joined once per column
template <class C, int K>
HALO_DEV void mul2_cols(uint64_t& acc, const uint32_t (&a)[NLIMB], const uint32_t (&b)[NLIMB], const uint32_t (&c)[NLIMB],
                        const uint32_t (&d)[NLIMB], uint32_t (&m)[NLIMB], uint32_t (&r)[NLIMB]) {
    if constexpr (K < 2 * NLIMB - 1) {
        uint64_t acc2;
        prod<K, false, K == 0>(acc, a, a, b);
        prod<K, false, true>(acc2, c, c, d);
        acc += acc2;
        red<C, K>(acc, m);
        finish<C, K>(acc, m, r);
        mul2_cols<C, K + 1>(acc, a, b, c, d, m, r);
    }
}
// two independent products, their column chains side by side
template <class C, int K>
HALO_DEV void mulx2_cols(uint64_t& acc1, uint64_t& acc2, const uint32_t (&a1)[NLIMB], const uint32_t (&b1)[NLIMB],
                         const uint32_t (&a2)[NLIMB], const uint32_t (&b2)[NLIMB], uint32_t (&m1)[NLIMB],
                         uint32_t (&m2)[NLIMB], uint32_t (&r1)[NLIMB], uint32_t (&r2)[NLIMB]) {
    if constexpr (K < 2 * NLIMB - 1) {
        prod<K, false, K == 0>(acc1, a1, a1, b1);
        prod<K, false, K == 0>(acc2, a2, a2, b2);
        red<C, K>(acc1, m1);
        red<C, K>(acc2, m2);
        finish<C, K>(acc1, m1, r1);
        finish<C, K>(acc2, m2, r2);
        mulx2_cols<C, K + 1>(acc1, acc2, a1, b1, a2, b2, m1, m2, r1, r2);
    }
}
}  // namespace colmul

template <class C>
HALO_DEV Fe<C> fe_mul(const Fe<C>& a, const Fe<C>& b) {
    uint32_t m[NLIMB];
    Fe<C> r;
    uint64_t acc;
    colmul::mul_cols<C, 0, false>(acc, a.v, a.v, b.v, m, r.v);
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}
template <class C>
HALO_DEV Fe<C> fe_mul2(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c, const Fe<C>& d) {
    uint32_t m[NLIMB];
    Fe<C> r;
    uint64_t acc;
    colmul::mul2_cols<C, 0>(acc, a.v, b.v, c.v, d.v, m, r.v);
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}
template <class C>
HALO_DEV void fe_mul_x2(const Fe<C>& a1, const Fe<C>& b1, const Fe<C>& a2, const Fe<C>& b2, Fe<C>& r1, Fe<C>& r2) {
    uint32_t m1[NLIMB], m2[NLIMB];
    uint64_t acc1, acc2;
    colmul::mulx2_cols<C, 0>(acc1, acc2, a1.v, b1.v, a2.v, b2.v, m1, m2, r1.v, r2.v);
    r1.v[NLIMB - 1] = (uint32_t)acc1;
    r2.v[NLIMB - 1] = (uint32_t)acc2;
}
template <class C>
HALO_DEV Fe<C> fe_sqr(const Fe<C>& a) {
    uint32_t m[NLIMB], a2[NLIMB];
#pragma unroll
    for (int i = 0; i < NLIMB; i++) a2[i] = a.v[i] << 1;
    Fe<C> r;
    uint64_t acc;
    colmul::mul_cols<C, 0, true>(acc, a.v, a2, a.v, m, r.v);
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}
#else
template <class C>
HALO_DEV Fe<C> fe_mul(const Fe<C>& a, const Fe<C>& b) {
    uint32_t m[NLIMB];
    Fe<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * NLIMB - 1; k++) {
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (j < 0 || j >= NLIMB) continue;
            acc = mad_acc(a.v[i], b.v[j], acc);
        }
        acc = fe_reduce_col<C>(m, k, acc);
        if (k < NLIMB) {
            const uint32_t mk = (0u - (uint32_t)acc) & LIMB_MASK;
            m[k] = mk;
            acc += mk;  // p[0] == 1: clears the low 29 bits
            acc >>= LIMB_BITS;
        } else {
            r.v[k - NLIMB] = (uint32_t)acc & LIMB_MASK;
            acc >>= LIMB_BITS;
        }
    }
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}

// Product sum a b + c d with ONE Montgomery reduction (81 + 81 + 45 mads instead of 2 x 126 and a
// modular addition).  Every input normalized (limbs < 2^29): a column holds <= 18 products + 5
// reduction products < 2^58, i.e. < 2^62.6.  Output < 2p when a b + c d < p 2^261 (~127 p^2).
template <class C>
HALO_DEV Fe<C> fe_mul2(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c, const Fe<C>& d) {
    uint32_t m[NLIMB];
    Fe<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * NLIMB - 1; k++) {
        // the two products' column sums run as two independent chains, joined once per column
        // (a single 18-deep dependent chain stalls issue: measured 0.61 vs 0.99 VALU/CU/clk in k_acc)
        uint64_t acc2 = 0;
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (j < 0 || j >= NLIMB) continue;
            acc = mad_acc(a.v[i], b.v[j], acc);
            acc2 = mad_acc(c.v[i], d.v[j], acc2);
        }
        acc += acc2;
        acc = fe_reduce_col<C>(m, k, acc);
        if (k < NLIMB) {
            const uint32_t mk = (0u - (uint32_t)acc) & LIMB_MASK;
            m[k] = mk;
            acc += mk;
            acc >>= LIMB_BITS;
        } else {
            r.v[k - NLIMB] = (uint32_t)acc & LIMB_MASK;
            acc >>= LIMB_BITS;
        }
    }
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}

// Two independent products r1 = a1 b1, r2 = a2 b2 with their column chains interleaved mad by mad:
// a single product's column is one dependent v_mad_u64_u32 chain, whose latency 4 waves per SIMD do
// not cover; two chains side by side do (same instruction count as two fe_mul).
template <class C>
HALO_DEV void fe_mul_x2(const Fe<C>& a1, const Fe<C>& b1, const Fe<C>& a2, const Fe<C>& b2, Fe<C>& r1, Fe<C>& r2) {
    uint32_t m1[NLIMB], m2[NLIMB];
    uint64_t acc1 = 0, acc2 = 0;
#pragma unroll
    for (int k = 0; k < 2 * NLIMB - 1; k++) {
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (j < 0 || j >= NLIMB) continue;
            acc1 = mad_acc(a1.v[i], b1.v[j], acc1);
            acc2 = mad_acc(a2.v[i], b2.v[j], acc2);
        }
        acc1 = fe_reduce_col<C>(m1, k, acc1);
        acc2 = fe_reduce_col<C>(m2, k, acc2);
        if (k < NLIMB) {
            const uint32_t mk1 = (0u - (uint32_t)acc1) & LIMB_MASK;
            const uint32_t mk2 = (0u - (uint32_t)acc2) & LIMB_MASK;
            m1[k] = mk1;
            m2[k] = mk2;
            acc1 = (acc1 + mk1) >> LIMB_BITS;
            acc2 = (acc2 + mk2) >> LIMB_BITS;
        } else {
            r1.v[k - NLIMB] = (uint32_t)acc1 & LIMB_MASK;
            r2.v[k - NLIMB] = (uint32_t)acc2 & LIMB_MASK;
            acc1 >>= LIMB_BITS;
            acc2 >>= LIMB_BITS;
        }
    }
    r1.v[NLIMB - 1] = (uint32_t)acc1;
    r2.v[NLIMB - 1] = (uint32_t)acc2;
}

// Squaring: cross products doubled up front (45 mads instead of 81).
template <class C>
HALO_DEV Fe<C> fe_sqr(const Fe<C>& a) {
    uint32_t m[NLIMB];
    uint32_t a2[NLIMB];
#pragma unroll
    for (int i = 0; i < NLIMB; i++) a2[i] = a.v[i] << 1;
    Fe<C> r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * NLIMB - 1; k++) {
#pragma unroll
        for (int i = 0; i < NLIMB; i++) {
            const int j = k - i;
            if (j <= i || j >= NLIMB) continue;
            acc = mad_acc(a2[i], a.v[j], acc);
        }
        if ((k & 1) == 0 && (k >> 1) < NLIMB) acc = mad_acc(a.v[k >> 1], a.v[k >> 1], acc);
        acc = fe_reduce_col<C>(m, k, acc);
        if (k < NLIMB) {
            const uint32_t mk = (0u - (uint32_t)acc) & LIMB_MASK;
            m[k] = mk;
            acc += mk;
            acc >>= LIMB_BITS;
        } else {
            r.v[k - NLIMB] = (uint32_t)acc & LIMB_MASK;
            acc >>= LIMB_BITS;
        }
    }
    r.v[NLIMB - 1] = (uint32_t)acc;
    return r;
}

#endif  // HALO_MAD_COL

// ----------------------------------------------------------------------------------------------
// Additive operations (results normalized, < 2p)
// ----------------------------------------------------------------------------------------------

// if x >= 2p then x - 2p  (x < 4p, normalized limbs)
template <class C>
HALO_DEV Fe<C> fe_reduce_2p(const Fe<C>& x) {
    Fe<C> t;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        int32_t d = (int32_t)x.v[i] - (int32_t)C::P2[i] + c;
        t.v[i] = (uint32_t)d & LIMB_MASK;
        c = d >> LIMB_BITS;
    }
    // c == 0 -> x >= 2p (take t); c == -1 -> x < 2p (take x)
    const bool ge = (c >= 0);
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = ge ? t.v[i] : x.v[i];
    return r;
}

template <class C>
HALO_DEV Fe<C> fe_add(const Fe<C>& a, const Fe<C>& b) {
    Fe<C> s;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        uint32_t x = a.v[i] + b.v[i] + c;
        s.v[i] = (i == NLIMB - 1) ? x : (x & LIMB_MASK);
        c = x >> LIMB_BITS;
    }
    return fe_reduce_2p(s);
}

template <class C>
HALO_DEV Fe<C> fe_sub(const Fe<C>& a, const Fe<C>& b) {
    // a - b + 2p in (0, 4p)
    Fe<C> s;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        int32_t x = (int32_t)a.v[i] - (int32_t)b.v[i] + (int32_t)C::P2[i] + c;
        s.v[i] = (i == NLIMB - 1) ? (uint32_t)x : ((uint32_t)x & LIMB_MASK);
        c = x >> LIMB_BITS;
    }
    return fe_reduce_2p(s);
}

template <class C>
HALO_DEV Fe<C> fe_neg(const Fe<C>& a) {
    return fe_sub(fe_zero<C>(), a);
}

template <class C>
HALO_DEV Fe<C> fe_dbl(const Fe<C>& a) {
    return fe_add(a, a);
}

// ---- lazy ("loose") operations: results are valid Montgomery-multiplication inputs (value < 8p,
// limbs < 2^30) but not reduced below 2p.  See DESIGN.md §3 for the bounds.

// a + b without carry propagation (a, b normalized, < 2p): limbs < 2^30, value < 4p.
template <class C>
HALO_DEV Fe<C> fe_add_nc(const Fe<C>& a, const Fe<C>& b) {
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = a.v[i] + b.v[i];
    return r;
}

// a - b + K p with signed carry propagation: a normalized (< 2p), b with limbs < 2^31 and b < K p;
// result normalized, in (0, 2p + K p).  K in {2, 4, 6, 8}.
template <int K, class C>
HALO_DEV Fe<C> fe_sub_k(const Fe<C>& a, const Fe<C>& b) {
    const uint32_t* kp = (K == 2) ? C::P2 : (K == 4) ? C::P4 : (K == 6) ? C::P6 : C::P8;
    Fe<C> s;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        int32_t x = (int32_t)a.v[i] - (int32_t)b.v[i] + (int32_t)kp[i] + c;
        s.v[i] = (i == NLIMB - 1) ? (uint32_t)x : ((uint32_t)x & LIMB_MASK);
        c = x >> LIMB_BITS;
    }
    return s;
}

// (+-a) - b + K p: the sign of a taken from negmask (0 or ~0u), folded into the limb loop (a limb-wise
// two's complement negation is the negation of the value; the signed carry chain absorbs it).
// Bounds as fe_sub_k, with a + b < K p when negated.
template <int K, class C>
HALO_DEV Fe<C> fe_sub_k_sgn(const Fe<C>& a, const Fe<C>& b, uint32_t negmask) {
    const uint32_t* kp = (K == 2) ? C::P2 : (K == 4) ? C::P4 : (K == 6) ? C::P6 : C::P8;
    Fe<C> s;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        const int32_t ai = (int32_t)((a.v[i] ^ negmask) - negmask);
        int32_t x = ai - (int32_t)b.v[i] + (int32_t)kp[i] + c;
        s.v[i] = (i == NLIMB - 1) ? (uint32_t)x : ((uint32_t)x & LIMB_MASK);
        c = x >> LIMB_BITS;
    }
    return s;
}

// carry-normalize limbs (value unchanged); input limbs < 2^31
template <class C>
HALO_DEV Fe<C> fe_norm(const Fe<C>& a) {
    Fe<C> r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        const uint32_t x = a.v[i] + c;
        r.v[i] = (i == NLIMB - 1) ? x : (x & LIMB_MASK);
        c = x >> LIMB_BITS;
    }
    return r;
}

// x < 8p (normalized) -> x < 2p
template <class C>
HALO_DEV Fe<C> fe_reduce_8p(const Fe<C>& x) {
    Fe<C> t;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        int32_t d = (int32_t)x.v[i] - (int32_t)C::P4[i] + c;
        t.v[i] = (uint32_t)d & LIMB_MASK;
        c = d >> LIMB_BITS;
    }
    const bool ge = (c >= 0);
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = ge ? t.v[i] : x.v[i];
    return fe_reduce_2p(r);
}

// x == 0 (mod p) for a normalized x < 4p
template <class C>
HALO_DEV bool fe_is_zero_4p(const Fe<C>& x) {
    return fe_is_zero(fe_reduce_2p(x));
}

// Canonical representative in [0, p)
template <class C>
HALO_DEV Fe<C> fe_canon(const Fe<C>& x) {
    Fe<C> t;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        int32_t d = (int32_t)x.v[i] - (int32_t)C::P[i] + c;
        t.v[i] = (uint32_t)d & LIMB_MASK;
        c = d >> LIMB_BITS;
    }
    const bool ge = (c >= 0);
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = ge ? t.v[i] : x.v[i];
    return r;
}

// x == 0 (mod p) for x < 2p: x is 0 or p
template <class C>
HALO_DEV bool fe_is_zero(const Fe<C>& x) {
    uint32_t z = 0, q = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        z |= x.v[i];
        q |= x.v[i] ^ C::P[i];
    }
    return z == 0 || q == 0;
}

template <class C>
HALO_DEV bool fe_eq(const Fe<C>& a, const Fe<C>& b) {
    return fe_is_zero(fe_sub(a, b));
}

template <class C>
HALO_DEV Fe<C> fe_select(bool c, const Fe<C>& a, const Fe<C>& b) {
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}

// a^e for a 256-bit exponent given as 4 x u64 (little endian), left-to-right 2-bit fixed window
// (small table: keeps register pressure low in latency-bound single-thread kernels).
template <class C>
HALO_DEV Fe<C> fe_pow(const Fe<C>& a, const uint64_t (&e)[4]) {
    const Fe<C> a2 = fe_sqr(a);
    const Fe<C> a3 = fe_mul(a2, a);
    Fe<C> r = fe_one<C>();
    for (int i = 127; i >= 0; i--) {
        r = fe_sqr(r);
        r = fe_sqr(r);
        const uint32_t d = (uint32_t)(e[i >> 5] >> ((i & 31) * 2)) & 3u;
        if (d) r = fe_mul(r, d == 1 ? a : (d == 2 ? a2 : a3));
    }
    return r;
}

// Fermat inverse a^(p-2) (349 dependent multiplications); inverse of 0 is 0.  Kept as the
// cross-check of fe_inv (k_field_op op 6).
template <class C>
HALO_DEV Fe<C> fe_inv_fermat(const Fe<C>& a) {
    uint64_t e[4] = {C::MODULUS64[0] - 2, C::MODULUS64[1], C::MODULUS64[2], C::MODULUS64[3]};
    return fe_pow(a, e);
}

// Inversion by Pornin's optimized binary GCD ("Optimized Binary GCD for Modular Inversion", 2020,
// algorithm 2 with k = 31): each round runs 30 binary-GCD steps on 62-bit approximations of a and
// b (their low 30 bits are exact, so the parity decisions are; the top 32 bits below their common
// length steer the comparisons), accumulating a 2x2 matrix of small signed factors, then applies it
// to the full a, b (exact division by 2^30) and to the coefficients u, v (mod p; the division by 2^30
// is a Montgomery step, trivial because p = 1 mod 2^32).  ceil((2 * 255 - 1) / 30) = 17 rounds reach
// b = gcd = 1 with v = x^-1.  All counts are fixed, so lanes never diverge, and the dependent chain is
// ~17 x 30 short steps instead of Fermat's 349 multiplications (k_final: ~160 -> ~30 us).
// Input: the canonical integer X of the Montgomery form x R'; X^-1 = x^-1 R'^-1, so one
// multiplication by R'^3 (INV_FIX) returns x^-1 R'.  Inverse of 0 is 0 (v stays 0).
namespace bgcd {
HALO_DEV int bitlen8(const uint32_t (&a)[8]) {
    int n = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (a[i]) n = 32 * i + 32 - (int)__clz(a[i]);
    return n;
}
// (a mod 2^30) + 2^30 floor(a / 2^(n - 32)), n >= 62 and a < 2^n
HALO_DEV uint64_t approx(const uint32_t (&a)[8], int n) {
    const int s = n - 32, i = s >> 5;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        if (j == i) lo = a[j];
        if (j == i + 1) hi = a[j];
    }
    const uint32_t top = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)(s & 31));
    return (uint64_t)(a[0] & 0x3fffffffu) | ((uint64_t)top << 30);
}
// r = |a f + b g| / 2^30 (exact), |f|, |g| <= 2^30; returns the sign
HALO_DEV bool lin(const uint32_t (&a)[8], const uint32_t (&b)[8], int64_t f, int64_t g, uint32_t (&r)[8]) {
    uint32_t t[8];
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int64_t x = (int64_t)a[i] * f + (int64_t)b[i] * g + c;
        t[i] = (uint32_t)x;
        c = x >> 32;
    }
    const bool neg = c < 0;
    uint64_t br = 1;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t s = __builtin_amdgcn_alignbit(i < 7 ? t[i + 1] : (uint32_t)c, t[i], 30u);
        const uint64_t ng = (uint64_t)(~s) + br;  // two's complement negation
        br = ng >> 32;
        r[i] = neg ? (uint32_t)ng : s;
    }
    return neg;
}
// r = (u f + v g) / 2^30 mod m for u, v in [0, m), |f|, |g| <= 2^30, m = 1 mod 2^32
HALO_DEV void lin_mod(const uint32_t (&u)[8], const uint32_t (&v)[8], int64_t f, int64_t g, const uint32_t (&m)[8],
                      uint32_t (&r)[8]) {
    uint32_t t[8];
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int64_t x = (int64_t)u[i] * f + (int64_t)v[i] * g + c;
        t[i] = (uint32_t)x;
        c = x >> 32;
    }
    // + q m with q = -t mod 2^30 (m = 1 mod 2^30): divisible by 2^30
    const uint32_t q = (0u - t[0]) & 0x3fffffffu;
    int64_t c2 = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int64_t x = (int64_t)t[i] + (int64_t)((uint64_t)q * m[i]) + c2;
        t[i] = (uint32_t)x;
        c2 = x >> 32;
    }
    const int64_t top = c + c2;  // value = t + top 2^256, |value / 2^30| < 2 m
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = __builtin_amdgcn_alignbit(i < 7 ? t[i + 1] : (uint32_t)top, t[i], 30u);
    int32_t hi = (int32_t)(top >> 30);  // bits 256.. of the quotient: 0 or -1
    // up to two additions of m while negative, then one conditional subtraction
#pragma unroll
    for (int k = 0; k < 2; k++) {
        uint64_t cy = 0;
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint64_t x = (uint64_t)s[i] + m[i] + cy;
            w[i] = (uint32_t)x;
            cy = x >> 32;
        }
        const bool add = hi < 0;
#pragma unroll
        for (int i = 0; i < 8; i++) s[i] = add ? w[i] : s[i];
        hi += add ? (int32_t)cy : 0;
    }
    uint64_t bw = 0;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t x = (uint64_t)s[i] - m[i] - bw;
        w[i] = (uint32_t)x;
        bw = (x >> 32) & 1u;
    }
    const bool ge = bw == 0;  // s >= m
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = ge ? w[i] : s[i];
}
}  // namespace bgcd

template <class C>
HALO_DEV Fe<C> fe_inv(const Fe<C>& x) {
    uint32_t a[8], b[8], u[8], v[8], m[8];
    fe_pack(fe_canon(x), a);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        m[i] = (uint32_t)(C::MODULUS64[i >> 1] >> (32 * (i & 1)));
        b[i] = m[i];
        u[i] = i == 0 ? 1u : 0u;
        v[i] = 0u;
    }
    constexpr int ROUNDS = (2 * 255 - 1 + 29) / 30;  // p < 2^255
    for (int it = 0; it < ROUNDS; it++) {
        const int n = max(max(bgcd::bitlen8(a), bgcd::bitlen8(b)), 62);
        uint64_t ab = bgcd::approx(a, n), bb = bgcd::approx(b, n);
        // |f|, |g| <= 2^30 after the 30 steps (Pornin, sec. 3): 32-bit registers
        int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 2
        for (int j = 0; j < 30; j++) {
            const bool odd = ab & 1u;
            const bool sw = odd && ab < bb;
            const uint64_t ta = sw ? bb : ab, tb = sw ? ab : bb;
            const int32_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
            ab = (odd ? ta - tb : ta) >> 1;
            bb = tb;
            f0 = odd ? tf0 - tf1 : tf0;
            g0 = odd ? tg0 - tg1 : tg0;
            f1 = tf1 * 2;
            g1 = tg1 * 2;
        }
        uint32_t na[8], nb[8], nu[8], nv[8];
        if (bgcd::lin(a, b, f0, g0, na)) {
            f0 = -f0;
            g0 = -g0;
        }
        if (bgcd::lin(a, b, f1, g1, nb)) {
            f1 = -f1;
            g1 = -g1;
        }
        bgcd::lin_mod(u, v, f0, g0, m, nu);
        bgcd::lin_mod(u, v, f1, g1, m, nv);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            a[i] = na[i];
            b[i] = nb[i];
            u[i] = nu[i];
            v[i] = nv[i];
        }
    }
    return fe_mul(fe_unpack<C>(v), fe_from_const<C>(C::INV_FIX));
}

// ----------------------------------------------------------------------------------------------
// ABI format conversions (ark: 4 x u64 Montgomery R = 2^256, canonical)
// ----------------------------------------------------------------------------------------------
template <class C>
HALO_DEV Fe<C> fe_from_ark(const uint4* p) {
    return fe_mul(fe_load<C>(p), fe_from_const<C>(C::ARK2INT));
}

template <class C>
HALO_DEV void fe_to_ark(uint4* p, const Fe<C>& x) {
    fe_store(p, fe_canon(fe_mul(x, fe_from_const<C>(C::INT2ARK))));
}

// canonical integer (not Montgomery) from ark format, as 8 x u32 words
template <class C>
HALO_DEV void fe_ark_to_canonical_words(const uint4* p, uint32_t (&w)[8]) {
    Fe<C> x = fe_canon(fe_mul(fe_load<C>(p), fe_from_const<C>(C::ARK2CANON)));
    fe_pack(x, w);
}

HALO_ARITH_END  // namespace halo
