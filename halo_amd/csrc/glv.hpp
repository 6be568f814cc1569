// GLV endomorphism helpers for the Pasta curves.
//
// phi(x, y) = (beta x, y) = lambda (x, y); a scalar k splits as k = k1 + lambda k2 (mod r) with
// |k1|, |k2| < 2^128 using the short lattice basis (a_i, b_i) (consts.hpp, gen_consts.py), so k P
// needs ~128 doublings instead of 255.  Used by the IPA fold (shared challenge, ipa.hip) and by the
// MSM's digit recoding when bases are not window-shifted (msm.hip).
#pragma once
#include "fields.hpp"

HALO_ARITH_BEGIN
// Decomposition xi = k1 + lambda k2 (mod r) with
// |k1|, |k2| < 2^128, using the short lattice basis (a_i, b_i) and c1 = round(b2 xi / r),
// c2 = round(-b1 xi / r) as (xi * G_i) >> 384 (consts.hpp, gen_consts.py).  The identity
// k1 + lambda k2 = xi holds for any integers c1, c2; the rounding only bounds the sizes.
namespace glv {
constexpr int TW = 10;  // two's complement width (320 bits)
HALO_DEV void mul_words(const uint32_t* a, int na, const uint32_t* b, int nb, uint32_t* c) {
    for (int i = 0; i < na + nb; i++) c[i] = 0;
    for (int i = 0; i < na; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < nb; j++) {
            const uint64_t t = (uint64_t)a[i] * b[j] + c[i + j] + carry;
            c[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
        c[i + nb] = (uint32_t)carry;
    }
}
HALO_DEV void tc_set(uint32_t (&t)[TW], const uint32_t* mag, int n, bool neg) {
    for (int i = 0; i < TW; i++) t[i] = i < n ? mag[i] : 0u;
    if (neg) {
        uint64_t c = 1;
        for (int i = 0; i < TW; i++) {
            c += (uint64_t)(~t[i]);
            t[i] = (uint32_t)c;
            c >>= 32;
        }
    }
}
HALO_DEV void tc_add(uint32_t (&a)[TW], const uint32_t (&b)[TW]) {
    uint64_t c = 0;
    for (int i = 0; i < TW; i++) {
        c += (uint64_t)a[i] + b[i];
        a[i] = (uint32_t)c;
        c >>= 32;
    }
}
// two's complement -> (neg, |x| as 5 words)
HALO_DEV void tc_get(const uint32_t (&t)[TW], bool& neg, uint32_t (&mag)[5]) {
    neg = (t[TW - 1] >> 31) != 0;
    uint32_t u[TW];
    for (int i = 0; i < TW; i++) u[i] = t[i];
    if (neg) {
        uint64_t c = 1;
        for (int i = 0; i < TW; i++) {
            c += (uint64_t)(~u[i]);
            u[i] = (uint32_t)c;
            c >>= 32;
        }
    }
    for (int i = 0; i < 5; i++) mag[i] = u[i];
}
// round((k * G) / 2^384): k 8 words, G 9 words -> 5 words
HALO_DEV void round_shift384(const uint32_t (&k)[8], const uint32_t (&G)[9], uint32_t (&c)[5]) {
    uint32_t p[17];
    mul_words(k, 8, G, 9, p);
    // + 2^383 then take words 12..16
    uint64_t carry = (uint64_t)p[11] + 0x80000000u;
    carry >>= 32;
    for (int i = 12; i < 17; i++) {
        carry += p[i];
        c[i - 12] = (uint32_t)carry;
        carry >>= 32;
    }
}
template <class K>
HALO_DEV void decompose(const uint32_t (&k)[8], bool& n1, uint32_t (&k1)[5], bool& n2, uint32_t (&k2)[5]) {
    uint32_t c1[5], c2[5];
    round_shift384(k, K::GLV_G1, c1);
    round_shift384(k, K::GLV_G2, c2);
    const bool c1n = K::GLV_G1_NEG, c2n = K::GLV_G2_NEG;
    uint32_t prod[10];
    uint32_t acc1[TW], acc2[TW], t[TW];
    tc_set(acc1, k, 8, false);
    // k1 = k - c1 a1 - c2 a2
    mul_words(c1, 5, K::GLV_A1, 5, prod);
    tc_set(t, prod, 10, !(c1n ^ (bool)K::GLV_A1_NEG));
    tc_add(acc1, t);
    mul_words(c2, 5, K::GLV_A2, 5, prod);
    tc_set(t, prod, 10, !(c2n ^ (bool)K::GLV_A2_NEG));
    tc_add(acc1, t);
    // k2 = -c1 b1 - c2 b2
    mul_words(c1, 5, K::GLV_B1, 5, prod);
    tc_set(acc2, prod, 10, !(c1n ^ (bool)K::GLV_B1_NEG));
    mul_words(c2, 5, K::GLV_B2, 5, prod);
    tc_set(t, prod, 10, !(c2n ^ (bool)K::GLV_B2_NEG));
    tc_add(acc2, t);
    tc_get(acc1, n1, k1);
    tc_get(acc2, n2, k2);
}
// NAF of a (<= 5-word) magnitude into naf[0..len); returns the top nonzero index (-1 if zero)
HALO_DEV int naf_digits(const uint32_t (&mag)[5], int8_t* naf, int len) {
    uint32_t k[6];
    for (int i = 0; i < 5; i++) k[i] = mag[i];
    k[5] = 0;
    int top = -1;
    for (int i = 0; i < len; i++) {
        int d = 0;
        if (k[0] & 1u) {
            d = 2 - (int)(k[0] & 3u);
            if (d == 1) {
                k[0] -= 1;
            } else {
                uint32_t c = 1;
                for (int q = 0; q < 6 && c; q++) {
                    k[q] += 1;
                    c = (k[q] == 0);
                }
            }
        }
        naf[i] = (int8_t)d;
        if (d) top = i;
        for (int q = 0; q < 5; q++) k[q] = (k[q] >> 1) | (k[q + 1] << 31);
        k[5] >>= 1;
    }
    return top;
}
}  // namespace glv

HALO_ARITH_END  // namespace halo
