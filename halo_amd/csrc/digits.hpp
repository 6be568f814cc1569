// Signed-window recoding of one MSM scalar (shared by k_digits in msm.hip and the fused first sort
// pass in sort.hip).
#pragma once
#include "fields.hpp"

namespace halo {

constexpr uint32_t DIGIT_NONE = 0xffffffffu;

// The W signed c-bit digits of an ark scalar, as sort entries: DIGIT_NONE for a zero digit, else
// (|d| - 1) with bit 31 = sign.  s > p / 2 is replaced by p - s and every digit's sign flipped
// (s P = -(p - s) P), so W = ceil(255 / c) windows suffice.  f(w, digit) is called for w < W in order.
// WMAX > 0: the window loop is unrolled WMAX times (W <= WMAX), so f sees a compile-time w (register
// arrays indexed by w stay in registers); WMAX = 0: a runtime loop.
template <class S, int WMAX = 0, class Fn>
HALO_DEV void scalar_signed_digits(const uint4* scalar, int c, int W, Fn&& f) {
    uint32_t w8[8];
    fe_ark_to_canonical_words<S>(scalar, w8);
    uint32_t t8[8];
    {
        int64_t br = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int64_t d = (int64_t)(uint32_t)(S::MODULUS64[q >> 1] >> (32 * (q & 1))) - (int64_t)w8[q] + br;
            t8[q] = (uint32_t)d;
            br = d >> 32;
        }
    }
    bool neg = false;  // p - s < s
#pragma unroll
    for (int q = 7; q >= 0; q--) {
        if (t8[q] != w8[q]) {
            neg = t8[q] < w8[q];
            break;
        }
    }
    if (neg)
#pragma unroll
        for (int q = 0; q < 8; q++) w8[q] = t8[q];
    const uint32_t nflip = neg ? 0x80000000u : 0u;
    const uint32_t half = 1u << (c - 1);
    const uint32_t full = 1u << c;
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < (WMAX ? WMAX : W); w++) {
        if (WMAX && w >= W) break;
        const int bit = w * c;
        uint32_t raw = 0;
        if (bit < 256) {
            const int q = bit >> 5, s = bit & 31;
            uint64_t lo = w8[q];
            uint64_t hi = (q + 1 < 8) ? w8[q + 1] : 0;
            raw = (uint32_t)(((hi << 32) | lo) >> s) & (full - 1);
        }
        uint32_t v = raw + carry;
        uint32_t out;
        if (v > half) {
            carry = 1;
            const uint32_t mag = full - v;  // |d|, d = v - 2^c < 0
            out = (mag == 0) ? DIGIT_NONE : (((mag - 1) | 0x80000000u) ^ nflip);
        } else {
            carry = 0;
            out = (v == 0) ? DIGIT_NONE : ((v - 1) | nflip);
        }
        f(w, out);
    }
}

}  // namespace halo
