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
// every lane gets the sum over its aligned group of G lanes (G a power of two <= 64)
template <class F>
HALO_DEV XYZZ<F> wave_group_sum(XYZZ<F> v, uint32_t G) {
    for (uint32_t m = G >> 1; m > 0; m >>= 1) v = xyzz_add(v, xyzz_shfl_xor(v, (int)m));
    return v;
}
// sum over aligned groups of G threads (G a power of two <= blockDim): valid in the group's first
// thread.  While a group spans several waves its upper half hands its points to the lower half
// through LDS (the number of waves that add halves each level, as in an LDS tree), then the last
// wave of each group finishes with lane shuffles (no barriers).  red: LDS scratch for blockDim / 2
// points.  Every thread of the block must call it.
template <class F>
HALO_DEV XYZZ<F> block_group_sum(XYZZ<F> v, uint32_t G, uint4* red) {
    const uint32_t gpos = threadIdx.x & (G - 1), gbase = threadIdx.x - gpos;
    for (uint32_t span = G; span > 64; span >>= 1) {  // active: gpos < span (wave-uniform tests)
        const uint32_t half = span >> 1;
        if (gpos >= half && gpos < span) xyzz_store(red + 8 * ((gbase >> 1) + gpos - half), v);
        __syncthreads();
        if (gpos < half) v = xyzz_add(v, xyzz_load<F>(red + 8 * ((gbase >> 1) + gpos)));
        __syncthreads();
    }
    if (gpos < 64) v = wave_group_sum<F>(v, G < 64 ? G : 64u);
    return v;
}

HALO_ARITH_END
