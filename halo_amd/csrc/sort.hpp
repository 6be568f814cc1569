// Device radix sort / scan used by the MSM (sort.hip).
#pragma once
#include "runtime.hpp"

namespace halo {

struct SortScratch {
    DevBuf keys[2], vals[2], hist, offs, count, scan_tmp, ctr;
};

// Exclusive scan of n u32 values: out[0..n) exclusive prefix, out[n] = total.
int device_exclusive_scan(const uint32_t* in, size_t n, uint32_t* out, DevBuf& tmp, hipStream_t s);

// Sorts the MSM digit entries (digits[e], DIGIT_NONE entries dropped) by key =
// (e / npw) * B + (|d| - 1), stable; values = (e mod npw) | sign.  key_bits = bits of the largest
// key.  Fills bstart[0..NB] when bstart is not null (bucket b's entries are [bstart[b], bstart[b+1])
// of the sorted arrays).
// Fused first pass (window-shifted MSM, one bucket set, W <= 16): the entries come from the scalars
// (digits.hpp recoding) instead of a digit array; `digits` is then unused.  P > 1 outputs (the IPA's
// L / R pair MSM, msm_srs_pairs): output p's n scalars at srcs[p], its keys offset by p 2^(c-1) and its
// values w n + i as for one output -- the layout k_digits_multi + a plain first pass produce.
struct RsFused {
    const void* scalars;  // ark scalars (device), P == 1
    size_t n;             // scalars per output
    int c, W, field;
    int P = 1;
    const void* srcs[8] = {};  // P > 1: output p's scalars
};
int msm_radix_sort(const uint32_t* digits, size_t E, size_t npw, uint32_t B, uint32_t key_bits, SortScratch& S,
                   uint32_t** keys_out, uint32_t** vals_out, const uint32_t** count_out, uint32_t* bstart, size_t NB,
                   hipStream_t s, const RsFused* fused = nullptr);

// bstart[b] (b <= NB) from the sorted keys (capacity E, device count)
int msm_bucket_starts(const uint32_t* keys, const uint32_t* count, size_t NB, size_t E, uint32_t* bstart, hipStream_t s);

}  // namespace halo
