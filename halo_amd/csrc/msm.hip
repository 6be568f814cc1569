// Pippenger multi-scalar multiplication on gfx950.
//
// Replaces `VariableBaseMSM::msm_unchecked` as called by group::point_dot_affine
// (crates/group/src/group.rs:48-50) and pedersen::commit (crates/accumulation/src/pedersen.rs:21),
// plus the SRS provider PublicParams (crates/group/src/pp.rs:26-94).
//
// Pipeline (all on the device, no host round trip):
//   1. digits   : scalar (ark Montgomery) -> canonical -> W signed c-bit digits
//                 (|d| <= 2^(c-1), W = ceil(256 / c)); key = (window, |d| - 1), value = index|sign.
//   2. sort     : stable LSD radix sort (8-bit digits, LDS-staged coalesced runs; sort.hip) of the
//                 W*n (bucket key, point ref) pairs; bucket starts from the sorted keys.
//   3. tasks    : every bucket is cut into tasks of <= K entries (skew-proof: an all-equal scalar
//                 vector becomes n/K equal tasks instead of one serial bucket).
//   4. acc      : one thread per task sums its points with XYZZ mixed additions (8M + 2S).
//   5. merge    : bucket sum = sum of its task partials.
//   6. reduce   : per window, segments of L buckets -> (sum_t t B_t, sum_t B_t) by running sums;
//                 one workgroup per window forms sum_j (acc_j + jL sum_j) and tree-reduces in LDS.
//   7. final    : Horner over the windows (+ w * S for hiding commitments), XYZZ -> affine -> ark.
#include <algorithm>
#include <type_traits>
#include <vector>
#include <cstdlib>

#include "digits.hpp"
#include "dispatch.hpp"
#include "glv.hpp"
#include "msm.hpp"
#include "runtime.hpp"
#include "sort.hpp"
#include "tree.hpp"

namespace halo {

// Columns of the bucket reduction grid (k_rowcol): 256 x 256 at 2^16 buckets keeps the row, column
// and bit-sliced tree depths at ~9 additions each (measured against 32 columns: single-MSM latency
// 2.15 -> 2.02 ms at 2^20, IPA opening 36.8 -> 35.2 ms; the pipelined step unchanged).
constexpr int MSM_SEG_L = 256;

// ---------------------------------------------------------------------------------------------
// synthetic bases / scalars (shared host/device definition)
// ---------------------------------------------------------------------------------------------
__host__ __device__ inline uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__host__ __device__ inline void synth_scalar(uint64_t seed, uint64_t j, uint64_t out[4]) {
    uint64_t st = seed ^ (j * 0xd1b54a32d192ed03ull);
    for (int i = 0; i < 4; i++) out[i] = splitmix64(st);
    out[3] &= 0x1fffffffffffffffull;  // < 2^253 < p
    if ((out[0] | out[1] | out[2] | out[3]) == 0) out[0] = 1;
}

// ---------------------------------------------------------------------------------------------
// conversion / generation kernels
// ---------------------------------------------------------------------------------------------
template <class F>
__global__ void k_wrapped_to_internal(const uint4* in, uint4* out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    aff_store(out + 4 * i, aff_from_wrapped<F>(in + 4 * i));
}

template <class F>
__global__ void k_internal_to_wrapped(const uint4* in, uint4* out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    aff_to_wrapped(out + 4 * i, aff_load<F>(in + 4 * i));
}

template <class Cv>
__global__ __launch_bounds__(64) void k_synth_bases(uint4* out, size_t n, uint64_t seed) {
    using F = typename Cv::Base;
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint64_t k[4];
    synth_scalar(seed, j, k);
    uint32_t w[8];
    for (int i = 0; i < 4; i++) {
        w[2 * i] = (uint32_t)k[i];
        w[2 * i + 1] = (uint32_t)(k[i] >> 32);
    }
    Affine<F> G;
    G.x = fe_from_const<F>(Cv::K::GX);
    G.y = fe_from_const<F>(Cv::K::GY);
    aff_store(out + 4 * j, xyzz_to_aff(xyzz_scalar_mul(G, w)));
}

// ---------------------------------------------------------------------------------------------
// 1. digits
// ---------------------------------------------------------------------------------------------
// digits[(w - w_lo) * ld + i] for the windows w_lo <= w < w_hi (ld >= n: the leading dimension, the
// batched MSMs' per-polynomial stride; a window range: one rank's share of a window-partitioned MSM)
template <class S>
__global__ void k_digits(const uint4* scalars, size_t n, int c, int W, uint32_t* digits, size_t ld, int w_lo,
                         int w_hi) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    scalar_signed_digits<S>(scalars + 2 * i, c, W, [&](int w, uint32_t out) {
        if (w >= w_lo && w < w_hi) digits[(size_t)(w - w_lo) * ld + i] = out;
    });
}

// k_digits over up to 8 scalar vectors of one length n in one launch (blockIdx.y = vector p, digits at
// digits + p SN): the pair MSMs' L and R sides, which took one launch each, one after the other
struct DigitSrcs {
    const uint4* s[8];
};
template <class S>
__global__ void k_digits_multi(DigitSrcs src, size_t n, int c, int W, uint32_t* digits, size_t SN) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* d = digits + (size_t)blockIdx.y * SN;
    scalar_signed_digits<S>(src.s[blockIdx.y] + 2 * i, c, W, [&](int w, uint32_t out) { d[(size_t)w * n + i] = out; });
}

// GLV recoding (bases not window-shifted): s = k1 + lambda k2 with |k1|, |k2| < 2^128, so each
// scalar gives W = ceil(129 / c) signed digits for point i (k1) and W for phi(G_i) (k2, entry
// n + i): the same number of bucket additions as W = ceil(255 / c) digits of s, but the Horner
// over the window sums needs ~128 doublings instead of ~255 (the latency of small MSMs).
template <class Cv>
__global__ void k_digits_glv(const uint4* scalars, size_t n, int c, int W, uint32_t* digits) {
    using S = typename Cv::Scalar;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t w8[8];
    fe_ark_to_canonical_words<S>(scalars + 2 * i, w8);
    bool neg[2];
    uint32_t mag[2][5];
    glv::decompose<typename Cv::K>(w8, neg[0], mag[0], neg[1], mag[1]);
    const uint32_t half = 1u << (c - 1);
    const uint32_t full = 1u << c;
    for (int h = 0; h < 2; h++) {
        const uint32_t nflip = neg[h] ? 0x80000000u : 0u;
        uint32_t carry = 0;
        for (int w = 0; w < W; w++) {
            const int bit = w * c;
            uint32_t raw = 0;
            if (bit < 160) {
                const int q = bit >> 5, sh = bit & 31;
                const uint64_t lo = mag[h][q];
                const uint64_t hi = (q + 1 < 5) ? mag[h][q + 1] : 0;
                raw = (uint32_t)(((hi << 32) | lo) >> sh) & (full - 1);
            }
            const uint32_t v = raw + carry;
            uint32_t out;
            if (v > half) {
                carry = 1;
                const uint32_t m = full - v;
                out = (m == 0) ? DIGIT_NONE : (((m - 1) | 0x80000000u) ^ nflip);
            } else {
                carry = 0;
                out = (v == 0) ? DIGIT_NONE : ((v - 1) | nflip);
            }
            digits[(size_t)w * 2 * n + (size_t)h * n + i] = out;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// 3-5. tasks, accumulation, merge
// ---------------------------------------------------------------------------------------------
// Uniform chunks: thread t accumulates the sorted entries [t K, t K + K) (every lane does the same
// number of mixed additions, whatever the bucket sizes).  A chunk may cross bucket boundaries: its
// first segment's sum goes to first[t], its last segment's (when there are >= 2) to last[t], and the
// buckets strictly inside the chunk are complete, so they go straight to bucket_sums.  k_merge then
// completes the buckets that straddle chunk boundaries.
// k_acc's register budget is sized for 4 workgroups per CU (the compiler's own allocation, 116 VGPRs;
// 5 / 6 per CU measured slower).
constexpr int ACC_MIN_BLOCKS = 4;
// npw_lg: log2 n_per_window when it is a power of two (the window of a shifted entry is a shift,
// not a division), else 0xff.
// (Measured and rejected: an LDS-DMA double buffer gathering entry e + 1's point while entry e's
// addition runs -- no change, 1.07 ms: the kernel is bound by its multiply-add issue, not the gathers.)
// One thread's chunk: the sorted entries [t K, t K + K) (see k_acc).
template <class Cv>
__device__ __forceinline__ void acc_chunk(size_t t, uint32_t cnt, const uint32_t* keys, const uint32_t* vals, uint32_t K,
                                          const uint4* bases, uint32_t n_per_window, uint32_t npw_lg, size_t stride,
                                          uint32_t blk_lg, uint32_t glv_n, uint4* first, uint4* last,
                                          uint4* bucket_sums, uint32_t* bstart, uint32_t NB, uint32_t key_lg,
                                          uint32_t poly_off, bool check_q) {
    using F = typename Cv::Base;
    const size_t beg = t * K;
    if (beg >= cnt) {
        if (t == 0)  // no entries at all: every bucket is empty
            for (uint32_t b = 0; b <= NB; b++) bstart[b] = 0;
        return;
    }
    const uint32_t end = (uint32_t)min((size_t)cnt, beg + K);
    uint32_t cur = keys[beg];
    // bucket starts (the tail's k_merge): bstart[b] = first sorted position of key b, for every b
    // whose first position (or, for empty buckets, the next bucket's) falls in this chunk
    {
        const uint32_t prev = beg ? keys[beg - 1] : 0xffffffffu;
        if (prev != cur)
            for (uint32_t b = prev + 1; b <= cur; b++) bstart[b] = (uint32_t)beg;
    }
    bool first_done = false;
    XYZZ<F> acc = xyzz_id<F>();
    bool fresh = true;  // acc is the identity (xyzz_madd_run)
    for (uint32_t e = (uint32_t)beg; e < end; e++) {
        const uint32_t k = keys[e];
        if (k != cur) {  // bucket boundary inside the chunk
            for (uint32_t b = cur + 1; b <= k; b++) bstart[b] = e;
            if (!first_done) {
                partial_store(first + PARTIAL_U4 * t, acc);
                first_done = true;
            } else {
                xyzz_store(bucket_sums + 8 * (size_t)cur, xyzz_settle(acc));
            }
            acc = xyzz_id<F>();
            fresh = true;
            cur = k;
        }
        const uint32_t v = vals[e];
        size_t idx = v & 0x7fffffffu;
        if (stride) {  // window-shifted SRS: entry w * n_per_window + i -> point w * stride + i
            const uint32_t w = npw_lg < 32 ? (uint32_t)idx >> npw_lg : (uint32_t)idx / n_per_window;
            uint32_t i = (uint32_t)idx - w * n_per_window;
            if (blk_lg < 32) i += (i >> blk_lg) << blk_lg;  // blocks of 2^blk_lg at stride 2^(blk_lg+1)
            // + the point offset of the entry's output (msm_srs_pairs: output k >> key_lg, odd = R at m)
            idx = (size_t)w * stride + i + (size_t)((k >> key_lg) & 1u) * poly_off;
        }
        const bool phi = glv_n && idx >= glv_n;  // GLV: phi(G_i)
        if (phi) idx -= glv_n;
        Affine<F> p = aff_load<F>(bases + 4 * idx);
        if (phi) p.x = fe_mul(p.x, fe_from_const<F>(Cv::K::BETA));
        acc = xyzz_madd_run(acc, fresh, p, (v & 0x80000000u) ? ~0u : 0u, check_q);
    }
    partial_store((first_done ? last : first) + PARTIAL_U4 * t, acc);
    if (end == cnt)
        for (uint32_t b = cur + 1; b <= NB; b++) bstart[b] = cnt;
}

template <class Cv>
__global__ __launch_bounds__(256, ACC_MIN_BLOCKS) void k_acc(const uint32_t* keys, const uint32_t* vals, const uint32_t* count,
                                             uint32_t K, const uint4* bases, uint32_t n_per_window, uint32_t npw_lg,
                                             size_t stride, uint32_t blk_lg, uint32_t glv_n, uint4* first, uint4* last,
                                             uint4* bucket_sums, uint32_t* bstart, uint32_t NB, uint32_t key_lg = 31,
                                             uint32_t poly_off = 0, uint32_t check_q = 1) {
    acc_chunk<Cv>((size_t)blockIdx.x * blockDim.x + threadIdx.x, *count, keys, vals, K, bases, n_per_window, npw_lg,
                  stride, blk_lg, glv_n, first, last, bucket_sums, bstart, NB, key_lg, poly_off, check_q != 0);
}

// ---------------------------------------------------------------------------------------------
// 7. final: Horner over the windows (wave 0), hiding term w * S from the table 2^i S (waves 1-4),
//    XYZZ -> affine -> ark WrappedPoint.
// ---------------------------------------------------------------------------------------------
// The hiding term w * P = sum of the 2^i P table entries over the set bits of w (an 8-level tree),
// -> hide_out (XYZZ).  glv: the table holds 2^i P for i < 128 only and w = k1 + lambda k2
// (|k1|, |k2| < 2^128, glv.hpp): lanes 0-127 take the bits of k1 with 2^i P, lanes 128-255 those of
// k2 with phi(2^i P) = (beta x, y) -- the IPA's 2^i H' table, whose doubling chain is then half as
// long.  Launched on the tail stream when the MSM starts, so it runs beside the digit / sort /
// accumulation phase instead of on the tail's critical path.
template <class Cv>
__device__ __forceinline__ void hide_term_block(const uint4* hide_table, const uint4* hide_scalar, int glv,
                                                uint4* hide_out) {
    using F = typename Cv::Base;
    using S = typename Cv::Scalar;
    __shared__ uint4 red[128 * 8];
    __shared__ uint32_t kw[8];
    __shared__ uint32_t neg[2];
    const int i = threadIdx.x;
    if (i == 0) {
        uint32_t w8[8];
        fe_ark_to_canonical_words<S>(hide_scalar, w8);
        if (glv) {
            bool n1, n2;
            uint32_t k1[5], k2[5];
            glv::decompose<typename Cv::K>(w8, n1, k1, n2, k2);
            for (int q = 0; q < 4; q++) {
                kw[q] = k1[q];
                kw[4 + q] = k2[q];
            }
            neg[0] = n1;
            neg[1] = n2;
        } else {
            for (int q = 0; q < 8; q++) kw[q] = w8[q];
        }
    }
    __syncthreads();
    XYZZ<F> v = xyzz_id<F>();
    if ((kw[i >> 5] >> (i & 31)) & 1u) {
        Affine<F> p = aff_load<F>(hide_table + 4 * (glv ? (i & 127) : i));
        if (glv) {
            if (i >= 128) p.x = fe_mul(p.x, fe_from_const<F>(Cv::K::BETA));
            if (neg[i >> 7]) p.y = fe_neg(p.y);
        }
        v = xyzz_from_aff(p);
    }
    v = block_group_sum<F>(v, 256, red);
    if (i == 0) xyzz_store(hide_out, v);
}

template <class Cv>
__global__ __launch_bounds__(256) void k_hide_term(const uint4* hide_table /* internal affine 2^i P */,
                                                   const uint4* hide_scalar /* ark */, int glv, uint4* hide_out) {
    hide_term_block<Cv>(hide_table, hide_scalar, glv, hide_out);
}

// up to 8 hiding terms (msm_srs_pairs): block b -> hide_out + 8 b
struct HideScalars {
    const uint4* sc[8];
};
template <class Cv>
__global__ __launch_bounds__(256) void k_hide_terms(const uint4* hide_table, HideScalars hs, int glv, uint4* hide_out) {
    hide_term_block<Cv>(hide_table, hs.sc[blockIdx.x], glv, hide_out + 8 * blockIdx.x);
}


// ---------------------------------------------------------------------------------------------
// SRS precomputation: window-shifted bases 2^(c w) G_i (w < W) and the hiding table 2^i S
// ---------------------------------------------------------------------------------------------
// copies w in [w_lo, w_hi) -> out[(w - w_lo) n + i] (a rank of a window partition holds only its own)
template <class Cv>
__global__ __launch_bounds__(64) void k_shift_windows(const uint4* gs, size_t n, int c, int w_lo, int w_hi, uint4* out,
                                                      uint32_t* has_id) {
    using F = typename Cv::Base;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Affine<F> g = aff_load<F>(gs + 4 * i);
    if (aff_is_id(g)) has_id[0] = 1u;  // (every copy of an identity is the identity; a prime-order
                                       // group has no other point with 2^(c w) g = 0)
    if (w_lo == 0) aff_store(out + 4 * i, g);
    XYZZ<F> p = xyzz_from_aff(g);
    for (int w = 1; w < w_hi; w++) {
        for (int k = 0; k < c; k++) p = xyzz_dbl(p);
        if (w >= w_lo) aff_store(out + 4 * ((size_t)(w - w_lo) * n + i), xyzz_to_aff(p));
    }
}

template <class Cv>
__global__ __launch_bounds__(64) void k_pow2_points(const uint4* P_int, uint4* out_xyzz, int count) {
    using F = typename Cv::Base;
    if (threadIdx.x != 0) return;
    XYZZ<F> p = xyzz_from_aff(aff_load<F>(P_int));
    for (int i = 0; i < count; i++) {
        xyzz_store(out_xyzz + 8 * i, p);
        p = xyzz_dbl(p);
    }
}

template <class Cv>
__global__ __launch_bounds__(64) void k_xyzz_to_aff(const uint4* in, uint4* out, int count) {
    using F = typename Cv::Base;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    aff_store(out + 4 * i, xyzz_to_aff(xyzz_load<F>(in + 8 * i)));
}

// ---------------------------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------------------------
// windows of c bits for scalars reduced to [0, p/2] (k_digits): 254 bits + the signed-digit carry
int msm_windows(int c) { return (255 + c - 1) / c; }

// window bits of the window-shifted SRS copies: one more bit than the plain MSM choice when that
// saves a window (c = 17 at 2^20: 15 windows instead of 16; the single bucket set of 2^16 buckets
// keeps the reduction and the 2-pass sort cheap)
int msm_shifted_window_bits(size_t n) {
    int c = msm_window_bits(n);
    if (msm_windows(c + 1) < msm_windows(c) && c + 1 <= 17) c++;
    // the top window holds only the 255 - (W - 1) c remaining bits, so its digits pile into the
    // lowest 2^(top - 1) buckets: n / 2^(top - 1) extra entries each, against W n / 2^(c - 1) on
    // average, and k_merge's longest runs (the latency of a small MSM) grow with that ratio.  Widen the
    // window until the ratio is at most 1/2 (c = 13 at 2^16: top 8 bits, ratio 1.6 -> c = 15, top 15).
    auto top_bits = [](int cc) { return 255 - (msm_windows(cc) - 1) * cc; };
    while (c < 17 && (1 << (c - top_bits(c))) * 2 > msm_windows(c)) c++;
    return c;
}

int msm_window_bits(size_t n) {
    unsigned lg = n > 1 ? ilog2(n - 1) + 1 : 1;
    int c = (int)lg - 4;
    return std::max(6, std::min(16, c));
}

static unsigned grid_for(size_t n, unsigned thr) { return (unsigned)std::max<size_t>(1, (n + thr - 1) / thr); }

// Chunk length K of k_acc for E sorted entries.  Large MSMs (E > 16 x the resident lanes, 256 CUs x
// 16 waves x 64): >= 4 rounds of resident lanes, 16 <= K <= 64 -- every lane does the same number
// of mixed additions, and several rounds absorb the CU slots held by the previous MSM's tail kernels,
// which one exact round would not (measured: K = 60 at 2^20 is 1 round and 15 % slower than K = 16;
// round 4, pipelined 2^20 step: 2 rounds (K = 30) 1.378, 3 rounds (K = 20) 1.365, 4 rounds 1.354 ms,
// and 6 / 8 rounds (K = 10 / 8: k_acc 0.87 / 0.85 ms, but twice the chunk partials for k_merge)
// 1.362 / 1.374 ms).
// Smaller MSMs are latency-bound (a commitment, an IPA round): their critical path is a lane's K
// dependent additions in k_acc plus k_merge's run of about E / (NB K) partials per bucket, so K =
// ceil(sqrt(E / NB)) balances the two -- but at least ceil(E / resident lanes), one round.
static uint32_t msm_chunk_len(const DeviceState* st, size_t E, size_t NB) {
    const size_t resident = (size_t)st->num_cu * 16 * 64;
    if (E > 16 * resident) return (uint32_t)std::max<size_t>(16, std::min<size_t>(64, (E + 4 * resident - 1) / (4 * resident)));
    size_t k = 1;
    while (k * k * std::max<size_t>(NB, 1) < E) k++;
    return (uint32_t)std::min<size_t>(16, std::max<size_t>(k, (E + resident - 1) / resident));
}

// Four scratch sets in two slots of two, a slot per issuing stream (least recently used slot
// reassigned): consecutive MSMs of one stream alternate between their slot's two sets (the tail of
// k overlaps k+1), two concurrent streams (two IPA openings in lockstep) never wait for each
// other's scratch, and a lone stream with a backlog borrows the idle slot (msm_pick_set).
// (Measured: rotating every MSM over all four sets made the 2^19-2^17 IPA rounds ~50 % slower,
// two sets only made back-to-back commitment batches slower.)
constexpr int MSM_SETS = 4;
struct MsmScratch {
    DevBuf digits, bstart, partials, bucket_sums, seg_acc, seg_sum, bits, window_sums, scan_tmp, conv;
    const uint32_t* skeys = nullptr;   // sorted keys of the current MSM (sort scratch)
    const uint32_t* scount = nullptr;  // device count of valid entries
    SortScratch sort;
    hipEvent_t acc_done = nullptr, tail_done = nullptr, start = nullptr, front_done = nullptr;
    bool tail_pending = false;
    hipStream_t owner = nullptr;  // stream the set's last MSM was enqueued on (msm_join)
};
// Two scratch sets per device: MSM k+1's digit/sort/accumulation phase (throughput-bound, whole
// GPU) runs on the caller's stream while MSM k's reduction tail (latency-bound, a few waves) runs
// on the per-device tail stream.
struct MsmPipe {
    MsmScratch set[MSM_SETS];
    hipStream_t slot_owner[2] = {nullptr, nullptr};
    int slot_next[2] = {0, 0};
    uint64_t slot_used[2] = {0, 0}, clock = 0;
    hipStream_t tail[MSM_SETS] = {};  // one per scratch set: consecutive tails run concurrently
};
static MsmPipe g_msm_pipe[64];  // per device

static bool set_busy(const MsmScratch& m) {
    return m.tail_pending && hipEventQuery(m.tail_done) == hipErrorNotReady;
}

// scratch set of the next MSM issued on stream s (advance: claim it).  A stream whose own slot is
// still busy (a batch of back-to-back commitments) borrows the other slot when that one is idle, so
// one stream alone pipelines four deep; a latency-bound caller (an IPA round, whose previous MSMs
// have completed) stays on its own two sets.
static int msm_pick_set(MsmPipe& P, hipStream_t s, bool advance) {
    int slot = (P.slot_owner[0] == s) ? 0 : (P.slot_owner[1] == s) ? 1 : -1;
    if (slot < 0) slot = (P.slot_used[0] <= P.slot_used[1]) ? 0 : 1;
    int set = 2 * slot + P.slot_next[slot];
    if (set_busy(P.set[set])) {
        const int o = slot ^ 1;
        const int oset = 2 * o + P.slot_next[o];
        if (!set_busy(P.set[2 * o]) && !set_busy(P.set[2 * o + 1])) {
            slot = o;
            set = oset;
        }
    }
    if (advance) {
        P.slot_owner[slot] = s;
        P.slot_next[slot] ^= 1;
        P.slot_used[slot] = ++P.clock;
    }
    return set;
}

// (Measured and rejected, round 4: tail streams restricted to a CU mask (32 / 64 / 128 of the 256
// CUs, hipExtStreamCreateWithCUMask) so that the tail would not share CUs with the next MSM's sort:
// 2^20 step 1.34 -> 2.71 / 2.08 / 1.89 ms -- the tail chain is throughput-bound on fewer CUs and
// becomes the critical path.)
static int pipe_init(MsmPipe& P) {
    if (P.tail[0]) return HALO_OK;
    for (auto& t : P.tail) HALO_HIP(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    for (auto& m : P.set) {
        HALO_HIP(hipEventCreateWithFlags(&m.acc_done, hipEventDisableTiming));
        HALO_HIP(hipEventCreateWithFlags(&m.tail_done, hipEventDisableTiming));
        HALO_HIP(hipEventCreateWithFlags(&m.start, hipEventDisableTiming));
        HALO_HIP(hipEventCreateWithFlags(&m.front_done, hipEventDisableTiming));
    }
    return HALO_OK;
}

// halo_shutdown: destroys the pipeline's streams and events while the HIP runtime is alive (a
// static destructor must not outlive it); pipe_init recreates them if the library is used again
void msm_shutdown() {
    for (auto& P : g_msm_pipe) {
        if (!P.tail[0]) continue;
        for (auto& t : P.tail) {
            (void)hipStreamSynchronize(t);
            (void)hipStreamDestroy(t);
            t = nullptr;
        }

        for (auto& m : P.set) {
            for (hipEvent_t* e : {&m.acc_done, &m.tail_done, &m.start, &m.front_done}) {
                if (*e) (void)hipEventDestroy(*e);
                *e = nullptr;
            }
            m.tail_pending = false;
            m.owner = nullptr;
        }
        P.slot_owner[0] = P.slot_owner[1] = nullptr;
    }
}

template <class Cv>
constexpr int curve_id() {
    return std::is_same<Cv, PallasCurve>::value ? HALO_PALLAS : HALO_VESTA;
}

// bases_int: n internal affine points, or (shifted) W * n window-shifted points (single bucket set).
template <class Cv>
static int msm_device_t(DeviceState* st, const uint4* bases_int, bool shifted, size_t shift_stride,
                        const uint4* scalars_ark, size_t n, int c_req, const uint4* hide_table, const uint4* hide_scalar,
                        uint4* d_out_wrapped, hipStream_t s, bool async, uint32_t blk_lg = 32,
                        bool hide_glv = false, bool out_xyzz = false, hipEvent_t hide_ready = nullptr,
                        int preset = -1, int w_lo = 0, int w_hi = 0, int base_w0 = 0) {
    MsmPipe& PP = g_msm_pipe[st->device & 63];
    HALO_CHECK(pipe_init(PP));
    // preset: the set the caller already claimed (and waited for) to stage converted bases in
    const int set = preset >= 0 ? preset : msm_pick_set(PP, s, true);
    MsmScratch& M = PP.set[set];
    // the previous user of this scratch set must have finished its tail
    if (M.tail_pending && preset < 0) HALO_HIP(hipStreamWaitEvent(s, M.tail_done, 0));
    const hipStream_t ts = PP.tail[set];
    const size_t nn = std::max<size_t>(n, 1);
    // non-shifted bases: GLV (2n half-size scalars, ~128-bit windows) -- see k_digits_glv
    const bool glv = !shifted;
    const size_t NP = glv ? 2 * nn : nn;  // digit entries per window
    const int c = c_req ? c_req : msm_window_bits(NP);
    const int W_all = glv ? (129 + c - 1) / c : msm_windows(c);
    // window range (shifted bases only): the windows [w_lo, w_hi) of the scalars, over the shifted
    // copies w_lo.. (the bases pointer is offset below); the partials of a partition add up
    if (w_hi <= 0 || glv) {
        w_lo = 0;
        w_hi = W_all;
    }
    if (w_lo < 0 || w_hi > W_all || w_lo >= w_hi)
        return set_error(HALO_EINVAL, "window range [%d, %d) outside [0, %d)", w_lo, w_hi, W_all);
    const int W = w_hi - w_lo;
    // (the copies start at window base_w0: a partially precomputed range)
    if (shifted && w_lo != base_w0) bases_int += 4 * (size_t)(w_lo - base_w0) * shift_stride;
    const uint32_t B = 1u << (c - 1);
    // sort geometry: SW windows of SN entries each (shifted: one window over all W * n digits)
    const int SW = shifted ? 1 : W;
    const size_t SN = shifted ? (size_t)W * nn : NP;
    const size_t NB = (size_t)SW * B;
    const uint32_t L = std::min<uint32_t>(MSM_SEG_L, B);
    const uint32_t logL = ilog2(L);
    const uint32_t H = B / L;
    const uint32_t logH = ilog2(H);
    const uint32_t NT = 1 + logH + logL;  // reduction bit terms per window (<= 64)
    const uint32_t key_bits = NB > 1 ? ilog2(NB - 1) + 1 : 1;
    HALO_CHECK(M.digits.reserve((size_t)W * NP * 4));
    HALO_CHECK(M.bstart.reserve((NB + 1) * 4));
    const size_t E = (size_t)W * NP;
    const uint32_t K = msm_chunk_len(st, E, NB);
    const size_t nchunks = (E + K - 1) / K;
    const size_t ng1 = nchunks / MSM_GROUP, ng2 = nchunks / (MSM_GROUP * MSM_GROUP);
    HALO_CHECK(M.partials.reserve((std::max<size_t>(nchunks, 1) * 2 + ng1 + ng2 + 2) * 16 * PARTIAL_U4));
    uint4* P_first = M.partials.as<uint4>();
    uint4* P_last = P_first + PARTIAL_U4 * std::max<size_t>(nchunks, 1);
    uint4* P_g1 = P_last + PARTIAL_U4 * std::max<size_t>(nchunks, 1);
    uint4* P_g2 = P_g1 + PARTIAL_U4 * (ng1 + 1);
    HALO_CHECK(M.bucket_sums.reserve(NB * 128));
    HALO_CHECK(M.seg_acc.reserve((size_t)SW * H * 128));  // row sums
    HALO_CHECK(M.seg_sum.reserve((size_t)SW * L * 128));  // column sums
    HALO_CHECK(M.bits.reserve((size_t)SW * NT * 128));
    HALO_CHECK(M.window_sums.reserve((size_t)(W + 1) * 128));  // + the hiding term's slot

    // the hiding term (k_hide_term) runs on the tail stream beside the accumulation phase
    uint4* hide_slot = nullptr;
    if (hide_table && hide_scalar) {
        hide_slot = M.window_sums.as<uint4>() + 8 * (size_t)W;
        HALO_HIP(hipEventRecord(M.start, s));
        HALO_HIP(hipStreamWaitEvent(ts, M.start, 0));
        if (hide_ready) HALO_HIP(hipStreamWaitEvent(ts, hide_ready, 0));  // table built on a side stream
        hipLaunchKernelGGL(k_hide_term<Cv>, dim3(1), dim3(256), 0, ts, hide_table, hide_scalar, (int)hide_glv,
                           hide_slot);
        HALO_HIP(hipGetLastError());
    }

    if (n > 0) {
        // shifted, all windows, W <= 16: digit recoding fused into the sort's first pass
        const bool fuse = shifted && w_lo == 0 && w_hi == W_all && W_all <= 16 && n < (1ull << 31) / 16;
        if (glv)
            hipLaunchKernelGGL(k_digits_glv<Cv>, dim3(grid_for(n, 256)), dim3(256), 0, s, scalars_ark, n, c, W,
                               M.digits.as<uint32_t>());
        else if (!fuse)
            hipLaunchKernelGGL(k_digits<typename Cv::Scalar>, dim3(grid_for(n, 256)), dim3(256), 0, s, scalars_ark,
                               n, c, W_all, M.digits.as<uint32_t>(), n, w_lo, w_hi);
        HALO_HIP(hipGetLastError());
        uint32_t *skeys = nullptr, *svals = nullptr;
        const uint32_t* scount = nullptr;
        RsFused fz{scalars_ark, n, c, W_all, curve_id<Cv>() == HALO_PALLAS ? HALO_FP : HALO_FQ};
        HALO_CHECK(msm_radix_sort(M.digits.as<const uint32_t>(), E, SN, B, key_bits, M.sort, &skeys, &svals, &scount,
                                  nullptr, NB, s, fuse ? &fz : nullptr));
        const uint32_t nblocks = (uint32_t)grid_for(nchunks, 256);
        // the resident window-shifted SRS without identity points: k_acc skips the bases' identity test
        const SrsState& srs_c = st->srs[curve_id<Cv>()];
        const bool srs_bases = shifted && srs_c.shifted_c != 0 && srs_c.shifted.ptr &&
                               (const char*)bases_int >= srs_c.shifted.as<const char>() &&
                               (const char*)bases_int < srs_c.shifted.as<const char>() + srs_c.shifted.bytes;
        const uint32_t check_q = (srs_bases && !srs_c.shifted_has_id) ? 0u : 1u;
        {
            ProfScope prof("msm_acc", s);
            HALO_LAUNCH(prof, k_acc<Cv>, dim3(nblocks), dim3(256), 0, s, (const uint32_t*)skeys,
                        (const uint32_t*)svals, scount, K, bases_int, (uint32_t)nn, is_pow2(nn) ? ilog2(nn) : 0xffu,
                        (shifted && (shift_stride != nn || blk_lg < 32)) ? shift_stride : (size_t)0, blk_lg,
                        glv ? (uint32_t)nn : 0u, P_first,
                        P_last, M.bucket_sums.as<uint4>(), M.bstart.as<uint32_t>(), (uint32_t)NB, 31u, 0u,
                        check_q);
        }
        M.skeys = skeys;
        M.scount = scount;
        HALO_HIP(hipGetLastError());
    } else {
        HALO_HIP(hipMemsetAsync(M.window_sums.ptr, 0, (size_t)SW * 128, s));
    }
    // ---- tail (latency-bound: task merge and bucket reduction) on the tail stream, overlapping the
    // caller's next MSM
    HALO_HIP(hipEventRecord(M.acc_done, s));
    HALO_HIP(hipStreamWaitEvent(ts, M.acc_done, 0));
    MsmTailArgs ta;
    ta.num_cu = (uint32_t)st->num_cu;
    ta.n = n;
    ta.skeys = M.skeys;
    ta.scount = M.scount;
    ta.K = K;
    ta.NB = NB;
    ta.E = E;
    ta.first = P_first;
    ta.last = P_last;
    ta.g1 = P_g1;
    ta.g2 = P_g2;
    ta.ng1 = ng1;
    ta.ng2 = ng2;
    ta.bstart = M.bstart.as<uint32_t>();
    ta.bucket_sums = M.bucket_sums.as<uint4>();
    ta.rows = M.seg_acc.as<uint4>();
    ta.cols = M.seg_sum.as<uint4>();
    ta.terms = M.bits.as<uint4>();
    ta.window_sums = M.window_sums.as<uint4>();
    ta.L = L;
    ta.H = H;
    ta.logH = logH;
    ta.logL = logL;
    ta.NT = NT;
    ta.SW = SW;
    ta.c = c;
    ta.hide_table = hide_table;
    ta.hide_scalar = hide_scalar;
    ta.out_wrapped = d_out_wrapped;
    // one window set with a nonempty MSM (the tail reaches k_bitcombine): it also finishes the MSM
    const bool fuse = SW == 1 && n > 0;
    if (fuse) {
        ta.final_mode = out_xyzz ? 2 : 1;
        ta.final_hide = (const uint4*)hide_slot;
        ta.final_out = (uint4*)d_out_wrapped;
    }
    HALO_CHECK(msm_tail_launch(curve_id<Cv>(), ta, ts));
    if (!fuse)
        HALO_CHECK(msm_final_launch(curve_id<Cv>(), M.window_sums.as<const uint4>(), SW, c, (const uint4*)hide_slot,
                                    d_out_wrapped, (int)out_xyzz, ts));
    HALO_HIP(hipGetLastError());
    HALO_HIP(hipEventRecord(M.tail_done, ts));
    M.tail_pending = true;
    M.owner = s;
    if (!async) HALO_HIP(hipStreamWaitEvent(s, M.tail_done, 0));
    return HALO_OK;
}

// ---------------------------------------------------------------------------------------------
// Batched commitments as ONE MSM (halo_msm_batch_dev for small polynomials): k scalar vectors over
// the resident window-shifted SRS share one digit pass, one sort (key = (polynomial, bucket)), one
// accumulation and one reduction tail with a window per polynomial; k_sums_out converts each
// polynomial's bucket-weighted sum.  At n = 2^16 one MSM is latency-bound (a few thousand
// workgroups, a ~1 ms reduction tail); sixteen of them in one pass fill the GPU once.
// ---------------------------------------------------------------------------------------------
template <class Cv>
__global__ __launch_bounds__(64) void k_sums_out(const uint4* window_sums, uint32_t k, uint4* out_wrapped) {
    using F = typename Cv::Base;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    aff_to_wrapped(out_wrapped + 4 * (size_t)i, xyzz_to_aff(xyzz_load<F>(window_sums + 8 * (size_t)i)));
}

template <class Cv>
static int msm_multi_device_t(DeviceState* st, const void* const* scalars, const size_t* lens, size_t k,
                              uint4* d_out, hipStream_t s) {
    SrsState& srs = st->srs[curve_id<Cv>()];
    MsmPipe& PP = g_msm_pipe[st->device & 63];
    HALO_CHECK(pipe_init(PP));
    const int set = msm_pick_set(PP, s, true);
    MsmScratch& M = PP.set[set];
    if (M.tail_pending) HALO_HIP(hipStreamWaitEvent(s, M.tail_done, 0));
    size_t nmax = 1;
    bool ragged = false;
    for (size_t p = 0; p < k; p++) nmax = std::max(nmax, lens[p]);
    size_t ld = 1;
    while (ld < nmax) ld <<= 1;
    if (ld > srs.n) ld = nmax;
    for (size_t p = 0; p < k; p++) ragged |= lens[p] != ld;
    const int c = srs.shifted_c, W = msm_windows(c);
    const uint32_t B = 1u << (c - 1);
    const size_t SN = (size_t)W * ld, E = k * SN, NB = k * (size_t)B;
    const int SW = (int)k;
    if (E >= (1ull << 32)) return set_error(HALO_EINVAL, "halo_msm_batch_dev: batch too large");
    const uint32_t L = std::min<uint32_t>(MSM_SEG_L, B), logL = ilog2(L), H = B / L, logH = ilog2(H);
    const uint32_t NT = 1 + logH + logL;
    const uint32_t key_bits = ilog2(NB - 1) + 1;
    const uint32_t K = msm_chunk_len(st, E, NB);
    const size_t nchunks = (E + K - 1) / K;
    const size_t ng1 = nchunks / MSM_GROUP, ng2 = nchunks / (MSM_GROUP * MSM_GROUP);
    HALO_CHECK(M.digits.reserve(E * 4));
    HALO_CHECK(M.bstart.reserve((NB + 1) * 4));
    HALO_CHECK(M.partials.reserve((nchunks * 2 + ng1 + ng2 + 2) * 16 * PARTIAL_U4));
    HALO_CHECK(M.bucket_sums.reserve(NB * 128));
    HALO_CHECK(M.seg_acc.reserve((size_t)SW * H * 128));
    HALO_CHECK(M.seg_sum.reserve((size_t)SW * L * 128));
    HALO_CHECK(M.bits.reserve((size_t)SW * NT * 128));
    HALO_CHECK(M.window_sums.reserve((size_t)SW * 128));
    uint4* P_first = M.partials.as<uint4>();
    uint4* P_last = P_first + PARTIAL_U4 * nchunks;
    uint4* P_g1 = P_last + PARTIAL_U4 * nchunks;
    uint4* P_g2 = P_g1 + PARTIAL_U4 * (ng1 + 1);
    uint32_t* digits = M.digits.as<uint32_t>();
    if (ragged) HALO_HIP(hipMemsetAsync(digits, 0xff, E * 4, s));  // DIGIT_NONE past each length
    for (size_t p = 0; p < k; p++)
        if (lens[p])
            hipLaunchKernelGGL(k_digits<typename Cv::Scalar>, dim3(grid_for(lens[p], 256)), dim3(256), 0, s,
                               (const uint4*)scalars[p], lens[p], c, W, digits + p * SN, ld, 0, W);
    HALO_HIP(hipGetLastError());
    uint32_t *skeys = nullptr, *svals = nullptr;
    const uint32_t* scount = nullptr;
    HALO_CHECK(msm_radix_sort(digits, E, SN, B, key_bits, M.sort, &skeys, &svals, &scount, nullptr, NB, s));
    {
        ProfScope prof("msm_acc", s);
        const uint32_t nblocks = (uint32_t)grid_for(nchunks, 256);
                HALO_LAUNCH(prof, k_acc<Cv>, dim3(nblocks), dim3(256), 0, s, (const uint32_t*)skeys, (const uint32_t*)svals, scount,
                    K, srs.shifted.as<const uint4>(), (uint32_t)ld, is_pow2(ld) ? ilog2(ld) : 0xffu, srs.n, 32u, 0u,
                    P_first, P_last, M.bucket_sums.as<uint4>(), M.bstart.as<uint32_t>(),
                    (uint32_t)NB, 31u, 0u, srs.shifted_has_id ? 1u : 0u);
        HALO_HIP(hipGetLastError());
    }
    MsmTailArgs ta;
    ta.num_cu = (uint32_t)st->num_cu;
    ta.n = E;
    ta.skeys = skeys;
    ta.scount = scount;
    ta.K = K;
    ta.NB = NB;
    ta.E = E;
    ta.first = P_first;
    ta.last = P_last;
    ta.g1 = P_g1;
    ta.g2 = P_g2;
    ta.ng1 = ng1;
    ta.ng2 = ng2;
    ta.bstart = M.bstart.as<uint32_t>();
    ta.bucket_sums = M.bucket_sums.as<uint4>();
    ta.rows = M.seg_acc.as<uint4>();
    ta.cols = M.seg_sum.as<uint4>();
    ta.terms = M.bits.as<uint4>();
    ta.window_sums = M.window_sums.as<uint4>();
    ta.L = L;
    ta.H = H;
    ta.logH = logH;
    ta.logL = logL;
    ta.NT = NT;
    ta.SW = SW;
    ta.c = c;
    ta.hide_table = nullptr;
    ta.hide_scalar = nullptr;
    ta.out_wrapped = nullptr;
    HALO_CHECK(msm_tail_launch(curve_id<Cv>(), ta, s));
    hipLaunchKernelGGL(k_sums_out<Cv>, dim3(grid_for(k, 64)), dim3(64), 0, s, M.window_sums.as<const uint4>(),
                       (uint32_t)k, d_out);
    HALO_HIP(hipGetLastError());
    HALO_HIP(hipEventRecord(M.tail_done, s));
    M.tail_pending = true;
    M.owner = s;
    return HALO_OK;
}

// ---------------------------------------------------------------------------------------------
// The IPA's weighted-round pairs (ipa.hip): L = sum_i sl[i] G[map(i)] and R = sum_i sr[i] G[m + map(i)],
// map(i) = i + (i >> lg m) << lg m (the left / right halves of the 2m-blocks), each plus its hiding
// term dot H' from the 2^i table, for np <= 4 sessions in lockstep -- ONE MSM over the window-shifted
// SRS with key (output, bucket): one digit pass, one sort, one accumulation and one reduction tail
// (SW = 2 np) instead of 2 np MSMs whose fronts and accumulations run one after the other.  Outputs
// packed XYZZ (128 B each).
// ---------------------------------------------------------------------------------------------
template <class Cv>
static int msm_srs_pairs_t(DeviceState* st, size_t np, const MsmPairIO* io, size_t half, uint32_t lgm,
                           const uint4* hide_table, hipStream_t s, hipEvent_t hide_ready, const MsmPreHide* pre_hide,
                           uint32_t* host_emit, uint32_t seq) {
    SrsState& srs = st->srs[curve_id<Cv>()];
    const size_t m = (size_t)1 << lgm;
    if (!srs.shifted_c) return set_error(HALO_EINVAL, "msm_srs_pairs: no window-shifted SRS");
    if (!np || np > 4) return set_error(HALO_EINVAL, "msm_srs_pairs: %zu pairs (1..4)", np);
    if (!half || (half & (half - 1)) || half % m || 2 * half > srs.n)
        return set_error(HALO_EINVAL, "msm_srs_pairs: %zu terms per side, blocks of %zu, SRS %zu", half, m, srs.n);
    MsmPipe& PP = g_msm_pipe[st->device & 63];
    HALO_CHECK(pipe_init(PP));
    const int set = msm_pick_set(PP, s, true);
    MsmScratch& M = PP.set[set];
    if (M.tail_pending) HALO_HIP(hipStreamWaitEvent(s, M.tail_done, 0));
    const hipStream_t ts = PP.tail[set];
    const int P = (int)(2 * np);  // outputs: L0, R0, L1, R1, ...
    const int c = srs.shifted_c, W = msm_windows(c);
    const uint32_t B = 1u << (c - 1);
    const size_t SN = (size_t)W * half, E = P * SN, NB = P * (size_t)B;
    const int SW = P;
    if (E >= (1ull << 32)) return set_error(HALO_EINVAL, "msm_srs_pairs: too large");
    const uint32_t L = std::min<uint32_t>(MSM_SEG_L, B), logL = ilog2(L), H = B / L, logH = ilog2(H);
    const uint32_t NT = 1 + logH + logL;
    const uint32_t key_bits = ilog2(NB - 1) + 1;
    const uint32_t K = msm_chunk_len(st, E, NB);
    const size_t nchunks = (E + K - 1) / K;
    const size_t ng1 = nchunks / MSM_GROUP, ng2 = nchunks / (MSM_GROUP * MSM_GROUP);
    HALO_CHECK(M.digits.reserve(E * 4));
    HALO_CHECK(M.bstart.reserve((NB + 1) * 4));
    HALO_CHECK(M.partials.reserve((nchunks * 2 + ng1 + ng2 + 2) * 16 * PARTIAL_U4));
    HALO_CHECK(M.bucket_sums.reserve(NB * 128));
    HALO_CHECK(M.seg_acc.reserve((size_t)SW * H * 128));
    HALO_CHECK(M.seg_sum.reserve((size_t)SW * L * 128));
    HALO_CHECK(M.bits.reserve((size_t)SW * NT * 128));
    HALO_CHECK(M.window_sums.reserve((size_t)(2 * SW) * 128));  // + the hiding terms
    uint4* P_first = M.partials.as<uint4>();
    uint4* P_last = P_first + PARTIAL_U4 * nchunks;
    uint4* P_g1 = P_last + PARTIAL_U4 * nchunks;
    uint4* P_g2 = P_g1 + PARTIAL_U4 * (ng1 + 1);
    uint4* hide_slot = M.window_sums.as<uint4>() + 8 * SW;
    // the hiding terms on the tail stream, beside the front and the accumulation
    HALO_HIP(hipEventRecord(M.start, s));
    HALO_HIP(hipStreamWaitEvent(ts, M.start, 0));
    if (hide_ready) HALO_HIP(hipStreamWaitEvent(ts, hide_ready, 0));
    if (pre_hide) {
        pre_hide->fn(ts, pre_hide->ctx);
        HALO_HIP(hipGetLastError());
    }
    HideScalars hs{};
    MsmOuts8 outs{};
    for (size_t q = 0; q < np; q++) {
        hs.sc[2 * q] = (const uint4*)io[q].hide_l;
        hs.sc[2 * q + 1] = (const uint4*)io[q].hide_r;
        outs.o[2 * q] = (uint4*)io[q].out_l;
        outs.o[2 * q + 1] = (uint4*)io[q].out_r;
    }
    hipLaunchKernelGGL(k_hide_terms<Cv>, dim3(P), dim3(256), 0, ts, hide_table, hs, 1, hide_slot);
    HALO_HIP(hipGetLastError());
    HALO_HIP(hipEventRecord(M.front_done, ts));
    uint32_t* digits = M.digits.as<uint32_t>();
    DigitSrcs ds{};
    for (int p = 0; p < P; p++) ds.s[p] = (const uint4*)(p & 1 ? io[p / 2].sr : io[p / 2].sl);
    // the digit recoding fused into the sort's first pass (thread = scalar, round = window), as the
    // headline MSM's: no digit array written and read back (W <= 16 windows and keys of <= 17 bits, so
    // the first pass is an 8-bit one)
    const bool fuse = W <= 16 && key_bits <= 17;
    RsFused fz{nullptr, half, c, W, curve_id<Cv>() == HALO_PALLAS ? HALO_FP : HALO_FQ, P, {}};
    for (int p = 0; p < P; p++) fz.srcs[p] = ds.s[p];
    if (!fuse) {
        hipLaunchKernelGGL(k_digits_multi<typename Cv::Scalar>, dim3(grid_for(half, 256), P), dim3(256), 0, s, ds, half,
                           c, W, digits, SN);
        HALO_HIP(hipGetLastError());
    }
    uint32_t *skeys = nullptr, *svals = nullptr;
    const uint32_t* scount = nullptr;
    HALO_CHECK(msm_radix_sort(digits, E, SN, B, key_bits, M.sort, &skeys, &svals, &scount, nullptr, NB, s,
                              fuse ? &fz : nullptr));
    {
        ProfScope prof("msm_acc", s);
        const uint32_t nblocks = (uint32_t)grid_for(nchunks, 256);
                HALO_LAUNCH(prof, k_acc<Cv>, dim3(nblocks), dim3(256), 0, s, (const uint32_t*)skeys, (const uint32_t*)svals, scount,
                    K, srs.shifted.as<const uint4>(), (uint32_t)half, ilog2(half), srs.n, lgm, 0u, P_first, P_last,
                    M.bucket_sums.as<uint4>(), M.bstart.as<uint32_t>(), (uint32_t)NB,
                    (uint32_t)(c - 1), (uint32_t)m, srs.shifted_has_id ? 1u : 0u);
        HALO_HIP(hipGetLastError());
    }
    MsmTailArgs ta;
    ta.num_cu = (uint32_t)st->num_cu;
    ta.n = E;
    ta.skeys = skeys;
    ta.scount = scount;
    ta.K = K;
    ta.NB = NB;
    ta.E = E;
    ta.first = P_first;
    ta.last = P_last;
    ta.g1 = P_g1;
    ta.g2 = P_g2;
    ta.ng1 = ng1;
    ta.ng2 = ng2;
    ta.bstart = M.bstart.as<uint32_t>();
    ta.bucket_sums = M.bucket_sums.as<uint4>();
    ta.rows = M.seg_acc.as<uint4>();
    ta.cols = M.seg_sum.as<uint4>();
    ta.terms = M.bits.as<uint4>();
    ta.window_sums = M.window_sums.as<uint4>();
    ta.L = L;
    ta.H = H;
    ta.logH = logH;
    ta.logL = logL;
    ta.NT = NT;
    ta.SW = SW;
    ta.c = c;
    ta.hide_table = nullptr;
    ta.hide_scalar = nullptr;
    ta.out_wrapped = nullptr;
    ta.pair_hide = hide_slot;  // k_bitcombine adds the hiding terms and writes the outputs
    ta.pair_outs = outs;
    if (np == 1) {
        ta.pair_host = host_emit;
        ta.pair_seq = seq;
    }
    HALO_HIP(hipStreamWaitEvent(s, M.front_done, 0));  // the hiding terms (done beside the front)
    HALO_CHECK(msm_tail_launch(curve_id<Cv>(), ta, s));
    HALO_HIP(hipGetLastError());
    HALO_HIP(hipEventRecord(M.tail_done, s));
    M.tail_pending = true;
    M.owner = s;
    return HALO_OK;
}

int msm_srs_pairs_device(DeviceState* st, int curve, size_t np, const MsmPairIO* io, size_t half, uint32_t lgm,
                         const void* hide_table, hipStream_t s, hipEvent_t hide_ready, const MsmPreHide* pre_hide,
                         uint32_t* host_emit, uint32_t seq) {
    int rc;
    DISPATCH_CURVE(curve, Cv, {
        rc = msm_srs_pairs_t<Cv>(st, np, io, half, lgm, (const uint4*)hide_table, s, hide_ready, pre_hide, host_emit,
                                 seq);
    });
    return rc;
}

// polynomials up to this length take the one-MSM batch path (tuning "msm_multi_max", default 2^18;
// 0 = off)
static size_t msm_multi_max() { return (size_t)tuning(TUNE_MSM_MULTI_MAX); }

// Claims the scratch set of the next MSM on stream s and orders s after that set's previous tail
// (the caller stages converted bases in its conv buffer before the MSM is enqueued; the MSM then
// runs on the same set, msm_device's preset).
int msm_claim_set(DeviceState* st, hipStream_t s, int* set, DevBuf** conv) {
    MsmPipe& PP = g_msm_pipe[st->device & 63];
    HALO_CHECK(pipe_init(PP));
    *set = msm_pick_set(PP, s, true);
    MsmScratch& M = PP.set[*set];
    if (M.tail_pending) HALO_HIP(hipStreamWaitEvent(s, M.tail_done, 0));
    *conv = &M.conv;
    return HALO_OK;
}

// Makes `s` wait (device-side) for the tails of the MSMs enqueued on `s` that are still in flight.
// Forgets which issuing streams own the two scratch-set slots and restarts each slot at its first set
// (only when no set's tail is still running; every set still waits for its own previous tail when
// reused).  An IPA opening calls it before its first two-stream round, so its two streams claim the
// same sets in the same order however many MSMs earlier callers issued on which streams (measured: after
// 23 two-stream MSMs the 2^20 opening took 21.7-22.6 ms, after 32 -- or after a reset -- 19.6-20.0).
void msm_slots_reset(DeviceState* st) {
    MsmPipe& P = g_msm_pipe[st->device & 63];
    for (const auto& m : P.set)
        if (set_busy(m)) return;
    for (int k = 0; k < 2; k++) {
        P.slot_owner[k] = nullptr;
        P.slot_next[k] = 0;
        P.slot_used[k] = 0;
    }
    P.clock = 0;
}

int msm_join(DeviceState* st, hipStream_t s) {
    MsmPipe& PP = g_msm_pipe[st->device & 63];
    for (auto& m : PP.set)
        if (m.tail_pending && m.owner == s) HALO_HIP(hipStreamWaitEvent(s, m.tail_done, 0));
    return HALO_OK;
}

int msm_device(DeviceState* st, int curve, const void* bases_int, const void* scalars_ark, size_t n,
               const void* hide_table, const void* hide_scalar, void* d_out_wrapped, hipStream_t s, bool async,
               bool hide_glv, bool out_xyzz, hipEvent_t hide_ready, int preset) {
    int rc;
    DISPATCH_CURVE(curve, Cv, {
        rc = msm_device_t<Cv>(st, (const uint4*)bases_int, false, 0, (const uint4*)scalars_ark, n, 0,
                              (const uint4*)hide_table, (const uint4*)hide_scalar, (uint4*)d_out_wrapped, s, async,
                              32, hide_glv, out_xyzz, hide_ready, preset);
    });
    return rc;
}

// MSM over the resident SRS prefix Gs[0..n): uses the window-shifted copies when present.
int msm_srs_device(DeviceState* st, int curve, const void* scalars_ark, size_t n, const void* hide_scalar,
                   void* d_out_wrapped, hipStream_t s, bool async, bool out_xyzz) {
    SrsState& srs = st->srs[curve];
    if (n > srs.n) return set_error(HALO_ESRSRANGE, "n (%zu) exceeds the resident SRS length (%zu)", n, srs.n);
    const void* table = hide_scalar ? srs.s_table.ptr : nullptr;
    if (hide_scalar && !srs.has_sh) return set_error(HALO_ESRSRANGE, "hiding commitment needs S: upload (S, H)");
    if (!async && n >= 1 && n <= srs_small_max())
        return msm_srs_small(st, curve, scalars_ark, n, hide_scalar, d_out_wrapped, s, out_xyzz);
    int rc;
    // the shifted copies hold W windows of srs.n points each; an MSM of n <= srs.n points uses the
    // prefix of every window (point index w * srs.n + i)
    const bool use_shifted = srs.shifted_c != 0;
    DISPATCH_CURVE(curve, Cv, {
        rc = msm_device_t<Cv>(st, use_shifted ? srs.shifted.as<const uint4>() : srs.gs.as<const uint4>(), use_shifted,
                              srs.n, (const uint4*)scalars_ark, n, use_shifted ? srs.shifted_c : 0, (const uint4*)table,
                              (const uint4*)hide_scalar, (uint4*)d_out_wrapped, s, async, 32, false, out_xyzz, nullptr,
                              -1);
    });
    return rc;
}

int msm_srs_range_device(DeviceState* st, int curve, size_t offset, const void* scalars_ark, size_t n,
                         const void* hide_table, const void* hide_scalar, void* d_out_wrapped, hipStream_t s,
                         bool async, uint32_t blk_lg, bool hide_glv, bool out_xyzz,
                         hipEvent_t hide_ready) {
    SrsState& srs = st->srs[curve];
    if (!srs.shifted_c) return set_error(HALO_EINVAL, "msm_srs_range_device: no window-shifted SRS");
    // highest point touched: offset + map(n - 1), map(i) = i + (i >> blk_lg) << blk_lg
    const size_t last = n ? (n - 1) + (blk_lg < 32 ? ((n - 1) >> blk_lg) << blk_lg : 0) : 0;
    if (n && offset + last >= srs.n)
        return set_error(HALO_ESRSRANGE, "range [%zu, %zu] exceeds the SRS (%zu)", offset, offset + last, srs.n);
    if (n >= (1u << 31)) return set_error(HALO_EINVAL, "msm_srs_range_device: n too large");
    int rc;
    // window w of point offset + i lives at shifted[w * srs.n + offset + i]: shift the base pointer
    DISPATCH_CURVE(curve, Cv, {
        rc = msm_device_t<Cv>(st, srs.shifted.as<const uint4>() + 4 * offset, true, srs.n, (const uint4*)scalars_ark, n,
                              srs.shifted_c, (const uint4*)hide_table, (const uint4*)hide_scalar,
                              (uint4*)d_out_wrapped, s, async, blk_lg, hide_glv, out_xyzz, hide_ready);
    });
    return rc;
}

// ---------------------------------------------------------------------------------------------
// Batched MSM with shared scalars (the IPA's switch from weighted to tail rounds, ipa.hip):
//   out[i] = sum_{u < T} w[u] bases[i + u len],  i < len.
// Every output has the same digit lists, so there is no sort: one workgroup groups the (window,
// scalar) digits by bucket (counting sort in LDS, k_batch_lists), and k_batch_expand replicates that
// order for every output (key = (i W + win) B + b, value = base index i + u len) -- exactly the
// sorted layout k_acc and the reduction tail take, with SW = len W windows of B buckets.  A batched
// Horner (one lane per output) finishes.
// ---------------------------------------------------------------------------------------------
constexpr int BATCH_C_MAX = 8;  // unshifted window bits: at most 32 windows of 128 buckets
constexpr uint32_t BATCH_B_MAX = 256;  // buckets per window (shifted: two 8-bit sub-digit windows)

__global__ __launch_bounds__(256) void k_batch_lists(const uint32_t* digits, uint32_t T, int W, uint32_t B,
                                                     uint32_t len, uint32_t* ent, uint32_t* ekey, uint32_t* tot) {
    __shared__ uint32_t cnt[BATCH_B_MAX + 1];
    __shared__ uint32_t base;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) base = 0;
    for (int w = 0; w < W; w++) {
        for (uint32_t b = tid; b < B; b += blockDim.x) cnt[b] = 0;
        __syncthreads();
        for (uint32_t u = tid; u < T; u += blockDim.x) {
            const uint32_t d = digits[(size_t)w * T + u];
            if (d != DIGIT_NONE) atomicAdd(&cnt[d & 0x7fffffffu], 1u);
        }
        __syncthreads();
        if (tid == 0) {  // exclusive scan over the B buckets, continuing after the previous windows
            uint32_t run = base;
            for (uint32_t b = 0; b < B; b++) {
                const uint32_t c = cnt[b];
                cnt[b] = run;
                run += c;
            }
            cnt[B] = run;
        }
        __syncthreads();
        for (uint32_t u = tid; u < T; u += blockDim.x) {
            const uint32_t d = digits[(size_t)w * T + u];
            if (d == DIGIT_NONE) continue;
            const uint32_t b = d & 0x7fffffffu;
            const uint32_t pos = atomicAdd(&cnt[b], 1u);
            ent[pos] = u | (d & 0x80000000u);
            ekey[pos] = (uint32_t)w * B + b;
        }
        __syncthreads();
        if (tid == 0) base = cnt[B];
        __syncthreads();
    }
    if (tid == 0) {
        tot[0] = base;        // entries per output
        tot[1] = base * len;  // entries in total (k_acc's count)
    }
}

// entry e of the lists: scalar u = e & tmask of shifted copy e >> tlog (tlog 31: no copies)
__global__ __launch_bounds__(256) void k_batch_expand(const uint32_t* ent, const uint32_t* ekey, const uint32_t* tot,
                                                      uint32_t len, uint32_t WB, uint32_t tlog, uint32_t wstride,
                                                      uint32_t* keys, uint32_t* vals) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t per = tot[0];
    if (per == 0 || p >= per * len) return;
    const uint32_t i = p / per, r = p - i * per;
    const uint32_t e = ent[r], ee = e & 0x7fffffffu;
    keys[p] = i * WB + ekey[r];
    vals[p] = (i + (ee & ((1u << tlog) - 1u)) * len + (ee >> tlog) * wstride) | (e & 0x80000000u);
}

// Shifted-SRS batches: the signed c_s-bit digit of (copy w, scalar u) -> nsub unsigned sub-digits
// d_0 + 2^cb d_1 (+ 2^(2 cb) d_2) of its magnitude (mag <= 2^(c_s - 1) <= 2^(nsub cb)), window q at
// sub[q][w T + u] (its sign carried along; DIGIT_NONE for 0).  Sub-digit values run 1 .. 2^cb (bucket
// v - 1 of B = 2^cb): the one magnitude whose top sub-digit would be 2^cb, mag = 2^(nsub cb), is written
// as top = 2^cb - 1 and 2^cb in the sub-digit below.  Two sub-digits while 2^(c_s / 2) <= BATCH_B_MAX
// (c_s <= 17), three above (window widths 18-20 would otherwise need 512-1024 buckets).
// (Round 4: two windows of 2^8 buckets instead of three of 2^6 at c_s = 17 -- a third fewer bucket
// additions, the dominant cost of the IPA's switch to the tail rounds: 47M -> 31M at 2^20.)
__global__ __launch_bounds__(256) void k_batch_subdigits(const uint32_t* digits, uint32_t TW, int cb, int nsub,
                                                         uint32_t* sub) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= TW) return;
    const uint32_t d = digits[e];
    const uint32_t mag = d == DIGIT_NONE ? 0u : (d & 0x7fffffffu) + 1u, sign = d & 0x80000000u;
    const uint32_t full = 1u << cb;
    uint32_t q[3];
    q[0] = mag & (full - 1u);
    q[1] = nsub == 2 ? mag >> cb : (mag >> cb) & (full - 1u);
    q[2] = nsub == 2 ? 0u : mag >> (2 * cb);
    if (q[nsub - 1] == full) {
        q[nsub - 1] = full - 1u;
        q[nsub - 2] += full;
    }
    for (int k = 0; k < nsub; k++) sub[(size_t)k * TW + e] = q[k] ? ((q[k] - 1u) | sign) : DIGIT_NONE;
}

template <class Cv>
__global__ __launch_bounds__(64) void k_batch_horner(const uint4* window_sums, uint32_t len, int W, int c,
                                                     uint4* out, int xyzz_out) {
    using F = typename Cv::Base;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    const uint4* ws = window_sums + 8 * (size_t)i * W;
    XYZZ<F> h = xyzz_id<F>();
    for (int w = W - 1; w >= 0; w--) {
        if (w != W - 1 && !xyzz_is_id(h)) {
            Jac<F> j = jac_from_xyzz(h);
            for (int k = 0; k < c; k++) j = jac_dbl(j);
            h = jac_to_xyzz(j);
        }
        h = xyzz_add(h, xyzz_load<F>(ws + 8 * w));
    }
    if (xyzz_out)
        xyzz_store(out + 8 * (size_t)i, h);
    else
        aff_store(out + 4 * (size_t)i, xyzz_to_aff(h));
}

template <class Cv>
static int msm_shared_batch_t(DeviceState* st, const uint4* bases, const uint4* w_ark, size_t T, size_t len,
                              uint4* out, bool xyzz_out, BatchScratch& S, hipStream_t s, size_t shift_stride, int c_s) {
    if (!T || !len) return set_error(HALO_EINVAL, "msm_shared_batch: empty batch");
    // shifted: the lists run over TS = W_s T (copy, scalar) entries with nsub sub-digit windows of
    // 2^cb buckets (magnitudes 1..2^(c_s-1) <= 2^(nsub cb), k_batch_subdigits)
    const bool shifted = shift_stride && c_s && (T & (T - 1)) == 0 &&
                         (size_t)msm_windows(c_s) * shift_stride < (1ull << 31);
    const int W_s = shifted ? msm_windows(c_s) : 1;
    const int nsub = (shifted && (1u << (c_s / 2)) > BATCH_B_MAX) ? 3 : 2;
    const int cb = shifted ? (nsub == 2 ? c_s / 2 : (c_s + 1) / 3) : 0;
    // unshifted window bits: about T / 4 buckets per window, so that the per-window reduction
    // (2 B additions) stays below the accumulation (T mixed additions)
    const int c = shifted ? cb : std::max(5, std::min(BATCH_C_MAX, (int)ilog2(std::max<size_t>(T, 2)) - 1));
    const int W = shifted ? nsub : msm_windows(c);
    const uint32_t B = shifted ? 1u << cb : 1u << (c - 1);
    const size_t TS = (size_t)W_s * T;
    const size_t SW = len * (size_t)W, NB = SW * B, E = SW * TS;
    if (E >= (1ull << 32) || T * len >= (1ull << 31) || B > BATCH_B_MAX)
        return set_error(HALO_EINVAL, "msm_shared_batch: batch too large (len %zu, T %zu)", len, T);
    const uint32_t L = std::min<uint32_t>(MSM_SEG_L, B), logL = ilog2(L), H = B / L, logH = ilog2(H);
    const uint32_t NT = 1 + logH + logL;
    const uint32_t K = msm_chunk_len(st, E, NB);
    const size_t nchunks = (E + K - 1) / K;
    const size_t ng1 = nchunks / MSM_GROUP, ng2 = nchunks / (MSM_GROUP * MSM_GROUP);
    HALO_CHECK(S.digits.reserve((size_t)(shifted ? W_s + W : W) * TS * 4));
    HALO_CHECK(S.lists.reserve((size_t)W * TS * 8 + 16));
    HALO_CHECK(S.keys.reserve(E * 4));
    HALO_CHECK(S.vals.reserve(E * 4));
    HALO_CHECK(S.bstart.reserve((NB + 1) * 4));
    HALO_CHECK(S.partials.reserve((nchunks * 2 + ng1 + ng2 + 2) * 16 * PARTIAL_U4));
    HALO_CHECK(S.bucket_sums.reserve(NB * 128));
    HALO_CHECK(S.window_sums.reserve(SW * 128));
    uint32_t* ent = S.lists.as<uint32_t>();
    uint32_t* ekey = ent + (size_t)W * TS;
    uint32_t* tot = ekey + (size_t)W * TS;
    uint4* P_first = S.partials.as<uint4>();
    uint4* P_last = P_first + PARTIAL_U4 * nchunks;
    uint4* P_g1 = P_last + PARTIAL_U4 * nchunks;
    uint4* P_g2 = P_g1 + PARTIAL_U4 * (ng1 + 1);

    const uint32_t* lists_in = S.digits.as<const uint32_t>();
    if (shifted) {
        hipLaunchKernelGGL(k_digits<typename Cv::Scalar>, dim3(grid_for(T, 256)), dim3(256), 0, s, w_ark, T, c_s, W_s,
                           S.digits.as<uint32_t>(), T, 0, W_s);
        uint32_t* sub = S.digits.as<uint32_t>() + TS;
        hipLaunchKernelGGL(k_batch_subdigits, dim3(grid_for(TS, 256)), dim3(256), 0, s, S.digits.as<const uint32_t>(),
                           (uint32_t)TS, cb, nsub, sub);
        lists_in = sub;
    } else {
        hipLaunchKernelGGL(k_digits<typename Cv::Scalar>, dim3(grid_for(T, 256)), dim3(256), 0, s, w_ark, T, c, W,
                           S.digits.as<uint32_t>(), T, 0, W);
    }
    hipLaunchKernelGGL(k_batch_lists, dim3(1), dim3(256), 0, s, lists_in, (uint32_t)TS, W, B, (uint32_t)len, ent, ekey,
                       tot);
    hipLaunchKernelGGL(k_batch_expand, dim3(grid_for(E, 256)), dim3(256), 0, s, (const uint32_t*)ent,
                       (const uint32_t*)ekey, (const uint32_t*)tot, (uint32_t)len, (uint32_t)(W * B),
                       shifted ? (uint32_t)ilog2(T) : 31u, shifted ? (uint32_t)shift_stride : 0u,
                       S.keys.as<uint32_t>(), S.vals.as<uint32_t>());
    hipLaunchKernelGGL(k_acc<Cv>, dim3(grid_for(nchunks, 256)), dim3(256), 0, s, S.keys.as<const uint32_t>(),
                       S.vals.as<const uint32_t>(), (const uint32_t*)(tot + 1), K, bases, 1u, 0u, (size_t)0, 32u, 0u,
                       P_first, P_last, S.bucket_sums.as<uint4>(), S.bstart.as<uint32_t>(), (uint32_t)NB, 31u, 0u, 1u);
    HALO_HIP(hipGetLastError());
    MsmTailArgs ta;
    ta.num_cu = (uint32_t)st->num_cu;
    ta.n = T;
    ta.skeys = S.keys.as<const uint32_t>();
    ta.scount = tot + 1;
    ta.K = K;
    ta.NB = NB;
    ta.E = E;
    ta.first = P_first;
    ta.last = P_last;
    ta.g1 = P_g1;
    ta.g2 = P_g2;
    ta.ng1 = ng1;
    ta.ng2 = ng2;
    ta.bstart = S.bstart.as<uint32_t>();
    ta.bucket_sums = S.bucket_sums.as<uint4>();
    ta.rows = ta.cols = ta.terms = nullptr;  // k_batch_window_sums needs no grid scratch
    ta.window_sums = S.window_sums.as<uint4>();
    ta.L = L;
    ta.H = H;
    ta.logH = logH;
    ta.logL = logL;
    ta.NT = NT;
    ta.SW = (int)SW;
    ta.c = c;
    ta.hide_table = nullptr;
    ta.hide_scalar = nullptr;
    ta.out_wrapped = nullptr;
    ta.batch_windows = true;
    HALO_CHECK(msm_tail_launch(curve_id<Cv>(), ta, s));
    hipLaunchKernelGGL(k_batch_horner<Cv>, dim3(grid_for(len, 64)), dim3(64), 0, s, S.window_sums.as<const uint4>(),
                       (uint32_t)len, W, c, out, (int)xyzz_out);
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

int msm_shared_batch(DeviceState* st, int curve, const void* bases_int, const void* w_ark, size_t T, size_t len,
                     void* out, bool xyzz_out, BatchScratch& S, hipStream_t s, size_t shift_stride, int c_s) {
    int rc;
    DISPATCH_CURVE(curve, Cv, {
        rc = msm_shared_batch_t<Cv>(st, (const uint4*)bases_int, (const uint4*)w_ark, T, len, (uint4*)out, xyzz_out,
                                    S, s, shift_stride, c_s);
    });
    return rc;
}

// ---------------------------------------------------------------------------------------------
// Host-side XYZZ -> affine (the IPA's per-round L and R, and every entry point that returns one point
// to the host): the lane-side conversion is a ~30 us dependent chain on one lane (fe_inv) at the end
// of the reduction tail; on the host it is a few microseconds.  A packed internal coordinate is an integer < 2p congruent to v 2^261, so
// x = X / ZZ and y = Y / ZZZ need no change of representation; 4 x 64-bit Montgomery arithmetic
// (R = 2^256) then yields x R mod p, which is the ark word form directly.
// ---------------------------------------------------------------------------------------------
namespace {
struct HostMont {
    uint64_t p[4], pinv, r2[4], one[4], inv_fix[4];
    uint32_t p32[8];
    explicit HostMont(const uint64_t (&m)[4]) {
        for (int i = 0; i < 4; i++) p[i] = m[i];
        uint64_t inv = 1;  // p[0]^-1 mod 2^64 by Newton's iteration
        for (int i = 0; i < 6; i++) inv *= 2 - p[0] * inv;
        pinv = 0 - inv;
        uint64_t x[4] = {1, 0, 0, 0};
        for (int i = 0; i < 512; i++) {  // 2^256 mod p (= one), then 2^512 mod p (= r2)
            dbl(x);
            if (i == 255)
                for (int k = 0; k < 4; k++) one[k] = x[k];
        }
        for (int k = 0; k < 4; k++) r2[k] = x[k];
        for (int k = 0; k < 8; k++) p32[k] = (uint32_t)(p[k >> 1] >> (32 * (k & 1)));
        mul(r2, r2, inv_fix);  // R^3 = 2^768 mod p (inv)
    }
    bool geq_p(const uint64_t (&a)[4]) const {
        for (int i = 3; i >= 0; i--)
            if (a[i] != p[i]) return a[i] > p[i];
        return true;
    }
    void sub_p(uint64_t (&a)[4]) const {
        unsigned __int128 b = 0;
        for (int i = 0; i < 4; i++) {
            const unsigned __int128 d = (unsigned __int128)a[i] - p[i] - b;
            a[i] = (uint64_t)d;
            b = (d >> 64) & 1;
        }
    }
    void dbl(uint64_t (&a)[4]) const {  // a < p (p < 2^255): 2a < 2^256
        uint64_t c = 0;
        for (int i = 0; i < 4; i++) {
            const uint64_t t = (a[i] << 1) | c;
            c = a[i] >> 63;
            a[i] = t;
        }
        if (geq_p(a)) sub_p(a);
    }
    void mul(const uint64_t (&a)[4], const uint64_t (&b)[4], uint64_t (&out)[4]) const {  // a b R^-1 mod p (CIOS)
        uint64_t t[6] = {0, 0, 0, 0, 0, 0};
        for (int i = 0; i < 4; i++) {
            unsigned __int128 c = 0;
            for (int j = 0; j < 4; j++) {
                c += (unsigned __int128)a[j] * b[i] + t[j];
                t[j] = (uint64_t)c;
                c >>= 64;
            }
            c += t[4];
            t[4] = (uint64_t)c;
            t[5] = (uint64_t)(c >> 64);
            const uint64_t m = t[0] * pinv;
            c = ((unsigned __int128)m * p[0] + t[0]) >> 64;
            for (int j = 1; j < 4; j++) {
                c += (unsigned __int128)m * p[j] + t[j];
                t[j - 1] = (uint64_t)c;
                c >>= 64;
            }
            c += t[4];
            t[3] = (uint64_t)c;
            t[4] = t[5] + (uint64_t)(c >> 64);
        }
        uint64_t r[4] = {t[0], t[1], t[2], t[3]};
        if (t[4] || geq_p(r)) sub_p(r);
        for (int i = 0; i < 4; i++) out[i] = r[i];
    }
    // Montgomery domain (a = x R mod p, a < p): Pornin's optimized binary GCD, the same algorithm as the
    // device's fe_inv (fields.hpp: 17 rounds of 30 steps on 62-bit approximations, each round's 2x2
    // factors applied to a, b and, with a Montgomery division by 2^30, to the coefficients u, v).  It
    // leaves v = a^-1 = x^-1 R^-1 (the invariants a = x u, b = x v mod p survive the rounds' common
    // division by 2^30); one product with inv_fix = R^3 makes it x^-1 R.
    // (Host: about 3x faster than the Fermat chain a^(p-2), 384 products, and 1.7x faster than a
    // plain binary extended Euclid.)
    static int bitlen8(const uint32_t (&a)[8]) {
        for (int i = 7; i >= 0; i--)
            if (a[i]) return 32 * i + 32 - __builtin_clz(a[i]);
        return 0;
    }
    static uint32_t align30(uint32_t hi, uint32_t lo, int s) { return (uint32_t)((((uint64_t)hi << 32) | lo) >> s); }
    static uint64_t approx(const uint32_t (&a)[8], int n) {  // (a mod 2^30) + 2^30 floor(a / 2^(n - 32))
        const int s = n - 32, i = s >> 5;
        const uint32_t lo = a[i], hi = i + 1 < 8 ? a[i + 1] : 0u;
        return (uint64_t)(a[0] & 0x3fffffffu) | ((uint64_t)align30(hi, lo, s & 31) << 30);
    }
    static bool lin(const uint32_t (&a)[8], const uint32_t (&b)[8], int64_t f, int64_t g, uint32_t (&r)[8]) {
        uint32_t t[8];
        int64_t c = 0;
        for (int i = 0; i < 8; i++) {  // |a f + b g| / 2^30, exact; returns the sign
            const int64_t x = (int64_t)a[i] * f + (int64_t)b[i] * g + c;
            t[i] = (uint32_t)x;
            c = x >> 32;
        }
        const bool neg = c < 0;
        uint64_t br = 1;
        for (int i = 0; i < 8; i++) {
            const uint32_t sh = align30(i < 7 ? t[i + 1] : (uint32_t)c, t[i], 30);
            const uint64_t ng = (uint64_t)(~sh) + br;
            br = ng >> 32;
            r[i] = neg ? (uint32_t)ng : sh;
        }
        return neg;
    }
    void lin_mod(const uint32_t (&u)[8], const uint32_t (&v)[8], int64_t f, int64_t g, uint32_t (&r)[8]) const {
        uint32_t t[8];
        int64_t c = 0;
        for (int i = 0; i < 8; i++) {  // (u f + v g) / 2^30 mod p (p = 1 mod 2^32)
            const int64_t x = (int64_t)u[i] * f + (int64_t)v[i] * g + c;
            t[i] = (uint32_t)x;
            c = x >> 32;
        }
        const uint32_t q = (0u - t[0]) & 0x3fffffffu;
        int64_t c2 = 0;
        for (int i = 0; i < 8; i++) {
            const int64_t x = (int64_t)t[i] + (int64_t)((uint64_t)q * p32[i]) + c2;
            t[i] = (uint32_t)x;
            c2 = x >> 32;
        }
        const int64_t top = c + c2;
        uint32_t s[8];
        for (int i = 0; i < 8; i++) s[i] = align30(i < 7 ? t[i + 1] : (uint32_t)top, t[i], 30);
        int32_t hi = (int32_t)(top >> 30);
        for (int k = 0; k < 2 && hi < 0; k++) {
            uint64_t cy = 0;
            for (int i = 0; i < 8; i++) {
                const uint64_t x = (uint64_t)s[i] + p32[i] + cy;
                s[i] = (uint32_t)x;
                cy = x >> 32;
            }
            hi += (int32_t)cy;
        }
        uint64_t bw = 0;
        uint32_t w[8];
        for (int i = 0; i < 8; i++) {
            const uint64_t x = (uint64_t)s[i] - p32[i] - bw;
            w[i] = (uint32_t)x;
            bw = (x >> 32) & 1u;
        }
        for (int i = 0; i < 8; i++) r[i] = bw == 0 ? w[i] : s[i];
    }
    void inv(const uint64_t (&x)[4], uint64_t (&out)[4]) const {
        uint32_t a[8], b[8], u[8], v[8];
        for (int i = 0; i < 8; i++) {
            a[i] = (uint32_t)(x[i >> 1] >> (32 * (i & 1)));
            b[i] = p32[i];
            u[i] = i == 0 ? 1u : 0u;
            v[i] = 0u;
        }
        for (int it = 0; it < 17; it++) {  // ceil((2 * 255 - 1) / 30) rounds: b = gcd = 1
            const int n = std::max(std::max(bitlen8(a), bitlen8(b)), 62);
            uint64_t ab = approx(a, n), bb = approx(b, n);
            int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
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
            if (lin(a, b, f0, g0, na)) {
                f0 = -f0;
                g0 = -g0;
            }
            if (lin(a, b, f1, g1, nb)) {
                f1 = -f1;
                g1 = -g1;
            }
            lin_mod(u, v, f0, g0, nu);
            lin_mod(u, v, f1, g1, nv);
            for (int i = 0; i < 8; i++) {
                a[i] = na[i];
                b[i] = nb[i];
                u[i] = nu[i];
                v[i] = nv[i];
            }
        }
        uint64_t r[4];
        for (int i = 0; i < 4; i++) r[i] = (uint64_t)v[2 * i] | ((uint64_t)v[2 * i + 1] << 32);
        mul(r, inv_fix, out);
    }
};

template <class F>
void host_xyzz_to_wrapped_t(const void* xyzz, void* wrapped) {
    static const HostMont M(F::MODULUS64);
    const uint64_t* q = (const uint64_t*)xyzz;
    uint64_t c[4][4];  // X, Y, ZZ, ZZZ reduced below p
    for (int k = 0; k < 4; k++) {
        for (int i = 0; i < 4; i++) c[k][i] = q[4 * k + i];
        if (M.geq_p(c[k])) M.sub_p(c[k]);
    }
    uint64_t* out = (uint64_t*)wrapped;
    if (!(c[2][0] | c[2][1] | c[2][2] | c[2][3])) {  // ZZ = 0: the identity, WrappedPoint (0, 0)
        for (int i = 0; i < 8; i++) out[i] = 0;
        return;
    }
    uint64_t m[4][4], t[4], iv[4], u[4], x[4], y[4];
    for (int k = 0; k < 4; k++) M.mul(c[k], M.r2, m[k]);  // to the Montgomery domain
    M.mul(m[2], m[3], t);
    M.inv(t, iv);  // (ZZ ZZZ)^-1
    M.mul(m[0], m[3], u);
    M.mul(u, iv, x);  // X / ZZ, times R
    M.mul(m[1], m[2], u);
    M.mul(u, iv, y);  // Y / ZZZ, times R
    for (int i = 0; i < 4; i++) {
        out[i] = x[i];
        out[4 + i] = y[i];
    }
}
// k points with one inversion (Montgomery's trick over the ZZ ZZZ products; k <= 16)
template <class F>
void host_xyzz_to_wrapped2_t(const void* const* xyzz, void* const* wrapped, int k) {
    static const HostMont M(F::MODULUS64);
    uint64_t m[16][4][4], t[16][4], pre[17][4];
    bool id[16];
    for (int j = 0; j < 4; j++) pre[0][j] = M.one[j];
    for (int i = 0; i < k; i++) {
        const uint64_t* q = (const uint64_t*)xyzz[i];
        uint64_t c[4][4];
        for (int a = 0; a < 4; a++) {
            for (int j = 0; j < 4; j++) c[a][j] = q[4 * a + j];
            if (M.geq_p(c[a])) M.sub_p(c[a]);
        }
        id[i] = !(c[2][0] | c[2][1] | c[2][2] | c[2][3]);
        for (int a = 0; a < 4; a++) M.mul(c[a], M.r2, m[i][a]);
        if (id[i])
            for (int j = 0; j < 4; j++) t[i][j] = M.one[j];
        else
            M.mul(m[i][2], m[i][3], t[i]);
        M.mul(pre[i], t[i], pre[i + 1]);
    }
    uint64_t inv[4];
    M.inv(pre[k], inv);  // (prod_i ZZ_i ZZZ_i)^-1
    for (int i = k - 1; i >= 0; i--) {
        uint64_t iv[4], u[4], x[4], y[4];
        M.mul(inv, pre[i], iv);  // (ZZ_i ZZZ_i)^-1
        M.mul(inv, t[i], inv);
        uint64_t* out = (uint64_t*)wrapped[i];
        if (id[i]) {
            for (int j = 0; j < 8; j++) out[j] = 0;
            continue;
        }
        M.mul(m[i][0], m[i][3], u);
        M.mul(u, iv, x);
        M.mul(m[i][1], m[i][2], u);
        M.mul(u, iv, y);
        for (int j = 0; j < 4; j++) {
            out[j] = x[j];
            out[4 + j] = y[j];
        }
    }
}
}  // namespace

void host_xyzz_to_wrapped2(int curve, const void* const* xyzz, void* const* wrapped, int k) {
    if (curve == HALO_PALLAS)
        host_xyzz_to_wrapped2_t<PallasCurve::Base>(xyzz, wrapped, k);
    else
        host_xyzz_to_wrapped2_t<VestaCurve::Base>(xyzz, wrapped, k);
}

template <class S>
static bool host_scalar_inverse_t(const void* x_ark, void* out_ark) {
    static const HostMont M(S::MODULUS64);
    uint64_t x[4];
    for (int i = 0; i < 4; i++) x[i] = ((const uint64_t*)x_ark)[i];
    if (M.geq_p(x)) M.sub_p(x);
    if (!(x[0] | x[1] | x[2] | x[3])) return false;
    uint64_t r[4];
    M.inv(x, r);  // Montgomery-domain inverse: (x R)^-1 R^2 = x^-1 R, the ark form of x^-1
    for (int i = 0; i < 4; i++) ((uint64_t*)out_ark)[i] = r[i];
    return true;
}
bool host_scalar_inverse(int curve, const void* x_ark, void* out_ark) {
    return curve == HALO_PALLAS ? host_scalar_inverse_t<PallasCurve::Scalar>(x_ark, out_ark)
                                : host_scalar_inverse_t<VestaCurve::Scalar>(x_ark, out_ark);
}

void host_xyzz_to_wrapped(int curve, const void* xyzz, void* wrapped) {
    if (curve == HALO_PALLAS)
        host_xyzz_to_wrapped_t<PallasCurve::Base>(xyzz, wrapped);
    else
        host_xyzz_to_wrapped_t<VestaCurve::Base>(xyzz, wrapped);
}

// Host-output entry points: the MSM leaves its sum as 128-B packed XYZZ on the device, and the affine
// conversion (one inversion) runs on the host after the copy -- not as a one-lane chain at the end
// of the reduction tail.
static int d2h_point(int curve, const void* d_xyzz, halo_wrapped_point_t* out, hipStream_t s) {
    alignas(16) uint64_t buf[16];
    HALO_CHECK(copy_d2h(buf, d_xyzz, 128, s));
    host_xyzz_to_wrapped(curve, buf, out);
    return HALO_OK;
}

int convert_wrapped_to_internal(int curve, const void* in, void* out, size_t n, hipStream_t s) {
    if (!n) return HALO_OK;
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_wrapped_to_internal<typename Cv::Base>, dim3(grid_for(n, 256)), dim3(256), 0, s,
                           (const uint4*)in, (uint4*)out, n);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

int convert_internal_to_wrapped(int curve, const void* in, void* out, size_t n, hipStream_t s) {
    if (!n) return HALO_OK;
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_internal_to_wrapped<typename Cv::Base>, dim3(grid_for(n, 256)), dim3(256), 0, s,
                           (const uint4*)in, (uint4*)out, n);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

// hiding table 2^i S (i < 256), internal affine
static int build_s_table(DeviceState* st, int curve, hipStream_t s) {
    SrsState& srs = st->srs[curve];
    HALO_CHECK(srs.s_table.reserve(256 * 64));
    HALO_CHECK(st->scratch[7].reserve(256 * 128 + 64));
    char* tmp = (char*)st->scratch[7].ptr;
    HALO_CHECK(copy_h2d(tmp + 256 * 128, srs.S, 64, s));
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_pow2_points<Cv>, dim3(1), dim3(64), 0, s, (const uint4*)(tmp + 256 * 128), (uint4*)tmp,
                           256);
        hipLaunchKernelGGL(k_xyzz_to_aff<Cv>, dim3(4), dim3(64), 0, s, (const uint4*)tmp, srs.s_table.as<uint4>(), 256);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

// The window-shifted copies 2^(c w) G_i for w in [w_lo, w_hi) (c = 0: the default width for the SRS
// length; w_hi = 0: every window).  The full set serves every SRS MSM; a partial range (one rank of a
// window-partitioned MSM, BASELINE configs[4]) serves halo_msm_srs_windows_dev over that range only.
int srs_precompute_windows(DeviceState* st, int curve, hipStream_t s, int c, int w_lo, int w_hi) {
    SrsState& srs = st->srs[curve];
    if (!srs.n) return set_error(HALO_ESRSRANGE, "no resident SRS to precompute");
    if (c == 0) c = msm_shifted_window_bits(srs.n);
    if (c < 2 || c > 20) return set_error(HALO_EINVAL, "window bits %d outside [2, 20]", c);
    const int W = msm_windows(c);
    if (w_hi == 0) w_hi = W;
    if (w_lo < 0 || w_hi > W || w_lo >= w_hi)
        return set_error(HALO_EINVAL, "window range [%d, %d) outside [0, %d)", w_lo, w_hi, W);
    srs.shifted_c = srs.part_c = 0;  // nothing valid while the copies are rewritten
    // asynchronous MSMs (halo_msm_srs_windows_dev, the pipelined MSM sets) and weighted IPA rounds on
    // other streams may still be reading the copies: drain the device before they are rewritten or
    // reallocated (a precompute is a setup step, never on a timed path)
    HALO_HIP(hipDeviceSynchronize());
    HALO_CHECK(srs.shifted.reserve((size_t)(w_hi - w_lo) * srs.n * 64));
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[7].reserve(4));
    uint32_t* flag = st->scratch[7].as<uint32_t>();
    HALO_HIP(hipMemsetAsync(flag, 0, 4, s));
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_shift_windows<Cv>, dim3(grid_for(srs.n, 64)), dim3(64), 0, s, srs.gs.as<const uint4>(),
                           srs.n, c, w_lo, w_hi, srs.shifted.as<uint4>(), flag);
    });
    HALO_HIP(hipGetLastError());
    uint32_t has_id = 1;
    HALO_HIP(hipMemcpyAsync(&has_id, flag, 4, hipMemcpyDeviceToHost, s));
    HALO_HIP(hipStreamSynchronize(s));
    srs.shifted_has_id = has_id != 0;
    if (w_lo == 0 && w_hi == W) {
        srs.shifted_c = c;
    } else {
        srs.part_c = c;
        srs.part_w0 = w_lo;
        srs.part_w1 = w_hi;
    }
    return HALO_OK;
}

}  // namespace halo

using namespace halo;

namespace halo {
// one block per row: row b sums the k WrappedPoints at pts_wrapped + 4 k b into out_wrapped + 4 b
template <class Cv>
__global__ __launch_bounds__(256) void k_point_sum(const uint4* pts_wrapped, size_t k, uint4* out_wrapped) {
    using F = typename Cv::Base;
    __shared__ uint4 red[256 * 8];
    pts_wrapped += 4 * k * (size_t)blockIdx.x;
    out_wrapped += 4 * (size_t)blockIdx.x;
    XYZZ<F> acc = xyzz_id<F>();
    for (size_t i = threadIdx.x; i < k; i += 256) acc = xyzz_madd(acc, aff_from_wrapped<F>(pts_wrapped + 4 * i));
    xyzz_store(red + 8 * threadIdx.x, acc);
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off)
            xyzz_store(red + 8 * threadIdx.x,
                       xyzz_add(xyzz_load<F>(red + 8 * threadIdx.x), xyzz_load<F>(red + 8 * (threadIdx.x + off))));
        __syncthreads();
    }
    if (threadIdx.x == 0) aff_to_wrapped(out_wrapped, xyzz_to_aff(xyzz_load<F>(red)));
}

// Sum of k packed XYZZ points (stride_bytes apart) -> packed XYZZ (no affine conversion on the device)
template <class Cv>
__global__ __launch_bounds__(256) void k_point_sum_xyzz(const uint4* pts, size_t k, size_t stride_u4, uint4* out) {
    using F = typename Cv::Base;
    __shared__ uint4 red[256 * 8];
    XYZZ<F> acc = xyzz_id<F>();
    for (size_t i = threadIdx.x; i < k; i += 256) acc = xyzz_add(acc, xyzz_load<F>(pts + stride_u4 * i));
    xyzz_store(red + 8 * threadIdx.x, acc);
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off)
            xyzz_store(red + 8 * threadIdx.x,
                       xyzz_add(xyzz_load<F>(red + 8 * threadIdx.x), xyzz_load<F>(red + 8 * (threadIdx.x + off))));
        __syncthreads();
    }
    if (threadIdx.x == 0) xyzz_store(out, xyzz_load<F>(red));
}

}  // namespace halo

static int check_curve(halo_curve_t c) {
    if (c != HALO_PALLAS && c != HALO_VESTA) return set_error(HALO_EINVAL, "unknown curve id %d", (int)c);
    return HALO_OK;
}

extern "C" int halo_msm_window_bits(size_t n) { return msm_window_bits(n); }

extern "C" int halo_srs_window_bits(halo_curve_t curve) {
    clear_error();
    if (curve != HALO_PALLAS && curve != HALO_VESTA) return set_error(HALO_EINVAL, "unknown curve id %d", (int)curve);
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    const SrsState& srs = st->srs[curve];
    return srs.shifted_c ? srs.shifted_c : srs.part_c;
}

extern "C" int halo_point_sum(halo_curve_t curve, const halo_wrapped_point_t* pts, size_t k, halo_wrapped_point_t* out) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!out || (k && !pts)) return set_error(HALO_EINVAL, "halo_point_sum: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(k, 1) * 64 + 64));
    char* buf = (char*)st->scratch[0].ptr;
    HALO_CHECK(copy_h2d(buf + 64, pts, k * 64, s));
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_point_sum<Cv>, dim3(1), dim3(256), 0, s, (const uint4*)(buf + 64), k, (uint4*)buf);
    });
    HALO_HIP(hipGetLastError());
    return copy_d2h(out, buf, 64, s);
}

extern "C" int halo_point_sum_dev(halo_curve_t curve, const void* d_pts, size_t k, size_t stride_bytes, void* d_out,
                                  void* stream) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!d_out || (k && !d_pts)) return set_error(HALO_EINVAL, "halo_point_sum_dev: null buffer");
    if (stride_bytes != 64) return set_error(HALO_EINVAL, "halo_point_sum_dev: only contiguous (64-B stride) points");
    hipStream_t s = (hipStream_t)stream;
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_point_sum<Cv>, dim3(1), dim3(256), 0, s, (const uint4*)d_pts, k, (uint4*)d_out);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_point_sum_rows_dev(halo_curve_t curve, const void* d_pts, size_t rows, size_t k, void* d_out,
                                       void* stream) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!rows) return HALO_OK;
    if (!d_out || (k && !d_pts)) return set_error(HALO_EINVAL, "halo_point_sum_rows_dev: null buffer");
    if (rows > 65535) return set_error(HALO_EINVAL, "halo_point_sum_rows_dev: %zu rows (at most 65535)", rows);
    hipStream_t s = (hipStream_t)stream;
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_point_sum<Cv>, dim3((unsigned)rows), dim3(256), 0, s, (const uint4*)d_pts, k, (uint4*)d_out);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_point_sum_xyzz_dev(halo_curve_t curve, const void* d_pts, size_t k, size_t stride_bytes, void* d_out,
                                       void* stream) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!d_out || (k && !d_pts)) return set_error(HALO_EINVAL, "halo_point_sum_xyzz_dev: null buffer");
    if (stride_bytes < 128 || stride_bytes % 16)
        return set_error(HALO_EINVAL, "halo_point_sum_xyzz_dev: stride %zu (a multiple of 16, at least 128)", stride_bytes);
    hipStream_t s = (hipStream_t)stream;
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_point_sum_xyzz<Cv>, dim3(1), dim3(256), 0, s, (const uint4*)d_pts, k, stride_bytes / 16,
                           (uint4*)d_out);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_xyzz_to_wrapped(halo_curve_t curve, const void* xyzz, size_t k, halo_wrapped_point_t* out) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (k && (!xyzz || !out)) return set_error(HALO_EINVAL, "halo_xyzz_to_wrapped: null buffer");
    for (size_t i = 0; i < k; i++) host_xyzz_to_wrapped(curve, (const char*)xyzz + 128 * i, out + i);
    return HALO_OK;
}

extern "C" int halo_srs_read(halo_curve_t curve, size_t offset, size_t n, halo_wrapped_point_t* out) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!out && n) return set_error(HALO_EINVAL, "halo_srs_read: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    if (offset + n > srs.n) return set_error(HALO_ESRSRANGE, "range [%zu, %zu) exceeds the SRS length %zu", offset, offset + n, srs.n);
    if (!n) return HALO_OK;
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(n * 64));
    HALO_CHECK(convert_internal_to_wrapped(curve, srs.gs.as<const char>() + offset * 64, st->scratch[0].ptr, n, s));
    return copy_d2h(out, st->scratch[0].ptr, n * 64, s);
}

extern "C" void halo_synth_scalar(halo_curve_t curve, uint64_t seed, uint64_t j, uint64_t out_canonical[4]) {
    (void)curve;
    synth_scalar(seed, j, out_canonical);
}

namespace halo {
// ark Projective (Jacobian X, Y, Z, Montgomery, 96 B) -> internal affine; Z = 0 -> (0, 0).  One
// Fermat inversion per lane (Projective::normalize_batch of point_dot, group.rs:53-56).
template <class Cv>
__global__ void k_jacobian_to_internal(const uint4* in, uint4* out, size_t n) {
    using F = typename Cv::Base;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Fe<F> Z = fe_from_ark<F>(in + 6 * i + 4);
    Affine<F> a;
    if (fe_is_zero(Z)) {
        a.x = fe_zero<F>();
        a.y = fe_zero<F>();
    } else {
        const Fe<F> zi = fe_inv(Z);
        const Fe<F> zi2 = fe_sqr(zi);
        a.x = fe_mul(fe_from_ark<F>(in + 6 * i), zi2);
        a.y = fe_mul(fe_from_ark<F>(in + 6 * i + 2), fe_mul(zi2, zi));
    }
    aff_store(out + 4 * i, a);
}
}  // namespace halo

// group::point_dot(xs, &[Projective]) (crates/group/src/group.rs:53-56): the bases arrive as ark
// Projective (Jacobian) points, normalised on the device, then the MSM of halo_msm.
extern "C" int halo_point_dot_projective(halo_curve_t curve, const halo_fe_t* scalars, size_t n_scalars,
                                         const uint64_t (*bases)[12], size_t n_bases, halo_wrapped_point_t* out) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    const size_t n = std::min(n_bases, n_scalars);
    if (!out || (n && (!bases || !scalars))) return set_error(HALO_EINVAL, "halo_point_dot_projective: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(n, 1) * 96));
    HALO_CHECK(st->scratch[1].reserve(std::max<size_t>(n, 1) * 64));
    HALO_CHECK(st->scratch[2].reserve(std::max<size_t>(n, 1) * 32));
    HALO_CHECK(st->scratch[3].reserve(128));
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, bases, n * 96, s));
    HALO_CHECK(copy_h2d(st->scratch[2].ptr, scalars, n * 32, s));
    if (n) {
        DISPATCH_CURVE(curve, Cv, {
            hipLaunchKernelGGL(k_jacobian_to_internal<Cv>, dim3(grid_for(n, 256)), dim3(256), 0, s,
                               st->scratch[0].as<const uint4>(), st->scratch[1].as<uint4>(), n);
        });
        HALO_HIP(hipGetLastError());
    }
    HALO_CHECK(msm_device(st, curve, st->scratch[1].ptr, st->scratch[2].ptr, n, nullptr, nullptr, st->scratch[3].ptr, s,
                          false, false, true));
    return d2h_point(curve, st->scratch[3].ptr, out, s);
}

// host arrays: bases (ark WrappedPoint), scalars (ark) -> out (host)
extern "C" int halo_msm(halo_curve_t curve, const halo_wrapped_point_t* bases, size_t n_bases,
                        const halo_fe_t* scalars, size_t n_scalars, halo_wrapped_point_t* out) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    const size_t n = std::min(n_bases, n_scalars);
    if (!out || (n && (!bases || !scalars))) return set_error(HALO_EINVAL, "halo_msm: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(n, 1) * 64));
    HALO_CHECK(st->scratch[1].reserve(std::max<size_t>(n, 1) * 64));
    HALO_CHECK(st->scratch[2].reserve(std::max<size_t>(n, 1) * 32));
    HALO_CHECK(st->scratch[3].reserve(128));
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, bases, n * 64, s));
    HALO_CHECK(copy_h2d(st->scratch[2].ptr, scalars, n * 32, s));
    HALO_CHECK(convert_wrapped_to_internal(curve, st->scratch[0].ptr, st->scratch[1].ptr, n, s));
    if (n >= 1 && n <= msm_tiny_max()) {  // a few points: GLV windows + one 32-window Horner (ipa.hip)
        HALO_CHECK(st->scratch[3].reserve(128 + 32 * 128));
        HALO_CHECK(msm_tiny(curve, st->scratch[1].ptr, st->scratch[2].ptr, n, st->scratch[3].as<char>() + 128,
                            st->scratch[3].ptr, s));
    } else {
        HALO_CHECK(msm_device(st, curve, st->scratch[1].ptr, st->scratch[2].ptr, n, nullptr, nullptr, st->scratch[3].ptr,
                              s, false, false, true));
    }
    return d2h_point(curve, st->scratch[3].ptr, out, s);
}

// SRS management --------------------------------------------------------------------------------
// Installs n WrappedPoints already in device memory (d_wrapped, may be scratch[0]) as the resident
// SRS of `curve`, plus (S, H) when given (host WrappedPoints).
static int srs_install(DeviceState* st, int curve, const void* d_wrapped, size_t n, const halo_wrapped_point_t* S,
                       const halo_wrapped_point_t* H, hipStream_t s) {
    SrsState& srs = st->srs[curve];
    HALO_CHECK(srs.gs.reserve(std::max<size_t>(n, 1) * 64));
    HALO_CHECK(convert_wrapped_to_internal(curve, d_wrapped, srs.gs.ptr, n, s));
    srs.n = n;
    srs.invalidate_derived();
    if (S && H) {
        HALO_CHECK(st->scratch[1].reserve(256));
        char* tmp = (char*)st->scratch[1].ptr;
        HALO_CHECK(copy_h2d(tmp, S, 64, s));
        HALO_CHECK(copy_h2d(tmp + 64, H, 64, s));
        HALO_CHECK(convert_wrapped_to_internal(curve, tmp, tmp + 128, 2, s));
        HALO_CHECK(copy_d2h(srs.S, tmp + 128, 64, s));
        HALO_CHECK(copy_d2h(srs.H, tmp + 192, 64, s));
        srs.H_wrapped = *H;
        srs.has_sh = true;
        HALO_CHECK(build_s_table(st, curve, s));
    }
    HALO_HIP(hipStreamSynchronize(s));
    return HALO_OK;
}

extern "C" int halo_srs_upload(halo_curve_t curve, const halo_wrapped_point_t* gs, size_t n,
                               const halo_wrapped_point_t* S, const halo_wrapped_point_t* H) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if ((n && !gs)) return set_error(HALO_EINVAL, "halo_srs_upload: null gs");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(n, 2) * 64));
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, gs, n * 64, s));
    return srs_install(st, curve, st->scratch[0].ptr, n, S, H, s);
}

// ---------------------------------------------------------------------------------------------
// the SRS wire format (bincode-v2 `standard()` Vec<WrappedPoint> per block,
// pp.rs:36-53; (S, H) tuple in sh.bin) decoded on the device.  A block whose records are all in the
// fixed 72-byte form (every u64 limb as 0xFD + 8 LE bytes -- what the reference's generator writes
// for Montgomery limbs >= 2^32) is decoded by k_decode_points, one record per lane; any other
// record (a small limb gets a shorter varint) sends that block through the sequential host decoder.
// Every point is then checked on the curve on the device (wrappers.rs:606 `assert!(is_on_curve)`).
// ---------------------------------------------------------------------------------------------
__global__ void k_decode_points(const uint8_t* rec0, size_t count, uint4* out, uint32_t* bad) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint8_t* r = rec0 + 72 * i;
    uint32_t w[16];
    bool ok = true;
#pragma unroll
    for (int l = 0; l < 8; l++) {
        const uint8_t* f = r + 9 * l;
        ok &= (f[0] == 0xFD);
        w[2 * l] = (uint32_t)f[1] | ((uint32_t)f[2] << 8) | ((uint32_t)f[3] << 16) | ((uint32_t)f[4] << 24);
        w[2 * l + 1] = (uint32_t)f[5] | ((uint32_t)f[6] << 8) | ((uint32_t)f[7] << 16) | ((uint32_t)f[8] << 24);
    }
    if (!ok) atomicOr(bad, 1u);
    out[4 * i] = make_uint4(w[0], w[1], w[2], w[3]);
    out[4 * i + 1] = make_uint4(w[4], w[5], w[6], w[7]);
    out[4 * i + 2] = make_uint4(w[8], w[9], w[10], w[11]);
    out[4 * i + 3] = make_uint4(w[12], w[13], w[14], w[15]);
}

template <class Cv>
__global__ void k_check_on_curve(const uint4* pts_wrapped, size_t n, uint32_t* bad) {
    using F = typename Cv::Base;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Affine<F> a = aff_from_wrapped<F>(pts_wrapped + 4 * i);
    // y^2 == x^3 + 5 (the identity (0, 0) is not on the curve, as for ark's Affine::new_unchecked)
    const Fe<F> lhs = fe_sqr(a.y);
    const Fe<F> rhs = fe_add(fe_mul(fe_sqr(a.x), a.x), fe_from_const<F>(Cv::K::B));
    if (!fe_eq(lhs, rhs)) atomicAdd(bad, 1u);
}

// bincode-v2 standard() unsigned varint
static bool bc_varint(const uint8_t* b, size_t len, size_t& off, uint64_t& v) {
    if (off >= len) return false;
    const uint8_t t = b[off];
    if (t < 251) {
        v = t;
        off += 1;
        return true;
    }
    const int width = t == 251 ? 2 : t == 252 ? 4 : t == 253 ? 8 : 0;
    if (!width || off + 1 + width > len) return false;
    v = 0;
    for (int i = 0; i < width; i++) v |= (uint64_t)b[off + 1 + i] << (8 * i);
    off += 1 + width;
    return true;
}

static bool bc_point(const uint8_t* b, size_t len, size_t& off, halo_wrapped_point_t& p) {
    for (int l = 0; l < 4; l++)
        if (!bc_varint(b, len, off, p.x[l])) return false;
    for (int l = 0; l < 4; l++)
        if (!bc_varint(b, len, off, p.y[l])) return false;
    return true;
}

extern "C" int halo_srs_load_bincode(halo_curve_t curve, const uint8_t* const* blocks, const size_t* block_lens,
                                     size_t nblocks, const uint8_t* sh, size_t sh_len, size_t n) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!is_pow2(n)) return set_error(HALO_ENOTPOW2, "assertion failed: n.is_power_of_two()");
    if (nblocks && (!blocks || !block_lens)) return set_error(HALO_EINVAL, "halo_srs_load_bincode: null blocks");
    halo_wrapped_point_t SH[2];
    if (sh) {
        size_t off = 0;
        if (!bc_point(sh, sh_len, off, SH[0]) || !bc_point(sh, sh_len, off, SH[1]))
            return set_error(HALO_EINVAL, "Failed to get SH data for curve %s", curve == HALO_PALLAS ? "pallas" : "vesta");
    }
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(n, 2) * 64));
    HALO_CHECK(st->scratch[2].reserve(16));
    uint4* d_pts = st->scratch[0].as<uint4>();
    uint32_t* d_bad = st->scratch[2].as<uint32_t>();
    size_t have = 0;
    std::vector<halo_wrapped_point_t> host_pts;
    for (size_t bi = 0; bi < nblocks && have < n; bi++) {
        const uint8_t* b = blocks[bi];
        const size_t len = block_lens[bi];
        size_t off = 0;
        uint64_t count = 0;
        if (!b || !bc_varint(b, len, off, count)) return set_error(HALO_EINVAL, "Failed to decode G_BLOCKS_NO %zu", bi);
        const size_t take = std::min<size_t>(count, n - have);
        bool fast = (len - off) >= 72 * take;
        if (fast && take) {
            HALO_CHECK(st->scratch[3].reserve(72 * take));
            HALO_HIP(hipMemsetAsync(d_bad, 0, 4, s));
            HALO_CHECK(copy_h2d(st->scratch[3].ptr, b + off, 72 * take, s));
            hipLaunchKernelGGL(k_decode_points, dim3(grid_for(take, 256)), dim3(256), 0, s,
                               st->scratch[3].as<const uint8_t>(), take, d_pts + 4 * have, d_bad);
            HALO_HIP(hipGetLastError());
            uint32_t bad = 0;
            HALO_CHECK(copy_d2h(&bad, d_bad, 4, s));
            fast = (bad == 0);
        }
        if (!fast) {  // general varints: sequential host decode of this block
            host_pts.resize(take);
            for (size_t i = 0; i < take; i++)
                if (!bc_point(b, len, off, host_pts[i])) return set_error(HALO_EINVAL, "Failed to decode G_BLOCKS_NO %zu", bi);
            HALO_CHECK(copy_h2d(d_pts + 4 * have, host_pts.data(), take * 64, s));
        }
        have += take;
    }
    if (have < n) return set_error(HALO_ESRSRANGE, "assertion failed: n <= N (%zu points available)", have);
    HALO_HIP(hipMemsetAsync(d_bad, 0, 4, s));
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_check_on_curve<Cv>, dim3(grid_for(n, 256)), dim3(256), 0, s, (const uint4*)d_pts, n, d_bad);
    });
    HALO_HIP(hipGetLastError());
    uint32_t bad = 0;
    HALO_CHECK(copy_d2h(&bad, d_bad, 4, s));
    if (bad) return set_error(HALO_EINVAL, "assertion failed: affine.is_on_curve() (%u points)", bad);
    return srs_install(st, curve, d_pts, n, sh ? &SH[0] : nullptr, sh ? &SH[1] : nullptr, s);
}

// PublicParams' (S, H) (pp.rs:26-61) as ark WrappedPoints
extern "C" int halo_srs_sh(halo_curve_t curve, halo_wrapped_point_t* S, halo_wrapped_point_t* H) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!S || !H) return set_error(HALO_EINVAL, "halo_srs_sh: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    if (!srs.has_sh) return set_error(HALO_ESRSRANGE, "no (S, H) uploaded");
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(256));
    char* b = st->scratch[0].as<char>();
    HALO_CHECK(copy_h2d(b, srs.S, 64, s));
    HALO_CHECK(copy_h2d(b + 64, srs.H, 64, s));
    HALO_CHECK(convert_internal_to_wrapped(curve, b, b + 128, 2, s));
    HALO_CHECK(copy_d2h(S, b + 128, 64, s));
    return copy_d2h(H, b + 192, 64, s);
}

extern "C" int halo_srs_len(halo_curve_t curve, size_t* n) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!n) return set_error(HALO_EINVAL, "null n");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    *n = st->srs[curve].n;
    return HALO_OK;
}

extern "C" int halo_srs_synthesize(halo_curve_t curve, size_t n, uint64_t seed) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    SrsState& srs = st->srs[curve];
    HALO_CHECK(srs.gs.reserve(std::max<size_t>(n, 1) * 64));
    if (n) {
        DISPATCH_CURVE(curve, Cv, {
            hipLaunchKernelGGL(k_synth_bases<Cv>, dim3(grid_for(n, 64)), dim3(64), 0, s, srs.gs.as<uint4>(), n, seed);
        });
        HALO_HIP(hipGetLastError());
    }
    HALO_HIP(hipStreamSynchronize(s));
    srs.n = n;
    srs.invalidate_derived();
    return HALO_OK;
}

extern "C" int halo_srs_precompute_windows(halo_curve_t curve) {
    return halo_srs_precompute_window_range(curve, 0, 0, 0);
}

extern "C" int halo_srs_precompute_window_range(halo_curve_t curve, int c, int w_lo, int w_hi) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    ScratchUse su(st, 0);
    return srs_precompute_windows(st, curve, 0, c, w_lo, w_hi);
}

extern "C" int halo_msm_srs(halo_curve_t curve, const halo_fe_t* scalars, size_t n, halo_wrapped_point_t* out) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!out || (n && !scalars)) return set_error(HALO_EINVAL, "halo_msm_srs: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[2].reserve(std::max<size_t>(n, 1) * 32));
    HALO_CHECK(st->scratch[3].reserve(128));
    HALO_CHECK(copy_h2d(st->scratch[2].ptr, scalars, n * 32, s));
    HALO_CHECK(msm_srs_device(st, curve, st->scratch[2].ptr, n, nullptr, st->scratch[3].ptr, s, false, true));
    return d2h_point(curve, st->scratch[3].ptr, out, s);
}

extern "C" int halo_msm_dev(halo_curve_t curve, const void* d_bases, const void* d_scalars, size_t n,
                            halo_wrapped_point_t* out, void* stream) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!out || (n && !d_scalars)) return set_error(HALO_EINVAL, "halo_msm_dev: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = (hipStream_t)stream;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[7].reserve(128));
    if (!d_bases) {
        HALO_CHECK(msm_srs_device(st, curve, d_scalars, n, nullptr, st->scratch[7].ptr, s, false, true));
    } else {
        HALO_CHECK(st->scratch[6].reserve(std::max<size_t>(n, 1) * 64));
        HALO_CHECK(convert_wrapped_to_internal(curve, d_bases, st->scratch[6].ptr, n, s));
        HALO_CHECK(msm_device(st, curve, st->scratch[6].ptr, d_scalars, n, nullptr, nullptr, st->scratch[7].ptr, s,
                              false, false, true));
    }
    return d2h_point(curve, st->scratch[7].ptr, out, s);
}

extern "C" int halo_msm_dev_async(halo_curve_t curve, const void* d_bases, const void* d_scalars, size_t n,
                                  void* d_out, void* stream) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!d_out || (n && !d_scalars)) return set_error(HALO_EINVAL, "halo_msm_dev_async: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = (hipStream_t)stream;
    if (!d_bases) return msm_srs_device(st, curve, d_scalars, n, nullptr, d_out, s, true);
    // the set is claimed once: its previous tail is waited for before the conversion overwrites conv,
    // and the MSM runs on that same set
    int set = -1;
    DevBuf* conv = nullptr;
    HALO_CHECK(msm_claim_set(st, s, &set, &conv));
    HALO_CHECK(conv->reserve(std::max<size_t>(n, 1) * 64));
    HALO_CHECK(convert_wrapped_to_internal(curve, d_bases, conv->ptr, n, s));
    return msm_device(st, curve, conv->ptr, d_scalars, n, nullptr, nullptr, d_out, s, true, false, false, nullptr,
                      set);
}

namespace halo {
// k commitments over the resident SRS prefix (lens[i] scalars at d_scalars[i]) -> d_out + 64 i,
// asynchronous on s (msm_join before reading)
int msm_batch_device(DeviceState* st, int curve, const void* const* d_scalars, const size_t* lens, size_t k, void* d_out,
                     hipStream_t s) {
    SrsState& srs = st->srs[curve];
    size_t nmax = 0;
    for (size_t i = 0; i < k; i++) {
        if (lens[i] && !d_scalars[i]) return set_error(HALO_EINVAL, "halo_msm_batch_dev: null scalars %zu", i);
        if (lens[i] > srs.n) return set_error(HALO_ESRSRANGE, "n (%zu) exceeds the resident SRS length (%zu)", lens[i], srs.n);
        nmax = std::max(nmax, lens[i]);
    }
    // (Measured and removed: the fronts on a side stream beside the accumulations -- slower, the
    // sort kernels starve beside k_acc's gathers)
    if (k > 1 && srs.shifted_c && nmax <= msm_multi_max()) {
        int rc;
        DISPATCH_CURVE(curve, Cv, { rc = msm_multi_device_t<Cv>(st, d_scalars, lens, k, (uint4*)d_out, s); });
        return rc;
    }
    for (size_t i = 0; i < k; i++)
        HALO_CHECK(msm_srs_device(st, curve, d_scalars[i], lens[i], nullptr, (char*)d_out + 64 * i, s, true));
    return HALO_OK;
}
}  // namespace halo

extern "C" int halo_msm_batch_dev(halo_curve_t curve, const void* const* d_scalars, const size_t* lens, size_t k,
                                  void* d_out, void* stream) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (k && (!d_scalars || !lens || !d_out)) return set_error(HALO_EINVAL, "halo_msm_batch_dev: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    return msm_batch_device(st, curve, d_scalars, lens, k, d_out, (hipStream_t)stream);
}

// One rank's share of a window-partitioned MSM over the resident window-shifted SRS (BASELINE
// configs[4]): the digits of windows [w_lo, w_hi) only, against the copies 2^(c w) G, w in range; the
// partials of a partition of [0, W) sum to the MSM.  Asynchronous like halo_msm_dev_async.
extern "C" int halo_msm_srs_windows_dev(halo_curve_t curve, const void* d_scalars, size_t n, int w_lo, int w_hi,
                                        void* d_out, void* stream) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!d_out || (n && !d_scalars)) return set_error(HALO_EINVAL, "halo_msm_srs_windows_dev: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    // the full set of copies, or this rank's range of them (halo_srs_precompute_window_range)
    const int c = srs.shifted_c ? srs.shifted_c : srs.part_c;
    const int w0 = srs.shifted_c ? 0 : srs.part_w0, w1 = srs.shifted_c ? msm_windows(c) : srs.part_w1;
    if (!c) return set_error(HALO_EINVAL, "halo_msm_srs_windows_dev: no window-shifted SRS");
    if (n > srs.n) return set_error(HALO_ESRSRANGE, "n (%zu) exceeds the resident SRS length (%zu)", n, srs.n);
    if (w_hi <= w_lo) return set_error(HALO_EINVAL, "empty window range [%d, %d)", w_lo, w_hi);
    if (w_lo < w0 || w_hi > w1)
        return set_error(HALO_EINVAL, "window range [%d, %d) not resident (copies of [%d, %d))", w_lo, w_hi, w0, w1);
    int rc;
    DISPATCH_CURVE(curve, Cv, {
        rc = msm_device_t<Cv>(st, srs.shifted.as<const uint4>(), true, srs.n, (const uint4*)d_scalars, n, c, nullptr,
                              nullptr, (uint4*)d_out, (hipStream_t)stream, true, 32, false, false, nullptr, -1, w_lo,
                              w_hi, w0);
    });
    return rc;
}

extern "C" int halo_srs_windows(halo_curve_t curve) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    const SrsState& srs = st->srs[curve];
    const int c = srs.shifted_c ? srs.shifted_c : srs.part_c;
    return c ? msm_windows(c) : 0;
}

extern "C" int halo_msm_join(void* stream) {
    clear_error();
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    return msm_join(st, (hipStream_t)stream);
}

// pedersen::commit(w, Gs, ms) -- crates/accumulation/src/pedersen.rs:7-27
extern "C" int halo_pedersen_commit(halo_curve_t curve, const halo_fe_t* w, const halo_wrapped_point_t* gs,
                                    size_t n_gs, const halo_fe_t* ms, size_t n_ms, halo_wrapped_point_t* out) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!out || (n_ms && !ms) || (n_gs && !gs)) return set_error(HALO_EINVAL, "halo_pedersen_commit: null buffer");
    if (n_gs < n_ms)
        return set_error(HALO_ELENGTH, "ms must be larger than Gs: (Gs: %zu), (ms: %zu)", n_gs, n_ms);
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    if (w && !srs.has_sh) return set_error(HALO_ESRSRANGE, "hiding commitment needs S: upload the SRS (S, H) first");
    hipStream_t s = 0;
    ScratchUse su(st, s);
    const size_t n = n_ms;
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(n, 1) * 64));
    HALO_CHECK(st->scratch[1].reserve(std::max<size_t>(n, 1) * 64));
    HALO_CHECK(st->scratch[2].reserve(std::max<size_t>(n, 1) * 32));
    HALO_CHECK(st->scratch[3].reserve(128 + 32));
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, gs, n * 64, s));
    HALO_CHECK(copy_h2d(st->scratch[2].ptr, ms, n * 32, s));
    HALO_CHECK(convert_wrapped_to_internal(curve, st->scratch[0].ptr, st->scratch[1].ptr, n, s));
    char* small = (char*)st->scratch[3].ptr;  // [0, 128) the XYZZ sum, [128, 160) w
    if (w) HALO_CHECK(copy_h2d(small + 128, w, 32, s));
    HALO_CHECK(msm_device(st, curve, st->scratch[1].ptr, st->scratch[2].ptr, n, w ? srs.s_table.ptr : nullptr,
                          w ? small + 128 : nullptr, small, s, false, false, true));
    return d2h_point(curve, small, out, s);
}

static size_t poly_degree(const halo_fe_t* c, size_t len) {
    // DensePolynomial::degree(): index of the last nonzero coefficient (0 for the zero polynomial)
    size_t n = len;
    while (n > 0 && !(c[n - 1].l[0] | c[n - 1].l[1] | c[n - 1].l[2] | c[n - 1].l[3])) n--;
    return n ? n - 1 : 0;
}

// pcdl::commit(p, d, w) -- crates/accumulation/src/pcdl.rs:275-287
extern "C" int halo_pcdl_commit(halo_curve_t curve, const halo_fe_t* coeffs, size_t len, size_t d,
                                const halo_fe_t* w, halo_wrapped_point_t* out) {
    clear_error();
    HALO_CHECK(check_curve(curve));
    if (!out || (len && !coeffs)) return set_error(HALO_EINVAL, "halo_pcdl_commit: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    if (!srs.n) return set_error(HALO_ESRSRANGE, "no resident SRS: call halo_srs_upload first");
    const size_t D = srs.n - 1;
    const size_t n = d + 1;
    const size_t p_deg = poly_degree(coeffs, len);
    if (!is_pow2(n)) return set_error(HALO_ENOTPOW2, "n (%zu) is not a power of two", n);
    if (p_deg > d) return set_error(HALO_EDEGREE, "p_deg (%zu) <= d (%zu)", p_deg, d);
    if (d > D) return set_error(HALO_ESRSRANGE, "d (%zu) <= D (%zu) (pp_len = %zu)", d, D, D + 1);
    if (w && !srs.has_sh) return set_error(HALO_ESRSRANGE, "hiding commitment needs S: upload the SRS (S, H) first");
    // coefficients past the degree are zero and contribute nothing to the MSM
    const size_t m = std::min(len, n);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[2].reserve(std::max<size_t>(m, 1) * 32));
    HALO_CHECK(st->scratch[3].reserve(128 + 32));
    HALO_CHECK(copy_h2d(st->scratch[2].ptr, coeffs, m * 32, s));
    char* small = (char*)st->scratch[3].ptr;  // [0, 128) the XYZZ sum, [128, 160) w
    if (w) HALO_CHECK(copy_h2d(small + 128, w, 32, s));
    HALO_CHECK(msm_srs_device(st, curve, st->scratch[2].ptr, m, w ? small + 128 : nullptr, small, s, false, true));
    return d2h_point(curve, small, out, s);
}
