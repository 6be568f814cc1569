// Stable LSD radix sort of the MSM's (bucket key, point reference) pairs (part of SURVEY §8 row a3).
//
// ark-ec's CPU Pippenger scatters every point straight into its bucket (a random read-modify-write
// per point per window).  On MI355X the buckets are instead formed by sorting the W*n digit entries
// by bucket key, so the accumulation kernel reads each bucket's points as one contiguous run.
//
// Design (per 8-bit digit pass, tiles of 8192 entries, 512 threads):
//   k_rs_hist    : per-tile LDS histogram of the digit -> hist[tile][digit] (coalesced)
//                  and, by the kernel's last arrivers, the digit-major exclusive prefix of that table
//                  without transposing it -> every tile's global run start per digit
//   k_rs_scatter : stable in-tile ranking (each wave ranks its own contiguous quarter of the tile with
//                  ballots that find equal digits among lanes; per-wave histograms order the waves),
//                  the tile is staged in LDS in digit order and written back as contiguous runs per
//                  digit (coalesced).
// Pass 0 reads the raw digit array (skipping zero digits) and forms key = window * B + |d| - 1 and
// value = point index | sign; later passes read the previous pass's pairs.  The number of valid
// entries is known only on the device (scan total) -- kernels bound themselves by it, so no host
// round trip is needed.
#include <algorithm>
#include <utility>
#include <vector>
#include <type_traits>
#include <cstdlib>

#include "digits.hpp"
#include "dispatch.hpp"
#include "fields.hpp"
#include "runtime.hpp"
#include "sort.hpp"

namespace halo {

constexpr int RS_THREADS = 512;
// Tiles of RS_THREADS x 16 rounds: 8192 entries, runs of ~32 entries = 128 B per digit, 64 KB of LDS
// staging.  (Measured: 4096-entry tiles, 4 workgroups per CU, were no faster.)
constexpr int RS_BINS = 256;      // bins of an 8-bit digit pass
constexpr int RS_BINS_MAX = 512;  // ... of a 9-bit pass (17- / 18-bit keys in two passes)
// tile rounds of a digit pass: 16 (8192 entries) for 8-bit digits; 14 for 9-bit digits, whose
// per-wave histograms (8 x 512 words) would otherwise leave one scatter workgroup per CU
template <int BITS>
constexpr int rs_rounds() { return BITS == 8 ? 16 : 14; }
constexpr size_t RS_STAGE_BYTES = 2 * 4 * RS_THREADS * 16;  // k_rs_scatter's key / value staging
constexpr uint32_t RS_NONE = 0xffffffffu;

// The scalars of a fused first pass: P outputs of n scalars each (output p at s[p], keys offset by p B)
struct RsScalars {
    const uint4* s[8] = {};
    uint32_t n = 0, P = 1, B = 0;
};
// (output p of the global scalar g and its scalar's address: a select chain, not a dynamic index into
// the kernel-argument array, which would go through scratch memory)
HALO_DEV const uint4* rs_scalar(const RsScalars& sc, uint32_t g, uint32_t& p, uint32_t& i) {
    p = sc.P == 1 ? 0u : g / sc.n;
    i = g - p * sc.n;
    const uint4* src = sc.s[0];
#pragma unroll
    for (uint32_t q = 1; q < 8; q++)
        if (p == q) src = sc.s[q];
    return src + 2 * (size_t)i;
}

struct RsIn {
    RsScalars sc;  // fused pass 0: the ark scalars (k_rs_hist_sc / k_rs_scatter<.., S>)
    int c = 0, W = 0;
    const uint32_t* digits;  // pass 0 only
    const uint32_t* keys;    // later passes
    const uint32_t* vals;
    const uint32_t* count;   // device count of valid entries (later passes)
    size_t E;                // pass 0: number of digit entries
    size_t npw;              // pass 0: entries per window (key = (e / npw) * B + |d| - 1)
    uint32_t B;
    uint32_t pass;
    uint32_t shift;  // digit = (key >> shift) & 255
};

// Entry e of the pass input, in two phases so that a thread's loads for all its rounds are issued
// back to back: rs_load reads the raw words at a clamped index (no control flow depends on loaded
// data; the arrays hold at least one word), rs_decode then forms (key, val) or rejects the entry.
// PASS0: a = digit (val unused); later passes: a = key, b = val (b only when WANT_VAL).
template <bool PASS0, bool WANT_VAL = true>
HALO_DEV void rs_load(const RsIn& in, size_t e, size_t limit, uint32_t& a, uint32_t& b) {
    const size_t ec = e < limit ? e : (limit ? limit - 1 : 0);
    if constexpr (PASS0) {
        a = in.digits[ec];
        b = 0;
    } else {
        a = in.keys[ec];
        b = WANT_VAL ? in.vals[ec] : 0u;
    }
}
template <bool PASS0>
HALO_DEV bool rs_decode(const RsIn& in, size_t e, size_t limit, uint32_t a, uint32_t b, uint32_t& key, uint32_t& val) {
    if (e >= limit) return false;
    if constexpr (PASS0) {
        if (a == RS_NONE) return false;
        // entries < 2^32; one window (npw >= E) needs no division
        const uint32_t w = (in.npw >= in.E) ? 0u : (uint32_t)e / (uint32_t)in.npw;
        key = w * in.B + (a & 0x7fffffffu);
        val = ((uint32_t)e - w * (uint32_t)in.npw) | (a & 0x80000000u);
    } else {
        key = a;
        val = b;
    }
    return true;
}

HALO_DEV size_t rs_limit(const RsIn& in) { return in.pass == 0 ? in.E : (size_t)*in.count; }

// Offsets from the tile-major histogram, by the histogram kernel's last arrivers (no separate scan
// launches, no spinning): each workgroup publishes its row (sc1 stores, drained) and counts itself in
// its chunk of RS_CH tiles; the chunk's last arriver scans the chunk's rows per digit (in-chunk
// exclusive prefix, in place) and publishes the chunk total; the last chunk to finish scans the chunk
// totals per digit and adds the digit's base (exclusive scan of the digit totals).  Tile t's run for
// digit d then starts at hist[t][d] + chunk[t / RS_CH][d].  Pass 0 also stores the number of valid
// entries.  Hand-off protocol (MI355X_MICROARCH.md, inter-workgroup visibility): every handed-off
// word stored sc1 and drained before a workgroup barrier and the agent-scope counter add; the
// consumer is the workgroup whose add returned the last count, which takes an agent-scope acquire
// before reading.  The counters (ctr[0..nchunks), ctr[nchunks]) are reset by their last arriver.
constexpr int RS_CH = 64;
#define RS_RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
HALO_DEV void rs_acquire() {  // one lane's agent acquire, then the whole workgroup waits for it
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}
// true in the workgroup whose add to *c returned total - 1 (every workgroup's stores drained first)
HALO_DEV bool rs_last_arriver(uint32_t* c, uint32_t total, uint32_t* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(c, 1u, RS_RLX_AGENT) == total - 1;
    __syncthreads();
    return *flag != 0;
}
template <int BINS>
HALO_DEV void rs_publish_and_scan(const uint32_t* h, uint32_t tile, uint32_t ntiles, uint32_t* hist, uint32_t* chunk,
                                  uint32_t* ctr, uint32_t* count) {
    static_assert(BINS <= RS_THREADS, "one thread per digit");
    constexpr int DPL = BINS / 64;  // digits per lane of the wave-0 scan
    __shared__ uint32_t flag;
    __shared__ uint32_t s[BINS];
    const uint32_t d = threadIdx.x;
    if (d < BINS) __hip_atomic_store(hist + (size_t)tile * BINS + d, h[d], RS_RLX_AGENT);
    const uint32_t ch = tile / RS_CH, nchunks = (ntiles + RS_CH - 1) / RS_CH;
    const uint32_t t0 = ch * RS_CH, nt = min((uint32_t)RS_CH, ntiles - t0);
    if (!rs_last_arriver(ctr + ch, nt, &flag)) return;
    rs_acquire();
    if (d < BINS) {
        uint32_t v[RS_CH];
#pragma unroll
        for (int i = 0; i < RS_CH; i++) v[i] = (i < (int)nt) ? hist[(size_t)(t0 + i) * BINS + d] : 0u;
        uint32_t run = 0;
#pragma unroll
        for (int i = 0; i < RS_CH; i++) {
            if (i < (int)nt) hist[(size_t)(t0 + i) * BINS + d] = run;  // read by the scatter launch
            run += v[i];
        }
        __hip_atomic_store(chunk + (size_t)ch * BINS + d, run, RS_RLX_AGENT);
    }
    if (d == 0) __hip_atomic_store(ctr + ch, 0u, RS_RLX_AGENT);
    if (!rs_last_arriver(ctr + nchunks, nchunks, &flag)) return;
    rs_acquire();
    // per digit: total over the chunks, then (after the digit scan) the chunks' exclusive prefix plus
    // the digit's base; the loads go in batches of U so their latencies overlap
    constexpr uint32_t U = 16;
    if (d < BINS) {
        uint32_t run = 0;
        for (uint32_t c0 = 0; c0 < nchunks; c0 += U) {
            uint32_t v[U];
#pragma unroll
            for (uint32_t i = 0; i < U; i++) v[i] = (c0 + i < nchunks) ? chunk[(size_t)(c0 + i) * BINS + d] : 0u;
#pragma unroll
            for (uint32_t i = 0; i < U; i++) run += v[i];
        }
        s[d] = run;
    }
    __syncthreads();
    // exclusive scan of the digit totals (wave 0: DPL digits per lane)
    if (d < 64) {
        uint32_t c[DPL], sum = 0;
#pragma unroll
        for (int q = 0; q < DPL; q++) {
            c[q] = s[d * DPL + q];
            sum += c[q];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(incl, off);
            if ((int)d >= off) incl += t;
        }
        uint32_t ex = incl - sum;
#pragma unroll
        for (int q = 0; q < DPL; q++) {
            s[d * DPL + q] = ex;
            ex += c[q];
        }
        if (d == 63 && count) *count = incl;
    }
    __syncthreads();
    if (d < BINS) {
        uint32_t run = s[d];
        for (uint32_t c0 = 0; c0 < nchunks; c0 += U) {
            uint32_t v[U];
#pragma unroll
            for (uint32_t i = 0; i < U; i++) v[i] = (c0 + i < nchunks) ? chunk[(size_t)(c0 + i) * BINS + d] : 0u;
#pragma unroll
            for (uint32_t i = 0; i < U; i++) {
                if (c0 + i < nchunks) chunk[(size_t)(c0 + i) * BINS + d] = run;
                run += v[i];
            }
        }
    }
    if (d == 0) __hip_atomic_store(ctr + nchunks, 0u, RS_RLX_AGENT);
}

template <int BITS, bool PASS0>
__global__ __launch_bounds__(RS_THREADS) void k_rs_hist(RsIn in, uint32_t ntiles, uint32_t* hist, uint32_t* chunk,
                                                        uint32_t* ctr, uint32_t* count) {
    constexpr int ROUNDS = rs_rounds<BITS>();
    constexpr int BINS = 1 << BITS;
    constexpr int RS_TILE = RS_THREADS * ROUNDS;
    __shared__ uint32_t h[BINS];
    if (threadIdx.x < BINS) h[threadIdx.x] = 0;
    const size_t limit = rs_limit(in);
    const size_t base = (size_t)blockIdx.x * RS_TILE;
    // every round's load in flight before the first use (keys only: the histogram needs no values)
    uint32_t A[ROUNDS], Bv[ROUNDS];
#pragma unroll
    for (int r = 0; r < ROUNDS; r++)
        rs_load<PASS0, false>(in, base + (size_t)r * RS_THREADS + threadIdx.x, limit, A[r], Bv[r]);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ROUNDS; r++) {
        uint32_t k, v;
        if (rs_decode<PASS0>(in, base + (size_t)r * RS_THREADS + threadIdx.x, limit, A[r], Bv[r], k, v))
            atomicAdd(&h[(k >> in.shift) & (BINS - 1u)], 1u);
    }
    __syncthreads();
    rs_publish_and_scan<BINS>(h, blockIdx.x, ntiles, hist, chunk, ctr, count);
}

// Fused first pass of the window-shifted MSM's sort (single bucket set): the entries are recoded
// from the scalars here instead of being written by k_digits and read back (32 B of scalar per
// W = 15 entries instead of 2 x 4 B per entry).  Thread = one scalar, round = window: a tile is
// RS_THREADS scalars x W windows.  Entry key = |d| - 1, value = (w n + i) | sign, as k_digits + pass 0.
// (P > 1 outputs: key p B + |d| - 1 has the same low byte as |d| - 1, B being a multiple of 256)
template <class S>
__global__ __launch_bounds__(RS_THREADS) void k_rs_hist_sc(const RsScalars sc, int c, int W, uint32_t ntiles,
                                                         uint32_t* hist, uint32_t* chunk, uint32_t* ctr,
                                                         uint32_t* count) {
    __shared__ uint32_t h[RS_BINS];
    if (threadIdx.x < RS_BINS) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t g = blockIdx.x * RS_THREADS + threadIdx.x;
    if (g < sc.P * sc.n) {
        uint32_t p, i;
        scalar_signed_digits<S>(rs_scalar(sc, g, p, i), c, W, [&](int, uint32_t d) {
            if (d != DIGIT_NONE) atomicAdd(&h[d & 255u], 1u);
        });
    }
    __syncthreads();
    rs_publish_and_scan<RS_BINS>(h, blockIdx.x, ntiles, hist, chunk, ctr, count);
}

// Each wave owns a contiguous eighth of the tile (1024 entries, 16 rounds of 64), so ranking is
// wave-local (ballots + a wave-private LDS run counter per digit) and the workgroup needs only
// three barriers: after the per-wave histograms, after the prefix, after staging.
// SF: void, or the scalar field of a fused first pass (k_rs_hist_sc's entries, in.sc != null)
template <int BITS, class SF = void, bool PASS0 = false>
__global__ __launch_bounds__(RS_THREADS) void k_rs_scatter(RsIn in, const uint32_t* tile_off, const uint32_t* chunk_off,
                                                           uint32_t* keys_out, uint32_t* vals_out) {
    constexpr int ROUNDS = rs_rounds<BITS>();
    constexpr int BINS = 1 << BITS;
    constexpr uint32_t DMASK = BINS - 1;
    constexpr int DPL = BINS / 64;
    constexpr int RS_TILE = RS_THREADS * ROUNDS;
    constexpr int WAVES = RS_THREADS / 64;
    constexpr int PER_WAVE = RS_TILE / WAVES;  // 1024 (8-bit digits) / 896 (9-bit)
    __shared__ uint32_t goff[BINS];           // global start of this tile's run per digit
    __shared__ uint32_t lstart[BINS];         // tile-local start per digit
    __shared__ uint32_t wpos[WAVES][BINS];    // per-wave histogram, then per-wave next position
    // the staging arrays (64 KB) are dynamic LDS (RS_STAGE_BYTES at launch): with a static size the
    // compiler derives the LDS-limited occupancy (4 waves per SIMD) and pads the VGPR allocation to
    // match it (76 used -> 97 allocated), which would keep the workgroup from being resident beside
    // the previous MSM's tail kernels (k_merge: 2 waves per SIMD of 161 VGPRs).  (Measured: 2^20
    // headline unchanged, 1.337 vs 1.336 ms -- the front and the tail contend for VALU issue, not slots.)
    static_assert(2 * 4 * RS_TILE <= RS_STAGE_BYTES, "staging size");
    extern __shared__ uint32_t rs_stage[];
    uint32_t* skey = rs_stage;
    uint32_t* sval = rs_stage + RS_TILE;
    __shared__ uint32_t total;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t limit = rs_limit(in);
    const size_t wbase = (size_t)blockIdx.x * RS_TILE + (size_t)wave * PER_WAVE;
    constexpr int R = PER_WAVE / 64;
    uint32_t K[R], V[R];
    uint32_t validmask = 0;
    if constexpr (!std::is_void<SF>::value) {
        // fused first pass: this lane's scalar, its W windows as the rounds
#pragma unroll
        for (int r = 0; r < R; r++) {
            K[r] = 0;
            V[r] = 0;
        }
        const uint32_t g = blockIdx.x * RS_THREADS + tid;
        if (g < in.sc.P * in.sc.n) {
            uint32_t p, i;
            const uint4* src = rs_scalar(in.sc, g, p, i);
            const uint32_t koff = p * in.sc.B;
            scalar_signed_digits<SF, R>(src, in.c, in.W, [&](int w, uint32_t d) {
                if (d != DIGIT_NONE) {
                    K[w] = koff + (d & 0x7fffffffu);
                    V[w] = ((uint32_t)w * in.sc.n + i) | (d & 0x80000000u);
                    validmask |= 1u << w;
                }
            });
        }
    } else {
        // all loads of the tile issued back to back (memory-level parallelism), kept in registers
        uint32_t A[R], Bv[R];
#pragma unroll
        for (int r = 0; r < R; r++) rs_load<PASS0>(in, wbase + (size_t)r * 64 + lane, limit, A[r], Bv[r]);
#pragma unroll
        for (int r = 0; r < R; r++) {
            K[r] = 0;
            V[r] = 0;
            if (rs_decode<PASS0>(in, wbase + (size_t)r * 64 + lane, limit, A[r], Bv[r], K[r], V[r])) validmask |= 1u << r;
        }
    }
    if (tid < BINS) {
        goff[tid] = tile_off[(size_t)blockIdx.x * BINS + tid] + chunk_off[(size_t)(blockIdx.x / RS_CH) * BINS + tid];
#pragma unroll
        for (int w = 0; w < WAVES; w++) wpos[w][tid] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; r++)
        if ((validmask >> r) & 1u) atomicAdd(&wpos[wave][(K[r] >> in.shift) & DMASK], 1u);
    __syncthreads();
    // thread tid = digit: tile-local exclusive prefix over digits (wave-0 shuffle scan of 4 digits/lane)
    if (tid < BINS) {
        uint32_t cnt = 0;
#pragma unroll
        for (int w = 0; w < WAVES; w++) cnt += wpos[w][tid];
        lstart[tid] = cnt;
    }
    __syncthreads();
    if (wave == 0) {
        uint32_t c[DPL];
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < DPL; q++) {
            c[q] = lstart[lane * DPL + q];
            sum += c[q];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(incl, off);
            if (lane >= off) incl += t;
        }
        uint32_t ex = incl - sum;
#pragma unroll
        for (int q = 0; q < DPL; q++) {
            lstart[lane * DPL + q] = ex;
            ex += c[q];
        }
        if (lane == 63) total = incl;
    }
    __syncthreads();
    if (tid < BINS) {
        uint32_t p = lstart[tid];
#pragma unroll
        for (int w = 0; w < WAVES; w++) {
            const uint32_t c = wpos[w][tid];
            wpos[w][tid] = p;
            p += c;
        }
    }
    __syncthreads();
    // The first pass needs no stability (the second, by the high byte, must keep the first's order,
    // but the order of equal full keys is free: k_acc's bucket sums do not depend on it), so it ranks
    // with the wave-private run counter's returning LDS add -- one ds_add_rtn per entry instead of the
    // eight-ballot match below (~40 VALU per round).
    if constexpr (PASS0 || !std::is_void<SF>::value) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (!((validmask >> r) & 1u)) continue;
            const uint32_t pos = atomicAdd(&wpos[wave][(K[r] >> in.shift) & DMASK], 1u);
            skey[pos] = K[r];
            sval[pos] = V[r];
        }
    } else {
    // stable, wave-local ranking: 16 rounds of 64 consecutive entries
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint32_t k = K[r], v = V[r];
        const bool valid = (validmask >> r) & 1u;
        const uint32_t dg = (k >> in.shift) & DMASK;
        uint64_t same = __ballot(valid);
#pragma unroll
        for (int b = 0; b < BITS; b++) {
            const uint64_t m = __ballot((dg >> b) & 1u);
            same &= ((dg >> b) & 1u) ? m : ~m;
        }
        const uint64_t below = same & ((1ull << lane) - 1ull);
        if (valid) {
            const uint32_t pos = wpos[wave][dg] + (uint32_t)__popcll(below);
            skey[pos] = k;
            sval[pos] = v;
        }
        __builtin_amdgcn_wave_barrier();
        if (valid && below == 0) wpos[wave][dg] += (uint32_t)__popcll(same);
        __builtin_amdgcn_wave_barrier();
    }
    }
    __syncthreads();
    // write runs: staging index i belongs to digit dg, global position goff[dg] + (i - lstart[dg])
    for (uint32_t i = tid; i < total; i += RS_THREADS) {
        const uint32_t k = skey[i];
        const uint32_t dg = (k >> in.shift) & DMASK;
        const uint32_t g = goff[dg] + (i - lstart[dg]);
        if (g >= in.E) continue;  // inconsistent offsets: never write outside the arrays
        keys_out[g] = k;
        vals_out[g] = sval[i];
    }
}

// bstart[b] = first position of key b in the sorted keys (b <= NB; bstart[NB] = count)
__global__ void k_bucket_starts(const uint32_t* keys, const uint32_t* count, size_t NB, size_t cap, uint32_t* bstart) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t n = *count;
    if (e > n || e > cap) return;
    const int64_t prev = (e == 0) ? -1 : (int64_t)keys[e - 1];
    const int64_t cur = (e == n) ? (int64_t)NB : (int64_t)keys[e];
    for (int64_t b = prev + 1; b <= cur; b++) bstart[b] = (uint32_t)e;
}

// exclusive scan (3 kernels) of n u32 -> out[0..n], out[n] = total
constexpr int SC_THREADS = 1024;
__device__ inline uint32_t sc_block_excl(uint32_t v, uint32_t* s, uint32_t* total) {
    s[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < SC_THREADS; off <<= 1) {
        const uint32_t t = ((int)threadIdx.x >= off) ? s[threadIdx.x - off] : 0;
        __syncthreads();
        s[threadIdx.x] += t;
        __syncthreads();
    }
    const uint32_t incl = s[threadIdx.x];
    *total = s[SC_THREADS - 1];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(SC_THREADS) void k_sc_reduce(const uint32_t* in, size_t n, size_t per, uint32_t* sums) {
    __shared__ uint32_t s[SC_THREADS];
    const size_t beg = (size_t)blockIdx.x * per, end = min(n, beg + per);
    uint32_t acc = 0;
    for (size_t i = beg + threadIdx.x; i < end; i += SC_THREADS) acc += in[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int off = SC_THREADS / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = s[0];
}

__global__ __launch_bounds__(SC_THREADS) void k_sc_sums(uint32_t* sums, int nb) {
    __shared__ uint32_t s[SC_THREADS];
    const int per = (nb + SC_THREADS - 1) / SC_THREADS;
    uint32_t loc[8];
    uint32_t acc = 0;
    for (int k = 0; k < per; k++) {
        const int i = threadIdx.x * per + k;
        loc[k] = (i < nb) ? sums[i] : 0;
        acc += loc[k];
    }
    uint32_t tot;
    uint32_t ex = sc_block_excl(acc, s, &tot);
    for (int k = 0; k < per; k++) {
        const int i = threadIdx.x * per + k;
        if (i < nb) sums[i] = ex;
        ex += loc[k];
    }
    if (threadIdx.x == 0) sums[nb] = tot;
}

__global__ __launch_bounds__(SC_THREADS) void k_sc_apply(const uint32_t* in, size_t n, size_t per, const uint32_t* sums,
                                                         uint32_t* out) {
    __shared__ uint32_t s[SC_THREADS];
    const size_t beg = (size_t)blockIdx.x * per, end = min(n, beg + per);
    uint32_t base = sums[blockIdx.x];
    for (size_t tile = beg; tile < end; tile += (size_t)SC_THREADS * 4) {
        uint32_t loc[4];
        uint32_t acc = 0;
        for (int k = 0; k < 4; k++) {
            const size_t i = tile + (size_t)threadIdx.x * 4 + k;
            loc[k] = (i < end) ? in[i] : 0;
            acc += loc[k];
        }
        uint32_t tot;
        uint32_t ex = sc_block_excl(acc, s, &tot) + base;
        for (int k = 0; k < 4; k++) {
            const size_t i = tile + (size_t)threadIdx.x * 4 + k;
            if (i < end) out[i] = ex;
            ex += loc[k];
        }
        base += tot;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = sums[gridDim.x];
}

int device_exclusive_scan(const uint32_t* in, size_t n, uint32_t* out, DevBuf& tmp, hipStream_t s) {
    const size_t per = (size_t)SC_THREADS * 16;
    size_t nb = std::max<size_t>(1, (n + per - 1) / per);
    if (nb > (size_t)SC_THREADS * 8) return set_error(HALO_EINVAL, "scan too large (%zu)", n);
    HALO_CHECK(tmp.reserve((nb + 1) * 4));
    hipLaunchKernelGGL(k_sc_reduce, dim3((unsigned)nb), dim3(SC_THREADS), 0, s, in, n, per, tmp.as<uint32_t>());
    hipLaunchKernelGGL(k_sc_sums, dim3(1), dim3(SC_THREADS), 0, s, tmp.as<uint32_t>(), (int)nb);
    hipLaunchKernelGGL(k_sc_apply, dim3((unsigned)nb), dim3(SC_THREADS), 0, s, in, n, per, tmp.as<const uint32_t>(),
                       out);
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

// Digit passes (shift, bits) for key_bits-bit keys: 8-bit passes up to 16 bits; 17 / 18 bits in two
// passes with a 9-bit one (the IPA's paired L / R MSMs: key = (side, 16-bit bucket)) instead of a third
// pass; wider keys in 8-bit passes.  A fused first pass (recoding from the scalars) is always 8 bits.
static std::vector<std::pair<uint32_t, uint32_t>> rs_plan(uint32_t key_bits, bool fused) {
    std::vector<std::pair<uint32_t, uint32_t>> P;
    if (key_bits == 17 || (key_bits == 18 && !fused)) {
        const uint32_t b0 = (key_bits == 18) ? 9 : 8;
        P.push_back({0, b0});
        P.push_back({b0, key_bits - b0});
        return P;
    }
    const uint32_t passes = std::max<uint32_t>(1, (key_bits + 7) / 8);
    for (uint32_t p = 0; p < passes; p++) P.push_back({8 * p, 8});
    return P;
}

int msm_radix_sort(const uint32_t* digits, size_t E, size_t npw, uint32_t B, uint32_t key_bits, SortScratch& S,
                   uint32_t** keys_out, uint32_t** vals_out, const uint32_t** count_out, uint32_t* bstart, size_t NB,
                   hipStream_t s, const RsFused* fused) {
    const auto plan = rs_plan(key_bits, fused != nullptr);
    auto tiles_of = [&](uint32_t bits) {
        const size_t tile = (size_t)RS_THREADS * (bits == 8 ? rs_rounds<8>() : rs_rounds<9>());
        return (uint32_t)std::max<size_t>(1, (E + tile - 1) / tile);
    };
    uint32_t ntmax = 1;
    for (auto& q : plan) ntmax = std::max(ntmax, tiles_of(q.second));
    // fused first pass: tiles of RS_THREADS scalars x W windows
    const size_t nsc = fused ? fused->n * (size_t)fused->P : 0;
    if (fused && (fused->P < 1 || fused->P > 8 || fused->W > rs_rounds<8>() || nsc >= (1ull << 31) / 16))
        return set_error(HALO_EINVAL, "fused sort pass: %d outputs, %d windows, %zu scalars", fused->P, fused->W, nsc);
    const uint32_t ntiles0 = fused ? (uint32_t)std::max<size_t>(1, (nsc + RS_THREADS - 1) / RS_THREADS) : 0u;
    ntmax = std::max(ntmax, ntiles0);
    HALO_CHECK(S.keys[0].reserve(std::max<size_t>(E, 1) * 4));
    HALO_CHECK(S.keys[1].reserve(std::max<size_t>(E, 1) * 4));
    HALO_CHECK(S.vals[0].reserve(std::max<size_t>(E, 1) * 4));
    HALO_CHECK(S.vals[1].reserve(std::max<size_t>(E, 1) * 4));
    HALO_CHECK(S.hist.reserve((size_t)RS_BINS_MAX * ntmax * 4));
    const size_t nchmax = (ntmax + RS_CH - 1) / RS_CH;
    HALO_CHECK(S.offs.reserve(nchmax * RS_BINS_MAX * 4));
    HALO_CHECK(S.count.reserve(16));
    // the last-arriver counters start at zero and are reset by their last arrivers
    // (a reallocation may return the freed address: the capacity, not the pointer, tells)
    const size_t ctr_had = S.ctr.bytes;
    HALO_CHECK(S.ctr.reserve((nchmax + 1) * 4));
    if (S.ctr.bytes != ctr_had) HALO_HIP(hipMemsetAsync(S.ctr.ptr, 0, S.ctr.bytes, s));
    int cur = 0;
    for (uint32_t p = 0; p < (uint32_t)plan.size(); p++) {
        const uint32_t bits = plan[p].second;
        RsIn in;
        in.digits = digits;
        in.keys = S.keys[cur ^ 1].as<const uint32_t>();
        in.vals = S.vals[cur ^ 1].as<const uint32_t>();
        in.count = S.count.as<const uint32_t>();
        in.E = E;
        in.npw = npw;
        in.B = B;
        in.pass = p;
        in.shift = plan[p].first;
        const bool fp = fused && p == 0;
        const uint32_t nt = fp ? ntiles0 : tiles_of(bits);
        uint32_t* hist = S.hist.as<uint32_t>();
        uint32_t* offs = S.offs.as<uint32_t>();
        if (fp) {
            for (int q = 0; q < 8; q++)
                in.sc.s[q] = (const uint4*)(fused->P == 1 ? (q == 0 ? fused->scalars : nullptr) : fused->srcs[q]);
            in.sc.n = (uint32_t)fused->n;
            in.sc.P = (uint32_t)fused->P;
            in.sc.B = B;
            in.c = fused->c;
            in.W = fused->W;
            DISPATCH_FIELD(fused->field, SF, {
                hipLaunchKernelGGL(k_rs_hist_sc<SF>, dim3(nt), dim3(RS_THREADS), 0, s, in.sc, in.c, in.W, nt,
                                   hist, offs, S.ctr.as<uint32_t>(), S.count.as<uint32_t>());
                hipLaunchKernelGGL((k_rs_scatter<8, SF>), dim3(nt), dim3(RS_THREADS), RS_STAGE_BYTES, s, in,
                                   (const uint32_t*)hist, (const uint32_t*)offs, S.keys[cur].as<uint32_t>(),
                                   S.vals[cur].as<uint32_t>());
            });
        } else {
            // pass 0 also stores the number of valid (nonzero-digit) entries
            uint32_t* cnt = p == 0 ? S.count.as<uint32_t>() : nullptr;
            if (bits == 9) {
                auto kh = p == 0 ? k_rs_hist<9, true> : k_rs_hist<9, false>;
                auto ks = p == 0 ? k_rs_scatter<9, void, true> : k_rs_scatter<9, void, false>;
                hipLaunchKernelGGL(kh, dim3(nt), dim3(RS_THREADS), 0, s, in, nt, hist, offs, S.ctr.as<uint32_t>(), cnt);
                // (the exact staging: 2 x 4 B x 7168 entries, so two workgroups fit in a CU's LDS)
                hipLaunchKernelGGL(ks, dim3(nt), dim3(RS_THREADS), 2 * 4 * RS_THREADS * rs_rounds<9>(), s, in,
                                   (const uint32_t*)hist, (const uint32_t*)offs, S.keys[cur].as<uint32_t>(),
                                   S.vals[cur].as<uint32_t>());
            } else {
                auto kh = p == 0 ? k_rs_hist<8, true> : k_rs_hist<8, false>;
                auto ks = p == 0 ? k_rs_scatter<8, void, true> : k_rs_scatter<8, void, false>;
                hipLaunchKernelGGL(kh, dim3(nt), dim3(RS_THREADS), 0, s, in, nt, hist, offs, S.ctr.as<uint32_t>(), cnt);
                hipLaunchKernelGGL(ks, dim3(nt), dim3(RS_THREADS), RS_STAGE_BYTES, s, in, (const uint32_t*)hist,
                                   (const uint32_t*)offs, S.keys[cur].as<uint32_t>(), S.vals[cur].as<uint32_t>());
            }
        }
        HALO_HIP(hipGetLastError());
        cur ^= 1;
    }
    *keys_out = S.keys[cur ^ 1].as<uint32_t>();
    *vals_out = S.vals[cur ^ 1].as<uint32_t>();
    *count_out = S.count.as<const uint32_t>();
    if (bstart) HALO_CHECK(msm_bucket_starts(*keys_out, S.count.as<const uint32_t>(), NB, E, bstart, s));
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

int msm_bucket_starts(const uint32_t* keys, const uint32_t* count, size_t NB, size_t E, uint32_t* bstart, hipStream_t s) {
    hipLaunchKernelGGL(k_bucket_starts, dim3((unsigned)((E + 1 + 255) / 256)), dim3(256), 0, s, keys, count, NB, E,
                       bstart);
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

}  // namespace halo
