// MSM reduction tail: chunk-partial merge, the bucket reduction
// sum_i (i + 1) B_i per window and the Horner over the windows (k_final; since the quad-cooperative
// doublings it is latency-bound like the rest, so it takes this unit's per-column multiplication).
//
// Every kernel here is latency-bound (a few waves doing dependent chains of curve additions).  They use
// the same per-column asm multiplication as the throughput kernels (round 3 measured it against the
// compiler's split column sums: 382 vs 418 ns per dependent modmul on one wave,
// tools/micro/fe_mul_bench.hip; the split form was removed in round 4).
#include <algorithm>
#include <cstdlib>

#include "dispatch.hpp"
#include "msm.hpp"
#include "runtime.hpp"
#include "sort.hpp"
#include "tree.hpp"


namespace halo {

// Skew guard: sums of MSM_GROUP consecutive chunk partials whose entries all belong to one bucket
// (level 1: groups of 64 chunks from first[]; level 2: groups of 64 level-1 groups), so that a huge
// bucket (all-equal scalars) is merged in O(chunks / 4096 + 128) sequential adds, not O(chunks).
template <class Cv>
__global__ __launch_bounds__(MSM_GROUP) void k_group_sums(const uint32_t* keys, const uint32_t* count, uint32_t K,
                                                          uint32_t span, const uint4* src, uint4* out) {
    using F = typename Cv::Base;
    static_assert(MSM_GROUP == 64, "one wave per group");
    const uint32_t g = blockIdx.x, i = threadIdx.x;
    const uint32_t cnt = *count;
    const size_t e0 = (size_t)g * MSM_GROUP * span * K, e1 = e0 + (size_t)MSM_GROUP * span * K;
    if (e1 > cnt || keys[e0] != keys[e1 - 1]) return;  // not one bucket throughout: never used (uniform)
    const XYZZ<F> v = wave_group_sum<F>(partial_load<F>(src + PARTIAL_U4 * ((size_t)g * MSM_GROUP + i)), 64);
    if (i == 0) partial_store(out + PARTIAL_U4 * (size_t)g, v);
}

// Buckets that touch a chunk boundary (or are empty): bucket b's entries [s, e) lie in chunks
// t0 = s / K .. t1 = (e - 1) / K.  Chunk t0 contributes first[t0] when the bucket starts it (s = t0 K),
// else last[t0]; every later chunk t <= t1 starts inside the bucket, so it contributes first[t] -- no
// key lookups, the sources follow from s, e and K alone; whole aligned groups strictly inside (t0, t1]
// come from the group sums.  A bucket strictly inside one chunk was written by k_acc.  The loop is
// software-pipelined: the next source's 128 B are loaded before the current addition, so each
// step's memory latency hides under the previous addition (the lane's chain is latency-bound).
template <class Cv, int LN>
__global__ __launch_bounds__(256) void k_merge(const uint32_t* bstart, const uint32_t* count, uint32_t K, size_t nb,
                                               const uint4* first, const uint4* last, const uint4* g1, const uint4* g2,
                                               uint4* bucket_sums) {
    using F = typename Cv::Base;
    // LN lanes per bucket (aligned groups of consecutive lanes): lane j sums the j-th contiguous part of
    // the bucket's sources, then the parts meet in a shuffle tree -- the chain per lane is 1 / LN as
    // long and the grid holds LN times the waves (one lane per bucket leaves one wave per SIMD, each
    // stalled on its dependent additions)
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t b = gid / LN;
    const uint32_t j = (uint32_t)(gid % LN);
    bool active = false, starts = false;
    uint32_t t0 = 0, t1 = 0;
    if (b < nb) {
        const uint32_t s = bstart[b], e = bstart[b + 1];
        if (s == e) {
            if (j == 0) xyzz_store(bucket_sums + 8 * b, xyzz_id<F>());
        } else {
            const uint32_t cnt = *count;
            t0 = s / K;
            t1 = (e - 1) / K;
            starts = s == t0 * K;  // the bucket is chunk t0's first segment
            active = !(t0 == t1 && !starts && e < min(cnt, (t0 + 1) * K));  // interior: done by k_acc
        }
    }
    XYZZ<F> acc = xyzz_id<F>();
    if (active) {
        // this lane's sources: chunks (t0, t1] split in LN contiguous parts [t, tb]
        const uint32_t total = t1 - t0, per = (total + LN - 1) / LN;
        uint32_t t = t0 + 1 + j * per;
        const uint32_t tb = min(t1, t0 + (j + 1) * per);
        constexpr uint32_t G2 = MSM_GROUP * MSM_GROUP;
        auto next_src = [&]() -> const uint4* {
            const uint4* src;
            if (t % G2 == 0 && t + G2 <= tb) {
                src = g2 + PARTIAL_U4 * (size_t)(t / G2);
                t += G2;
            } else if (t % MSM_GROUP == 0 && t + MSM_GROUP <= tb) {
                src = g1 + PARTIAL_U4 * (size_t)(t / MSM_GROUP);
                t += MSM_GROUP;
            } else {
                src = first + PARTIAL_U4 * (size_t)t;
                t++;
            }
            return src;
        };
        // chunk t0's partial starts lane 0's sum (no addition to the identity); one addition per step,
        // so lanes that take different sources do not execute several inlined copies of it
        if (j == 0) acc = partial_load<F>((starts ? first : last) + PARTIAL_U4 * (size_t)t0);
        else if (t <= tb) acc = partial_load<F>(next_src());
        if (t <= tb) {
            XYZZ<F> nxt = partial_load<F>(next_src());
            for (;;) {
                const XYZZ<F> cur = nxt;
                const bool more = t <= tb;
                if (more) nxt = partial_load<F>(next_src());
                acc = xyzz_add(acc, cur);
                if (!more) break;
            }
        }
    }
    for (int m = 1; m < LN; m <<= 1) acc = xyzz_add(acc, xyzz_shfl_xor(acc, m));
    if (active && j == 0) xyzz_store(bucket_sums + 8 * b, acc);
}

// ---------------------------------------------------------------------------------------------
// 6. per-window reduction  S_w = sum_{i<B} (i + 1) BS[w][i], organised for low dependency depth
//    (every stage is latency-bound: a lone XYZZ add is ~14 dependent modmuls).  View the buckets as
//    H rows x L columns, i = h L + l:
//      sum_i (i + 1) BS_i = sum_h R_h + L sum_h h R_h + sum_l l C_l,
//      R_h = sum_l BS[h L + l] (row sums), C_l = sum_h BS[h L + l] (column sums),
//      sum_h h R_h = sum_j 2^j U_j, U_j = sum_{h : bit j of h} R_h, and likewise V_j for the columns.
//    k_rowcol: R and C (tree sums, depth ~12); k_bitterms: sum_h R_h, U_j, V_j (independent tree
//    sums, depth ~12); k_bitcombine: lane k doubles its term (<= log B times), then a tree sum.
//    ~2.1 B adds in total at depth ~40 (a running-sum reduction needs 2 B adds at depth 2 B / #threads).
// ---------------------------------------------------------------------------------------------
// grid (rowcol_blocks(L, H, epl).x, SW), 256 threads.  epl: entries per lane (1, 2 or 4; rowcol_epl) --
// a lane first adds its epl entries of a row or column, then groups of L / epl (rows) or
// min(256, H / epl) (columns) lanes sum them as one tree each, several rows / columns to a block.  The
// launch is latency-bound: enough entries per lane keep it at one wave per SIMD (the 2^20 pair MSM's
// 2 x 2^16 buckets as 1024 one-entry blocks put four waves on each SIMD; a block per short column left
// three of its waves idle).
struct RowcolShape {
    uint32_t gr, rpb, nrb, gc, cpb, ncb;
};
__host__ __device__ __forceinline__ RowcolShape rowcol_shape(uint32_t L, uint32_t H, uint32_t epl) {
    RowcolShape r;
    r.gr = L / epl;
    r.rpb = 256 / r.gr;
    r.nrb = (H + r.rpb - 1) / r.rpb;
    r.gc = H / epl < 256 ? H / epl : 256;
    r.cpb = 256 / r.gc;
    r.ncb = (L + r.cpb - 1) / r.cpb;
    return r;
}
template <class Cv>
__global__ __launch_bounds__(256) void k_rowcol(const uint4* bucket_sums, uint32_t L, uint32_t H, uint32_t epl, uint4* rows,
                                                uint4* cols) {
    using F = typename Cv::Base;
    __shared__ uint4 red[128 * 8];
    const uint32_t w = blockIdx.y, tid = threadIdx.x;
    const uint4* bs = bucket_sums + 8 * (size_t)w * L * H;
    const RowcolShape sh = rowcol_shape(L, H, epl);
    XYZZ<F> v = xyzz_id<F>();
    if (blockIdx.x < sh.nrb) {  // (uniform per block) rows: groups of gr lanes
        const uint32_t h = blockIdx.x * sh.rpb + tid / sh.gr, l0 = tid % sh.gr;
        if (h < H)
            for (uint32_t l = l0; l < L; l += sh.gr) v = xyzz_add(v, xyzz_load<F>(bs + 8 * ((size_t)h * L + l)));
        v = block_group_sum<F>(v, sh.gr, red);
        if (l0 == 0 && h < H) xyzz_store(rows + 8 * ((size_t)w * H + h), v);
    } else {  // columns: groups of gc lanes
        const uint32_t l = (blockIdx.x - sh.nrb) * sh.cpb + tid / sh.gc, h0 = tid % sh.gc;
        if (l < L)
            for (uint32_t h = h0; h < H; h += sh.gc) v = xyzz_add(v, xyzz_load<F>(bs + 8 * ((size_t)h * L + l)));
        v = block_group_sum<F>(v, sh.gc, red);
        if (h0 == 0 && l < L) xyzz_store(cols + 8 * ((size_t)w * L + l), v);
    }
}

// grid (1 + logH + logL, SW), 256 threads.  out[w * NT + k]:
//   k == 0             : sum_h R_h
//   1 <= k <= logH     : U_{k-1} = sum_{h : bit k-1} R_h
//   k >  logH          : V_{k-1-logH} = sum_{l : bit k-1-logH} C_l
template <class Cv>
__global__ __launch_bounds__(256) void k_bitterms(const uint4* rows, const uint4* cols, uint32_t H, uint32_t L,
                                                  uint32_t logH, uint4* out) {
    using F = typename Cv::Base;
    __shared__ uint4 red[128 * 8];
    const uint32_t k = blockIdx.x, w = blockIdx.y, tid = threadIdx.x;
    const uint32_t NT = gridDim.x;
    const bool is_col = k > logH;
    const uint32_t cnt = is_col ? L : H;
    const uint4* src = is_col ? cols + 8 * (size_t)w * L : rows + 8 * (size_t)w * H;
    const uint32_t bit = is_col ? (k - 1 - logH) : (k - 1);
    XYZZ<F> acc = xyzz_id<F>();
    for (uint32_t j = tid; j < cnt; j += 256) {
        if (k != 0 && !((j >> bit) & 1u)) continue;
        acc = xyzz_add(acc, xyzz_load<F>(src + 8 * j));
    }
    acc = block_group_sum<F>(acc, 256, red);
    if (tid == 0) xyzz_store(out + 8 * ((size_t)w * NT + k), acc);
}

// grid SW, 64 threads: S_w = T_0 + sum_j 2^(j + logL) U_j + sum_j 2^j V_j.  fin (SW == 1): lane 0 then
// finishes the MSM as k_final would (+ hide, -> ark WrappedPoint (1) or packed XYZZ (2)), one
// lone-wave launch fewer on the tail's critical path.
// XYZZ point -> 32 words of pinned host memory (system-scope stores), then its flag = seq (release)
template <class F>
__device__ __forceinline__ void pair_emit_host(uint32_t* host, uint32_t* flag, const XYZZ<F>& v, uint32_t seq) {
    const Fe<F>* c[4] = {&v.X, &v.Y, &v.ZZ, &v.ZZZ};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t w[8];
        fe_pack(*c[k], w);
#pragma unroll
        for (int i = 0; i < 8; i++) __hip_atomic_store(host + 8 * k + i, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class Cv>
__global__ __launch_bounds__(64) void k_bitcombine(const uint4* terms, uint32_t NT, uint32_t logH, uint32_t logL,
                                                   uint4* window_sums, int fin, const uint4* hide, uint4* out,
                                                   const uint4* pair_hide, MsmOuts8 pair_outs, uint32_t* pair_host,
                                                   uint32_t pair_seq) {
    using F = typename Cv::Base;
    const uint32_t w = blockIdx.x, k = threadIdx.x;
    XYZZ<F> v = xyzz_id<F>();
    const uint32_t D = logH + logL;  // doubling classes d = 0 .. D - 1, one U or V term each (+ T_0 at d = 0)
    if (D <= 16) {
        // quad j (lanes 4j .. 4j + 3) doubles the term of class j j times with quad-cooperative doublings
        // (three product rounds per doubling instead of nine on one lane); then lanes 0 .. D - 1 take the
        // quads' results, lane D takes T_0, and a tree sums them
        const uint32_t j = k >> 2;
        if (j < D) {
            const uint32_t kt = j < logL ? 1 + logH + j : 1 + (j - logL);  // V_j or U_(j - logL)
            v = xyzz_load<F>(terms + 8 * ((size_t)w * NT + kt));
        }
        for (uint32_t i = 0; i + 1 < D; i++) {
            const XYZZ<F> d2 = xyzz_dbl_quad(v);
            if (i < j) v = d2;
        }
        v = xyzz_shfl(v, (int)((4 * k) & 63u));
        if (k == D) v = xyzz_load<F>(terms + 8 * (size_t)w * NT);
        if (k > D) v = xyzz_id<F>();
        uint32_t G = 1;
        while (G < D + 1) G <<= 1;
        v = wave_group_sum<F>(v, G);
    } else
    {
        if (k < NT) {
            v = xyzz_load<F>(terms + 8 * ((size_t)w * NT + k));
            const uint32_t d = (k == 0) ? 0 : (k <= logH ? (k - 1 + logL) : (k - 1 - logH));
            for (uint32_t i = 0; i < d; i++) v = xyzz_dbl(v);
        }
        // NT <= 64 terms: a tree over the wave's lanes
        uint32_t G = 1;
        while (G < NT) G <<= 1;
        v = wave_group_sum<F>(v, G);
    }
    if (k != 0) return;
    if (pair_hide) {  // a pair MSM's output w: + its hiding term (MsmTailArgs::pair_outs)
        const XYZZ<F> r = xyzz_add(v, xyzz_load<F>(pair_hide + 8 * w));
        xyzz_store(pair_outs.o[w], r);
        if (pair_host && w < 2) pair_emit_host(pair_host + 32 * w, pair_host + 64 + w, r, pair_seq);
        return;
    }
    if (fin == 0) {
        xyzz_store(window_sums + 8 * w, v);
        return;
    }
    if (hide) v = xyzz_add(v, xyzz_load<F>(hide));
    if (fin == 2)
        xyzz_store(out, v);
    else
        aff_to_wrapped(out, xyzz_to_aff(v));
}

// Many small windows (msm_shared_batch: SW = len * W windows of B = 16..128 buckets): 8 lanes per
// window, lane k owns the G = B / 8 buckets [G k, G k + G): a running sum gives R = sum B_b and
// S = sum (b - G k + 1) B_b over the segment (2 G additions), the lane adds G k R (lg G doublings
// and a 3-bit multiple), and a 3-level tree over the 8 lanes gives sum_b (b + 1) B_b.
constexpr uint32_t BATCH_SEGS = 8;  // lanes per window up to 64 buckets; B / 8 above (8 buckets a lane)
template <class Cv, uint32_t SEGS>
__global__ __launch_bounds__(256) void k_batch_window_sums(const uint4* bucket_sums, uint32_t SW, uint32_t B,
                                                           uint4* window_sums) {
    using F = typename Cv::Base;
    static_assert(SEGS >= 2 && SEGS <= 64 && (SEGS & (SEGS - 1)) == 0, "lanes per window");
    constexpr int KBITS = __builtin_ctz(SEGS);
    const uint32_t tid = threadIdx.x;
    const size_t t = (size_t)blockIdx.x * blockDim.x + tid;
    const uint32_t k = tid % SEGS, G = B / SEGS;
    const size_t w = t / SEGS;
    XYZZ<F> v = xyzz_id<F>();
    if (w < SW) {
        const uint4* bs = bucket_sums + 8 * (w * B + (size_t)k * G);
        XYZZ<F> R = xyzz_id<F>(), S = xyzz_id<F>();
        for (int j = (int)G - 1; j >= 0; j--) {
            R = xyzz_add(R, xyzz_load<F>(bs + 8 * j));
            S = xyzz_add(S, R);
        }
        if (k) {
            XYZZ<F> X = R;
            for (uint32_t g = G; g > 1; g >>= 1) X = xyzz_dbl(X);  // G R
            XYZZ<F> Y = xyzz_id<F>();
            for (int bit = KBITS - 1; bit >= 0; bit--) {
                Y = xyzz_dbl(Y);
                if ((k >> bit) & 1u) Y = xyzz_add(Y, X);
            }
            S = xyzz_add(S, Y);
        }
        v = S;
    }
    v = wave_group_sum<F>(v, SEGS);
    if (k == 0 && w < SW) xyzz_store(window_sums + 8 * w, v);
}

// Horner over the window sums (the c doublings per window run in Jacobian coordinates),
// plus the precomputed hiding term (or null), -> affine -> ark WrappedPoint.
template <class Cv>
__global__ __launch_bounds__(64) void k_final(const uint4* window_sums, int W, int c, const uint4* hide_xyzz,
                                              uint4* out_wrapped, int xyzz_out) {
    using F = typename Cv::Base;
    XYZZ<F> horner = xyzz_id<F>();
    // every quad of the wave runs the same Horner chain (identical data, so every branch is uniform):
    // quad-cooperative doublings (xyzz_dbl_quad: 4.0 k cycles per doubling against 6.3 k for the
    // Jacobian jac_dbl_quad, tools/micro/tree_parts.hip) and additions (4 product rounds instead of 14)
    const uint32_t s1 = threadIdx.x & 60u;
    for (int w = W - 1; w >= 0; w--) {
        if (w != W - 1 && !xyzz_is_id(horner))
            for (int k = 0; k < c; k++) horner = xyzz_dbl_quad(horner);
        const XYZZ<F> ws = xyzz_load<F>(window_sums + 8 * w);
        const bool idp = xyzz_is_id(horner), idq = xyzz_is_id(ws);
        if (idp || idq) {
            if (idp) horner = ws;
        } else {
            const XYZZ<F> r = xyzz_add_quad((threadIdx.x & 3u) == 1 ? ws : horner, s1, s1 + 1, false, false);
            horner = xyzz_shfl(r, (int)(s1 + 2));
        }
    }
    if (threadIdx.x != 0) return;
    if (hide_xyzz) horner = xyzz_add(horner, xyzz_load<F>(hide_xyzz));
    if (xyzz_out)  // 128 B packed XYZZ: the host converts (halo_ipa_round_lr, no inversion on the lane)
        xyzz_store(out_wrapped, horner);
    else
        aff_to_wrapped(out_wrapped, xyzz_to_aff(horner));
}

static unsigned grid_for_t(size_t n, unsigned thr) { return (unsigned)std::max<size_t>(1, (n + thr - 1) / thr); }

template <class Cv>
static int tail_launch_t(const MsmTailArgs& a, hipStream_t ts) {
    if (a.n > 0) {
        if (a.ng1)
            hipLaunchKernelGGL(k_group_sums<Cv>, dim3((unsigned)a.ng1), dim3(MSM_GROUP), 0, ts, a.skeys, a.scount, a.K,
                               1u, (const uint4*)a.first, a.g1);
        if (a.ng2)
            hipLaunchKernelGGL(k_group_sums<Cv>, dim3((unsigned)a.ng2), dim3(MSM_GROUP), 0, ts, a.skeys, a.scount, a.K,
                               MSM_GROUP, (const uint4*)a.g1, a.g2);
        // two lanes per bucket, each summing half of its chunk partials (measured per bucket: one lane
        // 167 us, two 138 us, four 172 us isolated at 2^20)
        constexpr int lanes = 2;
        hipLaunchKernelGGL((k_merge<Cv, lanes>), dim3(grid_for_t(a.NB * lanes, 256)), dim3(256), 0, ts, (const uint32_t*)a.bstart,
                           a.scount, a.K, a.NB, (const uint4*)a.first, (const uint4*)a.last,
                           (const uint4*)a.g1, (const uint4*)a.g2, a.bucket_sums);
        if (a.batch_windows) {
            const uint32_t B = a.L * a.H;
            if (B < 2 * BATCH_SEGS || B > 512 || (B & (B - 1)))
                return set_error(HALO_EINVAL, "batched window sums: %u buckets per window", B);
            // lanes per window: 8, or 8 buckets per lane above 64 buckets
            const uint32_t segs = std::max(BATCH_SEGS, B / 8);
            auto kws = segs == 8 ? k_batch_window_sums<Cv, 8> : segs == 16 ? k_batch_window_sums<Cv, 16>
                     : segs == 32 ? k_batch_window_sums<Cv, 32> : k_batch_window_sums<Cv, 64>;
            hipLaunchKernelGGL(kws, dim3(grid_for_t((size_t)a.SW * segs, 256)), dim3(256), 0, ts,
                               (const uint4*)a.bucket_sums, (uint32_t)a.SW, B, a.window_sums);
            HALO_HIP(hipGetLastError());
            return HALO_OK;
        }
        // entries per lane: the fewest (1, 2, 4) that keep the grid within one block per CU
        uint32_t epl = 1;
        while (epl < 4 && 2 * epl <= std::min(a.L, a.H)) {
            const RowcolShape sh = rowcol_shape(a.L, a.H, epl);
            if ((size_t)(sh.nrb + sh.ncb) * a.SW <= (size_t)a.num_cu) break;
            epl *= 2;
        }
        const RowcolShape sh = rowcol_shape(a.L, a.H, epl);
        hipLaunchKernelGGL(k_rowcol<Cv>, dim3(sh.nrb + sh.ncb, a.SW), dim3(256), 0, ts, (const uint4*)a.bucket_sums,
                           a.L, a.H, epl, a.rows, a.cols);
        hipLaunchKernelGGL(k_bitterms<Cv>, dim3(a.NT, a.SW), dim3(256), 0, ts, (const uint4*)a.rows,
                           (const uint4*)a.cols, a.H, a.L, a.logH, a.terms);
        const int fin = a.SW == 1 ? a.final_mode : 0;
        hipLaunchKernelGGL(k_bitcombine<Cv>, dim3(a.SW), dim3(64), 0, ts, (const uint4*)a.terms, a.NT, a.logH, a.logL,
                           a.window_sums, fin, a.final_hide, a.final_out, a.pair_hide, a.pair_outs, a.pair_host, a.pair_seq);
    }
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

int msm_final_launch(int curve, const uint4* window_sums, int W, int c, const uint4* hide, uint4* out, int xyzz_out,
                     hipStream_t s) {
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_final<Cv>, dim3(1), dim3(64), 0, s, window_sums, W, c, hide, out, xyzz_out);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

int msm_tail_launch(int curve, const MsmTailArgs& a, hipStream_t ts) {
    int rc;
    DISPATCH_CURVE(curve, Cv, { rc = tail_launch_t<Cv>(a, ts); });
    return rc;
}

}  // namespace halo
