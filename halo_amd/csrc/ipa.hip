// IPA inner-product folding, polynomial evaluation, dot products, powers, FFT multiplication
// (SURVEY §8 rows a7, a8, a9).
//
//  * IPA session: the round loop of pcdl::open_without_eval (crates/accumulation/src/pcdl.rs:404-438)
//    with G, c, z device-resident across rounds.  Per round the host (which owns the Poseidon
//    transcript, pcdl.rs:421-425) asks for L, R and then supplies xi.
//      L = <c_r, G_l> + H' <c_r, z_l>,  R = <c_l, G_r> + H' <c_l, z_r>     (pcdl.rs:412-418)
//      G_l[j] = (G_l[j] + xi G_r[j]).into_affine(); c_l[j] += xi^-1 c_r[j]; z_l[j] += xi z_r[j]
//                                                                       (pcdl.rs:427-435)
//    The G fold multiplies every lane by the SAME scalar xi, so all lanes follow one control path
//    (the NAF of xi, computed once per workgroup into LDS and read wave-uniformly); the dot products
//    are device reductions whose results feed the MSM's hiding-term slot (k_final) directly, so a
//    round never round-trips scalars through the host.
//  * DensePolynomial::evaluate (Horner, pcdl.rs:49,471): chunked Horner + z^offset + tree sum.
//  * group::scalar_dot / construct_powers (crates/group/src/group.rs:43-45,58-66).
//  * &Poly * &Poly (protocol.rs:132-139, pcdl.rs:215): NTT, pointwise product, iNTT, trim.
#include <algorithm>
#include <cstring>
#include <unordered_set>
#include <vector>

#include <chrono>
#include <thread>

#include "dispatch.hpp"
#include "glv.hpp"
#include "msm.hpp"
#include "runtime.hpp"
#include "tree.hpp"

namespace halo {

// ---------------------------------------------------------------------------------------------
// reductions / elementwise
// ---------------------------------------------------------------------------------------------
constexpr int RED_THREADS = 256;

// partial[blockIdx] = sum_{i in block range} x[i] * y[i].  x is read raw (ark value X = x 2^256) and
// y converted to internal (y R'), so fe_mul(X, Y) = x y 2^256: every partial is the product already
// in ark form and the final sum only needs canonicalising.
template <class F>
__global__ __launch_bounds__(RED_THREADS) void k_dot_partial(const uint4* x, const uint4* y, size_t n, size_t per_block,
                                                             uint4* partial) {
    __shared__ uint4 red[RED_THREADS * 2];
    const size_t beg = (size_t)blockIdx.x * per_block, end = min(n, beg + per_block);
    Fe<F> acc = fe_zero<F>();
    for (size_t i = beg + threadIdx.x; i < end; i += RED_THREADS)
        acc = fe_add(acc, fe_mul(fe_load<F>(x + 2 * i), fe_from_ark<F>(y + 2 * i)));
    fe_store(red + 2 * threadIdx.x, acc);
    __syncthreads();
    for (int off = RED_THREADS / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off)
            fe_store(red + 2 * threadIdx.x, fe_add(fe_load<F>(red + 2 * threadIdx.x), fe_load<F>(red + 2 * (threadIdx.x + off))));
        __syncthreads();
    }
    if (threadIdx.x == 0) fe_store(partial + 2 * blockIdx.x, fe_load<F>(red));
}

// out_ark = ARK(sum_b partial[b]) where partial values are "ark-valued products" (see above)
template <class F>
__global__ __launch_bounds__(RED_THREADS) void k_sum_partials_to_ark(const uint4* partial, size_t nb, uint4* out_ark) {
    __shared__ uint4 red[RED_THREADS * 2];
    Fe<F> acc = fe_zero<F>();
    for (size_t i = threadIdx.x; i < nb; i += RED_THREADS) acc = fe_add(acc, fe_load<F>(partial + 2 * i));
    fe_store(red + 2 * threadIdx.x, acc);
    __syncthreads();
    for (int off = RED_THREADS / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off)
            fe_store(red + 2 * threadIdx.x, fe_add(fe_load<F>(red + 2 * threadIdx.x), fe_load<F>(red + 2 * (threadIdx.x + off))));
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        // acc holds sum of ark-form values (x y 2^256 mod p, weakly reduced): canonicalize
        fe_store(out_ark, fe_canon(fe_reduce_2p(fe_load<F>(red))));
    }
}

// out[i] = z^i, i < n (ark in / out); each thread produces a run of `run` consecutive powers
template <class F>
__global__ void k_powers(const uint4* z_ark, size_t n, size_t run, uint4* out) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t beg = t * run;
    if (beg >= n) return;
    const Fe<F> z = fe_from_ark<F>(z_ark);
    Fe<F> p = fe_one<F>(), b = z;
    for (size_t e = beg; e; e >>= 1) {
        if (e & 1) p = fe_mul(p, b);
        b = fe_sqr(b);
    }
    const size_t end = min(n, beg + run);
    for (size_t i = beg; i < end; i++) {
        fe_to_ark(out + 2 * i, p);
        p = fe_mul(p, z);
    }
}

// Chunked Horner: partial[(poly, chunk)] = z^start * sum_{i in chunk} c_i z^(i - start)  (internal)
template <class F>
__global__ __launch_bounds__(RED_THREADS) void k_eval_chunks(const uint4* const* polys, const size_t* lens,
                                                             const uint4* z_ark, size_t chunk, int nchunks,
                                                             uint4* partial) {
    __shared__ uint4 red[RED_THREADS * 2];
    const int pi = blockIdx.y;
    const size_t len = lens[pi];
    const uint4* c = polys[pi];
    const Fe<F> z = fe_from_ark<F>(z_ark);
    const size_t per_block = chunk * RED_THREADS;
    const size_t tbeg = (size_t)blockIdx.x * per_block + (size_t)threadIdx.x * chunk;
    Fe<F> acc = fe_zero<F>();
    if (tbeg < len) {
        const size_t tend = min(len, tbeg + chunk);
        for (size_t i = tend; i-- > tbeg;) acc = fe_add(fe_mul(acc, z), fe_from_ark<F>(c + 2 * i));
        Fe<F> p = fe_one<F>(), b = z;
        for (size_t e = tbeg; e; e >>= 1) {
            if (e & 1) p = fe_mul(p, b);
            b = fe_sqr(b);
        }
        acc = fe_mul(acc, p);
    }
    fe_store(red + 2 * threadIdx.x, acc);
    __syncthreads();
    for (int off = RED_THREADS / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off)
            fe_store(red + 2 * threadIdx.x, fe_add(fe_load<F>(red + 2 * threadIdx.x), fe_load<F>(red + 2 * (threadIdx.x + off))));
        __syncthreads();
    }
    if (threadIdx.x == 0) fe_store(partial + 2 * ((size_t)pi * nchunks + blockIdx.x), fe_load<F>(red));
}

template <class F>
__global__ __launch_bounds__(RED_THREADS) void k_sum_internal_to_ark(const uint4* partial, int per, uint4* out_ark) {
    __shared__ uint4 red[RED_THREADS * 2];
    const int pi = blockIdx.x;
    Fe<F> acc = fe_zero<F>();
    for (int i = threadIdx.x; i < per; i += RED_THREADS) acc = fe_add(acc, fe_load<F>(partial + 2 * ((size_t)pi * per + i)));
    fe_store(red + 2 * threadIdx.x, acc);
    __syncthreads();
    for (int off = RED_THREADS / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off)
            fe_store(red + 2 * threadIdx.x, fe_add(fe_load<F>(red + 2 * threadIdx.x), fe_load<F>(red + 2 * (threadIdx.x + off))));
        __syncthreads();
    }
    if (threadIdx.x == 0) fe_to_ark(out_ark + 2 * pi, fe_load<F>(red));
}

// pointwise a[i] *= b[i] (ark in / out)
template <class F>
__global__ void k_pointwise_mul(uint4* a, const uint4* b, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe_to_ark(a + 2 * i, fe_mul(fe_from_ark<F>(a + 2 * i), fe_from_ark<F>(b + 2 * i)));
}

// ---------------------------------------------------------------------------------------------
// IPA fold
// ---------------------------------------------------------------------------------------------

// G'[j] = G_l[j] + xi G_r[j] for j < m, c'[j] = c_l + xi^-1 c_r, z'[j] = z_l + xi z_r.
// gs: internal affine (2m points), cs/zs: ark scalars (2m).  xi / xi_inv: ark.
// xi G_r = k1 G_r + k2 phi(G_r), phi(x, y) = (beta x, y) (GLV): one interleaved NAF double-and-add
// of ~128 doublings (digit schedule wave-uniform, in LDS) instead of 255.  The affine conversion
// shares one inversion per workgroup (Montgomery's trick over prefix / suffix product scans).
constexpr int FOLD_THREADS = 128;
template <class Cv>
__global__ __launch_bounds__(FOLD_THREADS, 4) void k_ipa_fold(uint4* gs, uint4* cs, uint4* zs, size_t m,
                                                           const uint4* xi_ark, const uint4* xi_inv_ark) {
    using F = typename Cv::Base;
    using S = typename Cv::Scalar;
    constexpr int ND = 132;
    __shared__ int8_t naf1[ND], naf2[ND];
    __shared__ int top_s, neg1_s, neg2_s;
    __shared__ uint32_t pre[FOLD_THREADS][NLIMB], suf[FOLD_THREADS][NLIMB];
    __shared__ uint32_t tinv[NLIMB];
    const int tid = threadIdx.x;
    if (tid == 0) {
        uint32_t w8[8];
        fe_ark_to_canonical_words<S>(xi_ark, w8);
        bool n1, n2;
        uint32_t k1[5], k2[5];
        glv::decompose<typename Cv::K>(w8, n1, k1, n2, k2);
        const int t1 = glv::naf_digits(k1, naf1, ND), t2 = glv::naf_digits(k2, naf2, ND);
        top_s = t1 > t2 ? t1 : t2;
        neg1_s = n1;
        neg2_s = n2;
    }
    __syncthreads();
    const int top = top_s;
    const size_t j = (size_t)blockIdx.x * FOLD_THREADS + tid;
    const bool live = j < m;
    XYZZ<F> acc = xyzz_id<F>();
    if (live) {
        const Fe<S> xi = fe_from_ark<S>(xi_ark);
        const Fe<S> xinv = fe_from_ark<S>(xi_inv_ark);
        fe_to_ark(cs + 2 * j, fe_add(fe_from_ark<S>(cs + 2 * j), fe_mul(fe_from_ark<S>(cs + 2 * (j + m)), xinv)));
        fe_to_ark(zs + 2 * j, fe_add(fe_from_ark<S>(zs + 2 * j), fe_mul(fe_from_ark<S>(zs + 2 * (j + m)), xi)));
        const Affine<F> gr = aff_load<F>(gs + 4 * (j + m));
        Affine<F> p1 = gr, p2;
        p2.x = fe_mul(gr.x, fe_from_const<F>(Cv::K::BETA));
        p2.y = gr.y;
        if (aff_is_id(gr)) p2 = gr;
        const int s1 = neg1_s ? -1 : 1, s2 = neg2_s ? -1 : 1;
        for (int i = top; i >= 0; i--) {
            acc = xyzz_dbl(acc);
            const int d1 = __builtin_amdgcn_readfirstlane((int)naf1[i] * s1);
            const int d2 = __builtin_amdgcn_readfirstlane((int)naf2[i] * s2);
            if (d1) {
                Affine<F> q = p1;
                if (d1 < 0) q.y = fe_neg(q.y);
                acc = xyzz_madd(acc, q);
            }
            if (d2) {
                Affine<F> q = p2;
                if (d2 < 0) q.y = fe_neg(q.y);
                acc = xyzz_madd(acc, q);
            }
        }
        acc = xyzz_madd(acc, aff_load<F>(gs + 4 * j));
    }
    // batched affine conversion: z = ZZ * ZZZ (1 for identity / idle lanes)
    // (measured and rejected: a Jacobian accumulator (dbl-2009-l + madd-2007-bl, ~27 % fewer
    // multiplications) was 13 % slower -- its fully reduced additions cost more than they save)
    const bool id = xyzz_is_id(acc);
    const Fe<F> z = (live && !id) ? fe_mul(acc.ZZ, acc.ZZZ) : fe_one<F>();
    // inclusive prefix and suffix products (Hillis-Steele in LDS)
    Fe<F> pv = z, sv = z;
    for (int off = 1; off < FOLD_THREADS; off <<= 1) {
        for (int l = 0; l < NLIMB; l++) {
            pre[tid][l] = pv.v[l];
            suf[tid][l] = sv.v[l];
        }
        __syncthreads();
        if (tid >= off) {
            Fe<F> o;
            for (int l = 0; l < NLIMB; l++) o.v[l] = pre[tid - off][l];
            pv = fe_mul(pv, o);
        }
        if (tid + off < FOLD_THREADS) {
            Fe<F> o;
            for (int l = 0; l < NLIMB; l++) o.v[l] = suf[tid + off][l];
            sv = fe_mul(sv, o);
        }
        __syncthreads();
    }
    for (int l = 0; l < NLIMB; l++) {
        pre[tid][l] = pv.v[l];
        suf[tid][l] = sv.v[l];
    }
    __syncthreads();
    if (tid == FOLD_THREADS - 1) {
        const Fe<F> t = fe_inv(pv);  // inverse of the product of all z
        for (int l = 0; l < NLIMB; l++) tinv[l] = t.v[l];
    }
    __syncthreads();
    if (!live) return;
    Fe<F> inv;
    for (int l = 0; l < NLIMB; l++) inv.v[l] = tinv[l];
    if (tid > 0) {
        Fe<F> o;
        for (int l = 0; l < NLIMB; l++) o.v[l] = pre[tid - 1][l];
        inv = fe_mul(inv, o);
    }
    if (tid + 1 < FOLD_THREADS) {
        Fe<F> o;
        for (int l = 0; l < NLIMB; l++) o.v[l] = suf[tid + 1][l];
        inv = fe_mul(inv, o);
    }
    Affine<F> r;
    if (id) {
        r.x = fe_zero<F>();
        r.y = fe_zero<F>();
    } else {
        r.x = fe_mul(acc.X, fe_mul(inv, acc.ZZZ));  // X / ZZ
        r.y = fe_mul(acc.Y, fe_mul(inv, acc.ZZ));   // Y / ZZZ
    }
    aff_store(gs + 4 * j, r);
}

// 2^i P (i < count) as XYZZ from a WrappedPoint: one doubling chain (one thread)
template <class Cv>
__global__ __launch_bounds__(64) void k_pow2_xyzz_from_wrapped(const uint4* P_wrapped, uint4* out_xyzz, int count) {
    using F = typename Cv::Base;
    // quad-cooperative XYZZ doublings on lanes 0-3 (xyzz_dbl_quad: three product rounds, 4.0 k cycles
    // against 6.3 k for the Jacobian jac_dbl_quad with its longer add / double tail, tools/micro/tree_parts.hip)
    if (threadIdx.x >= 4) return;
    XYZZ<F> q = xyzz_from_aff(aff_from_wrapped<F>(P_wrapped));
    for (int i = 0; i < count; i++) {
        if (threadIdx.x == 0) xyzz_store(out_xyzz + 8 * i, q);
        q = xyzz_dbl_quad(q);
    }
}

// XYZZ -> internal affine, one inversion per lane (all lanes in parallel)
template <class Cv>
__global__ __launch_bounds__(64) void k_xyzz_to_aff_ipa(const uint4* in, uint4* out, int count) {
    using F = typename Cv::Base;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) aff_store(out + 4 * i, xyzz_to_aff(xyzz_load<F>(in + 8 * i)));
}

template <class Cv>
__global__ void k_copy_first_wrapped(const uint4* gs_int, const uint4* cs, uint4* out_U, uint4* out_c) {
    using F = typename Cv::Base;
    if (threadIdx.x != 0) return;
    aff_to_wrapped(out_U, aff_load<F>(gs_int));
    out_c[0] = cs[0];
    out_c[1] = cs[1];
}

// ---------------------------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------------------------
static unsigned gridn(size_t n, unsigned t) { return (unsigned)std::max<size_t>(1, (n + t - 1) / t); }

// dot product of two device ark vectors -> device ark scalar (out_ark), using tmp (>= 2048*32 B)
static int dot_device(int field, const void* x, const void* y, size_t n, void* out_ark, void* tmp, hipStream_t s) {
    const size_t per_block = std::max<size_t>(RED_THREADS * 8, (n + 1023) / 1024);
    const size_t nb = std::max<size_t>(1, (n + per_block - 1) / per_block);
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_dot_partial<F>, dim3((unsigned)nb), dim3(RED_THREADS), 0, s, (const uint4*)x,
                           (const uint4*)y, n, per_block, (uint4*)tmp);
        hipLaunchKernelGGL(k_sum_partials_to_ark<F>, dim3(1), dim3(RED_THREADS), 0, s, (const uint4*)tmp, nb,
                           (uint4*)out_ark);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

// ---------------------------------------------------------------------------------------------
// Tail rounds of the opening (length <= IPA_TAIL_N): instead of folding G (one ~128-doubling scalar
// multiplication per element per round, a ~1 ms dependent chain however few elements are left) the
// session keeps G0 = G at the switch round and the fold weights w (G_j[i] = sum_u w[u] G0[i + u len],
// fold: w' = interleave(w, xi w)).  L and R are then direct sums over G0 with expanded scalars
//   k = j + u len:  s[k] = c[m + j] w[u] (j < m, -> L),  c[j - m] w[u] (j >= m, -> R),
// evaluated from a table d 2^(4 win) G0[k] (win < 32, 1 <= d <= 8, built once per session): each
// scalar is split by GLV, s = k1 + lambda k2 with |k1|, |k2| < 0.47 x 2^128, so every (k, win, half)
// term is one table entry (or phi of it, x -> beta x, or its negative) selected by a signed 4-bit
// digit in [-8, 7] -- no per-term double-and-add chain on the rounds' critical path -- and the terms
// go through block trees.  The table's doubling chain is 124 doublings instead of 248; the 8
// multiples of each 2^(4 win) G0[k] cost 7 curve operations per (win, k), once (round 5: signed
// digits, was 15 unsigned multiples -- half the table build and half the table's footprint).
// U = sum_u w[u] G0[u] at the end.  c and z keep their ordinary elementwise folds (pcdl.rs:430-435).
constexpr size_t IPA_TAIL_N = 2048;
constexpr int IPA_HTAB = 128;  // entries 2^i H' of the session's hiding table (GLV split of the scalar)
constexpr int TAIL_DB = 4;                            // digit bits
constexpr int TAIL_TBL = 128 / TAIL_DB;               // table windows per 128-bit GLV half
constexpr int TAIL_MUL = 1 << (TAIL_DB - 1);           // multiples d = 1..8 per window (signed digits)
constexpr int TAIL_WIN = 2 * TAIL_TBL;  // terms per point: 32 windows x (k1, k2)
// threads per tail block: 256, one wave per SIMD (512 measured slower, opening 2^10 1.93 -> 2.13 ms: two
// waves' quad trees then share a SIMD's issue slots)
constexpr int TAIL_THREADS = 256;

// the doubling chain by a quad of lanes per point (xyzz_dbl_quad: three product rounds per doubling,
// 4.0 k cycles against 6.3 k for the Jacobian jac_dbl_quad -- fewer products, but a longer tail of
// additions and doublings on every lane; tools/micro/tree_parts.hip; TAIL_TABLE_LANES = 4) -- the
// chain is latency-bound and the grid is small (n0 <= 8192 points)
constexpr int TAIL_TABLE_LANES = 4;
template <class Cv>
__global__ __launch_bounds__(64) void k_tail_table(const uint4* gs, int gs_xyzz, size_t n0, uint4* table) {
    using F = typename Cv::Base;
    const size_t k = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TAIL_TABLE_LANES;
    if (k >= n0) return;  // (whole quads leave)
    const bool lead = threadIdx.x % TAIL_TABLE_LANES == 0;
    const XYZZ<F> p0 = gs_xyzz ? xyzz_load<F>(gs + 8 * k) : xyzz_from_aff(aff_load<F>(gs + 4 * k));
    if (lead) xyzz_store(table + 8 * k, p0);
    XYZZ<F> q = p0;
    for (int w = 1; w < TAIL_TBL; w++) {
        for (int b = 0; b < TAIL_DB; b++) q = xyzz_dbl_quad(q);
        if (lead) xyzz_store(table + 8 * ((size_t)w * TAIL_MUL * n0 + k), q);
    }
}

// entry (w, d, k) of the tail table: d 2^(4 w) G0[k], 1 <= d <= 8 (XYZZ); ld = the number of
// points the table was built for (a session may use a prefix of the SRS's table)
HALO_DEV size_t tail_entry(size_t w, uint32_t d, size_t ld, size_t k) {
    return 8 * ((w * TAIL_MUL + (d - 1)) * ld + k);
}

// Signed windows: a GLV half |k| < 0.47 x 2^128 (the lattice bound, tests/test_field_bounds.py) is kept
// as k + 0x8888...8 (< 2^128), whose nibble e of window w is the digit e - 8 in [-8, 7] of k.
HALO_DEV void tail_bias(uint32_t (&k)[5]) {
    uint64_t c = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        c += (uint64_t)k[q] + 0x88888888u;
        k[q] = (uint32_t)c;
        c >>= 32;
    }
}
// window bw of a biased word: |digit| (0..8) and whether the digit is negative
HALO_DEV uint32_t tail_digit(uint32_t word, uint32_t bw, bool& neg) {
    const uint32_t e = (word >> (TAIL_DB * (bw % (32 / TAIL_DB)))) & 15u;
    neg = e < 8;
    return neg ? 8 - e : e - 8;
}

// The multiples 2..8 of each window base P = 2^(4 w) G0[k] written by k_tail_table.  Lane
// (j, w, k), j < 4, owns d = 2j + 1, 2j + 2: it forms (2j + 1) P by double-and-add, then adds P --
// at most 5 dependent curve operations per lane.
constexpr int TAIL_MLANES = 4;
template <class Cv>
__global__ __launch_bounds__(64) void k_tail_mults(size_t n0, uint4* table) {
    using F = typename Cv::Base;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)TAIL_MLANES * TAIL_TBL * n0) return;
    const uint32_t j = (uint32_t)(t / ((size_t)TAIL_TBL * n0));
    const size_t r = t % ((size_t)TAIL_TBL * n0), w = r / n0, k = r % n0;
    const XYZZ<F> p = xyzz_load<F>(table + tail_entry(w, 1, n0, k));
    const uint32_t s = 2 * j + 1;
    XYZZ<F> cur = p;
#pragma unroll 1
    for (int b = 31 - __clz(s) - 1; b >= 0; b--) {  // s P, s = 2 j + 1 (bit 0 set: the last step adds)
        cur = xyzz_dbl(cur);
        if ((s >> b) & 1u) cur = xyzz_add(cur, p);
    }
    if (j) xyzz_store(table + tail_entry(w, s, n0, k), cur);
    xyzz_store(table + tail_entry(w, s + 1, n0, k), j ? xyzz_add(cur, p) : xyzz_dbl(p));
}

// mode 0: L/R scalars of the current round (len = 2m); mode 1: U's scalars s[k] = w[k]
// the GLV digits of term k's scalar v (internal form) and its side
template <class Cv>
HALO_DEV void tail_scalar_val(const Fe<typename Cv::Scalar>& v, uint8_t sd, size_t k, uint32_t* scal, uint8_t* side) {
    using S = typename Cv::Scalar;
    Fe<S> one_raw = fe_zero<S>();  // internal (x 2^261) -> canonical: Montgomery product with 1
    one_raw.v[0] = 1;
    uint32_t w8[8], k1[5], k2[5];
    bool n1, n2;
    fe_pack(fe_canon(fe_mul(v, one_raw)), w8);
    glv::decompose<typename Cv::K>(w8, n1, k1, n2, k2);
    tail_bias(k1);
    tail_bias(k2);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        scal[8 * k + q] = k1[q];
        scal[8 * k + 4 + q] = k2[q];
    }
    side[k] = sd | (n1 ? 2 : 0) | (n2 ? 4 : 0);
}

template <class Cv>
HALO_DEV void tail_scalar_one(const uint4* cs, const uint4* w, size_t k, size_t len, size_t m, int mode, uint32_t* scal,
                              uint8_t* side) {
    using S = typename Cv::Scalar;
    if (mode == 0) {
        const size_t j = k % len, u = k / len;
        const size_t ci = (j < m) ? m + j : j - m;
        tail_scalar_val<Cv>(fe_mul(fe_from_ark<S>(cs + 2 * ci), fe_from_ark<S>(w + 2 * u)), (j < m) ? 0 : 1, k, scal,
                            side);
    } else {
        tail_scalar_val<Cv>(fe_from_ark<S>(w + 2 * k), 0, k, scal, side);
    }
}

template <class Cv>
__global__ __launch_bounds__(256) void k_tail_scalars(const uint4* cs, const uint4* w, size_t n0, size_t len, size_t m,
                                                      int mode, uint32_t* scal, uint8_t* side) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n0) tail_scalar_one<Cv>(cs, w, k, len, m, mode, scal, side);
}

template <class Cv>
HALO_DEV void glv_split_words(const uint4* x_ark, uint32_t* out10) {
    using S = typename Cv::Scalar;
    uint32_t w8[8], k1[5], k2[5];
    bool n1, n2;
    fe_ark_to_canonical_words<S>(x_ark, w8);
    glv::decompose<typename Cv::K>(w8, n1, k1, n2, k2);
    for (int q = 0; q < 4; q++) {
        out10[q] = k1[q];
        out10[4 + q] = k2[q];
    }
    out10[8] = n1;
    out10[9] = n2;
}

// The previous round's fold (pcdl.rs:430-435, w' = interleave(w, xi w)) deferred into this launch:
// halo_ipa_fold only records xi (passed here by value -- no H2D copy, no k_tail_fold launch); the
// scalar blocks read the unfolded c, w and fold the entries they need on the fly, the dots block
// writes the folded c, z, w to the other buffers of their ping-pong pairs.
struct TailFoldArgs {
    uint4 xi[2], xinv[2];  // ark
    uint4 *cs_out, *zs_out, *w_out;
    size_t wlen_in;  // fold weights before the fold
    int active;
    uint4* w_one;  // the first tail round: w = [1] (not yet in memory): use 1, and store it here
};

// The hiding term dot * P' of one side as lane terms: lane t < 256 returns the table entry for bit t
// of the GLV split dot = k1 + lambda k2 (lanes 0-127: k1 with 2^t P', 128-255: k2 with phi(2^(t-128) P'))
// or the identity.  Block-uniform call (it synchronises).
// pre: the split already formed (glv_split_words, 10 words), else lane 0 forms it.
template <class Cv>
HALO_DEV XYZZ<typename Cv::Base> hiding_lane_term(const uint4* htab, const uint4* dot_ark, const uint32_t* pre,
                                                  uint32_t (&kw)[10]) {
    using F = typename Cv::Base;
    const int tid = threadIdx.x;
    if (pre) {
        if (tid < 10) kw[tid] = pre[tid];
    } else if (tid == 0) {
        glv_split_words<Cv>(dot_ark, kw);
    }
    __syncthreads();
    XYZZ<F> acc = xyzz_id<F>();
    if ((kw[tid >> 5] >> (tid & 31)) & 1u) {
        Affine<F> p = aff_load<F>(htab + 4 * (tid & 127));
        if (tid >= 128) p.x = fe_mul(p.x, fe_from_const<F>(Cv::K::BETA));
        if (kw[8 + (tid >> 7)]) p.y = fe_neg(p.y);
        acc = xyzz_from_aff(p);
    }
    return acc;
}

// A tail round's side sum straight into the session's pinned staging (coherent host memory): 32
// words with system-scope stores, then the side's flag = seq with a system-scope release.  The host
// polls the two flags instead of a D2H copy plus a stream synchronisation (round 3 measurement,
// tools/micro/sync_bench.hip: 5.8 vs 11 us per host round trip).  host: L at [0, 32), R at [32, 64)
// words; flags[0..2).
template <class F>
HALO_DEV void tail_emit_host(uint32_t* host, uint32_t* flags, uint32_t sd, const XYZZ<F>& v, uint32_t seq) {
    const Fe<F>* c[4] = {&v.X, &v.Y, &v.ZZ, &v.ZZZ};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t w[8];
        fe_pack(*c[k], w);
#pragma unroll
        for (int i = 0; i < 8; i++)
            __hip_atomic_store(host + 32 * sd + 8 * k + i, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(flags + sd, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block partial sums part[block][side].  mode 0 (L and R of a round, 2m = len): the first nbs blocks
// take side 0's terms, the rest side 1's (each block one side: one tree, not two); the term q of a
// side is (win, u, j) = window, fold weight, j < m, at point k = j + u 2m + side m.  mode 1 (U): terms
// t = win n0 + k, all on side 0.
template <class Cv>
// With htab: side sd's first block also adds the hiding term dots[sd] * P (GLV table htab of 2^i P;
// hkw: the dots' GLV splits when already formed) into its tree; with out_xyzz and nbs == 1 (the side
// is one block) it writes the side's sum straight to out_xyzz + 8 sd (no k_tail_final).  Mode 1 is
// one side of nbs blocks.
__global__ __launch_bounds__(TAIL_THREADS) void k_tail_msm(const uint4* table, size_t ld, const uint32_t* scal,
                                                            const uint8_t* side, size_t n0, size_t m, int mode, uint32_t nbs,
                                                            uint4* part, const uint4* htab, const uint4* dots_ark,
                                                            const uint32_t* hkw, uint4* out_xyzz,
                                                            uint32_t* host = nullptr, uint32_t seq = 0,
                                                            const uint4* plus_wrapped = nullptr,
                                                            const uint4* copy_src = nullptr, uint4* copy_dst = nullptr,
                                                            uint32_t tpl = 1) {
    using F = typename Cv::Base;
    __shared__ uint4 red[TAIL_THREADS / 2 * 8];
    __shared__ uint32_t kw[10];
    const int tid = threadIdx.x;
    XYZZ<F> acc = xyzz_id<F>();
    const uint32_t bsd = mode == 0 ? (uint32_t)(blockIdx.x >= nbs) : 0u;
    const bool first = htab && blockIdx.x == bsd * nbs;
    if (first) acc = hiding_lane_term<Cv>(htab, dots_ark + 2 * bsd, hkw ? hkw + 10 * bsd : nullptr, kw);
    const uint32_t sd = bsd;
    const size_t hn = n0 / 2, total = mode == 0 ? (size_t)TAIL_WIN * hn : (size_t)TAIL_WIN * n0;
    const size_t q0 = (size_t)(blockIdx.x - sd * nbs) * TAIL_THREADS + tid, qstride = (size_t)nbs * TAIL_THREADS;
    // term q of the side: mode 0 (win, u, j) at point k = j + u 2m + sd m; mode 1 t = win n0 + k
    auto term = [&](size_t q) {
        XYZZ<F> t = xyzz_id<F>();
        if (q >= total) return t;
        size_t win, k;
        if (mode == 0) {
            win = q / hn;
            const size_t r = q % hn, u = r / m, j = r % m;
            k = j + u * 2 * m + sd * m;
        } else {
            win = q / n0;
            k = q % n0;
        }
        constexpr uint32_t DPW = 32 / TAIL_DB;  // digits per scalar word
        const uint32_t half = (uint32_t)win / TAIL_TBL, bw = (uint32_t)win % TAIL_TBL;
        bool dneg;
        const uint32_t d = tail_digit(scal[8 * k + 4 * half + bw / DPW], bw, dneg);
        const uint32_t sk = side[k];
        if (d) {
            t = xyzz_load<F>(table + tail_entry(bw, d, ld, k));
            if (half) t.X = fe_mul(t.X, fe_from_const<F>(Cv::K::BETA));  // phi
            if ((((sk >> (1 + half)) & 1u) != 0) != dneg) t = xyzz_neg(t);
        }
        return t;
    };
    // tpl = 2 (grids beyond one block per CU): each lane first adds its two terms, so the trees run at
    // one wave per SIMD instead of two sharing a SIMD's issue slots
    XYZZ<F> t = term(q0);
    if (tpl == 2) t = xyzz_add(t, term(q0 + qstride));
    acc = first ? xyzz_add(acc, t) : t;
    acc = block_group_sum<F>(acc, TAIL_THREADS, red);
    if (out_xyzz && nbs == 1) {
        if (tid == 0) {
            if (plus_wrapped) acc = xyzz_madd(acc, aff_from_wrapped<F>(plus_wrapped));
            xyzz_store(out_xyzz + 8 * bsd, acc);
            if (copy_src) {  // 32 B beside the result, so that one D2H copy takes both
                copy_dst[0] = copy_src[0];
                copy_dst[1] = copy_src[1];
            }
            if (host) tail_emit_host(host, host + 64, bsd, acc, seq);
        }
    } else if (tid == 0) {
        xyzz_store(part + 8 * (2 * (size_t)blockIdx.x + sd), acc);
        xyzz_store(part + 8 * (2 * (size_t)blockIdx.x + (sd ^ 1)), xyzz_id<F>());
    }
}

// One tail round (L and R with their hiding terms) in ONE launch (round 4; was k_tail_prep + k_tail_msm +
// k_tail_final).  Blocks [0, 2 nbs) own 4 points each (one per wave), all on one side: side sd's point
// q = (block - sd nbs) 4 + wave (q < n0 / 2) is k = j + u 2m + sd m with u = q / m, j = q % m, and its
// 64 lanes are its 64 window terms (32 4-bit GLV windows x (k1, k2)).  Every lane of the wave forms the
// point's scalar c[ci] w[u] and its GLV split itself (wave-uniform work: the SIMD issues it once), so
// no preparation launch is needed; with a deferred fold the unfolded c / w are folded on the fly as
// k_tail_prep did.  Blocks 2 nbs + sd form side sd's dot product (with a deferred fold they also write
// their halves of the folded c, z, w), scale it by xi_0 in xi mode, and add the side's hiding term
// dot_sd * H' as one more partial -- one block per side, in parallel with the point blocks.  Each block
// publishes its partial (relaxed agent-scope stores drained, then an agent-scope release add on its
// side's counter); the last block to arrive on a side takes an agent acquire, sums the side's nbs + 1
// partials and writes the side's XYZZ sum to out_xyzz + 8 sd, then resets the counter.  No block waits
// for another.
struct TailRoundArgs {
    const uint4* table;
    size_t ld, n0, m;
    const uint4 *cs, *zs, *w;
    uint32_t nbs;              // point blocks per side
    const uint4* xi0_ark;      // xi mode: dots scaled by xi_0
    const uint4* htab;         // 2^i H' (or 2^i H in xi mode), i < 128
    uint4* dots_ark;           // [2] out
    uint4* part;               // [2][nbs + 1] XYZZ partials
    uint32_t* ctr;             // [2] arrival counters (zero between launches)
    uint4* out_xyzz;           // [2] L, R
    uint32_t* host;            // the session's pinned L | R staging (tail_emit_host) or null
    uint32_t seq;              // this round's flag value
};

// n0 up to this: one launch per round (k_tail_round, scalars formed in the points' waves); above it the
// three-launch round (k_tail_digits, k_tail_msm, k_tail_final) is faster (measured per 2^10 / 2^12 round:
// 0.118 / 0.195 vs 0.125-0.131 / 0.206 ms fused; 2^4 / 2^6 / 2^8: 0.103 / 0.110 / 0.114 vs 0.092-0.094 /
// 0.094-0.097 / 0.097-0.109 ms for the fused one)
constexpr size_t TAIL_FUSE_N = 256;

HALO_DEV uint32_t tail_word(const uint32_t (&k)[5], uint32_t i) {  // k[i], i < 4, without dynamic indexing
    uint32_t r = k[0];
    r = i == 1 ? k[1] : r;
    r = i == 2 ? k[2] : r;
    return i == 3 ? k[3] : r;
}

template <class F>
HALO_DEV void tail_publish_fe(uint32_t* d, const Fe<F>& v) {
    uint32_t x[8];
    fe_pack(v, x);
#pragma unroll
    for (int i = 0; i < 8; i++) __hip_atomic_store(d + i, x[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class F>
HALO_DEV void tail_publish(uint4* dst, const XYZZ<F>& v) {  // relaxed agent-scope stores (sc1), one lane
    uint32_t* d = (uint32_t*)dst;
    tail_publish_fe(d, v.X);
    tail_publish_fe(d + 8, v.Y);
    tail_publish_fe(d + 16, v.ZZ);
    tail_publish_fe(d + 24, v.ZZZ);
}

// true in the block whose release add on *c returned total - 1 (then acquired); block-uniform
HALO_DEV bool tail_arrive(uint32_t* c, uint32_t total, uint32_t* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t got = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        *flag = got == total - 1;
        if (*flag) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return *flag != 0;
}

template <class Cv>
HALO_DEV void tail_side_final(const TailRoundArgs& a, uint32_t sd, uint4* red) {
    using F = typename Cv::Base;
    const uint32_t np = a.nbs + 1;
    // partial j to lane j / 4 of wave j % 4: every wave gets a quarter, and its tree skips the identity
    // lanes above them (as k_tail_final deals them)
    const uint32_t tid = threadIdx.x, j0 = (tid & 63) * (TAIL_THREADS / 64) + (tid >> 6);
    XYZZ<F> acc = xyzz_id<F>();
    for (uint32_t j = j0; j < np; j += TAIL_THREADS) acc = xyzz_add(acc, xyzz_load<F>(a.part + 8 * ((size_t)sd * np + j)));
    acc = block_group_sum<F>(acc, TAIL_THREADS, red);
    if (tid == 0) {
        xyzz_store(a.out_xyzz + 8 * sd, acc);
        if (a.host) tail_emit_host(a.host, a.host + 64, sd, acc, a.seq);
        __hip_atomic_store(a.ctr + sd, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Side sd's dot (0: <c_r, z_l>, 1: <c_l, z_r>) by one block, scaled by xi_0 in xi mode, to dots_ark +
// 2 sd and its GLV split to kw (10 words: k1, k2 words, signs; visible to the block on return).  With a
// deferred fold the block folds the halves its dot reads and writes them to the ping-pong buffers (side
// 0: c_r, z_l and the even w'; side 1: c_l, z_r and the odd w').
template <class Cv>
HALO_DEV void tail_side_dot(const uint4* cs, const uint4* zs, const uint4* w, size_t m, uint32_t sd, const TailFoldArgs& f,
                            const uint4* xi0_ark, uint4* dots_ark, uint32_t* kw) {
    using S = typename Cv::Scalar;
    const int tid = threadIdx.x;
    const size_t len = 2 * m;
    const size_t oc = sd ? 0 : m, oz = sd ? m : 0;  // c_r z_l (side 0), c_l z_r (side 1)
    Fe<S> acc_s = fe_zero<S>();
    if (f.active) {
        const Fe<S> xi = fe_from_ark<S>(f.xi), xinv = fe_from_ark<S>(f.xinv);
        for (size_t i = tid; i < m; i += TAIL_THREADS) {
            const Fe<S> c = fe_add(fe_from_ark<S>(cs + 2 * (oc + i)), fe_mul(fe_from_ark<S>(cs + 2 * (oc + i + len)), xinv));
            const Fe<S> z = fe_add(fe_from_ark<S>(zs + 2 * (oz + i)), fe_mul(fe_from_ark<S>(zs + 2 * (oz + i + len)), xi));
            fe_to_ark(f.cs_out + 2 * (oc + i), c);
            fe_to_ark(f.zs_out + 2 * (oz + i), z);
            acc_s = fe_add(acc_s, fe_mul(c, z));
        }
        for (size_t u = tid; u < f.wlen_in; u += TAIL_THREADS) {
            const Fe<S> wv = fe_from_ark<S>(w + 2 * u);
            fe_to_ark(f.w_out + 2 * (2 * u + sd), sd ? fe_mul(wv, xi) : wv);
        }
    } else {
        for (size_t i = tid; i < m; i += TAIL_THREADS)
            acc_s = fe_add(acc_s, fe_mul(fe_from_ark<S>(cs + 2 * (oc + i)), fe_from_ark<S>(zs + 2 * (oz + i))));
    }
    // block sum: lane shuffles inside each wave, then the four wave sums through LDS
    for (int off = 32; off > 0; off >>= 1) {
        Fe<S> o;
#pragma unroll
        for (int l = 0; l < NLIMB; l++) o.v[l] = __shfl_xor(acc_s.v[l], off);
        acc_s = fe_add(acc_s, o);
    }
    __shared__ uint4 wsum[TAIL_THREADS / 64][2];
    if ((tid & 63) == 0) fe_store(wsum[tid >> 6], acc_s);
    __syncthreads();
    if (tid == 0) {
        Fe<S> d = fe_load<S>(wsum[0]);
        for (int q = 1; q < TAIL_THREADS / 64; q++) d = fe_add(d, fe_load<S>(wsum[q]));
        if (xi0_ark) d = fe_mul(d, fe_from_ark<S>(xi0_ark));
        fe_to_ark(dots_ark + 2 * sd, d);
        Fe<S> one_raw = fe_zero<S>();
        one_raw.v[0] = 1;
        uint32_t w8[8], k1[5], k2[5];
        bool n1, n2;
        fe_pack(fe_canon(fe_mul(d, one_raw)), w8);
        glv::decompose<typename Cv::K>(w8, n1, k1, n2, k2);
        for (int i = 0; i < 4; i++) {
            kw[i] = k1[i];
            kw[4 + i] = k2[i];
        }
        kw[8] = n1;
        kw[9] = n2;
    }
    __syncthreads();
}

// The round's n0 point scalars c[ci] w[u] (with a deferred fold applied on the fly) as GLV words, one
// lane per point, and (the last two blocks) the two sides' dots with their GLV splits (hkw, for
// k_tail_msm's hiding terms) and the folded c, z, w: the first launch of a tail round over more than
// TAIL_FUSE_N points, where forming the scalars once per point beats forming them in each point's
// wave of k_tail_round (64 times the instructions).
template <class Cv>
__global__ __launch_bounds__(256) void k_tail_digits(const uint4* cs, const uint4* zs, const uint4* w, size_t n0, size_t m,
                                                     const TailFoldArgs f, uint32_t* scal, uint8_t* side,
                                                     const uint4* xi0_ark, uint4* dots_ark, uint32_t* hkw) {
    using S = typename Cv::Scalar;
    const uint32_t nsb = (uint32_t)((n0 + 255) / 256);
    if (blockIdx.x >= nsb) {
        __shared__ uint32_t kw[10];
        const uint32_t sd = blockIdx.x - nsb;
        tail_side_dot<Cv>(cs, zs, w, m, sd, f, xi0_ark, dots_ark, kw);
        if (threadIdx.x < 10) hkw[10 * sd + threadIdx.x] = kw[threadIdx.x];
        return;
    }
    const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n0) return;
    const size_t len = 2 * m, j = k % len, u = k / len;
    const size_t ci = (j < m) ? m + j : j - m;
    Fe<S> c, wu;
    if (f.active) {
        c = fe_add(fe_from_ark<S>(cs + 2 * ci), fe_mul(fe_from_ark<S>(cs + 2 * (ci + len)), fe_from_ark<S>(f.xinv)));
        wu = fe_from_ark<S>(w + 2 * (u >> 1));
        if (u & 1) wu = fe_mul(wu, fe_from_ark<S>(f.xi));
    } else {
        c = fe_from_ark<S>(cs + 2 * ci);
        wu = f.w_one ? fe_one<S>() : fe_from_ark<S>(w + 2 * u);
        if (f.w_one && k == 0) fe_to_ark(f.w_one, wu);
    }
    tail_scalar_val<Cv>(fe_mul(c, wu), (j < m) ? 0 : 1, k, scal, side);
}

template <class Cv>
__global__ __launch_bounds__(TAIL_THREADS, 1) void k_tail_round(const TailRoundArgs a, const TailFoldArgs f) {
    using F = typename Cv::Base;
    using S = typename Cv::Scalar;
    __shared__ uint4 red[TAIL_THREADS / 2 * 8];
    __shared__ uint32_t flag;
    const int tid = threadIdx.x;
    const size_t m = a.m, len = 2 * m, hn = a.n0 / 2;
    if (blockIdx.x < 2 * a.nbs) {
        const uint32_t sd = blockIdx.x >= a.nbs;
        const size_t q = (size_t)(blockIdx.x - sd * a.nbs) * (TAIL_THREADS / 64) + (tid >> 6);
        XYZZ<F> acc = xyzz_id<F>();
        if (q < hn) {  // (wave-uniform)
            const size_t u = q / m, j = q % m, k = j + u * len + sd * m;
            const size_t ci = sd ? j : m + j;
            Fe<S> c, wu;
            if (f.active) {  // c' = c_l + xi^-1 c_r over the unfolded c; w'[u] = w[u / 2] (xi w[u / 2] for odd u)
                c = fe_add(fe_from_ark<S>(a.cs + 2 * ci), fe_mul(fe_from_ark<S>(a.cs + 2 * (ci + len)), fe_from_ark<S>(f.xinv)));
                wu = fe_from_ark<S>(a.w + 2 * (u >> 1));
                if (u & 1) wu = fe_mul(wu, fe_from_ark<S>(f.xi));
            } else {
                c = fe_from_ark<S>(a.cs + 2 * ci);
                wu = f.w_one ? fe_one<S>() : fe_from_ark<S>(a.w + 2 * u);
                if (f.w_one && k == 0 && (tid & 63) == 0) fe_to_ark(f.w_one, wu);
            }
            Fe<S> one_raw = fe_zero<S>();  // internal (x 2^261) -> canonical: Montgomery product with 1
            one_raw.v[0] = 1;
            uint32_t w8[8], k1[5], k2[5];
            bool n1, n2;
            fe_pack(fe_canon(fe_mul(fe_mul(c, wu), one_raw)), w8);
            glv::decompose<typename Cv::K>(w8, n1, k1, n2, k2);
            tail_bias(k1);
            tail_bias(k2);
            constexpr uint32_t DPW = 32 / TAIL_DB;  // digits per scalar word
            const uint32_t win = tid & 63, half = win / TAIL_TBL, bw = win % TAIL_TBL;
            const uint32_t word = half ? tail_word(k2, bw / DPW) : tail_word(k1, bw / DPW);
            bool dneg;
            const uint32_t d = tail_digit(word, bw, dneg);
            if (d) {
                XYZZ<F> t = xyzz_load<F>(a.table + tail_entry(bw, d, a.ld, k));
                if (half) t.X = fe_mul(t.X, fe_from_const<F>(Cv::K::BETA));  // phi
                if ((half ? n2 : n1) != dneg) t = xyzz_neg(t);
                acc = t;
            }
        }
        acc = block_group_sum<F>(acc, TAIL_THREADS, red);
        if (tid == 0) tail_publish(a.part + 8 * ((size_t)sd * (a.nbs + 1) + (blockIdx.x - sd * a.nbs)), acc);
        if (tail_arrive(a.ctr + sd, a.nbs + 1, &flag)) tail_side_final<Cv>(a, sd, red);
        return;
    }
    // ---- hiding blocks 2 nbs + sd: side sd's dot, its GLV split and the term dot_sd H'
    const uint32_t sd = blockIdx.x - 2 * a.nbs;
    __shared__ uint32_t kw[10];
    tail_side_dot<Cv>(a.cs, a.zs, a.w, m, sd, f, a.xi0_ark, a.dots_ark, kw);
    // dot H': lane t < 128 bit t of k1 with 2^t H', t >= 128 bit t - 128 of k2 with phi(2^(t-128) H')
    XYZZ<F> acc = xyzz_id<F>();
    if ((kw[tid >> 5] >> (tid & 31)) & 1u) {
        Affine<F> p = aff_load<F>(a.htab + 4 * (tid & 127));
        if (tid >= 128) p.x = fe_mul(p.x, fe_from_const<F>(Cv::K::BETA));
        if (kw[8 + (tid >> 7)]) p.y = fe_neg(p.y);
        acc = xyzz_from_aff(p);
    }
    acc = block_group_sum<F>(acc, TAIL_THREADS, red);
    if (tid == 0) tail_publish(a.part + 8 * ((size_t)sd * (a.nbs + 1) + a.nbs), acc);
    if (tail_arrive(a.ctr + sd, a.nbs + 1, &flag)) tail_side_final<Cv>(a, sd, red);
}

// block b (0: L, 1: R): sum of the partials + dot_b * H' (from the 2^i H' table), -> WrappedPoint
template <class Cv>
__global__ __launch_bounds__(TAIL_THREADS) void k_tail_final(const uint4* part, int nblk, const uint4* htab,
                                                              const uint4* dots_ark, uint4* out_wrapped,
                                                              int xyzz_out, uint32_t* host = nullptr,
                                                              uint32_t seq = 0, const uint4* plus_wrapped = nullptr,
                                                              const uint4* copy_src = nullptr, uint4* copy_dst = nullptr) {
    using F = typename Cv::Base;
    using S = typename Cv::Scalar;
    __shared__ uint4 red[TAIL_THREADS / 2 * 8];
    __shared__ uint32_t kw[8];
    __shared__ uint32_t neg[2];
    const int tid = threadIdx.x, b = blockIdx.x;
    if (htab && tid == 0) {  // dot_b = k1 + lambda k2: lanes 0-127 k1 with 2^i H', 128-255 k2 with phi(2^i H')
        uint32_t w8[8], k1[5], k2[5];
        bool n1, n2;
        fe_ark_to_canonical_words<S>(dots_ark + 2 * b, w8);
        glv::decompose<typename Cv::K>(w8, n1, k1, n2, k2);
        for (int q = 0; q < 4; q++) {
            kw[q] = k1[q];
            kw[4 + q] = k2[q];
        }
        neg[0] = n1;
        neg[1] = n2;
    }
    __syncthreads();
    // lane tid: its partials plus, for bit tid of (k1 | k2), the table entry -- one tree
    XYZZ<F> acc = xyzz_id<F>();
    if (htab && ((kw[tid >> 5] >> (tid & 31)) & 1u)) {
        Affine<F> p = aff_load<F>(htab + 4 * (tid & 127));
        if (tid >= 128) p.x = fe_mul(p.x, fe_from_const<F>(Cv::K::BETA));
        if (neg[tid >> 7]) p.y = fe_neg(p.y);
        acc = xyzz_from_aff(p);
    }
    // this side's partials (blocks [b per_side, (b + 1) per_side)), dealt round-robin over the waves so
    // that every SIMD's wave sums a quarter of them
    const int per_side = nblk / (int)gridDim.x, j0 = (tid & 63) * (TAIL_THREADS / 64) + (tid >> 6);
    for (int j = j0; j < per_side; j += TAIL_THREADS)
        acc = xyzz_add(acc, xyzz_load<F>(part + 8 * (2 * (size_t)(b * per_side + j) + b)));
    acc = block_group_sum<F>(acc, TAIL_THREADS, red);
    if (tid == 0) {
        if (plus_wrapped) acc = xyzz_madd(acc, aff_from_wrapped<F>(plus_wrapped));  // (the combine's + C)
        if (copy_src) {  // 32 B beside the result, so that one D2H copy takes both
            copy_dst[0] = copy_src[0];
            copy_dst[1] = copy_src[1];
        }
        if (xyzz_out) {  // 128 B per side, converted on the host (host_xyzz_to_wrapped)
            xyzz_store(out_wrapped + 8 * b, acc);
            if (host) tail_emit_host(host, host + 64, b, acc, seq);
        } else {
            aff_to_wrapped(out_wrapped + 4 * b, xyzz_to_aff(acc));
        }
    }
}

template <class S>
__global__ void k_set_one_ark(uint4* out) {
    if (threadIdx.x == 0) fe_to_ark(out, fe_one<S>());
}

// Small host values passed by value and stored by one launch (instead of one H2D copy per value, each
// a blit kernel of ~4 us on the stream): segment i is cnt[i] uint4 at dst[i], taken in order from v.
struct PutArgs {
    uint4* dst[4];
    int cnt[4];
    uint4 v[16];
};
__global__ void k_put_args(PutArgs a) {
    int base = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if ((int)threadIdx.x < a.cnt[i]) a.dst[i][threadIdx.x] = a.v[base + threadIdx.x];
        base += a.cnt[i];
    }
}

// x[i] *= k (ark scalars, i < count): the IPA's dots scaled by xi_0 in xi mode
template <class S>
__global__ void k_scale_ark(uint4* x, int count, const uint4* k) {
    const int i = threadIdx.x;
    if (i < count) fe_to_ark(x + 2 * i, fe_mul(fe_from_ark<S>(x + 2 * i), fe_from_ark<S>(k)));
}

// c / z folds (pcdl.rs:430-435) and the weight update w' = interleave(w, xi w)
// xi | xi^-1 (ark words) as one by-value kernel argument
struct ArkScalarPair {
    uint4 v[4];
};

template <class Cv>
__global__ __launch_bounds__(256) void k_tail_fold(uint4* cs, uint4* zs, size_t m, ArkScalarPair x,
                                                   const uint4* w_in, uint4* w_out, size_t wlen) {
    using S = typename Cv::Scalar;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const Fe<S> xi = fe_from_ark<S>(x.v);
    if (i < m) {
        const Fe<S> xinv = fe_from_ark<S>(x.v + 2);
        fe_to_ark(cs + 2 * i, fe_add(fe_from_ark<S>(cs + 2 * i), fe_mul(fe_from_ark<S>(cs + 2 * (i + m)), xinv)));
        fe_to_ark(zs + 2 * i, fe_add(fe_from_ark<S>(zs + 2 * i), fe_mul(fe_from_ark<S>(zs + 2 * (i + m)), xi)));
    }
    if (i < wlen) {
        const Fe<S> wv = fe_from_ark<S>(w_in + 2 * i);
        fe_to_ark(w_out + 2 * (2 * i), wv);
        fe_to_ark(w_out + 2 * (2 * i + 1), fe_mul(wv, xi));
    }
}

// Weighted rounds (sessions over the resident SRS, length > IPA_TAIL_N): G is never folded.  With
// len = 2m and the fold weights w (as in the tail rounds, G_i = sum_u w[u] SRS[i + u len]),
//   L = sum_{u, i < m} c[m + i] w[u] SRS[u len + i],   R = sum_{u, i < m} c[i] w[u] SRS[u len + m + i],
// two MSMs of n/2 terms over the resident window-shifted SRS (msm_srs_range_device, block map
// blk_lg = lg m).  Term j = u m + i of both: sl[j] = c[m + i] w[u], sr[j] = c[i] w[u].
template <class S>
__global__ __launch_bounds__(256) void k_weighted_scalars(const uint4* cs, const uint4* w, size_t m, int lgm,
                                                          size_t total, uint4* sl, uint4* sr) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= total) return;
    const size_t u = j >> lgm, i = j & (m - 1);
    const Fe<S> wu = fe_from_ark<S>(w + 2 * u);
    fe_to_ark(sl + 2 * j, fe_mul(fe_from_ark<S>(cs + 2 * (m + i)), wu));
    fe_to_ark(sr + 2 * j, fe_mul(fe_from_ark<S>(cs + 2 * i), wu));
}

// A weighted round's preparation in one launch (was five: two dot products of two kernels each, the
// xi_0 scaling and k_weighted_scalars): the weighted scalars of both sides (when sl is non-null: w has
// more than one entry), and the two dots <c_r, z_l>, <c_l, z_r> as block partials whose last arriving
// block (release / acquire on *ctr, reset by it) sums them, canonicalises, scales by xi_0 (xi0_ark
// non-null) and writes dots_ark[0..2).  Same products and sums as k_dot_partial /
// k_sum_partials_to_ark / k_scale_ark, so the results are identical.  part: 2 x ndot elements
// (ndot <= gridDim.x blocks carry the dots).
template <class S>
__global__ __launch_bounds__(256) void k_weighted_prep(const uint4* cs, const uint4* zs, const uint4* w, size_t m,
                                                       int lgm, size_t total, uint4* sl, uint4* sr, uint4* part,
                                                       uint32_t* ctr, const uint4* xi0_ark, uint4* dots_ark,
                                                       uint32_t ndot) {
    __shared__ uint4 red[256 * 4];
    __shared__ uint32_t flag;
    const uint32_t tid = threadIdx.x;
    const size_t j = (size_t)blockIdx.x * 256 + tid;
    if (sl && j < total) {
        const size_t u = j >> lgm, i = j & (m - 1);
        const Fe<S> wu = fe_from_ark<S>(w + 2 * u);
        fe_to_ark(sl + 2 * j, fe_mul(fe_from_ark<S>(cs + 2 * (m + i)), wu));
        fe_to_ark(sr + 2 * j, fe_mul(fe_from_ark<S>(cs + 2 * i), wu));
    }
    // the dots: the first ndot blocks only (grid-stride over m), so that at most ndot arrivals meet on
    // the one counter (2048 same-address adds cost more than the launches they replace)
    if (blockIdx.x >= ndot) return;
    const size_t stride = (size_t)ndot * 256;
    Fe<S> a = fe_zero<S>(), b = fe_zero<S>();
    for (size_t i = j; i < m; i += stride) {
        a = fe_add(a, fe_mul(fe_load<S>(cs + 2 * (m + i)), fe_from_ark<S>(zs + 2 * i)));
        b = fe_add(b, fe_mul(fe_load<S>(cs + 2 * i), fe_from_ark<S>(zs + 2 * (m + i))));
    }
    auto block_sum2 = [&](Fe<S>& x, Fe<S>& y) {
        fe_store(red + 4 * tid, x);
        fe_store(red + 4 * tid + 2, y);
        __syncthreads();
        for (uint32_t off = 128; off > 0; off >>= 1) {
            if (tid < off) {
                fe_store(red + 4 * tid, fe_add(fe_load<S>(red + 4 * tid), fe_load<S>(red + 4 * (tid + off))));
                fe_store(red + 4 * tid + 2, fe_add(fe_load<S>(red + 4 * tid + 2), fe_load<S>(red + 4 * (tid + off) + 2)));
            }
            __syncthreads();
        }
        x = fe_load<S>(red);
        y = fe_load<S>(red + 2);
    };
    block_sum2(a, b);
    if (tid == 0) {
        tail_publish_fe((uint32_t*)(part + 4 * (size_t)blockIdx.x), a);
        tail_publish_fe((uint32_t*)(part + 4 * (size_t)blockIdx.x + 2), b);
    }
    if (!tail_arrive(ctr, ndot, &flag)) return;
    a = fe_zero<S>();
    b = fe_zero<S>();
    for (uint32_t q = tid; q < ndot; q += 256) {
        a = fe_add(a, fe_load<S>(part + 4 * (size_t)q));
        b = fe_add(b, fe_load<S>(part + 4 * (size_t)q + 2));
    }
    __syncthreads();  // (red is reused)
    block_sum2(a, b);
    if (tid != 0) return;
    *ctr = 0u;
    Fe<S> d[2] = {fe_canon(fe_reduce_2p(a)), fe_canon(fe_reduce_2p(b))};
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (xi0_ark) {
            fe_store(dots_ark + 2 * k, d[k]);  // (ark words, as k_sum_partials_to_ark leaves them)
            fe_to_ark(dots_ark + 2 * k, fe_mul(fe_from_ark<S>(dots_ark + 2 * k), fe_from_ark<S>(xi0_ark)));
        } else {
            fe_store(dots_ark + 2 * k, d[k]);
        }
    }
}

// The dot blocks of k_weighted_prep alone (no scalars), as a MsmPreHide hook of the pair MSM
struct WeightedDots {
    const uint4 *cs, *zs;
    size_t m;
    uint4* part;
    uint32_t* ctr;
    const uint4* xi0;
    uint4* dots;
    uint32_t ndot;
    int curve;
};
static void weighted_dots_launch(hipStream_t ts, void* ctx) {
    const WeightedDots& d = *(const WeightedDots*)ctx;
    DISPATCH_CURVE(d.curve, Cv, {
        hipLaunchKernelGGL(k_weighted_prep<typename Cv::Scalar>, dim3(d.ndot), dim3(256), 0, ts, d.cs, d.zs,
                           (const uint4*)nullptr, d.m, 0, (size_t)0, (uint4*)nullptr, (uint4*)nullptr, d.part, d.ctr,
                           d.xi0, d.dots, d.ndot);
    });
}

}  // namespace halo

using namespace halo;

// One opening.  Sessions are pooled per device (ipa_acquire / ipa_release): the streams, events,
// pinned staging and every device buffer survive halo_ipa_end and are reused by the next opening,
// so an opening allocates nothing once the pool is warm (~11 hipMallocs, two stream
// creations and a pinned allocation per opening; ADVICE r02: the buffers leaked at end).
struct halo_ipa_session {
    // ---- resources (kept across pooled uses)
    int device = -1;
    hipStream_t s = nullptr;
    hipStream_t s2 = nullptr;           // weighted rounds above ipa_pair_max: R's MSM (created on first use)
    bool solo = true;                   // the round call advances this session alone (s2 is used then)
    bool slots_reset = false;           // this opening restarted the MSM slot assignment (msm_slots_reset)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t htab_ready = nullptr;  // recorded after the session's own 2^i H' table
    hipEvent_t lr_ready = nullptr;    // halo_ipa_round_lr_dev: L, R copied out (created on first use)
    uint8_t* pinned = nullptr;  // [128, 192) xi|xi_inv (H2D), [256, 512) L|R XYZZ (D2H or tail_emit_host),
                                // [512, 520) the L / R flags of tail_emit_host: coherent, several sessions in flight
    uint32_t poll_seq = 0;      // the last tail round's flag value (monotonic over the session object's life)
    bool poll_pending = false;  // the last round emits L / R to `pinned` itself: poll instead of synchronising
    DevBuf gs, cs, zs, htab, small, tmp, pbar;
    DevBuf cs2, zs2;  // ping-pong partners of cs / zs (tail rounds with a deferred fold)
    DevBuf own_table, w[2], scal, side, part;
    BatchScratch mat;  // weighted -> tail switch (msm_shared_batch)
    // handed out by ipa_acquire and not yet returned by ipa_release (guarded by g_pool_mu): every
    // session entry point refuses a handle that is not open, and a second end cannot pool it twice
    bool in_use = false;
    // ---- per-opening state (reset by ipa_acquire)
    int curve = 0;
    size_t n = 0, m = 0;
    // tail rounds (length <= IPA_TAIL_N, sessions over the SRS only): see k_tail_table
    bool allow_tail = false, tail = false;
    bool srs_round0 = false;  // G is still the SRS prefix (no fold yet): L/R on the resident shifted SRS
    bool gs_srs_prefix = false;  // G (length 2m) = Gs[0..2m): the tail can use the SRS's multiples table
    bool tail_from_srs = false;  // n <= ipa_srs_tail_max(): tail rounds from round 1 over the SRS's table
    bool gs_xyzz = false;     // gs holds XYZZ points (materialised for the tail table only)
    bool gs_valid = false;    // gs holds the current G (halo_ipa_state may read it)
    bool weighted = false;    // G is never folded: L/R over the resident shifted SRS (k_weighted_scalars)
    size_t n0 = 0, wlen = 0;
    int wcur = 0;
    const uint4* table = nullptr;  // tail multiples table: own_table, or the SRS's small table
    size_t table_ld = 0;
    std::shared_ptr<DevBuf> table_ref;  // keeps the SRS's table alive while the session reads it
    bool fold_inflight = false;       // a fold's H2D copy of xi may still read `pinned`
    bool fold_pending = false;        // tail rounds: the last fold is applied by the next launch (k_tail_prep)
    bool w_one_pending = false;       // entered the tail rounds: w = [1] is written by the next tail launch
    halo_fe_t pend_xi{}, pend_xinv{};
    size_t pend_m = 0;                // the half-length m the pending fold folds (before its m /= 2)
    bool htab_waited = false;         // round 1 waited for it (later rounds follow a host sync of round 1)
    // xi mode (halo_ipa_begin_xi / _dev_xi / halo_pcdl_open_start): the hiding terms use the resident
    // 2^i H table and the dots scaled by xi_0 (dot H' = (dot xi_0) H), so there is neither H' nor a
    // per-session table
    bool xi_mode = false;
    const void* htab_ptr = nullptr;  // 2^i H' (own table) or 2^i H (SrsState::h_tables)
    bool started = false;            // rounds may run (a pcdl open session starts at halo_pcdl_open_start)
    bool blinded = false;            // halo_pcdl_open_blind ran (pbar holds p_bar)
    bool combined = false;           // halo_pcdl_open_combine ran

    void reset_state() {
        curve = 0;
        n = m = 0;
        allow_tail = tail = srs_round0 = gs_srs_prefix = tail_from_srs = gs_xyzz = gs_valid = weighted = false;
        n0 = wlen = 0;
        wcur = 0;
        table = nullptr;
        table_ld = 0;
        fold_inflight = htab_waited = xi_mode = fold_pending = slots_reset = w_one_pending = false;
        htab_ptr = nullptr;
        started = blinded = combined = false;
    }
    size_t buffer_bytes() const {
        size_t b = 0;
        for (const DevBuf* d : {&gs, &cs, &zs, &cs2, &zs2, &htab, &small, &tmp, &pbar, &own_table, &w[0], &w[1], &scal,
                                &side, &part, &mat.digits, &mat.lists, &mat.keys, &mat.vals, &mat.bstart, &mat.partials,
                                &mat.bucket_sums, &mat.window_sums})
            b += d->bytes;
        return b;
    }
    void release_large() {  // everything sized by n (the small staging and the H' table stay)
        for (DevBuf* d : {&gs, &cs, &zs, &cs2, &zs2, &tmp, &pbar, &own_table, &w[0], &w[1], &scal, &side, &part,
                          &mat.digits, &mat.lists, &mat.keys, &mat.vals, &mat.bstart, &mat.partials, &mat.bucket_sums,
                          &mat.window_sums})
            d->release();
    }
    void destroy() {
        if (s) (void)hipStreamSynchronize(s);
        if (s2) (void)hipStreamSynchronize(s2);
        if (htab_ready) (void)hipEventDestroy(htab_ready);
        if (lr_ready) (void)hipEventDestroy(lr_ready);
        lr_ready = nullptr;
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (s) (void)hipStreamDestroy(s);
        if (s2) (void)hipStreamDestroy(s2);
        s2 = nullptr;
        ev_fork = ev_join = nullptr;
        if (pinned) (void)hipHostFree(pinned);
        s = nullptr;
        htab_ready = nullptr;
        pinned = nullptr;
        for (DevBuf* b : {&gs, &cs, &zs, &cs2, &zs2, &htab, &small, &tmp, &pbar, &own_table, &w[0], &w[1], &scal, &side,
                          &part})
            b->release();
        for (DevBuf* b : {&mat.digits, &mat.lists, &mat.keys, &mat.vals, &mat.bstart, &mat.partials, &mat.bucket_sums,
                          &mat.window_sums})
            b->release();
    }
};

namespace {
constexpr size_t IPA_POOL_MAX = 8;  // idle sessions kept per device
std::mutex g_pool_mu;
std::vector<halo_ipa_session*> g_pool;
// every session object that exists (open or pooled), guarded by g_pool_mu: a handle is looked up here
// before anything dereferences it, so a handle whose session was destroyed (the pool was full at its
// end, or halo_shutdown ran) is refused instead of read after free
std::unordered_set<const halo_ipa_session*> g_live;

void ipa_destroy(halo_ipa_session* ses) {
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        g_live.erase(ses);
    }
    ses->destroy();
    delete ses;
}

// A session for the current device: from the pool, or new with its streams and pinned staging.
halo_ipa_session* ipa_acquire(DeviceState* st) {
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = g_pool.size(); i-- > 0;)
            if (g_pool[i]->device == st->device) {
                halo_ipa_session* ses = g_pool[i];
                g_pool.erase(g_pool.begin() + i);
                ses->reset_state();
                ses->in_use = true;
                return ses;
            }
    }
    auto* ses = new halo_ipa_session();
    ses->device = st->device;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        g_live.insert(ses);
    }
    // one stream per session (a side stream for the H' table of explicit-H' sessions was measured: with
    // HIP's default 4 hardware queues it shares a queue with the MSM tail streams, ~0.3 ms per 2^16
    // round; the prover's and pcdl::open's sessions use the resident 2^i H tables and build none)
    if (hipStreamCreateWithFlags(&ses->s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ses->htab_ready, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void**)&ses->pinned, 1024, hipHostMallocCoherent) != hipSuccess) {
        ipa_destroy(ses);
        set_error(HALO_EDEVICE, "halo_ipa_begin: stream / pinned buffer allocation failed");
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        ses->in_use = true;
    }
    return ses;
}

// the handle is an open session (checked before anything touches its state).  A
// handle of a destroyed session, or of one idle in the pool, is refused; a pooled session handed to a
// later opening is that opening's again, so a handle must not be used after its end (halo_gpu.h)
bool ipa_is_open(const halo_ipa_session* ses) {
    std::lock_guard<std::mutex> g(g_pool_mu);
    return ses && g_live.count(ses) && ses->in_use;
}

// Back to the pool once its stream is idle (the pinned staging is then free); beyond IPA_POOL_MAX
// idle sessions on the device the resources are released.
void ipa_release(halo_ipa_session* ses) {
    if (!ses) return;
    {
        // a handle that is not open (a second end of the same handle) is neither touched nor pooled
        // twice: two later openings would otherwise share its streams and buffers
        std::lock_guard<std::mutex> g(g_pool_mu);
        if (!g_live.count(ses) || !ses->in_use) return;
        ses->in_use = false;
    }
    if (ses->s) (void)hipStreamSynchronize(ses->s);
    ses->table_ref.reset();  // a retired SRS multiples table is freed with its last session
    // an idle session keeps at most "ipa_pool_keep_bytes" of device buffers (tuning, default 1 GB: a
    // 2^20 opening's ~0.6 GB stay pooled for the next one): above it the per-size buffers
    // are released here
    if ((long long)ses->buffer_bytes() > tuning(TUNE_IPA_POOL_KEEP)) ses->release_large();
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        size_t same = 0;
        for (halo_ipa_session* p : g_pool) same += p->device == ses->device;
        if (same < IPA_POOL_MAX) {
            g_pool.push_back(ses);
            return;
        }
    }
    ipa_destroy(ses);
}
}  // namespace

// halo_shutdown: releases the pooled sessions while the HIP runtime is alive.
void halo::ipa_shutdown() {
    std::lock_guard<std::mutex> g(g_pool_mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (halo_ipa_session* ses : g_pool) {
        (void)hipSetDevice(ses->device);
        g_live.erase(ses);
        ses->destroy();
        delete ses;
    }
    g_pool.clear();
    (void)hipSetDevice(cur);
}

static int check_field_i(halo_field_t f) {
    if (f != HALO_FP && f != HALO_FQ) return set_error(HALO_EINVAL, "unknown field id %d", (int)f);
    return HALO_OK;
}

extern "C" int halo_scalar_dot(halo_field_t field, const halo_fe_t* xs, const halo_fe_t* ys, size_t n, halo_fe_t* out) {
    clear_error();
    HALO_CHECK(check_field_i(field));
    if (!out || (n && (!xs || !ys))) return set_error(HALO_EINVAL, "halo_scalar_dot: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(n, 1) * 32));
    HALO_CHECK(st->scratch[1].reserve(std::max<size_t>(n, 1) * 32));
    HALO_CHECK(st->scratch[2].reserve(2048 * 32 + 64));
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, xs, n * 32, s));
    HALO_CHECK(copy_h2d(st->scratch[1].ptr, ys, n * 32, s));
    char* t = (char*)st->scratch[2].ptr;
    HALO_CHECK(dot_device(field, st->scratch[0].ptr, st->scratch[1].ptr, n, t + 2048 * 32, t, s));
    return copy_d2h(out, t + 2048 * 32, 32, s);
}

extern "C" int halo_construct_powers(halo_field_t field, const halo_fe_t* z, size_t n, halo_fe_t* out) {
    clear_error();
    HALO_CHECK(check_field_i(field));
    if (!z || (n && !out)) return set_error(HALO_EINVAL, "halo_construct_powers: null buffer");
    if (!n) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(n * 32 + 32));
    char* b = (char*)st->scratch[0].ptr;
    HALO_CHECK(copy_h2d(b, z, 32, s));
    const size_t run = 16;
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_powers<F>, dim3(gridn((n + run - 1) / run, 128)), dim3(128), 0, s, (const uint4*)b, n, run,
                           (uint4*)(b + 32));
    });
    HALO_HIP(hipGetLastError());
    return copy_d2h(out, b + 32, n * 32, s);
}

extern "C" int halo_poly_eval_batch(halo_field_t field, const halo_fe_t* const* polys, const size_t* lens, size_t k,
                                    const halo_fe_t* z, halo_fe_t* out) {
    clear_error();
    HALO_CHECK(check_field_i(field));
    if (!z || (k && (!polys || !lens || !out))) return set_error(HALO_EINVAL, "halo_poly_eval_batch: null buffer");
    if (!k) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    size_t total = 0, maxlen = 0;
    for (size_t i = 0; i < k; i++) {
        if (lens[i] && !polys[i]) return set_error(HALO_EINVAL, "halo_poly_eval_batch: null polynomial %zu", i);
        total += lens[i];
        maxlen = std::max(maxlen, lens[i]);
    }
    const size_t chunk = 32;
    const int nchunks = (int)std::max<size_t>(1, (maxlen + chunk * RED_THREADS - 1) / (chunk * RED_THREADS));
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(total, 1) * 32));
    HALO_CHECK(st->scratch[1].reserve(k * (sizeof(void*) + sizeof(size_t)) + 64));
    HALO_CHECK(st->scratch[2].reserve((size_t)k * nchunks * 32 + k * 32));
    std::vector<const void*> dptr(k);
    size_t off = 0;
    char* base = (char*)st->scratch[0].ptr;
    for (size_t i = 0; i < k; i++) {
        dptr[i] = base + off * 32;
        HALO_CHECK(copy_h2d(base + off * 32, polys[i], lens[i] * 32, s));
        off += lens[i];
    }
    char* meta = (char*)st->scratch[1].ptr;
    HALO_CHECK(copy_h2d(meta, dptr.data(), k * sizeof(void*), s));
    HALO_CHECK(copy_h2d(meta + k * sizeof(void*), lens, k * sizeof(size_t), s));
    HALO_CHECK(copy_h2d(meta + k * (sizeof(void*) + sizeof(size_t)), z, 32, s));
    char* part = (char*)st->scratch[2].ptr;
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_eval_chunks<F>, dim3(nchunks, (unsigned)k), dim3(RED_THREADS), 0, s,
                           (const uint4* const*)meta, (const size_t*)(meta + k * sizeof(void*)),
                           (const uint4*)(meta + k * (sizeof(void*) + sizeof(size_t))), chunk, nchunks, (uint4*)part);
        hipLaunchKernelGGL(k_sum_internal_to_ark<F>, dim3((unsigned)k), dim3(RED_THREADS), 0, s, (const uint4*)part,
                           nchunks, (uint4*)(part + (size_t)k * nchunks * 32));
    });
    HALO_HIP(hipGetLastError());
    return copy_d2h(out, part + (size_t)k * nchunks * 32, k * 32, s);
}

// Device-resident variant (the prover's 78 evaluations at xi, protocol.rs:315-323): d_polys is a
// host array of k device pointers (ark coefficients), results (ark) to d_out[k].  Stream-ordered;
// the pointer table is staged through a per-device buffer, so calls on one stream may be queued back
// to back.
extern "C" int halo_poly_eval_batch_dev(halo_field_t field, const void* const* d_polys, const size_t* lens, size_t k,
                                        const halo_fe_t* z, void* d_out, void* stream) {
    clear_error();
    HALO_CHECK(check_field_i(field));
    if (!z || (k && (!d_polys || !lens || !d_out))) return set_error(HALO_EINVAL, "halo_poly_eval_batch_dev: null buffer");
    if (!k) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = (hipStream_t)stream;
    ScratchUse su(st, s);
    size_t maxlen = 0;
    for (size_t i = 0; i < k; i++) {
        if (lens[i] && !d_polys[i]) return set_error(HALO_EINVAL, "halo_poly_eval_batch_dev: null polynomial %zu", i);
        maxlen = std::max(maxlen, lens[i]);
    }
    const size_t chunk = 32;
    const int nchunks = (int)std::max<size_t>(1, (maxlen + chunk * RED_THREADS - 1) / (chunk * RED_THREADS));
    const size_t meta_bytes = k * (sizeof(void*) + sizeof(size_t)) + 32;
    HALO_CHECK(st->eval_meta[0].reserve(meta_bytes));
    HALO_CHECK(st->eval_meta[1].reserve((size_t)k * nchunks * 32));
    std::vector<unsigned char> host(meta_bytes);
    memcpy(host.data(), d_polys, k * sizeof(void*));
    memcpy(host.data() + k * sizeof(void*), lens, k * sizeof(size_t));
    memcpy(host.data() + k * (sizeof(void*) + sizeof(size_t)), z, 32);
    char* meta = (char*)st->eval_meta[0].ptr;
    HALO_CHECK(copy_h2d(meta, host.data(), meta_bytes, s));
    char* part = (char*)st->eval_meta[1].ptr;
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_eval_chunks<F>, dim3(nchunks, (unsigned)k), dim3(RED_THREADS), 0, s,
                           (const uint4* const*)meta, (const size_t*)(meta + k * sizeof(void*)),
                           (const uint4*)(meta + k * (sizeof(void*) + sizeof(size_t))), chunk, nchunks, (uint4*)part);
        hipLaunchKernelGGL(k_sum_internal_to_ark<F>, dim3((unsigned)k), dim3(RED_THREADS), 0, s, (const uint4*)part,
                           nchunks, (uint4*)d_out);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_poly_mul(halo_field_t field, const halo_fe_t* a, size_t la, const halo_fe_t* b, size_t lb,
                             halo_fe_t* out, size_t* out_len) {
    clear_error();
    HALO_CHECK(check_field_i(field));
    if ((la && !a) || (lb && !b) || !out_len) return set_error(HALO_EINVAL, "halo_poly_mul: null buffer");
    if (la == 0 || lb == 0) {
        *out_len = 0;  // the zero polynomial
        return HALO_OK;
    }
    if (!out) return set_error(HALO_EINVAL, "halo_poly_mul: null out");
    const size_t rl = la + lb - 1;
    unsigned logn = 0;
    while (((size_t)1 << logn) < rl) logn++;
    if (logn > 28) return set_error(HALO_EINVAL, "halo_poly_mul: product too large");
    const size_t N = (size_t)1 << logn;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    for (int i = 0; i < 5; i++) HALO_CHECK(st->scratch[i].reserve(N * 32));
    char* A = (char*)st->scratch[0].ptr;
    char* Bv = (char*)st->scratch[1].ptr;
    char* FA = (char*)st->scratch[2].ptr;
    char* FB = (char*)st->scratch[3].ptr;
    char* T = (char*)st->scratch[4].ptr;
    HALO_HIP(hipMemsetAsync(A, 0, N * 32, s));
    HALO_HIP(hipMemsetAsync(Bv, 0, N * 32, s));
    HALO_CHECK(copy_h2d(A, a, la * 32, s));
    HALO_CHECK(copy_h2d(Bv, b, lb * 32, s));
    HALO_CHECK(ntt_device_dispatch(st, field, A, FA, T, logn, 1, 0, s));
    HALO_CHECK(ntt_device_dispatch(st, field, Bv, FB, T, logn, 1, 0, s));
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_pointwise_mul<F>, dim3(gridn(N, 256)), dim3(256), 0, s, (uint4*)FA, (const uint4*)FB, N);
    });
    HALO_HIP(hipGetLastError());
    HALO_CHECK(ntt_device_dispatch(st, field, FA, A, T, logn, 1, 1, s));
    std::vector<halo_fe_t> tmp(rl);
    HALO_CHECK(copy_d2h(tmp.data(), A, rl * 32, s));
    size_t n = rl;
    while (n > 0 && !(tmp[n - 1].l[0] | tmp[n - 1].l[1] | tmp[n - 1].l[2] | tmp[n - 1].l[3])) n--;
    std::copy(tmp.begin(), tmp.begin() + n, out);
    *out_len = n;
    return HALO_OK;
}

// ------------------------------------------------------------------------------------------ IPA
// Session start shared by halo_ipa_begin (G = resident SRS prefix, z powers generated on the
// device) and halo_ipa_begin_vectors (explicit G, c, z: a shard of a distributed opening or its
// final collapsed rounds, halo_amd/dist.py).
static size_t ipa_tail_n() { return IPA_TAIL_N; }

// 8192 points (0.5 GB of XYZZ multiples per curve): the small MSMs up to 2^13 and the openings up to
// 2^13 run entirely on the table (tail rounds from round 1, no weighted rounds, no materialisation)
size_t halo::srs_tab_n() { return 8192; }
size_t halo::srs_small_max() { return srs_tab_n(); }
// SRS sessions of n <= this start in the tail rounds over the SRS's table.  A tail round costs ~64 n0
// table terms: measured per round (hiding open, tools/pcdl_open_time.py) 0.23 ms at n0 = 4096 against
// 0.29 ms for the weighted path's average (opening 2^12: 5.95 -> 3.86 ms), but 0.33 ms at n0 = 8192,
// where the weighted rounds are cheaper.
static size_t ipa_srs_tail_max() {  // tuning "ipa_srs_tail_n" (default 4096; the tests pin the other paths)
    return std::min((size_t)tuning(TUNE_IPA_SRS_TAIL_N), srs_tab_n());
}

// Length at which weighted rounds materialise G = sum_u w[u] SRS[i + u len] (one batched MSM with
// the fold weights as shared scalars, msm_shared_batch) and continue as tail rounds: a weighted
// round costs two n/2-term MSMs whatever the length (~0.75 ms at 2^16), a tail round ~0.25 ms.
// Measured (opening 2^12 / 2^16 / 2^20, ms): 1024: 6.2 / 10.4 / 29.3; 2048: 5.6 / 9.3 / 27.6;
// 4096 (tail 4096): 6.5 / 10.7 / 27.4; 8192: 6.4 / 12.8 / 28.4.
// (tuning "ipa_mat_n", default 2048)
static size_t ipa_mat_n() {  // 0 keeps the weighted rounds to the end
    return (size_t)tuning(TUNE_IPA_MAT_N);
}

// The 2^i H tables (i < IPA_HTAB, internal affine) of xi-mode sessions, kept per device and curve,
// one per distinct H and never rewritten (open sessions hold pointers into them; ADVICE r02: a new H
// used to rebuild the one shared table under live sessions).  One ~1 ms doubling chain per H, then
// shared by every later opening.  Past IPA_HTABLES_MAX distinct H, *out = nullptr: the session builds
// its own table.
constexpr size_t IPA_HTABLES_MAX = 8;
static int ipa_h_table(DeviceState* st, int curve, const halo_wrapped_point_t* Hpt, const void** out) {
    SrsState& srs = st->srs[curve];
    *out = nullptr;
    for (auto& t : srs.h_tables)
        if (!memcmp(t->key, Hpt, 64)) {
            *out = t->t.ptr;
            return HALO_OK;
        }
    if (srs.h_tables.size() >= IPA_HTABLES_MAX) return HALO_OK;
    auto ht = std::make_unique<SrsState::HTable>();
    HALO_CHECK(ht->t.reserve(IPA_HTAB * 64));
    const hipStream_t s = nullptr;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[7].reserve(IPA_HTAB * 128 + 64));
    char* tmp = (char*)st->scratch[7].ptr;
    HALO_CHECK(copy_h2d(tmp + IPA_HTAB * 128, Hpt, 64, s));
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_pow2_xyzz_from_wrapped<Cv>, dim3(1), dim3(64), 0, s, (const uint4*)(tmp + IPA_HTAB * 128),
                           (uint4*)tmp, IPA_HTAB);
        hipLaunchKernelGGL(k_xyzz_to_aff_ipa<Cv>, dim3(IPA_HTAB / 64), dim3(64), 0, s, (const uint4*)tmp,
                           ht->t.as<uint4>(), IPA_HTAB);
    });
    HALO_HIP(hipGetLastError());
    HALO_HIP(hipStreamSynchronize(s));  // sessions on other streams read it
    memcpy(ht->key, Hpt, 64);
    *out = ht->t.ptr;
    srs.h_tables.push_back(std::move(ht));
    return HALO_OK;
}

// small-buffer layout of a session (ses->small, device):
//   [0, 32) z | [64, 128) H' (or H) | [128, 192) dots | [192, 224) xi_0 | [256, 384) U | c
//   [384, 448) xi | xi^-1 | [512, 768) L | R XYZZ
//   hiding open: [1024) w_bar, [1056) alpha, [1088) w, [1120) w' out, [1152) C, [1216) C_bar out,
//   [1280) S (internal), [1344) C' out
constexpr size_t SM_BYTES = 2048;
constexpr size_t SM_WBAR = 1024, SM_ALPHA = 1056, SM_W = 1088, SM_WP = 1120, SM_C = 1152, SM_CBAR = 1216, SM_S = 1280,
                 SM_CP = 1344, SM_NEGW = 1408, SM_T = 1536, SM_V = 1696,  // SM_T: 128 B XYZZ
                 SM_HKW = 1728,  // 2 x 10 words: the dots' GLV splits (k_tail_digits -> k_tail_round)
                 SM_CTR = 1856;  // 2 x u32 arrival counters of k_tail_round, 1 of k_weighted_prep (zero between launches)

// Phase 1 of a session: G (resident SRS prefix, or explicit gs_host), c (cs_len coefficients, host or
// device (ordered on the null stream), zero-padded to n), z = powers of z (or explicit zs_host) on the
// device.  st->mu held; ses freshly acquired.
static int ipa_setup(DeviceState* st, halo_ipa_session* ses, int curve, size_t n, const halo_wrapped_point_t* gs_host,
                     const halo_fe_t* cs, size_t cs_len, bool cs_on_device, const halo_fe_t* zs_host, const halo_fe_t* z) {
    SrsState& srs = st->srs[curve];
    ses->curve = curve;
    {
        // tuning "ipa_tail" / "ipa_weighted" (default 1): 0 = no tail rounds / fold G every round
        ses->allow_tail = !gs_host && tuning(TUNE_IPA_TAIL) != 0;
        ses->tail_from_srs = ses->allow_tail && n <= std::min(ipa_srs_tail_max(), srs.n);
        ses->weighted = !gs_host && srs.shifted_c != 0 && n > ipa_tail_n() && !ses->tail_from_srs &&
                        tuning(TUNE_IPA_WEIGHTED) != 0;
        if (ses->weighted) ses->allow_tail = false;
        ses->srs_round0 = !gs_host && srs.shifted_c != 0 && !ses->weighted;
        ses->gs_srs_prefix = !gs_host && !ses->weighted;
    }
    ses->n = n;
    ses->m = n / 2;
    hipStream_t s = ses->s;
    // an SRS session that starts in the tail rounds never reads G itself (the SRS's table does)
    const bool need_gs = !ses->weighted && !(ses->gs_srs_prefix && ses->allow_tail && (n <= ipa_tail_n() || ses->tail_from_srs));
    if (need_gs || gs_host) HALO_CHECK(ses->gs.reserve(n * 64));
    ses->gs_valid = need_gs || gs_host;
    if (ses->weighted) {  // w = [1]; scal holds the two n/2-term scalar vectors of a round
        HALO_CHECK(ses->w[0].reserve(n * 32));
        HALO_CHECK(ses->w[1].reserve(n * 32));
        HALO_CHECK(ses->scal.reserve(n * 32));
        DISPATCH_CURVE(curve, Cv, {
            hipLaunchKernelGGL(k_set_one_ark<typename Cv::Scalar>, dim3(1), dim3(64), 0, s, ses->w[0].as<uint4>());
        });
        ses->n0 = n;
        ses->wlen = 1;
        ses->wcur = 0;
    }
    HALO_CHECK(ses->cs.reserve(n * 32));
    HALO_CHECK(ses->zs.reserve(n * 32));
    HALO_CHECK(ses->small.reserve(SM_BYTES));
    HALO_HIP(hipMemsetAsync(ses->small.as<char>() + SM_CTR, 0, 12, s));  // k_tail_round's / k_weighted_prep's counters
    // (n / 4: k_weighted_prep's block partials, 64 B per 256 terms of a side)
    HALO_CHECK(ses->tmp.reserve(std::max<size_t>({4096 * 32, gs_host ? n * 64 : 0, n / 4})));
    if (gs_host) {
        HALO_CHECK(copy_h2d(ses->tmp.ptr, gs_host, n * 64, s));
        HALO_CHECK(convert_wrapped_to_internal(curve, ses->tmp.ptr, ses->gs.ptr, n, s));
    } else if (need_gs) {
        HALO_HIP(hipMemcpyAsync(ses->gs.ptr, srs.gs.ptr, n * 64, hipMemcpyDeviceToDevice, s));
    }
    if (cs_len < n) HALO_HIP(hipMemsetAsync(ses->cs.as<char>() + cs_len * 32, 0, (n - cs_len) * 32, s));
    if (cs_on_device) {  // the producer ran on the null stream: order the session's stream after it
        hipEvent_t ev;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, 0) != hipSuccess ||
            hipStreamWaitEvent(s, ev, 0) != hipSuccess || hipEventDestroy(ev) != hipSuccess)
            return set_error(HALO_EDEVICE, "halo_ipa_begin_dev: stream ordering failed");
        if (cs_len) HALO_HIP(hipMemcpyAsync(ses->cs.ptr, cs, cs_len * 32, hipMemcpyDeviceToDevice, s));
    } else {
        HALO_CHECK(copy_h2d(ses->cs.ptr, cs, cs_len * 32, s));
    }
    char* sm = (char*)ses->small.ptr;
    if (zs_host) {
        HALO_CHECK(copy_h2d(ses->zs.ptr, zs_host, n * 32, s));
    } else {
        HALO_CHECK(copy_h2d(sm, z, 32, s));
        // consecutive powers per thread: a thread's chain is its exponentiation (~log2 n + popcount
        // products) plus `run`; small n is latency-bound (short runs), large n throughput-bound
        const size_t run = n <= 4096 ? 2 : 16;
        DISPATCH_CURVE(curve, Cv, {
            hipLaunchKernelGGL(k_powers<typename Cv::Scalar>, dim3(gridn((n + run - 1) / run, 128)), dim3(128), 0, s,
                               (const uint4*)sm, n, run, ses->zs.as<uint4>());
        });
        HALO_HIP(hipGetLastError());
    }
    if (gs_host) HALO_HIP(hipStreamSynchronize(s));  // tmp held the staged bases
    return HALO_OK;
}

// G of a session that skipped its copy of the SRS prefix (ipa_setup: it was to start in the tail
// rounds) but folds G before any round ran (pcdl.rs:627-687 test_u_check drives folds only).
static int ipa_ensure_gs(DeviceState* st, halo_ipa_session* ses) {
    if (ses->gs_valid) return HALO_OK;
    if (!ses->gs_srs_prefix) return set_error(HALO_EINVAL, "ipa: G is not resident");
    const size_t len = 2 * ses->m;
    HALO_CHECK(ses->gs.reserve(ses->n * 64));
    HALO_HIP(hipMemcpyAsync(ses->gs.ptr, st->srs[ses->curve].gs.ptr, len * 64, hipMemcpyDeviceToDevice, ses->s));
    ses->gs_valid = true;
    return HALO_OK;
}

// Phase 2: the hiding terms' table.  xi mode (xi0 and H): the shared 2^i H table and dots scaled by
// xi_0; otherwise (H_prime) a per-session 2^i H' table.  The rounds may run afterwards.
static int ipa_start(DeviceState* st, halo_ipa_session* ses, const halo_wrapped_point_t* H_prime, const halo_fe_t* xi0,
                     const halo_wrapped_point_t* Hpt) {
    hipStream_t s = ses->s;
    char* sm = (char*)ses->small.ptr;
    ses->xi_mode = xi0 != nullptr;
    const halo_wrapped_point_t* own = H_prime;  // the point of a per-session table, if one is needed
    if (ses->xi_mode) {  // xi_0 at [192, 224)
        HALO_CHECK(ipa_h_table(st, ses->curve, Hpt, &ses->htab_ptr));
        HALO_CHECK(copy_h2d(sm + 192, xi0, 32, s));
        own = ses->htab_ptr ? nullptr : Hpt;
    }
    ses->started = true;
    if (!own) {
        ses->htab_waited = true;
        return HALO_OK;
    }
    HALO_CHECK(ses->htab.reserve(IPA_HTAB * (64 + 128)));  // affine table + XYZZ chain scratch
    ses->htab_ptr = ses->htab.ptr;
    HALO_CHECK(copy_h2d(sm + 64, own, 64, s));
    // 2^i H' for i < 128 (the hiding terms use the GLV split of their scalar, k_hide_term): a
    // quad-cooperative doubling chain on the session's stream; the hiding-term kernels wait for htab_ready
    const hipStream_t hs = s;
    uint4* chain = ses->htab.as<uint4>() + 4 * IPA_HTAB;  // XYZZ scratch after the affine table
    DISPATCH_CURVE(ses->curve, Cv, {
        hipLaunchKernelGGL(k_pow2_xyzz_from_wrapped<Cv>, dim3(1), dim3(64), 0, hs, (const uint4*)(sm + 64), chain, IPA_HTAB);
        hipLaunchKernelGGL(k_xyzz_to_aff_ipa<Cv>, dim3(IPA_HTAB / 64), dim3(64), 0, hs, (const uint4*)chain,
                           ses->htab.as<uint4>(), IPA_HTAB);
    });
    HALO_HIP(hipGetLastError());
    HALO_HIP(hipEventRecord(ses->htab_ready, hs));
    ses->htab_waited = false;
    return HALO_OK;
}

static int ipa_begin(halo_curve_t curve, size_t n, const halo_wrapped_point_t* gs_host, const halo_fe_t* cs,
                     const halo_fe_t* zs_host, const halo_fe_t* z, const halo_wrapped_point_t* H_prime,
                     halo_ipa_session** out, bool cs_on_device = false, const halo_fe_t* xi0 = nullptr,
                     const halo_wrapped_point_t* Hpt = nullptr) {
    if (curve != HALO_PALLAS && curve != HALO_VESTA) return set_error(HALO_EINVAL, "unknown curve");
    if (!cs || !(z || zs_host) || !(H_prime || (xi0 && Hpt)) || !out)
        return set_error(HALO_EINVAL, "halo_ipa_begin: null argument");
    if (n <= 1) return set_error(HALO_EINVAL, "assertion failed: n > 1");
    if (!is_pow2(n)) return set_error(HALO_ENOTPOW2, "n (%zu) is not a power of two", n);
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    if (!gs_host && n > srs.n) return set_error(HALO_ESRSRANGE, "d (%zu) <= D (%zu)", n - 1, srs.n ? srs.n - 1 : 0);
    halo_ipa_session* ses = ipa_acquire(st);
    if (!ses) return HALO_EDEVICE;
    int rc = ipa_setup(st, ses, curve, n, gs_host, cs, n, cs_on_device, zs_host, z);
    if (!rc) rc = ipa_start(st, ses, H_prime, xi0, Hpt);
    if (rc) {
        ipa_release(ses);
        return rc;
    }
    *out = ses;
    return HALO_OK;
}

extern "C" int halo_ipa_begin(halo_curve_t curve, const halo_fe_t* cs, size_t n, const halo_fe_t* z,
                              const halo_wrapped_point_t* H_prime, halo_ipa_session** out) {
    clear_error();
    return ipa_begin(curve, n, nullptr, cs, nullptr, z, H_prime, out);
}

// Device-resident coefficients (the prover's opened polynomials never leave HBM): d_cs holds n ark
// coefficients on the device, ordered on the null stream.
extern "C" int halo_ipa_begin_dev(halo_curve_t curve, const void* d_cs, size_t n, const halo_fe_t* z,
                                  const halo_wrapped_point_t* H_prime, halo_ipa_session** out) {
    clear_error();
    return ipa_begin(curve, n, nullptr, (const halo_fe_t*)d_cs, nullptr, z, H_prime, out, true);
}

// pcdl::open_without_eval's H' = xi_0 H (pcdl.rs:390-391) inside the session: the caller passes H and
// xi_0 instead of H'; the hiding terms use a cached 2^i H table with the dots scaled by xi_0.
extern "C" int halo_ipa_begin_xi(halo_curve_t curve, const halo_fe_t* cs, size_t n, const halo_fe_t* z,
                                 const halo_wrapped_point_t* H, const halo_fe_t* xi0, halo_ipa_session** out) {
    clear_error();
    if (!xi0 || !H) return set_error(HALO_EINVAL, "halo_ipa_begin_xi: null argument");
    return ipa_begin(curve, n, nullptr, cs, nullptr, z, nullptr, out, false, xi0, H);
}
extern "C" int halo_ipa_begin_dev_xi(halo_curve_t curve, const void* d_cs, size_t n, const halo_fe_t* z,
                                     const halo_wrapped_point_t* H, const halo_fe_t* xi0, halo_ipa_session** out) {
    clear_error();
    if (!xi0 || !H) return set_error(HALO_EINVAL, "halo_ipa_begin_dev_xi: null argument");
    return ipa_begin(curve, n, nullptr, (const halo_fe_t*)d_cs, nullptr, z, nullptr, out, true, xi0, H);
}

extern "C" int halo_ipa_begin_vectors(halo_curve_t curve, const halo_wrapped_point_t* gs, const halo_fe_t* cs,
                                      const halo_fe_t* zs, size_t n, const halo_wrapped_point_t* H_prime,
                                      halo_ipa_session** out) {
    clear_error();
    if (!gs || !zs) return set_error(HALO_EINVAL, "halo_ipa_begin_vectors: null argument");
    return ipa_begin(curve, n, gs, cs, zs, nullptr, H_prime, out);
}

// v = c(z) over the session's first len coefficients, to the host (stream sync): the dot product of c
// with the session's z^i vector (ipa_setup wrote it), one parallel multiplication per coefficient
// instead of chunked Horner chains (2^10: 44 + 5 us of dependent chains -> one short dot launch pair)
static int ipa_eval_cs(halo_ipa_session* ses, size_t len, halo_fe_t* v_out) {
    hipStream_t s = ses->s;
    char* sm = ses->small.as<char>();
    if (!len) {
        memset(v_out, 0, 32);
        return HALO_OK;
    }
    HALO_CHECK(ses->tmp.reserve(4096 * 32));  // dot_device: at most 1024 block partials
    const int sf = ses->curve == HALO_PALLAS ? HALO_FP : HALO_FQ;
    HALO_CHECK(dot_device(sf, ses->cs.ptr, ses->zs.ptr, len, sm + SM_V, ses->tmp.ptr, s));
    HALO_HIP(hipMemcpyAsync(ses->pinned, sm + SM_V, 32, hipMemcpyDeviceToHost, s));
    HALO_HIP(hipStreamSynchronize(s));
    memcpy(v_out, ses->pinned, 32);
    return HALO_OK;
}

// k_tail_msm's terms per lane: 2 once a one-term grid would put more than one block on a CU (two waves
// sharing a SIMD's issue slots through the whole tree): a lane's own addition of its two terms costs
// less than the slower tree (opening 2^16, n0 = 2048: 512 blocks of one term or 256 of two)
static uint32_t tail_terms_per_lane(const DeviceState* st, size_t blocks_one_term) {
    return blocks_one_term > (size_t)st->num_cu ? 2u : 1u;
}

// ---------------------------------------------------------------------------------------------
// pcdl::open_without_eval (pcdl.rs:326-392) with p, p_bar and p' kept in the session's buffers
// (the hiding open used to download p_bar / p' and upload p, p_bar, p' between three
// host calls).  The caller owns the transcript, as in the reference:
//   halo_pcdl_open_begin(p, d, z)          asserts of pcdl.rs:338-341; c = p padded to n on the device
//   [hiding] halo_pcdl_open_blind(q, w_bar) -> C_bar      p_bar = (X - z) q, C_bar = commit(p_bar, w_bar)
//            (transcript: absorb C, C_bar, z, v; alpha = challenge)
//            halo_pcdl_open_combine(alpha, C, w) -> C', w'   c = p + alpha p_bar (in place), pcdl.rs:366-371
//   (transcript: absorb C', z, v; xi_0 = challenge)
//   halo_pcdl_open_start(H, xi_0)           H' = xi_0 H; then halo_ipa_round_lr / fold / end
// ---------------------------------------------------------------------------------------------
// scratch of a small SRS MSM over n points: GLV words (n x 32 B) | sides (n B, 256-B aligned) | partials;
// stream s waits for the previous small MSM (done with the scratch) and for the SRS multiples table
static int small_msm_scratch(DeviceState* st, int curve, size_t n, hipStream_t s, char** scr, size_t* o_side,
                             size_t* o_part, size_t* nblk) {
    SrsState& srs = st->srs[curve];
    const size_t nmax = std::min(srs_small_max(), srs.n);
    if (n < 1 || n > nmax) return set_error(HALO_EINVAL, "small SRS MSM: n (%zu) outside [1, %zu]", n, nmax);
    const uint32_t tpl = tail_terms_per_lane(st, (TAIL_WIN * n + TAIL_THREADS - 1) / TAIL_THREADS);
    *nblk = (TAIL_WIN * n + TAIL_THREADS * tpl - 1) / (TAIL_THREADS * tpl);
    *o_side = n * 32;
    *o_part = *o_side + ((n + 255) & ~(size_t)255);
    if (srs.small_ev) HALO_HIP(hipStreamWaitEvent(s, srs.small_ev, 0));  // the previous small MSM is done with small_scr
    else HALO_HIP(hipEventCreateWithFlags(&srs.small_ev, hipEventDisableTiming));
    HALO_CHECK(srs.small_scr.reserve(*o_part + *nblk * 256));
    HALO_CHECK(srs_small_table(st, curve, s));
    *scr = (char*)srs.small_scr.ptr;
    return HALO_OK;
}

// The small MSM after its scalars' GLV words are in the scratch (small_msm_scratch): the table sums with
// the hiding term w S in block 0 (2^i S table), an XYZZ result from the one block or k_tail_final, plus an
// optional point added at the end and a 32-B side copy (copy_src -> copy_dst) beside it.
static int small_msm_sums(DeviceState* st, int curve, char* scr, size_t o_side, size_t o_part, size_t nblk, size_t n,
                          const void* hide_scalar, void* d_out, hipStream_t s, bool out_xyzz, const void* plus_wrapped,
                          const void* copy_src, void* copy_dst) {
    SrsState& srs = st->srs[curve];
    DISPATCH_CURVE(curve, Cv, {
        const bool direct = out_xyzz && nblk == 1;
        const uint32_t tpl = tail_terms_per_lane(st, (TAIL_WIN * n + TAIL_THREADS - 1) / TAIL_THREADS);
        hipLaunchKernelGGL(k_tail_msm<Cv>, dim3((unsigned)nblk), dim3(TAIL_THREADS), 0, s,
                           srs.small_tab->as<const uint4>(), srs.small_n0, (const uint32_t*)scr,
                           (const uint8_t*)(scr + o_side), n, (size_t)0, 1, (uint32_t)nblk, (uint4*)(scr + o_part),
                           hide_scalar ? srs.s_table.as<const uint4>() : (const uint4*)nullptr, (const uint4*)hide_scalar,
                           (const uint32_t*)nullptr, direct ? (uint4*)d_out : (uint4*)nullptr, (uint32_t*)nullptr, 0u,
                           (const uint4*)plus_wrapped, (const uint4*)copy_src, (uint4*)copy_dst, tpl);
        if (!direct)
            hipLaunchKernelGGL(k_tail_final<Cv>, dim3(1), dim3(TAIL_THREADS), 0, s, (const uint4*)(scr + o_part),
                               (int)nblk, (const uint4*)nullptr, (const uint4*)nullptr, (uint4*)d_out, (int)out_xyzz,
                               (uint32_t*)nullptr, 0u, (const uint4*)plus_wrapped, (const uint4*)copy_src,
                               (uint4*)copy_dst);
    });
    HALO_HIP(hipGetLastError());
    HALO_HIP(hipEventRecord(srs.small_ev, s));
    return HALO_OK;
}

// The hiding combine's scalars for a small SRS MSM in one launch (was k_put_args + k_combine_scalars +
// k_tail_scalars): p' = p + alpha p_bar in place, p_bar <- alpha p_bar, the MSM scalars alpha p_bar as
// GLV words and sides in the small MSM's scratch, w' = w + alpha w_bar and -w, and C (by value) to its
// staging slot for the final's + C.  alpha, w, C by value (no host-to-device copy).
struct CombineSmallArgs {
    uint4 alpha[2], w[2], C[4];  // ark / WrappedPoint words
};
template <class Cv>
__global__ __launch_bounds__(256) void k_combine_small(const CombineSmallArgs a, uint4* p, uint4* pb, size_t n,
                                                       const uint4* w_bar, uint4* w_prime, uint4* negw, uint4* C_out,
                                                       uint32_t* scal, uint8_t* side) {
    using S = typename Cv::Scalar;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const Fe<S> al = fe_from_ark<S>(a.alpha);
    if (i < n) {
        const Fe<S> t = fe_mul(al, fe_from_ark<S>(pb + 2 * i));
        fe_to_ark(p + 2 * i, fe_add(fe_from_ark<S>(p + 2 * i), t));
        fe_to_ark(pb + 2 * i, t);
        tail_scalar_val<Cv>(t, 0, i, scal, side);
    }
    if (i == 0) {
        const Fe<S> wv = fe_from_ark<S>(a.w);
        fe_to_ark(w_prime, fe_add(wv, fe_mul(al, fe_from_ark<S>(w_bar))));
        fe_to_ark(negw, fe_neg(wv));
#pragma unroll
        for (int k = 0; k < 4; k++) C_out[k] = a.C[k];
    }
}

// The hiding blind's scalars for a small SRS MSM in one launch (was an H2D copy of w_bar + k_pbar +
// k_tail_scalars): p_bar = (X - z) q (d + 1 coefficients, pcdl.rs:344-347) to p_bar_out and as GLV words
// and sides in the small MSM's scratch, and w_bar (by value) to its staging slot (the MSM's hiding scalar).
template <class Cv>
__global__ __launch_bounds__(256) void k_pbar_small(const uint4* q, size_t d, const uint4* z, const ArkScalarPair wb,
                                                    uint4* w_bar_out, uint4* p_bar_out, uint32_t* scal, uint8_t* side) {
    using S = typename Cv::Scalar;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        w_bar_out[0] = wb.v[0];
        w_bar_out[1] = wb.v[1];
    }
    if (i > d) return;
    const Fe<S> a = i >= 1 ? fe_from_ark<S>(q + 2 * (i - 1)) : fe_zero<S>();
    const Fe<S> b = i < d ? fe_from_ark<S>(q + 2 * i) : fe_zero<S>();
    const Fe<S> t = fe_sub(a, fe_mul(fe_from_ark<S>(z), b));
    fe_to_ark(p_bar_out + 2 * i, t);
    tail_scalar_val<Cv>(t, 0, i, scal, side);
}

// Up to COMBINE_MSM_MAX coefficients halo_pcdl_open_combine forms C' through an MSM of alpha p_bar (see there)
constexpr size_t COMBINE_MSM_MAX = (size_t)1 << 16;

extern "C" int halo_pcdl_open_begin(halo_curve_t curve, const halo_fe_t* p, size_t len, size_t d, const halo_fe_t* z,
                                    halo_fe_t* v_out, halo_ipa_session** out) {
    clear_error();
    if (curve != HALO_PALLAS && curve != HALO_VESTA) return set_error(HALO_EINVAL, "unknown curve");
    if ((len && !p) || !z || !out) return set_error(HALO_EINVAL, "halo_pcdl_open_begin: null argument");
    const size_t n = d + 1;
    if (n <= 1) return set_error(HALO_EINVAL, "assertion failed: n > 1");
    if (!is_pow2(n)) return set_error(HALO_ENOTPOW2, "n (%zu) is not a power of two", n);
    // p.degree() <= d: trailing zero coefficients do not count towards the degree
    size_t deg_len = len;
    while (deg_len > 0 && !(p[deg_len - 1].l[0] | p[deg_len - 1].l[1] | p[deg_len - 1].l[2] | p[deg_len - 1].l[3]))
        deg_len--;
    if (deg_len > n) return set_error(HALO_EDEGREE, "assertion failed: p.degree() <= d");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    if (!srs.n || d > srs.n - 1) return set_error(HALO_ESRSRANGE, "assertion failed: d <= pp.D");
    halo_ipa_session* ses = ipa_acquire(st);
    if (!ses) return HALO_EDEVICE;
    int rc = ipa_setup(st, ses, curve, n, nullptr, p, deg_len, false, nullptr, z);
    if (!rc && v_out) rc = ipa_eval_cs(ses, deg_len, v_out);  // v = p(z) (pcdl::open, pcdl.rs:471)
    if (rc) {
        ipa_release(ses);
        return rc;
    }
    *out = ses;
    return HALO_OK;
}

extern "C" int halo_pcdl_open_blind(halo_ipa_session* ses, const halo_fe_t* q, const halo_fe_t* w_bar,
                                    halo_wrapped_point_t* C_bar) {
    clear_error();
    if (!ses || !q || !w_bar || !C_bar) return set_error(HALO_EINVAL, "halo_pcdl_open_blind: null argument");
    if (ses->started || ses->blinded) return set_error(HALO_EINVAL, "halo_pcdl_open_blind: session already blinded or started");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[ses->curve];
    if (!srs.has_sh) return set_error(HALO_ESRSRANGE, "hiding commitment needs S: upload the SRS (S, H) first");
    hipStream_t s = ses->s;
    const size_t n = ses->n, d = n - 1;
    char* sm = ses->small.as<char>();
    HALO_CHECK(ses->pbar.reserve(n * 32));
    HALO_CHECK(ses->tmp.reserve(std::max<size_t>(4096 * 32, d * 32)));
    HALO_CHECK(copy_h2d(ses->tmp.ptr, q, d * 32, s));
    // C_bar as packed XYZZ, converted on the host: the MSM's last lane no longer runs an inversion (~0.1 ms
    // of dependent multiplications at the end of the blind)
    if (n <= std::min(srs_small_max(), srs.n)) {  // p_bar, its GLV words and w_bar in one launch (k_pbar_small)
        char* scr;
        size_t o_side, o_part, nblk;
        HALO_CHECK(small_msm_scratch(st, ses->curve, n, s, &scr, &o_side, &o_part, &nblk));
        ArkScalarPair wb;
        memcpy(&wb.v[0], w_bar, 32);
        DISPATCH_CURVE(ses->curve, Cv, {
            hipLaunchKernelGGL(k_pbar_small<Cv>, dim3(gridn(n, 256)), dim3(256), 0, s, ses->tmp.as<const uint4>(), d,
                               (const uint4*)sm, wb, (uint4*)(sm + SM_WBAR), ses->pbar.as<uint4>(), (uint32_t*)scr,
                               (uint8_t*)(scr + o_side));  // z at sm[0, 32)
        });
        HALO_HIP(hipGetLastError());
        HALO_CHECK(small_msm_sums(st, ses->curve, scr, o_side, o_part, nblk, n, sm + SM_WBAR, sm + SM_T, s, true, nullptr,
                                  nullptr, nullptr));
    } else {
        HALO_CHECK(copy_h2d(sm + SM_WBAR, w_bar, 32, s));
        HALO_CHECK(pcdl_pbar_device(ses->curve, ses->tmp.ptr, d, sm, ses->pbar.ptr, s));  // z at sm[0, 32)
        HALO_CHECK(msm_srs_device(st, ses->curve, ses->pbar.ptr, n, sm + SM_WBAR, sm + SM_T, s, false, true));
    }
    HALO_HIP(hipMemcpyAsync(ses->pinned + 128, sm + SM_T, 128, hipMemcpyDeviceToHost, s));
    HALO_HIP(hipStreamSynchronize(s));
    host_xyzz_to_wrapped(ses->curve, ses->pinned + 128, C_bar);
    if (n > COMBINE_MSM_MAX) {  // pcdl_combine_device reads C_bar on the device
        memcpy(ses->pinned + 128, C_bar, 64);
        HALO_HIP(hipMemcpyAsync(sm + SM_CBAR, ses->pinned + 128, 64, hipMemcpyHostToDevice, s));
    }
    ses->blinded = true;
    return HALO_OK;
}

extern "C" int halo_pcdl_open_combine(halo_ipa_session* ses, const halo_fe_t* alpha, const halo_wrapped_point_t* C,
                                      const halo_fe_t* w, halo_fe_t* w_prime, halo_wrapped_point_t* C_prime) {
    clear_error();
    if (!ses || !alpha || !C || !w || !w_prime || !C_prime)
        return set_error(HALO_EINVAL, "halo_pcdl_open_combine: null argument");
    if (!ses->blinded || ses->combined || ses->started)
        return set_error(HALO_EINVAL, "halo_pcdl_open_combine: needs exactly one halo_pcdl_open_blind before it");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = ses->s;
    char* sm = ses->small.as<char>();
    const bool small = ses->n <= std::min(srs_small_max(), st->srs[ses->curve].n);  // (k_combine_small takes them by value)
    if (!small) {  // alpha, w, C and S (internal) in one launch
        PutArgs a{};
        const void* src[4] = {alpha, w, C, st->srs[ses->curve].S};
        const size_t off[4] = {SM_ALPHA, SM_W, SM_C, SM_S};
        const int cnt[4] = {2, 2, 4, 4};
        int k = 0;
        for (int i = 0; i < 4; i++) {
            a.dst[i] = (uint4*)(sm + off[i]);
            a.cnt[i] = cnt[i];
            memcpy(&a.v[k], src[i], 16 * cnt[i]);
            k += cnt[i];
        }
        hipLaunchKernelGGL(k_put_args, dim3(1), dim3(64), 0, s, a);
        HALO_HIP(hipGetLastError());
    }
    // c (= p padded) += alpha p_bar in place: p' (pcdl.rs:366); C' = C + alpha C_bar - w' S, w' = w + alpha w_bar.
    // Up to COMBINE_MSM_MAX coefficients C' is formed as C + MSM(G, alpha p_bar) - w S (= C + alpha C_bar - w' S,
    // since C_bar = MSM(G, p_bar) + w_bar S): an MSM (the table path, or the bucket pipeline) instead of
    // the lone-lane scalar multiplications of k_hiding_point (~1.3 ms of dependent curve operations).
    if (ses->n <= COMBINE_MSM_MAX) {
        // the MSM as packed XYZZ (no inversion on the device), + C, converted on the host below
        if (small) {
            // one launch for every scalar (k_combine_small), then the small MSM whose final block adds C and
            // puts w' beside the sum: one device-to-host copy of both
            char* scr;
            size_t o_side, o_part, nblk;
            HALO_CHECK(small_msm_scratch(st, ses->curve, ses->n, s, &scr, &o_side, &o_part, &nblk));
            CombineSmallArgs a;
            memcpy(a.alpha, alpha, 32);
            memcpy(a.w, w, 32);
            memcpy(a.C, C, 64);
            DISPATCH_CURVE(ses->curve, Cv, {
                hipLaunchKernelGGL(k_combine_small<Cv>, dim3(gridn(ses->n, 256)), dim3(256), 0, s, a, ses->cs.as<uint4>(),
                                   ses->pbar.as<uint4>(), ses->n, (const uint4*)(sm + SM_WBAR), (uint4*)(sm + SM_WP),
                                   (uint4*)(sm + SM_NEGW), (uint4*)(sm + SM_C), (uint32_t*)scr, (uint8_t*)(scr + o_side));
            });
            HALO_HIP(hipGetLastError());
            HALO_CHECK(small_msm_sums(st, ses->curve, scr, o_side, o_part, nblk, ses->n, sm + SM_NEGW, sm + SM_T, s, true,
                                      sm + SM_C, sm + SM_WP, sm + SM_T + 128));
            HALO_HIP(hipMemcpyAsync(ses->pinned + 128, sm + SM_T, 160, hipMemcpyDeviceToHost, s));
            HALO_HIP(hipStreamSynchronize(s));
            memcpy(w_prime, ses->pinned + 256, 32);
            host_xyzz_to_wrapped(ses->curve, ses->pinned + 128, C_prime);
            ses->combined = true;
            return HALO_OK;
        } else {
            HALO_CHECK(pcdl_combine_scalars_device(ses->curve, ses->cs.ptr, ses->pbar.ptr, ses->n, sm + SM_ALPHA,
                                                   sm + SM_W, sm + SM_WBAR, sm + SM_WP, sm + SM_NEGW, s));
            HALO_CHECK(msm_srs_device(st, ses->curve, ses->pbar.ptr, ses->n, sm + SM_NEGW, sm + SM_T, s, false, true));
            HALO_CHECK(xyzz_add_wrapped_device(ses->curve, sm + SM_T, sm + SM_C, s, false));
        }
        HALO_HIP(hipMemcpyAsync(ses->pinned, sm + SM_WP, 32, hipMemcpyDeviceToHost, s));
        HALO_HIP(hipMemcpyAsync(ses->pinned + 128, sm + SM_T, 128, hipMemcpyDeviceToHost, s));
        HALO_HIP(hipStreamSynchronize(s));
        memcpy(w_prime, ses->pinned, 32);
        host_xyzz_to_wrapped(ses->curve, ses->pinned + 128, C_prime);
    } else {
        HALO_CHECK(pcdl_combine_device(ses->curve, ses->cs.ptr, ses->n, ses->pbar.ptr, ses->n, sm + SM_ALPHA, sm + SM_W,
                                       sm + SM_WBAR, sm + SM_C, sm + SM_CBAR, sm + SM_S, ses->cs.ptr, sm + SM_CP,
                                       sm + SM_WP, s));
        HALO_HIP(hipMemcpyAsync(ses->pinned, sm + SM_WP, 32, hipMemcpyDeviceToHost, s));
        HALO_HIP(hipMemcpyAsync(ses->pinned + 32, sm + SM_CP, 64, hipMemcpyDeviceToHost, s));
        HALO_HIP(hipStreamSynchronize(s));
        memcpy(w_prime, ses->pinned, 32);
        memcpy(C_prime, ses->pinned + 32, 64);
    }
    ses->combined = true;
    return HALO_OK;
}

extern "C" int halo_pcdl_open_start(halo_ipa_session* ses, const halo_wrapped_point_t* H, const halo_fe_t* xi0) {
    clear_error();
    if (!ses || !xi0) return set_error(HALO_EINVAL, "halo_pcdl_open_start: null argument");
    if (ses->started) return set_error(HALO_EINVAL, "halo_pcdl_open_start: session already started");
    if (ses->blinded && !ses->combined)
        return set_error(HALO_EINVAL, "halo_pcdl_open_start: a blinded opening needs halo_pcdl_open_combine first");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    if (!H) {  // the resident SRS's H (pp.H, pcdl.rs:390)
        const SrsState& srs = st->srs[ses->curve];
        if (!srs.has_sh) return set_error(HALO_ESRSRANGE, "no (S, H) uploaded");
        H = &srs.H_wrapped;
    }
    return ipa_start(st, ses, nullptr, xi0, H);
}

// Switch to the tail rounds: G0 = current G (length 2m), w = [1], and the multiples table of G0:
// the SRS's own table when G0 is still the SRS prefix (a session of n <= IPA_TAIL_N over the SRS:
// the reference's small pcdl_open shapes, benches/pcdl.rs:35-57), else built for the session.
static int ipa_enter_tail(DeviceState* st, halo_ipa_session* ses, hipStream_t s) {
    const size_t n0 = 2 * ses->m;
    const size_t nblk = (TAIL_WIN * n0 + TAIL_THREADS - 1) / TAIL_THREADS + 2;  // (+ mode 0's per-side rounding)
    HALO_CHECK(ses->w[0].reserve(n0 * 32));
    HALO_CHECK(ses->w[1].reserve(n0 * 32));
    HALO_CHECK(ses->cs2.reserve(n0 * 32));
    HALO_CHECK(ses->zs2.reserve(n0 * 32));
    HALO_CHECK(ses->scal.reserve(n0 * 32));
    HALO_CHECK(ses->side.reserve(n0));
    HALO_CHECK(ses->part.reserve(nblk * 2 * 128));
    SrsState& srs = st->srs[ses->curve];
    if (ses->gs_srs_prefix && n0 <= std::min(srs_tab_n(), srs.n)) {
        HALO_CHECK(srs_small_table(st, ses->curve, s));
        ses->table_ref = srs.small_tab;  // an SRS write rebuilds into a fresh buffer while this is held
        ses->table = srs.small_tab->as<const uint4>();
        ses->table_ld = srs.small_n0;
    } else {
        // a session that skipped its copy of the SRS prefix (ipa_setup: need_gs) but builds its own
        // table here (the SRS table is off or shorter than n0) copies the prefix now
        HALO_CHECK(ipa_ensure_gs(st, ses));
        HALO_CHECK(ses->own_table.reserve((size_t)TAIL_TBL * TAIL_MUL * n0 * 128));
        DISPATCH_CURVE(ses->curve, Cv, {
            hipLaunchKernelGGL(k_tail_table<Cv>, dim3(gridn((size_t)TAIL_TABLE_LANES * n0, 64)), dim3(64), 0, s, ses->gs.as<const uint4>(),
                               (int)ses->gs_xyzz, n0, ses->own_table.as<uint4>());
            hipLaunchKernelGGL(k_tail_mults<Cv>, dim3(gridn((size_t)TAIL_MLANES * TAIL_TBL * n0, 64)), dim3(64), 0, s, n0,
                               ses->own_table.as<uint4>());
        });
        HALO_HIP(hipGetLastError());
        ses->table = ses->own_table.as<const uint4>();
        ses->table_ld = n0;
    }
    // w = [1]: the next round's first launch uses 1 and stores it (TailFoldArgs::w_one), no launch here
    ses->w_one_pending = true;
    ses->n0 = n0;
    ses->wlen = 1;
    ses->wcur = 0;
    ses->tail = true;
    return HALO_OK;
}

// mode 0: L, R of the current round (with their dot * H' terms) -> small[512..768) as XYZZ; the round's
// scalars and dots come from k_tail_prep (one launch), the hiding terms ride in each side's first
// k_tail_msm block, and k_tail_final runs only when a side spans several blocks.
// mode 1: U = sum_u w[u] G0[u] -> small[256..384) as XYZZ (converted on the host).
static int ipa_tail_sums(const DeviceState* st, halo_ipa_session* ses, int mode, hipStream_t s, const void* copy_src = nullptr,
                         void* copy_dst = nullptr) {
    const size_t n0 = ses->n0, m = ses->m;
    char* sm = (char*)ses->small.ptr;
    if (mode == 0) {  // one fused launch (k_tail_round) up to TAIL_FUSE_N points, three above
        TailFoldArgs f{};
        f.active = ses->fold_pending;
        if (ses->w_one_pending) {  // (no fold is pending right after the switch to the tail rounds)
            f.w_one = ses->w[ses->wcur].as<uint4>();
            ses->w_one_pending = false;
        }
        if (f.active) {  // the previous round's fold, applied here (halo_ipa_fold deferred it)
            memcpy(&f.xi, &ses->pend_xi, 32);
            memcpy(&f.xinv, &ses->pend_xinv, 32);
            f.cs_out = ses->cs2.as<uint4>();
            f.zs_out = ses->zs2.as<uint4>();
            f.w_out = ses->w[ses->wcur ^ 1].as<uint4>();
            f.wlen_in = ses->wlen;
        }
        TailRoundArgs ra{};
        ra.table = ses->table;
        ra.ld = ses->table_ld;
        ra.n0 = n0;
        ra.m = m;
        ra.cs = ses->cs.as<const uint4>();
        ra.zs = ses->zs.as<const uint4>();
        ra.w = ses->w[ses->wcur].as<const uint4>();
        ra.nbs = (uint32_t)((n0 / 2 + TAIL_THREADS / 64 - 1) / (TAIL_THREADS / 64));
        ra.xi0_ark = ses->xi_mode ? (const uint4*)(sm + 192) : nullptr;
        ra.htab = (const uint4*)ses->htab_ptr;
        ra.dots_ark = (uint4*)(sm + 128);
        ra.part = ses->part.as<uint4>();
        ra.ctr = (uint32_t*)(sm + SM_CTR);
        ra.out_xyzz = (uint4*)(sm + 512);
        ra.host = (uint32_t*)(ses->pinned + 256);
        ra.seq = ++ses->poll_seq;
        if (ra.seq == 0) ra.seq = ++ses->poll_seq;  // (0 is the flags' initial value)
        ses->poll_pending = true;
        if (n0 <= TAIL_FUSE_N) {
            DISPATCH_CURVE(ses->curve, Cv, {
                hipLaunchKernelGGL(k_tail_round<Cv>, dim3(2 * ra.nbs + 2), dim3(TAIL_THREADS), 0, s, ra, f);
            });
        } else {  // k_tail_digits (the point scalars and the dots) + k_tail_msm + k_tail_final
            const size_t nbs1 = (TAIL_WIN * (n0 / 2) + TAIL_THREADS - 1) / TAIL_THREADS;
            const uint32_t tpl = tail_terms_per_lane(st, 2 * nbs1);
            const size_t nbs = (TAIL_WIN * (n0 / 2) + TAIL_THREADS * tpl - 1) / (TAIL_THREADS * tpl), nblk = 2 * nbs;
            DISPATCH_CURVE(ses->curve, Cv, {
                hipLaunchKernelGGL(k_tail_digits<Cv>, dim3(gridn(n0, 256) + 2), dim3(256), 0, s, ses->cs.as<const uint4>(),
                                   ses->zs.as<const uint4>(), ses->w[ses->wcur].as<const uint4>(), n0, m, f,
                                   ses->scal.as<uint32_t>(), ses->side.as<uint8_t>(), ra.xi0_ark, ra.dots_ark,
                                   (uint32_t*)(sm + SM_HKW));
                hipLaunchKernelGGL(k_tail_msm<Cv>, dim3((unsigned)nblk), dim3(TAIL_THREADS), 0, s, ses->table, ses->table_ld,
                                   ses->scal.as<const uint32_t>(), ses->side.as<const uint8_t>(), n0, m, 0, (uint32_t)nbs,
                                   ses->part.as<uint4>(), (const uint4*)ses->htab_ptr, (const uint4*)(sm + 128),
                                   (const uint32_t*)(sm + SM_HKW), (uint4*)(sm + 512), ra.host, ra.seq, (const uint4*)nullptr,
                                   (const uint4*)nullptr, (uint4*)nullptr, tpl);
                if (nbs > 1)
                    hipLaunchKernelGGL(k_tail_final<Cv>, dim3(2), dim3(TAIL_THREADS), 0, s, ses->part.as<const uint4>(),
                                       (int)nblk, (const uint4*)nullptr, (const uint4*)nullptr, (uint4*)(sm + 512), 1,
                                       ra.host, ra.seq);
            });
        }
        HALO_HIP(hipGetLastError());
        if (f.active) {
            std::swap(ses->cs.ptr, ses->cs2.ptr);
            std::swap(ses->cs.bytes, ses->cs2.bytes);
            std::swap(ses->zs.ptr, ses->zs2.ptr);
            std::swap(ses->zs.bytes, ses->zs2.bytes);
            ses->wcur ^= 1;
            ses->wlen *= 2;
            ses->fold_pending = false;
        }
        return HALO_OK;
    }
    // mode 1: U = sum_u w[u] G0[u]
    if (ses->w_one_pending) {
        DISPATCH_CURVE(ses->curve, Cv, {
            hipLaunchKernelGGL(k_set_one_ark<typename Cv::Scalar>, dim3(1), dim3(64), 0, s, ses->w[ses->wcur].as<uint4>());
        });
        HALO_HIP(hipGetLastError());
        ses->w_one_pending = false;
    }
    const uint32_t tpl = tail_terms_per_lane(st, (TAIL_WIN * n0 + TAIL_THREADS - 1) / TAIL_THREADS);
    const size_t nblk = (TAIL_WIN * n0 + TAIL_THREADS * tpl - 1) / (TAIL_THREADS * tpl);
    uint4* out = (uint4*)(sm + 256);
    DISPATCH_CURVE(ses->curve, Cv, {
        hipLaunchKernelGGL(k_tail_scalars<Cv>, dim3(gridn(n0, 256)), dim3(256), 0, s, ses->cs.as<const uint4>(),
                           ses->w[ses->wcur].as<const uint4>(), n0, 2 * m, m, 1, ses->scal.as<uint32_t>(),
                           ses->side.as<uint8_t>());
        hipLaunchKernelGGL(k_tail_msm<Cv>, dim3((unsigned)nblk), dim3(TAIL_THREADS), 0, s, ses->table, ses->table_ld,
                           ses->scal.as<const uint32_t>(), ses->side.as<const uint8_t>(), n0, m, 1, (uint32_t)nblk,
                           ses->part.as<uint4>(), (const uint4*)nullptr, (const uint4*)nullptr, (const uint32_t*)nullptr,
                           out, (uint32_t*)nullptr, 0u, (const uint4*)nullptr, (const uint4*)copy_src, (uint4*)copy_dst, tpl);
        if (nblk > 1)
            hipLaunchKernelGGL(k_tail_final<Cv>, dim3(1), dim3(TAIL_THREADS), 0, s, ses->part.as<const uint4>(), (int)nblk,
                               (const uint4*)nullptr, (const uint4*)nullptr, out, 1, (uint32_t*)nullptr, 0u,
                               (const uint4*)nullptr, (const uint4*)copy_src, (uint4*)copy_dst);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

// MSM of at most TINY_MSM_MAX caller points (acc::prover's C = sum alpha^i U_i, acc.rs:166): the bucket
// pipeline's latency there is its Horner over 43 windows of 6 bits (~250 quad doublings in k_final).
// Here every scalar is split by GLV into two 128-bit halves with signed 4-bit windows (tail_bias), so
// 32 windows suffice: wave w forms window w's term d P_i (or phi(d P_i)) for its 2n (point, half) lanes
// by double-and-add (|d| <= 8: at most four curve operations), sums them with the wave's quad tree, and
// k_final's Horner over the 32 window sums (4 quad doublings each) finishes: ~124 doublings in all.
constexpr size_t TINY_MSM_MAX = 32;
template <class Cv>
__global__ __launch_bounds__(256) void k_tiny_window_sums(const uint4* bases, const uint4* scalars_ark, uint32_t n,
                                                          uint4* window_sums) {
    using F = typename Cv::Base;
    using S = typename Cv::Scalar;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    XYZZ<F> acc = xyzz_id<F>();
    if (lane < 2 * n && w < (uint32_t)TAIL_TBL) {
        const uint32_t i = lane >> 1, half = lane & 1u;
        uint32_t w8[8], k1[5], k2[5];
        bool n1, n2;
        fe_ark_to_canonical_words<S>(scalars_ark + 2 * i, w8);
        glv::decompose<typename Cv::K>(w8, n1, k1, n2, k2);
        tail_bias(k1);
        tail_bias(k2);
        bool dneg;
        const uint32_t bw = w, word = half ? tail_word(k2, bw / 8) : tail_word(k1, bw / 8);
        const uint32_t d = tail_digit(word, bw, dneg);
        Affine<F> a = aff_load<F>(bases + 4 * i);
        if (d && !aff_is_id(a)) {
            if (half) a.x = fe_mul(a.x, fe_from_const<F>(Cv::K::BETA));  // phi
            if ((half ? n2 : n1) != dneg) a.y = fe_neg(a.y);
            const XYZZ<F> P = xyzz_from_aff(a);
            XYZZ<F> t = P;
#pragma unroll 1
            for (int b = 31 - __clz(d) - 1; b >= 0; b--) {
                t = xyzz_dbl(t);
                if ((d >> b) & 1u) t = xyzz_add(t, P);
            }
            acc = t;
        }
    }
    acc = wave_group_sum<F>(acc, 64u);
    if (lane == 0 && w < (uint32_t)TAIL_TBL) xyzz_store(window_sums + 8 * w, acc);
}

// sum_i scalars[i] bases[i] (internal affine bases, ark scalars, n <= TINY_MSM_MAX) -> packed XYZZ at
// out_xyzz (device), stream-ordered on s; scratch: 32 XYZZ window sums (4 KiB).
int halo::msm_tiny(int curve, const void* bases_int, const void* scalars_ark, size_t n, void* scratch, void* out_xyzz,
                   hipStream_t s) {
    if (n < 1 || n > TINY_MSM_MAX) return set_error(HALO_EINVAL, "tiny MSM: n (%zu) outside [1, %zu]", n, TINY_MSM_MAX);
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_tiny_window_sums<Cv>, dim3(TAIL_TBL / 4), dim3(256), 0, s, (const uint4*)bases_int,
                           (const uint4*)scalars_ark, (uint32_t)n, (uint4*)scratch);
    });
    HALO_HIP(hipGetLastError());
    return msm_final_launch(curve, (const uint4*)scratch, TAIL_TBL, TAIL_DB, nullptr, (uint4*)out_xyzz, 1, s);
}
size_t halo::msm_tiny_max() { return TINY_MSM_MAX; }

// The SRS prefix's multiples table d 2^(4 w) G_k (k < n0 = min(srs_tab_n(), srs.n)), built on first
// use per SRS (k_tail_table + k_tail_mults on stream s; small_tab_ev marks its completion for other
// streams).  SrsState::invalidate_derived() (every writer of the SRS points) forces a rebuild.  The
// table is versioned: while an open IPA session holds the current buffer (table_ref),
// the rebuild goes into a fresh one and the old buffer lives until its last session is released;
// otherwise it is rebuilt in place after the last small MSM that read it (small_ev).
int halo::srs_small_table(DeviceState* st, int curve, hipStream_t s) {
    SrsState& srs = st->srs[curve];
    const size_t n0 = std::min(srs_tab_n(), srs.n);
    if (!n0) return set_error(HALO_ESRSRANGE, "no resident SRS: call halo_srs_upload first");
    if (!srs.small_tab_ev) HALO_HIP(hipEventCreateWithFlags(&srs.small_tab_ev, hipEventDisableTiming));
    if (srs.small_n0 == n0 && srs.small_tab) {
        HALO_HIP(hipStreamWaitEvent(s, srs.small_tab_ev, 0));
        return HALO_OK;
    }
    if (!srs.small_tab || srs.small_tab.use_count() > 1) srs.small_tab = std::make_shared<DevBuf>();
    if (srs.small_ev) HALO_HIP(hipStreamWaitEvent(s, srs.small_ev, 0));  // the old table's last small MSM
    HALO_CHECK(srs.small_tab->reserve((size_t)TAIL_TBL * TAIL_MUL * n0 * 128));
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_tail_table<Cv>, dim3(gridn((size_t)TAIL_TABLE_LANES * n0, 64)), dim3(64), 0, s, srs.gs.as<const uint4>(), 0, n0,
                           srs.small_tab->as<uint4>());
        hipLaunchKernelGGL(k_tail_mults<Cv>, dim3(gridn((size_t)TAIL_MLANES * TAIL_TBL * n0, 64)), dim3(64), 0, s, n0,
                           srs.small_tab->as<uint4>());
    });
    HALO_HIP(hipGetLastError());
    HALO_HIP(hipEventRecord(srs.small_tab_ev, s));
    srs.small_n0 = n0;
    return HALO_OK;
}

// Small MSM over the resident SRS prefix (msm.hpp): the tail rounds' machinery over G0 = Gs[0..n)
// with the SRS's multiples table (leading dimension small_n0 >= n); mode 1 of k_tail_scalars /
// k_tail_msm gives sum_k s[k] G0[k] (64 n table terms), k_tail_final adds w S from the 2^i S table.
int halo::msm_srs_small(DeviceState* st, int curve, const void* scalars_ark, size_t n, const void* hide_scalar,
                  void* d_out_wrapped, hipStream_t s, bool out_xyzz, const void* plus_wrapped) {
    if (plus_wrapped && !out_xyzz) return set_error(HALO_EINVAL, "small SRS MSM: + point needs the XYZZ output");
    char* scr;
    size_t o_side, o_part, nblk;
    HALO_CHECK(small_msm_scratch(st, curve, n, s, &scr, &o_side, &o_part, &nblk));
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_tail_scalars<Cv>, dim3(gridn(n, 256)), dim3(256), 0, s, (const uint4*)nullptr,
                           (const uint4*)scalars_ark, n, (size_t)1, (size_t)0, 1, (uint32_t*)scr, (uint8_t*)(scr + o_side));
    });
    HALO_HIP(hipGetLastError());
    return small_msm_sums(st, curve, scr, o_side, o_part, nblk, n, hide_scalar, d_out_wrapped, s, out_xyzz, plus_wrapped,
                          nullptr, nullptr);
}

static int ipa_copy_out(halo_ipa_session* ses) {
    // L, R as packed XYZZ (128 B each): the affine conversion runs on the host (host_xyzz_to_wrapped)
    HALO_HIP(hipMemcpyAsync(ses->pinned + 256, (char*)ses->small.ptr + 512, 256, hipMemcpyDeviceToHost, ses->s));
    return HALO_OK;
}

// Enqueues one round's L and R (with their H' terms) and their D2H copy into ses->pinned.
static int ipa_round_launch(DeviceState* st, halo_ipa_session* ses) {
    if (ses->m == 0) return set_error(HALO_EINVAL, "halo_ipa_round_lr: no rounds left");
    if (!ses->started) return set_error(HALO_EINVAL, "halo_ipa_round_lr: session not started (halo_pcdl_open_start)");
    hipStream_t s = ses->s;
    const size_t m = ses->m;
    const int sf = ses->curve == HALO_PALLAS ? HALO_FP : HALO_FQ;
    char* sm = (char*)ses->small.ptr;  // [0,32) z, [64,128) H', [128,192) dots, [256,384) U|c, [512,768) L|R XYZZ
    const char* cs = ses->cs.as<const char>();
    const char* zs = ses->zs.as<const char>();
    if (ses->weighted && 2 * m <= ipa_mat_n()) {
        // G (length 2m) = sum_u w[u] SRS[i + u 2m]: from here on an ordinary (tail) session
        ses->allow_tail = tuning(TUNE_IPA_TAIL) != 0;
        const bool to_tail = ses->allow_tail && 2 * m <= ipa_tail_n();  // the tail table reads XYZZ directly
        HALO_CHECK(ses->gs.reserve(2 * m * 128));
        // over the window-shifted copies (three-window Horner) when they are resident
        const SrsState& srs = st->srs[ses->curve];
        const bool sh = srs.shifted_c != 0;
        HALO_CHECK(msm_shared_batch(st, ses->curve, sh ? srs.shifted.ptr : srs.gs.ptr, ses->w[ses->wcur].ptr,
                                    ses->wlen, 2 * m, ses->gs.ptr, to_tail, ses->mat, s, sh ? srs.n : 0,
                                    sh ? srs.shifted_c : 0));
        ses->gs_xyzz = to_tail;
        ses->gs_valid = true;
        ses->gs_srs_prefix = false;
        ses->weighted = false;
    }
    if (!ses->tail && ses->allow_tail && (2 * m <= ipa_tail_n() || ses->tail_from_srs)) HALO_CHECK(ipa_enter_tail(st, ses, s));
    const char* gs = ses->gs.as<const char>();  // (materialised above in a weighted session)
    // only round 1 orders its hiding terms after the side-stream table: every later round starts after
    // the host has synchronised on round 1's results, which needed the table (a cross-stream wait in
    // every round cost ~0.3 ms per 2^16 round)
    hipEvent_t hr = ses->htab_waited ? nullptr : ses->htab_ready;
    ses->htab_waited = true;
    if (ses->tail) {  // k_tail_prep forms the dots (scaled by xi_0) with the round's scalars
        if (hr) HALO_HIP(hipStreamWaitEvent(s, hr, 0));
        HALO_CHECK(ipa_tail_sums(st, ses, 0, s));  // (L and R reach `pinned` from the kernels: no copy)
        return HALO_OK;
    }
    if (ses->weighted) {
        // the round's weighted scalars (k_weighted_prep without its dot blocks) on s, and in the pair path
        // its two dots (scaled by xi_0) on the MSM's tail stream just before the hiding terms that read
        // them (MsmPreHide), beside the digit / sort / accumulation phase
        const size_t half = ses->n0 / 2;  // = wlen * m terms per side
        const uint32_t lgm = ilog2(m);
        const char* sl = cs + m * 32;     // round 0 (w = [1]): the scalars are c_r, c_l themselves
        const char* sr = cs;
        char* sb = (char*)ses->scal.ptr;
        const unsigned nbk = gridn(half, 256), ndot = std::min(nbk, 256u);
        HALO_CHECK(ses->tmp.reserve((size_t)ndot * 64));
        const bool pair = half <= (size_t)tuning(TUNE_IPA_PAIR_MAX);
        WeightedDots wd{(const uint4*)cs, (const uint4*)zs, m, ses->tmp.as<uint4>(), (uint32_t*)(sm + SM_CTR + 8),
                        ses->xi_mode ? (const uint4*)(sm + 192) : nullptr, (uint4*)(sm + 128), ndot, ses->curve};
        if (ses->wlen > 1 || !pair) {
            DISPATCH_CURVE(ses->curve, Cv, {
                hipLaunchKernelGGL(k_weighted_prep<typename Cv::Scalar>, dim3(ses->wlen > 1 ? nbk : ndot), dim3(256), 0,
                                   s, (const uint4*)cs, (const uint4*)zs, ses->w[ses->wcur].as<const uint4>(), m,
                                   (int)lgm, half, ses->wlen > 1 ? (uint4*)sb : nullptr, (uint4*)(sb + half * 32),
                                   wd.part, wd.ctr, wd.xi0, wd.dots, pair ? 0u : ndot);
            });
            HALO_HIP(hipGetLastError());
        }
        if (ses->wlen > 1) {
            sl = sb;
            sr = sb + half * 32;
        }
        // L and R as one MSM (key = (side, bucket)) while the round is latency-bound; at 2^19 terms per
        // side two MSMs win (R's front and accumulation overlap L's reduction tail).  Measured, opening
        // 2^14 / 2^17 / 2^18 / 2^19 / 2^20 ms, two MSMs vs one: 7.5 / 11.3 / 14.4 / 19.3 / 27.2 vs
        // 6.9 / 10.3 / 13.2 / 17.8 / 29.0 (round 4, after the sort and accumulation changes: 2^20
        // 21.7 vs 22.7 ms)
        if (pair) {
            // L and R reach `pinned` from k_bitcombine itself (polled, as the tail rounds): no copy
            const MsmPairIO io{sl, sr, sm + 128, sm + 160, sm + 512, sm + 640};
            const MsmPreHide pre{weighted_dots_launch, &wd};
            uint32_t seq = ++ses->poll_seq;
            if (seq == 0) seq = ++ses->poll_seq;  // (0 is the flags' initial value)
            HALO_CHECK(msm_srs_pairs_device(st, ses->curve, 1, &io, half, lgm, ses->htab_ptr, s, hr, &pre,
                                            (uint32_t*)(ses->pinned + 256), seq));
            HALO_CHECK(msm_join(st, s));
            ses->poll_pending = true;
            return HALO_OK;
        } else if (ses->solo) {
            // L on the session stream and R on its second stream: the two MSMs' fronts, accumulations and
            // reduction tails overlap, instead of R's front waiting for L's accumulation (measured, 2^20
            // opening 20.5-20.8 -> 19.7-19.9 ms; with k sessions in lockstep their streams already overlap,
            // and 2k streams over the default 4 hardware queues made the prover's three openings ~2 ms
            // slower, so lockstep rounds keep one stream per session)
            if (!ses->s2) {
                HALO_HIP(hipStreamCreateWithFlags(&ses->s2, hipStreamNonBlocking));
                HALO_HIP(hipEventCreateWithFlags(&ses->ev_fork, hipEventDisableTiming));
                HALO_HIP(hipEventCreateWithFlags(&ses->ev_join, hipEventDisableTiming));
            }
            if (!ses->slots_reset) {
                msm_slots_reset(st);
                ses->slots_reset = true;
            }
            HALO_HIP(hipEventRecord(ses->ev_fork, s));
            HALO_HIP(hipStreamWaitEvent(ses->s2, ses->ev_fork, 0));
            HALO_CHECK(msm_srs_range_device(st, ses->curve, 0, sl, half, ses->htab_ptr, sm + 128, sm + 512, s, true,
                                            lgm, true, true, hr));
            HALO_CHECK(msm_srs_range_device(st, ses->curve, m, sr, half, ses->htab_ptr, sm + 160, sm + 640, ses->s2,
                                            true, lgm, true, true, hr));
            HALO_CHECK(msm_join(st, ses->s2));
            HALO_HIP(hipEventRecord(ses->ev_join, ses->s2));
            HALO_HIP(hipStreamWaitEvent(s, ses->ev_join, 0));
        } else {
            HALO_CHECK(msm_srs_range_device(st, ses->curve, 0, sl, half, ses->htab_ptr, sm + 128, sm + 512, s, true,
                                            lgm, true, true, hr));
            HALO_CHECK(msm_srs_range_device(st, ses->curve, m, sr, half, ses->htab_ptr, sm + 160, sm + 640, s, true,
                                            lgm, true, true, hr));
        }
        HALO_CHECK(msm_join(st, s));
        return ipa_copy_out(ses);
    }
    HALO_CHECK(dot_device(sf, cs + m * 32, zs, m, sm + 128, ses->tmp.ptr, s));        // <c_r, z_l>
    HALO_CHECK(dot_device(sf, cs, zs + m * 32, m, sm + 160, ses->tmp.ptr, s));        // <c_l, z_r>
    if (ses->xi_mode) {  // dot H' = (dot xi_0) H
        DISPATCH_CURVE(ses->curve, Cv, {
            hipLaunchKernelGGL(k_scale_ark<typename Cv::Scalar>, dim3(1), dim3(64), 0, s, (uint4*)(sm + 128), 2,
                               (const uint4*)(sm + 192));
        });
        HALO_HIP(hipGetLastError());
    }
    {
        // L and R are independent: the second MSM's accumulation overlaps the first one's tail
        if (ses->srs_round0) {  // G_l = SRS[0, m), G_r = SRS[m, 2m): resident window-shifted copies, no Horner
            HALO_CHECK(msm_srs_range_device(st, ses->curve, 0, cs + m * 32, m, ses->htab_ptr, sm + 128, sm + 512, s, true,
                                            32, true, true, hr));
            HALO_CHECK(msm_srs_range_device(st, ses->curve, m, cs, m, ses->htab_ptr, sm + 160, sm + 640, s, true, 32,
                                            true, true, hr));
        } else {
            HALO_CHECK(msm_device(st, ses->curve, gs, cs + m * 32, m, ses->htab_ptr, sm + 128, sm + 512, s, true, true,
                                  true, hr));
            HALO_CHECK(msm_device(st, ses->curve, gs + m * 64, cs, m, ses->htab_ptr, sm + 160, sm + 640, s, true, true,
                                  true, hr));
        }
        HALO_CHECK(msm_join(st, s));
    }
    return ipa_copy_out(ses);
}

// Enqueues one fold with challenge xi (pcdl.rs:427-435); the session advances to the next round.
static int ipa_fold_now(DeviceState* st, halo_ipa_session* ses, const halo_fe_t* xi, const halo_fe_t* xi_inv);

// A deferred tail-round fold applied on its own (before U at the end, a state read, or a second fold).
static int ipa_apply_pending_fold(DeviceState* st, halo_ipa_session* ses) {
    if (!ses->fold_pending) return HALO_OK;
    ses->fold_pending = false;
    ses->m = ses->pend_m;  // ipa_fold_now halves it again
    return ipa_fold_now(st, ses, &ses->pend_xi, &ses->pend_xinv);
}

static int ipa_fold_launch(DeviceState* st, halo_ipa_session* ses, const halo_fe_t* xi, const halo_fe_t* xi_inv) {
    if (ses->m == 0) return set_error(HALO_EINVAL, "halo_ipa_fold: no rounds left");
    if (!ses->started) return set_error(HALO_EINVAL, "halo_ipa_fold: session not started (halo_pcdl_open_start)");
    if (ses->tail) {  // applied by the next round's k_tail_prep (no launch, no copy now)
        HALO_CHECK(ipa_apply_pending_fold(st, ses));
        ses->pend_xi = *xi;
        ses->pend_xinv = *xi_inv;
        ses->pend_m = ses->m;
        ses->fold_pending = true;
        ses->srs_round0 = false;
        ses->m /= 2;
        return HALO_OK;
    }
    return ipa_fold_now(st, ses, xi, xi_inv);
}

static int ipa_fold_now(DeviceState* st, halo_ipa_session* ses, const halo_fe_t* xi, const halo_fe_t* xi_inv) {
    hipStream_t s = ses->s;
    char* sm = (char*)ses->small.ptr;
    // the previous fold's H2D copy from the pinned staging must have completed (a round in between
    // synchronises the stream; two folds in a row wait here)
    if (ses->fold_inflight) HALO_HIP(hipStreamSynchronize(s));
    const size_t m = ses->m;
    if (ses->tail || ses->weighted) {
        // xi, xi^-1 as kernel arguments: no staging copy, so nothing for a later fold to wait on
        ArkScalarPair x;
        memcpy(&x.v[0], xi, 32);
        memcpy(&x.v[2], xi_inv, 32);
        ses->srs_round0 = false;
        DISPATCH_CURVE(ses->curve, Cv, {
            hipLaunchKernelGGL(k_tail_fold<Cv>, dim3(gridn(std::max(m, ses->wlen), 256)), dim3(256), 0, s,
                               ses->cs.as<uint4>(), ses->zs.as<uint4>(), m, x, ses->w[ses->wcur].as<const uint4>(),
                               ses->w[ses->wcur ^ 1].as<uint4>(), ses->wlen);
        });
        HALO_HIP(hipGetLastError());
        ses->wcur ^= 1;
        ses->wlen *= 2;
        ses->m /= 2;
        return HALO_OK;
    }
    ses->fold_inflight = true;
    memcpy(ses->pinned + 128, xi, 32);
    memcpy(ses->pinned + 160, xi_inv, 32);
    HALO_HIP(hipMemcpyAsync(sm + 384, ses->pinned + 128, 64, hipMemcpyHostToDevice, s));
    ses->srs_round0 = false;
    if (!ses->tail && !ses->weighted) {  // G itself is folded below
        HALO_CHECK(ipa_ensure_gs(st, ses));
        ses->gs_srs_prefix = false;
    }
    {
        DISPATCH_CURVE(ses->curve, Cv, {
            ProfScope prof("ipa_fold", s);
            HALO_LAUNCH(prof, k_ipa_fold<Cv>, dim3(gridn(m, FOLD_THREADS)), dim3(FOLD_THREADS), 0, s, ses->gs.as<uint4>(),
                        ses->cs.as<uint4>(), ses->zs.as<uint4>(), m, (const uint4*)(sm + 384),
                        (const uint4*)(sm + 416));
        });
        HALO_HIP(hipGetLastError());
    }
    ses->m /= 2;
    return HALO_OK;
}

// Waits for a tail round's L and R in `pinned` (tail_emit_host): spins on the two flags; after 2 s
// (a failed or very late launch) it synchronises the stream, which reports a launch error, and takes
// L, R from the device copy instead.
static int ipa_poll_lr(halo_ipa_session* ses) {
    ses->poll_pending = false;
    const volatile uint32_t* fl = (const volatile uint32_t*)(ses->pinned + 512);
    const uint32_t seq = ses->poll_seq;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; spin++) {
        if (__atomic_load_n(&fl[0], __ATOMIC_ACQUIRE) == seq && __atomic_load_n(&fl[1], __ATOMIC_ACQUIRE) == seq) {
            // the flags are the round's last stores, stream-ordered after any fold it followed
            ses->fold_inflight = false;
            return HALO_OK;
        }
        // spin politely: a pause per probe, and past ~1 ms (a round is 0.1-2 ms) give the core up between
        // probes (the spin holds the device mutex)
        __builtin_ia32_pause();
        if (spin > (1u << 16)) std::this_thread::yield();
        if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
    }
    HALO_HIP(hipStreamSynchronize(ses->s));
    HALO_HIP(hipMemcpy(ses->pinned + 256, (char*)ses->small.ptr + 512, 256, hipMemcpyDeviceToHost));
    return HALO_OK;
}

extern "C" int halo_ipa_round_lr(halo_ipa_session* ses, halo_wrapped_point_t* L, halo_wrapped_point_t* R) {
    clear_error();
    if (!ses || !L || !R) return set_error(HALO_EINVAL, "halo_ipa_round_lr: null argument");
    return halo_ipa_round_lr_multi(&ses, 1, L, R);
}

// k independent openings advanced in lockstep: every session's round is enqueued on its own stream
// before any is waited for, so their latency-bound kernels overlap on the device.
extern "C" int halo_ipa_round_lr_multi(halo_ipa_session* const* ses, size_t k, halo_wrapped_point_t* L,
                                       halo_wrapped_point_t* R) {
    clear_error();
    if (!ses || !L || !R) return set_error(HALO_EINVAL, "halo_ipa_round_lr_multi: null argument");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    for (size_t i = 0; i < k; i++) {
        if (!ses[i]) return set_error(HALO_EINVAL, "halo_ipa_round_lr_multi: null session %zu", i);
        if (!ipa_is_open(ses[i])) return set_error(HALO_EINVAL, "halo_ipa_round_lr_multi: session %zu is not open", i);
        ses[i]->solo = k == 1;
        HALO_CHECK(ipa_round_launch(st, ses[i]));
    }
    for (size_t i = 0; i < k; i++) {
        if (ses[i]->poll_pending) {
            HALO_CHECK(ipa_poll_lr(ses[i]));
        } else {
            HALO_HIP(hipStreamSynchronize(ses[i]->s));
            ses[i]->fold_inflight = false;
        }
        const void* src[2] = {ses[i]->pinned + 256, ses[i]->pinned + 384};
        void* dst[2] = {&L[i], &R[i]};
        host_xyzz_to_wrapped2(ses[i]->curve, src, dst, 2);
    }
    return HALO_OK;
}

// One round whose L and R stay on the device (the distributed opening's per-round reduce):
// the round is enqueued as halo_ipa_round_lr enqueues it, L and R (packed XYZZ, 2 x 128 B) are copied to
// d_lr on the session's stream, and `stream` is ordered after that copy.  No host wait: the caller
// gathers and sums the ranks' pairs on the device (halo_point_sum_xyzz_dev) and brings one sum home.
extern "C" int halo_ipa_round_lr_dev(halo_ipa_session* ses, void* d_lr, void* stream) {
    clear_error();
    if (!ses || !d_lr) return set_error(HALO_EINVAL, "halo_ipa_round_lr_dev: null argument");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    if (!ipa_is_open(ses)) return set_error(HALO_EINVAL, "halo_ipa_round_lr_dev: the session is not open");
    ses->solo = true;
    HALO_CHECK(ipa_round_launch(st, ses));
    ses->poll_pending = false;  // (the copy a tail / pair round emits to the pinned staging is not waited for)
    HALO_HIP(hipMemcpyAsync(d_lr, (char*)ses->small.ptr + 512, 256, hipMemcpyDeviceToDevice, ses->s));
    if (!ses->lr_ready) HALO_HIP(hipEventCreateWithFlags(&ses->lr_ready, hipEventDisableTiming));
    HALO_HIP(hipEventRecord(ses->lr_ready, ses->s));
    HALO_HIP(hipStreamWaitEvent((hipStream_t)stream, ses->lr_ready, 0));
    return HALO_OK;
}

extern "C" int halo_ipa_fold(halo_ipa_session* ses, const halo_fe_t* xi, const halo_fe_t* xi_inv) {
    clear_error();
    if (!ses || !xi) return set_error(HALO_EINVAL, "halo_ipa_fold: null argument");
    return halo_ipa_fold_multi(&ses, 1, xi, xi_inv);
}

extern "C" int halo_ipa_fold_multi(halo_ipa_session* const* ses, size_t k, const halo_fe_t* xi,
                                   const halo_fe_t* xi_inv) {
    clear_error();
    if (!ses || !xi) return set_error(HALO_EINVAL, "halo_ipa_fold_multi: null argument");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    // every session checked and every inverse formed before the first fold is enqueued: an argument
    // error leaves all k sessions where they were (lockstep openings stay in step)
    std::vector<halo_fe_t> inv(xi_inv ? 0 : k);
    for (size_t i = 0; i < k; i++) {
        if (!ses[i]) return set_error(HALO_EINVAL, "halo_ipa_fold_multi: null session %zu", i);
        if (!ipa_is_open(ses[i])) return set_error(HALO_EINVAL, "halo_ipa_fold_multi: session %zu is not open", i);
        for (size_t j = 0; j < i; j++)
            if (ses[j] == ses[i]) return set_error(HALO_EINVAL, "halo_ipa_fold_multi: session %zu listed twice", i);
        // xi_inv == NULL: xi^-1 formed here, as the reference's fold does (pcdl.rs:430)
        if (!xi_inv && !host_scalar_inverse(ses[i]->curve, &xi[i], &inv[i]))
            return set_error(HALO_EINVAL, "halo_ipa_fold_multi: xi %zu is zero (no inverse)", i);
    }
    for (size_t i = 0; i < k; i++) HALO_CHECK(ipa_fold_launch(st, ses[i], &xi[i], xi_inv ? &xi_inv[i] : &inv[i]));
    // no host wait: the fold is stream-ordered before the next round (which synchronises), so the host
    // goes on to the transcript and the next round's launches while it runs
    return HALO_OK;
}

extern "C" int halo_ipa_state(halo_ipa_session* ses, size_t* m, halo_wrapped_point_t* gs, halo_fe_t* cs, halo_fe_t* zs) {
    clear_error();
    if (!ses) return set_error(HALO_EINVAL, "halo_ipa_state: null session");
    if (!ipa_is_open(ses)) return set_error(HALO_EINVAL, "halo_ipa_state: the session is not open");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = ses->s;
    HALO_CHECK(ipa_apply_pending_fold(st, ses));
    const size_t len = std::max<size_t>(2 * ses->m, 1);
    if (m) *m = ses->m;
    if (gs && (ses->tail || ses->weighted || !ses->gs_valid))
        return set_error(HALO_EINVAL,
                         "halo_ipa_state: G is not materialised in the weighted / tail rounds (HALO_IPA_WEIGHTED=0, "
                         "HALO_IPA_TAIL=0)");
    if (gs) {
        HALO_CHECK(ses->tmp.reserve(std::max<size_t>(len * 64, 4096 * 32)));
        HALO_CHECK(convert_internal_to_wrapped(ses->curve, ses->gs.ptr, ses->tmp.ptr, len, s));
        HALO_CHECK(copy_d2h(gs, ses->tmp.ptr, len * 64, s));
    }
    if (cs) HALO_CHECK(copy_d2h(cs, ses->cs.ptr, len * 32, s));
    if (zs) HALO_CHECK(copy_d2h(zs, ses->zs.ptr, len * 32, s));
    return HALO_OK;
}

// halo_ipa_end in two halves: the device work enqueued on the session's stream (st->mu held), then the
// wait, the host conversion and the release -- halo_ipa_end_multi enqueues every session's end before
// it waits for any, so the lockstep openings' final U sums overlap on the device.
static int ipa_end_enqueue(DeviceState* st, halo_ipa_session* ses) {
    hipStream_t s = ses->s;
    char* sm = (char*)ses->small.ptr;
    int rc = HALO_OK;
    if (!ses->started) {
        rc = set_error(HALO_EINVAL, "halo_ipa_end: session not started");
    } else if ((rc = ipa_apply_pending_fold(st, ses))) {
    } else if (ses->tail || ses->weighted) {
        // U = G_0 = sum_u w[u] G0[u] (len = 1 once every round ran)
        if (ses->m != 0)
            rc = set_error(HALO_EINVAL, "halo_ipa_end: U needs every round in the weighted / tail rounds (m = %zu)",
                           ses->m);
        else if (ses->tail)  // XYZZ at [256, 384), converted below; c = cs[0] copied to [384, 416) by its last block
            rc = ipa_tail_sums(st, ses, 1, s, ses->cs.ptr, sm + 384);
        else
            rc = msm_srs_range_device(st, ses->curve, 0, ses->w[ses->wcur].ptr, ses->n0, nullptr, nullptr, sm + 256, s,
                                      false);
        if (!rc && !ses->tail && hipMemcpyAsync(sm + 320, ses->cs.ptr, 32, hipMemcpyDeviceToDevice, s) != hipSuccess)
            rc = set_error(HALO_EDEVICE, "ipa end copy failed");
    } else if ((rc = ipa_ensure_gs(st, ses))) {
    } else {
        DISPATCH_CURVE(ses->curve, Cv, {
            hipLaunchKernelGGL(k_copy_first_wrapped<Cv>, dim3(1), dim3(64), 0, s, ses->gs.as<const uint4>(),
                               ses->cs.as<const uint4>(), (uint4*)(sm + 256), (uint4*)(sm + 320));
        });
        if (hipGetLastError() != hipSuccess) rc = set_error(HALO_EDEVICE, "ipa end launch failed");
    }
    // one copy through the pinned staging: U (wrapped, or XYZZ [256, 384) after tail rounds), c
    if (!rc && hipMemcpyAsync(ses->pinned + 256, sm + 256, ses->tail ? 160 : 96, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = set_error(HALO_EDEVICE, "ipa end copy failed");
    return rc;
}

static int ipa_end_finish(halo_ipa_session* ses, halo_wrapped_point_t* U, halo_fe_t* c) {
    const bool u_xyzz = ses->tail;
    if (hipStreamSynchronize(ses->s) != hipSuccess) return set_error(HALO_EDEVICE, "ipa end synchronisation failed");
    if (U) {
        if (u_xyzz)
            host_xyzz_to_wrapped(ses->curve, ses->pinned + 256, U);
        else
            memcpy(U, ses->pinned + 256, 64);
    }
    if (c) memcpy(c, ses->pinned + (u_xyzz ? 384 : 320), 32);
    return HALO_OK;
}

extern "C" int halo_ipa_end(halo_ipa_session* ses, halo_wrapped_point_t* U, halo_fe_t* c) {
    clear_error();
    if (!ses) return set_error(HALO_EINVAL, "halo_ipa_end: null session");
    if (!ipa_is_open(ses)) return set_error(HALO_EINVAL, "halo_ipa_end: the session is not open (already ended)");
    int rc = HALO_OK;
    if (U || c) {
        DeviceState* st = current_state();
        if (!st) {
            ipa_release(ses);
            return HALO_EDEVICE;
        }
        std::lock_guard<std::mutex> g(st->mu);
        rc = ipa_end_enqueue(st, ses);
        if (!rc) rc = ipa_end_finish(ses, U, c);
    }
    ipa_release(ses);
    return rc;
}

extern "C" int halo_ipa_end_multi(halo_ipa_session* const* ses, size_t k, halo_wrapped_point_t* U, halo_fe_t* c) {
    clear_error();
    if (k && !ses) return set_error(HALO_EINVAL, "halo_ipa_end_multi: null session list");
    for (size_t i = 0; i < k; i++) {
        if (!ses[i]) return set_error(HALO_EINVAL, "halo_ipa_end_multi: null session %zu", i);
        if (!ipa_is_open(ses[i]))
            return set_error(HALO_EINVAL, "halo_ipa_end_multi: session %zu is not open (already ended)", i);
        for (size_t j = 0; j < i; j++)
            if (ses[j] == ses[i]) return set_error(HALO_EINVAL, "halo_ipa_end_multi: session %zu listed twice", i);
    }
    int rc = HALO_OK;
    if (k && (U || c)) {
        DeviceState* st = current_state();
        if (!st) {
            for (size_t i = 0; i < k; i++) ipa_release(ses[i]);
            return HALO_EDEVICE;
        }
        std::lock_guard<std::mutex> g(st->mu);
        for (size_t i = 0; i < k && !rc; i++) rc = ipa_end_enqueue(st, ses[i]);
        // every stream is drained before any session goes back to the pool, failed or not
        for (size_t i = 0; i < k; i++) {
            const int r = rc ? (hipStreamSynchronize(ses[i]->s) == hipSuccess ? HALO_OK : HALO_EDEVICE)
                             : ipa_end_finish(ses[i], U ? U + i : nullptr, c ? c + i : nullptr);
            if (!rc && r) rc = r;
        }
    }
    for (size_t i = 0; i < k; i++) ipa_release(ses[i]);
    return rc;
}

extern "C" int halo_ipa_fold_host(halo_curve_t curve, halo_wrapped_point_t* gs, halo_fe_t* cs, halo_fe_t* zs, size_t m,
                                  const halo_fe_t* xi, const halo_fe_t* xi_inv) {
    clear_error();
    if (curve != HALO_PALLAS && curve != HALO_VESTA) return set_error(HALO_EINVAL, "unknown curve");
    if (!xi || !xi_inv || (m && (!gs || !cs || !zs))) return set_error(HALO_EINVAL, "halo_ipa_fold_host: null argument");
    if (!m) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(2 * m * 64));
    HALO_CHECK(st->scratch[1].reserve(2 * m * 64));
    HALO_CHECK(st->scratch[2].reserve(2 * m * 32));
    HALO_CHECK(st->scratch[3].reserve(2 * m * 32));
    HALO_CHECK(st->scratch[4].reserve(64));
    char* sm = (char*)st->scratch[4].ptr;
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, gs, 2 * m * 64, s));
    HALO_CHECK(copy_h2d(st->scratch[2].ptr, cs, 2 * m * 32, s));
    HALO_CHECK(copy_h2d(st->scratch[3].ptr, zs, 2 * m * 32, s));
    HALO_CHECK(copy_h2d(sm, xi, 32, s));
    HALO_CHECK(copy_h2d(sm + 32, xi_inv, 32, s));
    HALO_CHECK(convert_wrapped_to_internal(curve, st->scratch[0].ptr, st->scratch[1].ptr, 2 * m, s));
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_ipa_fold<Cv>, dim3(gridn(m, 128)), dim3(128), 0, s, st->scratch[1].as<uint4>(),
                           st->scratch[2].as<uint4>(), st->scratch[3].as<uint4>(), m, (const uint4*)sm,
                           (const uint4*)(sm + 32));
    });
    HALO_HIP(hipGetLastError());
    HALO_CHECK(convert_internal_to_wrapped(curve, st->scratch[1].ptr, st->scratch[0].ptr, m, s));
    HALO_CHECK(copy_d2h(gs, st->scratch[0].ptr, m * 64, s));
    HALO_CHECK(copy_d2h(cs, st->scratch[2].ptr, m * 32, s));
    HALO_CHECK(copy_d2h(zs, st->scratch[3].ptr, m * 32, s));
    return HALO_OK;
}

// ---------------------------------------------------------------------------------------------
// h(X) coefficients and the decider commitment.
//
// HPoly::get_poly (crates/accumulation/src/pcdl.rs:198-219) builds
//   h(X) = prod_{i < lg n} (1 + xi_{lg n - i} X^(2^i))
// with lg n growing FFT multiplications; its coefficient j is simply the product of
// xi_{lg n - b} over the set bits b of j (the identity pcdl.rs:735-758 tests).  Generated directly:
// j = hi * 2^LB + lo, coef[j] = T_lo[lo] * T_hi[hi] (two small tables, one multiplication per
// coefficient).  The ASDL combination sum_i alpha_i h_i(X) (acc.rs:89) folds alpha_i into T_hi,i.
// ---------------------------------------------------------------------------------------------
template <class F>
__global__ void k_hpoly_tables(const uint4* xis_ark, size_t k, uint32_t lg_n, uint32_t lb, const uint4* alphas_ark,
                               uint4* t_lo, uint4* t_hi) {
    const size_t nlo = (size_t)1 << lb, nhi = (size_t)1 << (lg_n - lb);
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= k * (nlo + nhi)) return;
    const size_t i = idx / (nlo + nhi), x = idx % (nlo + nhi);
    const uint4* xi = xis_ark + 2 * i * (lg_n + 1);
    Fe<F> v = fe_one<F>();
    if (x < nlo) {
        for (uint32_t b = 0; b < lb; b++)
            if ((x >> b) & 1) v = fe_mul(v, fe_from_ark<F>(xi + 2 * (lg_n - b)));
        fe_store(t_lo + 2 * (i * nlo + x), v);
    } else {
        const size_t y = x - nlo;
        if (alphas_ark) v = fe_from_ark<F>(alphas_ark + 2 * i);
        for (uint32_t b = 0; b < lg_n - lb; b++)
            if ((y >> b) & 1) v = fe_mul(v, fe_from_ark<F>(xi + 2 * (lg_n - lb - b)));
        fe_store(t_hi + 2 * (i * nhi + y), v);
    }
}

template <class F>
__global__ void k_hpoly_coeffs(const uint4* t_lo, const uint4* t_hi, size_t k, uint32_t lg_n, uint32_t lb,
                               uint4* out_ark) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >> lg_n) return;
    const size_t nlo = (size_t)1 << lb, nhi = (size_t)1 << (lg_n - lb);
    const size_t lo = j & (nlo - 1), hi = j >> lb;
    Fe<F> acc = fe_zero<F>();
    for (size_t i = 0; i < k; i++)
        acc = fe_add(acc, fe_mul(fe_load<F>(t_lo + 2 * (i * nlo + lo)), fe_load<F>(t_hi + 2 * (i * nhi + hi))));
    fe_to_ark(out_ark + 2 * j, acc);
}

// k h-polynomials (xis: k rows of n_xis ark elements) -> sum_i alpha_i h_i coefficients (ark) at d_out
// (2^(n_xis - 1) entries), on stream s.  Uses scratch[6] for the xis/alphas and tables.
static int hpoly_device(DeviceState* st, int field, const halo_fe_t* xis, size_t k, size_t n_xis,
                        const halo_fe_t* alphas, void* d_out, hipStream_t s) {
    const uint32_t lg_n = (uint32_t)(n_xis - 1);
    const uint32_t lb = lg_n / 2;
    const size_t nlo = (size_t)1 << lb, nhi = (size_t)1 << (lg_n - lb);
    const size_t in_elems = k * n_xis + (alphas ? k : 0);
    HALO_CHECK(st->scratch[6].reserve((in_elems + k * (nlo + nhi)) * 32));
    uint4* d_xis = st->scratch[6].as<uint4>();
    uint4* d_alpha = alphas ? d_xis + 2 * k * n_xis : nullptr;
    uint4* t_lo = d_xis + 2 * in_elems;
    uint4* t_hi = t_lo + 2 * k * nlo;
    HALO_CHECK(copy_h2d(d_xis, xis, k * n_xis * 32, s));
    if (alphas) HALO_CHECK(copy_h2d(d_alpha, alphas, k * 32, s));
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_hpoly_tables<F>, dim3(gridn(k * (nlo + nhi), 128)), dim3(128), 0, s, (const uint4*)d_xis, k,
                           lg_n, lb, (const uint4*)d_alpha, t_lo, t_hi);
        hipLaunchKernelGGL(k_hpoly_coeffs<F>, dim3(gridn((size_t)1 << lg_n, 256)), dim3(256), 0, s, (const uint4*)t_lo,
                           (const uint4*)t_hi, k, lg_n, lb, (uint4*)d_out);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_hpoly_combine(halo_field_t field, const halo_fe_t* xis, size_t k, size_t n_xis,
                                  const halo_fe_t* alphas, halo_fe_t* out, size_t* out_len) {
    clear_error();
    HALO_CHECK(check_field_i(field));
    if (n_xis < 1 || n_xis > 29) return set_error(HALO_EINVAL, "halo_hpoly: n_xis %zu out of range [1, 29]", n_xis);
    if (!k || !xis || !out) return set_error(HALO_EINVAL, "halo_hpoly: null buffer or k = 0");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    const size_t n = (size_t)1 << (n_xis - 1);
    HALO_CHECK(st->scratch[7].reserve(n * 32));
    HALO_CHECK(hpoly_device(st, field, xis, k, n_xis, alphas, st->scratch[7].ptr, s));
    HALO_CHECK(copy_d2h(out, st->scratch[7].ptr, n * 32, s));
    if (out_len) {  // DensePolynomial trims trailing zeros
        size_t m = n;
        while (m > 0 && !(out[m - 1].l[0] | out[m - 1].l[1] | out[m - 1].l[2] | out[m - 1].l[3])) m--;
        *out_len = m;
    }
    return HALO_OK;
}

// Device-resident variant (acc::prover's h(X), acc.rs:89 / pcdl.rs:198-219): the 2^(n_xis - 1)
// coefficients (ark, untrimmed) go to d_out on `stream`; h never crosses PCIe.
extern "C" int halo_hpoly_combine_dev(halo_field_t field, const halo_fe_t* xis, size_t k, size_t n_xis,
                                      const halo_fe_t* alphas, void* d_out, void* stream) {
    clear_error();
    HALO_CHECK(check_field_i(field));
    if (n_xis < 1 || n_xis > 29) return set_error(HALO_EINVAL, "halo_hpoly: n_xis %zu out of range [1, 29]", n_xis);
    if (!k || !xis || !d_out) return set_error(HALO_EINVAL, "halo_hpoly: null buffer or k = 0");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = (hipStream_t)stream;
    ScratchUse su(st, s);
    return hpoly_device(st, field, xis, k, n_xis, alphas, d_out, s);
}

extern "C" int halo_hpoly_coeffs(halo_field_t field, const halo_fe_t* xis, size_t n_xis, halo_fe_t* out) {
    return halo_hpoly_combine(field, xis, 1, n_xis, nullptr, out, nullptr);
}

// pcdl::check step 5 (pcdl.rs:579): U' = pedersen::commit(None, &pp.Gs[0..d+1], &h.get_poly().coeffs),
// computed without leaving the device (h coefficients -> resident-SRS MSM).
extern "C" int halo_pcdl_decider_commit(halo_curve_t curve, const halo_fe_t* xis, size_t n_xis, size_t d,
                                        halo_wrapped_point_t* out) {
    clear_error();
    if (curve != HALO_PALLAS && curve != HALO_VESTA) return set_error(HALO_EINVAL, "unknown curve id %d", (int)curve);
    if (n_xis < 1 || n_xis > 29) return set_error(HALO_EINVAL, "halo_pcdl_decider_commit: n_xis %zu out of range", n_xis);
    if (!xis || !out) return set_error(HALO_EINVAL, "halo_pcdl_decider_commit: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    const size_t n = (size_t)1 << (n_xis - 1);
    if (d + 1 > srs.n)
        return set_error(HALO_ESRSRANGE, "range end index %zu out of range for slice of length %zu", d + 1, srs.n);
    // all coefficients are products of nonzero challenges: no trailing zeros, ms.len() = n
    if (d + 1 < n)
        return set_error(HALO_ELENGTH, "ms must be larger than Gs: (Gs: %zu), (ms: %zu)", d + 1, n);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[7].reserve(n * 32 + 128));
    const int field = (curve == HALO_PALLAS) ? HALO_FP : HALO_FQ;
    HALO_CHECK(hpoly_device(st, field, xis, 1, n_xis, nullptr, st->scratch[7].ptr, s));
    char* d_out = (char*)st->scratch[7].ptr + n * 32;
    HALO_CHECK(msm_srs_device(st, curve, st->scratch[7].ptr, n, nullptr, d_out, s, false, true));
    alignas(16) uint64_t xyzz[16];  // converted on the host (msm.hip d2h_point)
    HALO_CHECK(copy_d2h(xyzz, d_out, 128, s));
    host_xyzz_to_wrapped(curve, xyzz, out);
    return HALO_OK;
}

// ---------------------------------------------------------------------------------------------
// Trace::new's interpolate + commit batch (crates/plonk/src/circuit/trace.rs
// :165-192): k evaluation vectors on the 2^log_n domain -> Evals::from_vec_and_domain (rotate right
// by one, poly.rs:21-31) -> interpolate_by_ref (iNTT, trailing zeros trimmed) -> pcdl::commit(poly,
// d, None).  One batched iNTT, then k resident-SRS MSMs enqueued back to back (pipelined: each
// MSM's reduction tail overlaps the next one's accumulation), one host sync at the end.
// ---------------------------------------------------------------------------------------------
__global__ void k_rotate_right(const uint4* in, uint4* out, size_t k, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k * n) return;
    const size_t r = i / n, j = i % n;
    const size_t from = r * n + (j == 0 ? n - 1 : j - 1);
    out[2 * i] = in[2 * from];
    out[2 * i + 1] = in[2 * from + 1];
}

// lens[r] = 1 + index of the last nonzero element of row r (0 if all zero); one block per row
__global__ __launch_bounds__(256) void k_row_lengths(const uint4* a, size_t n, uint32_t* lens) {
    __shared__ uint32_t best;
    if (threadIdx.x == 0) best = 0;
    __syncthreads();
    const uint4* row = a + 2 * (size_t)blockIdx.x * n;
    uint32_t m = 0;
    for (size_t j = threadIdx.x; j < n; j += 256) {
        const uint4 x = row[2 * j], y = row[2 * j + 1];
        if (x.x | x.y | x.z | x.w | y.x | y.y | y.z | y.w) m = (uint32_t)j + 1;
    }
    if (m) atomicMax(&best, m);
    __syncthreads();
    if (threadIdx.x == 0) lens[blockIdx.x] = best;
}

extern "C" int halo_trace_commit_batch(halo_curve_t curve, const halo_fe_t* evals, size_t k, unsigned log_n, size_t d,
                                       halo_fe_t* coeffs_out, size_t* lens_out, halo_wrapped_point_t* commits_out) {
    clear_error();
    if (curve != HALO_PALLAS && curve != HALO_VESTA) return set_error(HALO_EINVAL, "unknown curve id %d", (int)curve);
    if (!k) return HALO_OK;
    if (!evals || !commits_out) return set_error(HALO_EINVAL, "halo_trace_commit_batch: null buffer");
    if (log_n > 28) return set_error(HALO_EINVAL, "log_n %u too large", log_n);
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    SrsState& srs = st->srs[curve];
    if (!srs.n) return set_error(HALO_ESRSRANGE, "no resident SRS: call halo_srs_upload first");
    const size_t n = (size_t)1 << log_n, D = srs.n - 1, nc = d + 1;
    if (!is_pow2(nc)) return set_error(HALO_ENOTPOW2, "n (%zu) is not a power of two", nc);
    if (d > D) return set_error(HALO_ESRSRANGE, "d (%zu) <= D (%zu) (pp_len = %zu)", d, D, D + 1);
    const int field = (curve == HALO_PALLAS) ? HALO_FP : HALO_FQ;
    hipStream_t s = 0;
    ScratchUse su(st, s);
    const size_t bytes = k * n * 32;
    HALO_CHECK(st->scratch[0].reserve(bytes));
    HALO_CHECK(st->scratch[1].reserve(bytes));
    HALO_CHECK(st->scratch[2].reserve(bytes));
    HALO_CHECK(st->scratch[3].reserve(bytes));
    HALO_CHECK(st->scratch[7].reserve(k * (64 + 4)));
    uint4* A = st->scratch[0].as<uint4>();
    uint4* B = st->scratch[1].as<uint4>();
    HALO_CHECK(copy_h2d(A, evals, bytes, s));
    hipLaunchKernelGGL(k_rotate_right, dim3(gridn(k * n, 256)), dim3(256), 0, s, (const uint4*)A, B, k, n);
    HALO_HIP(hipGetLastError());
    // batched in-place iNTT of the k rows of B (ping-pong through scratch 2 and 3)
    HALO_CHECK(ntt_device_dispatch(st, field, B, B, st->scratch[2].ptr, log_n, k, 1, s, st->scratch[3].ptr));
    uint32_t* d_lens = (uint32_t*)((char*)st->scratch[7].ptr + k * 64);
    hipLaunchKernelGGL(k_row_lengths, dim3((unsigned)k), dim3(256), 0, s, (const uint4*)B, n, d_lens);
    HALO_HIP(hipGetLastError());
    std::vector<uint32_t> lens(k);
    HALO_CHECK(copy_d2h(lens.data(), d_lens, k * 4, s));
    for (size_t r = 0; r < k; r++) {
        const size_t p_deg = lens[r] ? lens[r] - 1 : 0;
        if (p_deg > d) return set_error(HALO_EDEGREE, "p_deg (%zu) <= d (%zu)", p_deg, d);
    }
    uint4* d_commits = st->scratch[7].as<uint4>();
    std::vector<const void*> ptrs(k);
    std::vector<size_t> szs(k);
    for (size_t r = 0; r < k; r++) {
        ptrs[r] = B + 2 * r * n;
        szs[r] = lens[r];
    }
    HALO_CHECK(msm_batch_device(st, curve, ptrs.data(), szs.data(), k, d_commits, s));
    HALO_CHECK(msm_join(st, s));
    HALO_CHECK(copy_d2h(commits_out, d_commits, k * 64, s));
    if (coeffs_out) HALO_CHECK(copy_d2h(coeffs_out, B, bytes, s));
    if (lens_out)
        for (size_t r = 0; r < k; r++) lens_out[r] = lens[r];
    return HALO_OK;
}
