// Radix-2 NTT / iNTT over the Pasta scalar fields.
//
// Replaces ark-poly 0.5.0 `Radix2EvaluationDomain::{fft, ifft}` as reached from
// `Evals::from_poly(_ref)` / `Evals::interpolate(_by_ref)` (crates/group/src/poly.rs:56-64,133-139),
// `DensePolynomial::evaluate_over_domain_by_ref` (crates/plonk/src/plonk/protocol.rs:89-106,140-141)
// and FFT polynomial multiplication (`&Poly * &Poly`, protocol.rs:132-139, pcdl.rs:215).
//
// Algorithm: Stockham auto-sort, radix R = 2^r per pass (Σ r = log N; the pass split is
// `ntt_radices` below: two passes of up to 11 bits for 2^17..2^22, passes of <= 8 bits otherwise),
// natural order in and out, out-of-place ping-pong.  One workgroup owns T = E / R consecutive
// columns j of a pass (E = 1024 or 2048 elements per workgroup): it loads x[j + r N/R] (T-element
// contiguous runs), multiplies by the Stockham twiddle read coalesced from the per-pass
// pre-twiddle table, performs the R-point DFT as radix-4 register groups (two radix-2 DIT stages
// per LDS round trip), and writes y[(j / Ns) Ns R + (j mod Ns) + k Ns].  Field elements live in LDS
// in the 9 x 29-bit limb form, limb-major with an XOR bank swizzle (see NttSwz).  The first pass
// takes ark words unconverted and the last pass multiplies by 2^261 (or 2^261 / N for the inverse),
// see NttPassArgs::out_const; the intermediate buffers hold the internal packed format.
#include <algorithm>
#include <cstdlib>

#include "dispatch.hpp"
#include "msm.hpp"
#include "runtime.hpp"

namespace halo {

constexpr int NTT_E = 1024;        // elements per workgroup for passes with R <= 256
constexpr int NTT_E_BIG = 2048;    // ... and for the two-pass split of 2^17..2^22 (R up to 2048)
constexpr int NTT_EPT = 4;         // elements per thread (radix-4 register groups) on 1024-element blocks
// ... and on the 2048-element blocks of the 2^17..2^22 passes.  HALO_NTT_EPT_BIG=8 selects radix-8
// register groups there (three stages per LDS round trip: an 11-bit pass makes 4 LDS round trips and
// 4 barriers instead of 6), measured slower: 2^22 pair 1.05 -> 1.09 ms (192 VGPRs and 256-thread
// blocks: 2 waves per SIMD instead of 4, so the barrier waits are hidden worse than they are saved)
#ifndef HALO_NTT_EPT_BIG
#define HALO_NTT_EPT_BIG 4
#endif
constexpr int NTT_EPT_BIG = HALO_NTT_EPT_BIG;
constexpr int ntt_lg(int ept) { return ept == 8 ? 3 : 2; }
#ifndef HALO_NTT_WAVE_SYNC
#define HALO_NTT_WAVE_SYNC 1
#endif
constexpr bool NTT_WAVE_SYNC = HALO_NTT_WAVE_SYNC;
constexpr int NTT_MAX_LOG_R_MULTI = 8;
constexpr int NTT_TW_MAX = 2048;  // stage-twiddle table entries (stages 0..10), read through L1/L2
constexpr unsigned NTT_FULL_TABLE_MAX_LOG = 24;  // per-pass twiddle tables up to 2^24

struct NttPassArgs {
    const uint4* in;
    uint4* out;
    const uint4* tw;        // per-pass pre-twiddle table tw[rho * Ns + jj] (internal packed), or null
    const uint4* tw_hi;     // 2-level fallback (logn > NTT_FULL_TABLE_MAX_LOG)
    const uint4* tw_lo;
    const uint4* stage_tw;  // entry 2^s - 1 + k = omega_{2^(s+1)}^k (s < 8, k < 2^s)
    uint32_t logn, log_r, log_ns, lo_bits;
    uint32_t in_ark, out_ark;
    // pass 0 of a forward transform whose inputs beyond N / 2^prune are zero: the first `prune`
    // radix-2 stages only replicate each nonzero input across its 2^prune-element group (b = 0 in every
    // butterfly), so the pass loads one element per group and starts at stage `prune`
    uint32_t prune;
    // Output multiplier.  The first pass takes the ark words (x 2^256 mod p) directly as internal
    // values, i.e. as x 2^-5 in Montgomery form with R' = 2^261; the transform is linear, so the last
    // pass multiplies by 2^261 (forward) or 2^261 / N (inverse) and emits ark words again: the
    // input conversion costs no multiplication.
    uint32_t out_const[NLIMB];
    // out_scaled: the pass's pre-twiddle table already holds M(w, out_const) (the last pass of a
    // table-driven transform): the rho = 0 inputs take M(x, out_const), the outputs no multiplication
    // (the transform is linear and M(M(a, t), c) = M(M(a, c), t)), one multiplication per element fewer
    uint32_t out_scaled;
    size_t stride;              // elements between consecutive transforms of a batch
};

// LDS layout: limb-major (SoA), limb l of position p at smem[l * NE + swz(p)].  swz XORs the bank
// bits with a linear function of p >> 5, chosen (by exhaustive check over every access pattern of
// the load, group and store phases, tools: see DESIGN.md) so that every ds_read_b32 / ds_write_b32
// is conflict-free: for NE = 1024 over r = 1..8, for NE = 2048 over r = 9..11.  (A 4096-element
// variant for 2 x 12-bit passes at 2^24 was measured 47 % slower than 3 x 8 bits: one 1024-thread
// block per CU and 32-byte strided column loads; not kept.)
template <int NE>
struct NttSwz;
template <>
struct NttSwz<1024> {
    static constexpr int NB = 5;
    static constexpr uint32_t C[5] = {31, 22, 5, 27, 10};
};
template <>
struct NttSwz<2048> {
    static constexpr int NB = 6;
    static constexpr uint32_t C[6] = {10, 29, 31, 20, 30, 17};
};

template <int NE>
HALO_DEV uint32_t ntt_swz_hi(uint32_t hi) {  // linear map of (p >> 5) onto the bank bits
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < NttSwz<NE>::NB; b++) m ^= ((hi >> b) & 1u) ? NttSwz<NE>::C[b] : 0u;
    return m;
}
template <int NE>
HALO_DEV uint32_t ntt_swz(uint32_t p) {
    return p ^ ntt_swz_hi<NE>(p >> 5);
}

template <class F>
HALO_DEV Fe<F> lds_get_soa(const uint32_t* s, uint32_t idx, uint32_t stride) {
    Fe<F> r;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) r.v[l] = s[l * stride + idx];
    return r;
}
template <class F>
HALO_DEV void lds_put_soa(uint32_t* s, uint32_t idx, uint32_t stride, const Fe<F>& a) {
#pragma unroll
    for (int l = 0; l < NLIMB; l++) s[l * stride + idx] = a.v[l];
}

// x < 2^259 with normalized limbs -> x mod p in [0, 2p): subtract (q - 1) p with q = floor(x / 2^254)
// (p = 2^254 + delta, delta < 2^126, for both Pasta fields).
template <class C>
HALO_DEV Fe<C> fe_reduce_q(const Fe<C>& x) {
    const int32_t qm = 1 - (int32_t)(x.v[NLIMB - 1] >> 22);
    Fe<C> r;
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        int64_t d = (int64_t)x.v[i] + c;
        if (C::P[i] != 0) d += (int64_t)qm * (int64_t)C::P[i];
        r.v[i] = (i == NLIMB - 1) ? (uint32_t)d : ((uint32_t)d & LIMB_MASK);
        c = d >> LIMB_BITS;
    }
    return r;
}

// G radix-2 DIT stages s .. s+G-1 over the EPT register-resident elements at positions base + m 2^s
// (m < EPT).  Stage s' pairs m and m + 2^(s'-s) and multiplies the upper element by
// omega_{2^(s'+1)}^k, k = (base + m 2^s) mod 2^s'.  Lazy reduction: values entering a pass are < 4p
// (< 2p except raw ark words), stage 0 doubles that bound, every later stage adds at most 2p
// (u + t and u - t + 2p with t = v w < 2p), so after 8 stages they are < 22p: still valid
// Montgomery inputs (< 64p), reduced once at the end of the pass (fe_reduce_q, < 32p).
// K0ZERO: k0 == 0 (the pass's first group, from the global loads): the butterflies with k = 0 have
// twiddle omega^0 = 1 and skip their multiplication (stage 1: one of the thread's two)
template <class F, int EPT, int LG, bool K0ZERO = false>
HALO_DEV void ntt_group(Fe<F> (&v)[EPT], uint32_t s, uint32_t G, uint32_t k0, const uint4* twg) {
#pragma unroll
    for (int g = 0; g < LG; g++) {
        if ((uint32_t)g >= G) break;
        const uint32_t sp = s + (uint32_t)g;
#pragma unroll
        for (int m = 0; m < EPT; m++) {
            if (m & (1 << g)) continue;
            const int m2 = m + (1 << g);
            Fe<F> t = v[m2];
            const bool unit = K0ZERO && sp != 0 && (m & ((1 << g) - 1)) == 0;
            if (sp != 0 && !unit) {
                const uint32_t k = k0 + ((uint32_t)(m & ((1 << g) - 1)) << s);
                t = fe_mul(t, fe_load<F>(twg + 2 * ((1u << sp) - 1u + k)));
            }
            // stage 0 (no multiplication): t is a pass input, < 4p even for non-canonical ark words;
            // a unit-twiddle butterfly at stage 1 takes t < 8p unmultiplied (its sums < 16p, so after
            // 8 stages the bound is 28p instead of 22p: still < 32p for fe_reduce_q)
            v[m2] = (sp == 0) ? fe_sub_k<4>(v[m], t) : unit ? fe_sub_k<8>(v[m], t) : fe_sub_k<2>(v[m], t);
            v[m] = fe_norm(fe_add_nc(v[m], t));
        }
    }
}

// The stage twiddles one thread needs for a radix-4 group at stages s, s + 1 (LG = 2, EPT = 4):
// stage s uses omega_{2^(s+1)}^k0 for both of its butterflies, stage s + 1 omega_{2^(s+2)}^(k0) and
// ^(k0 + 2^s).  Loaded packed (3 x 32 B) BEFORE the barrier that precedes the group's LDS reads, so
// the L2 round trip of the table overlaps the barrier wait instead of following it.
// (LG = 3: stage s + 2 omega_{2^(s+3)}^(k0 + j 2^s), j < 4, as well: 7 twiddles)
template <int LG>
struct NttGroupTw {
    uint4 w[(1 << LG) - 1][2];
};
template <int LG>
HALO_DEV void ntt_group_tw_load(NttGroupTw<LG>& t, uint32_t s, uint32_t G, uint32_t k0, const uint4* twg) {
    // stage s + g: omega_{2^(s+g+1)}^(k0 + j 2^s), j < 2^g, at entry 2^(s+g) - 1 + k0 + j 2^s
#pragma unroll
    for (int g = 0; g < LG; g++) {
        if ((uint32_t)g >= G) break;
#pragma unroll
        for (int j = 0; j < (1 << g); j++) {
            const uint32_t i = ((1u << (s + g)) - 1u) + k0 + ((uint32_t)j << s);
            t.w[(1 << g) - 1 + j][0] = twg[2 * i];
            t.w[(1 << g) - 1 + j][1] = twg[2 * i + 1];
        }
    }
}
template <class F>
HALO_DEV Fe<F> ntt_tw_unpack(const uint4 (&w)[2]) {
    uint32_t x[8] = {w[0].x, w[0].y, w[0].z, w[0].w, w[1].x, w[1].y, w[1].z, w[1].w};
    return fe_unpack<F>(x);
}
// ntt_group for EPT = 4, LG = 2, s >= 1 with the twiddles already loaded (same arithmetic and value
// bounds).  The first stage's sums stay limb-unnormalized (limbs < 2^30): the second stage takes them
// as a multiplication input (a column of 9 products < 2^59 plus the reduction stays < 2^63) or as the
// minuend of fe_sub_k (int32 limb chain, |x| < 2^31), and only the values leaving the group are
// carry-normalized -- two fe_norm per group instead of four.
template <class F>
HALO_DEV void ntt_group4_pre(Fe<F> (&v)[4], uint32_t G, const NttGroupTw<2>& t) {
    {
        const Fe<F> w = ntt_tw_unpack<F>(t.w[0]);
#pragma unroll
        for (int m = 0; m < 4; m += 2) {
            const Fe<F> x = fe_mul(v[m + 1], w);
            v[m + 1] = fe_sub_k<2>(v[m], x);
            v[m] = fe_add_nc(v[m], x);
        }
    }
    if (G > 1) {
#pragma unroll
        for (int m = 0; m < 2; m++) {
            const Fe<F> x = fe_mul(v[m + 2], ntt_tw_unpack<F>(t.w[1 + m]));
            v[m + 2] = fe_sub_k<2>(v[m], x);
            v[m] = fe_norm(fe_add_nc(v[m], x));
        }
    } else {
        v[0] = fe_norm(v[0]);
        v[2] = fe_norm(v[2]);
    }
}

// The radix-8 group (EPT = 8, three stages s, s + 1, s + 2; always full on the 2048-element blocks:
// the host splits every such pass so that r - G0 and r - prune are multiples of 3).  Same arithmetic
// and value bounds as ntt_group: stage s's sums stay limb-unnormalized (limbs < 2^30; they enter stage
// s + 1 only as multiplication inputs or fe_sub_k minuends), stage s + 1's and s + 2's sums are
// carry-normalized.
template <class F>
HALO_DEV void ntt_group8_pre(Fe<F> (&v)[8], const NttGroupTw<3>& t) {
    {
        const Fe<F> w = ntt_tw_unpack<F>(t.w[0]);
#pragma unroll
        for (int m = 0; m < 8; m += 2) {
            const Fe<F> x = fe_mul(v[m + 1], w);
            v[m + 1] = fe_sub_k<2>(v[m], x);
            v[m] = fe_add_nc(v[m], x);
        }
    }
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const Fe<F> w = ntt_tw_unpack<F>(t.w[1 + j]);
#pragma unroll
        for (int m = j; m < 8; m += 4) {
            const Fe<F> x = fe_mul(v[m + 2], w);
            v[m + 2] = fe_sub_k<2>(v[m], x);
            v[m] = fe_norm(fe_add_nc(v[m], x));
        }
    }
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const Fe<F> x = fe_mul(v[m + 4], ntt_tw_unpack<F>(t.w[3 + m]));
        v[m + 4] = fe_sub_k<2>(v[m], x);
        v[m] = fe_norm(fe_add_nc(v[m], x));
    }
}

// raw workgroup barrier: LDS writes complete, global loads left in flight (a __syncthreads() would
// also drain them).  wave_only: the LDS positions the wave reads next are exactly the ones it just
// wrote (its own EPT * 64-position chunk), so its own writes completing is enough -- no s_barrier.
HALO_DEV void ntt_lds_barrier(bool wave_only = false) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!wave_only) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// One Stockham pass: R = 2^log_r point DFTs over the columns j of the N/R x R view.  A workgroup
// owns T = NTT_E / R consecutive columns.  Each thread holds EPT elements in registers; the first
// LG stages are done straight from the global loads, the rest in groups of LG stages through LDS,
// and a final coalesced store phase writes y[(j / Ns) Ns R + (j mod Ns) + k Ns].
template <class F, int NE, int EPT>
__global__ __launch_bounds__(NE / EPT) void k_ntt_pass(NttPassArgs a) {
    constexpr int LG = ntt_lg(EPT);
    constexpr uint32_t TH = NE / EPT;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* data = smem;
    const uint32_t r = a.log_r;
    const uint32_t R = 1u << r;
    const size_t N = (size_t)1 << a.logn;
    const size_t NJ = N >> r;
    const uint32_t T = (uint32_t)((NJ < (size_t)(NE >> r)) ? NJ : (NE >> r));
    const uint32_t EB = T * R;  // elements in this block
    const size_t Ns = (size_t)1 << a.log_ns;
    // XCD-aware order for the wide passes (few columns per block): blocks b, b + 8, ... run on one
    // XCD, so give them consecutive column groups -- neighbouring columns share 128-B lines in L2
    uint32_t bx = blockIdx.x;
    if (NE >= NTT_E_BIG && (gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
    const size_t j0 = (size_t)bx * T;
    const uint4* in = a.in + (size_t)blockIdx.y * a.stride * 2;
    uint4* out = a.out + (size_t)blockIdx.y * a.stride * 2;
    const uint32_t tau = threadIdx.x;

    // ---- load + pre-twiddle + first LG stages (positions base + m)
    uint32_t base;
    if (R >= (uint32_t)EPT) {
        const uint32_t q = tau / T, t = tau % T;
        base = t * R + EPT * q;
    } else {
        base = EPT * tau;
    }
    Fe<F> v[EPT];
    const size_t tw_step = N >> (a.log_ns + r);  // N / (Ns R)
#pragma unroll
    for (int m = 0; m < EPT; m++) {
        const uint32_t pos = base + m;
        if (pos < EB) {
            const uint32_t t = pos >> r;
            const uint32_t pl = a.prune ? (pos & ~((1u << a.prune) - 1u)) : pos;  // the group's nonzero input
            const uint32_t rho = r ? (__brev(pl & (R - 1)) >> (32 - r)) : 0;
            const size_t j = j0 + t;
            const uint4* src = in + 2 * (j + (size_t)rho * NJ);
            Fe<F> x = fe_load<F>(src);  // ark words are used as internal values (see out_const)
            if (a.out_scaled && rho == 0) {
                Fe<F> oc;
#pragma unroll
                for (int l = 0; l < NLIMB; l++) oc.v[l] = a.out_const[l];
                x = fe_mul(x, oc);
            }
            if (!a.in_ark && a.log_ns != 0 && rho != 0) {
                const size_t jj = j & (Ns - 1);
                Fe<F> w;
                if (a.tw) {
                    w = fe_load<F>(a.tw + 2 * ((size_t)rho * Ns + jj));
                } else {
                    const size_t e = (size_t)rho * jj * tw_step;
                    const uint32_t lo_mask = (1u << a.lo_bits) - 1;
                    w = fe_load<F>(a.tw_lo + 2 * (e & lo_mask));
                    const size_t eh = e >> a.lo_bits;
                    if (eh) w = fe_mul(w, fe_load<F>(a.tw_hi + 2 * eh));
                }
                x = fe_mul(x, w);
            }
            v[m] = x;
        } else {
            v[m] = fe_zero<F>();
        }
    }
    // on the wide blocks the short group goes first (r mod LG stages), so later groups stay in range
    const uint32_t G0 = (NE >= NTT_E_BIG && (r % LG)) ? r % LG : (r < (uint32_t)LG ? r : (uint32_t)LG);
    if (!a.prune) ntt_group<F, EPT, LG, true>(v, 0, G0, 0, a.stage_tw);  // (pruned: host guarantees prune >= G0)
    {
        const uint32_t pb = ntt_swz<NE>(base);
#pragma unroll
        for (int m = 0; m < EPT; m++)
            if (base + m < EB) lds_put_soa(data, pb ^ (uint32_t)m, NE, v[m]);
    }
    // ---- remaining stages in groups of LG through LDS; each group's twiddles are loaded before the
    // barrier that precedes its LDS reads
    uint32_t s = a.prune ? a.prune : G0;
    NttGroupTw<LG> tw;
    if (s < r) ntt_group_tw_load(tw, s, (r - s) < (uint32_t)LG ? (r - s) : (uint32_t)LG, tau & ((1u << s) - 1),
                                 a.stage_tw);
    // Wave-local exchanges: a group at stage s <= 6 (2^s <= 64) reads and writes exactly its wave's
    // chunk of EPT * 64 consecutive positions [EPT 64 w, EPT 64 (w + 1)), and so does the load phase
    // of a one-column block (base = EPT tau); between two such phases the wave only waits for its own
    // LDS writes (HALO_NTT_WAVE_SYNC=0 A/B: s_barrier everywhere).
    const bool wave_sync = NTT_WAVE_SYNC && (T == 1u || R < (uint32_t)EPT);
    bool chunk = wave_sync;
    ntt_lds_barrier(chunk && s < r && s <= 6);
    for (; s < r; s += LG) {
        const uint32_t G = (r - s) < (uint32_t)LG ? (r - s) : (uint32_t)LG;
        const uint32_t h = 1u << s;
        const uint32_t gb = (tau & (h - 1)) | ((tau >> s) << (s + LG));
        const uint32_t shb = ntt_swz_hi<NE>(gb >> 5);
#pragma unroll
        for (int m = 0; m < EPT; m++) {
            const uint32_t pos = gb + (uint32_t)m * h;
            const uint32_t ph = (pos ^ shb) ^ ntt_swz_hi<NE>(((uint32_t)m * h) >> 5);
            if (pos < EB) v[m] = lds_get_soa<F>(data, ph, NE);
        }
        if constexpr (LG == 3)
            ntt_group8_pre<F>(v, tw);  // (G == 3 on every group, see G0)
        else
            ntt_group4_pre<F>(v, G, tw);
        // (no barrier here: a thread writes back exactly the positions it read)
#pragma unroll
        for (int m = 0; m < EPT; m++) {
            const uint32_t pos = gb + (uint32_t)m * h;
            const uint32_t ph = (pos ^ shb) ^ ntt_swz_hi<NE>(((uint32_t)m * h) >> 5);
            if (pos < EB) lds_put_soa(data, ph, NE, v[m]);
        }
        const uint32_t sn = s + LG;
        if (sn < r)
            ntt_group_tw_load(tw, sn, (r - sn) < (uint32_t)LG ? (r - sn) : (uint32_t)LG, tau & ((1u << sn) - 1),
                              a.stage_tw);
        chunk = NTT_WAVE_SYNC && s <= 6;
        ntt_lds_barrier(chunk && sn < r && sn <= 6);
    }

    // ---- store y[(j / Ns) Ns R + (j mod Ns) + k Ns]
    Fe<F> oc;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) oc.v[l] = a.out_const[l];
#pragma unroll
    for (int i = 0; i < EPT; i++) {
        const uint32_t idx = tau + TH * (uint32_t)i;
        if (idx >= EB) continue;
        uint32_t k, t;
        if (a.log_ns == 0) {
            t = idx >> r;
            k = idx & (R - 1);
        } else {
            k = idx / T;
            t = idx % T;
        }
        const size_t j = j0 + t;
        const size_t dst = ((j >> a.log_ns) << (a.log_ns + r)) + (j & (Ns - 1)) + (size_t)k * Ns;
        Fe<F> x = lds_get_soa<F>(data, ntt_swz<NE>(t * R + k), NE);
        if (a.out_ark) {
            fe_store(out + 2 * dst, fe_canon(a.out_scaled ? fe_reduce_q(x) : fe_mul(x, oc)));
        } else {
            fe_store(out + 2 * dst, fe_reduce_q(x));
        }
    }
}

// Per-pass pre-twiddle table: tab[rho * Ns + jj] = omega_N^(rho jj N / (Ns R)) (internal packed).
template <class F>
__global__ void k_pass_twiddles(uint4* tab, uint32_t log_r, uint32_t log_ns, uint32_t logn, const uint4* lo,
                                const uint4* hi, uint32_t lo_bits, Fe<F> scale, int scaled) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t cnt = (size_t)1 << (log_r + log_ns);
    if (i >= cnt) return;
    const size_t rho = i >> log_ns, jj = i & (((size_t)1 << log_ns) - 1);
    const size_t e = rho * jj * ((size_t)1 << (logn - log_ns - log_r));
    Fe<F> w = fe_load<F>(lo + 2 * (e & (((size_t)1 << lo_bits) - 1)));
    const size_t eh = e >> lo_bits;
    if (eh) w = fe_mul(w, fe_load<F>(hi + 2 * eh));
    if (scaled) w = fe_mul(w, scale);  // the last pass's table: M(w, out_const), NttPassArgs::out_scaled
    fe_store(tab + 2 * i, w);
}

// out[i] = base^(i * step) for i < count (internal packed format).  base given in internal form.
template <class F>
__global__ void k_pow_table(uint4* out, size_t count, Fe<F> base, uint64_t step) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint64_t e = (uint64_t)i * step;
    Fe<F> r = fe_one<F>();
    Fe<F> b = base;
    while (e) {
        if (e & 1) r = fe_mul(r, b);
        b = fe_sqr(b);
        e >>= 1;
    }
    fe_store(out + 2 * i, r);
}

// Reduce coefficients mod X^N - 1: out[i] = sum_k in[i + kN] (ark format in and out).
template <class F>
__global__ void k_fold(const uint4* in, size_t len, uint4* out, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    Fe<F> acc = fe_zero<F>();
    for (size_t k = i; k < len; k += N) acc = fe_add(acc, fe_from_ark<F>(in + 2 * k));
    fe_to_ark(out + 2 * i, acc);
}

// Four-step twiddle: x[a][b] (ark) *= omega^((row0 + a)(col0 + b) mod N), omega from the two-level
// tables (lo: omega^e for e < 2^lo_bits, hi: omega^(e 2^lo_bits)).
template <class F>
__global__ void k_twiddle_mat(uint4* x, size_t rows, size_t cols, size_t row0, size_t col0, uint32_t logn,
                              const uint4* lo, const uint4* hi, uint32_t lo_bits) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * cols) return;
    const size_t a = i / cols, b = i % cols;
    const uint64_t mask = ((uint64_t)1 << logn) - 1;
    const uint64_t e = (uint64_t)(((unsigned __int128)(row0 + a) * (col0 + b)) & mask);
    Fe<F> w = fe_load<F>(lo + 2 * (e & (((uint64_t)1 << lo_bits) - 1)));
    const uint64_t eh = e >> lo_bits;
    if (eh) w = fe_mul(w, fe_load<F>(hi + 2 * eh));
    fe_to_ark(x + 2 * i, fe_mul(fe_from_ark<F>(x + 2 * i), w));
}

// Batched transpose of 32-byte elements through LDS tiles (32 x 32 elements, padded).
__global__ __launch_bounds__(256) void k_transpose32(const uint4* src, uint4* dst, size_t rows, size_t cols) {
    __shared__ uint4 t[32][33][2];
    const size_t s = blockIdx.z;
    const size_t r0 = (size_t)blockIdx.y * 32, c0 = (size_t)blockIdx.x * 32;
    const uint4* S = src + 2 * s * rows * cols;
    uint4* D = dst + 2 * s * rows * cols;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int k = ty; k < 32; k += 8) {
        const size_t r = r0 + k, c = c0 + tx;
        if (r < rows && c < cols) {
            t[k][tx][0] = S[2 * (r * cols + c)];
            t[k][tx][1] = S[2 * (r * cols + c) + 1];
        }
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        const size_t c = c0 + k, r = r0 + tx;
        if (r < rows && c < cols) {
            D[2 * (c * rows + r)] = t[tx][k][0];
            D[2 * (c * rows + r) + 1] = t[tx][k][1];
        }
    }
}

// Transpose of matrices whose elements are runs of `run` 32-byte values (block permutation)
__global__ void k_transpose_runs(const uint4* src, uint4* dst, size_t batch, size_t rows, size_t cols, size_t run) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // destination 32-byte element
    const size_t per = rows * cols * run;
    if (i >= batch * per) return;
    const size_t s = i / per, rem = i % per;
    const size_t j = rem % run, q = rem / run;  // q = c * rows + r in the destination
    const size_t c = q / rows, r = q % rows;
    const size_t from = s * per + (r * cols + c) * run + j;
    dst[2 * i] = src[2 * from];
    dst[2 * i + 1] = src[2 * from + 1];
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------

template <class F>
static Fe<F> host_fe(const uint32_t (&k)[NLIMB]) {
    Fe<F> r;
    for (int i = 0; i < NLIMB; i++) r.v[i] = k[i];
    return r;
}

template <class F>
static int launch_pow_table(uint4* out, size_t count, const Fe<F>& base, uint64_t step, hipStream_t s) {
    if (!count) return HALO_OK;
    const unsigned thr = 256, blocks = (unsigned)((count + thr - 1) / thr);
    hipLaunchKernelGGL(k_pow_table<F>, dim3(blocks), dim3(thr), 0, s, out, count, base, step);
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

// Pass split: N <= 2^8 in one pass; 2^17..2^22 in two passes of up to 11 bits on 2048-element
// blocks (one fewer pass than the 8-bit split: one pre-twiddle multiplication and one HBM round
// trip per element saved; measured A/B on one box: 2^20 pair 0.28 -> 0.25 ms, 2^22 equal at
// 1.03 ms, where the single-column 11-bit pass loses on its strided 32-B loads what it saves in
// work); everything else in passes of <= 8 bits on 1024-element blocks.
constexpr unsigned NTT_MAX_LOG_R_BIG = 11;
static std::vector<unsigned> ntt_radices(unsigned logn) {
    std::vector<unsigned> r;
    if (logn <= NTT_MAX_LOG_R_MULTI) {
        r.push_back(logn);
        return r;
    }
    if (logn >= 17 && logn <= 2 * NTT_MAX_LOG_R_BIG) {
        r.push_back((logn + 1) / 2);
        r.push_back(logn / 2);
        return r;
    }
    const unsigned passes = (logn + NTT_MAX_LOG_R_MULTI - 1) / NTT_MAX_LOG_R_MULTI;
    unsigned left = logn;
    for (unsigned p = 0; p < passes; p++) {
        unsigned take = (left + (passes - p) - 1) / (passes - p);
        r.push_back(take);
        left -= take;
    }
    return r;
}

// Stages of pass 0 (radix 2^lr) that a zero tail lets the pass skip (NttPassArgs::prune): only when
// they cover its first register group; on one-column wide blocks a trailing single-stage group would
// reach past the column, so the stages left after the pruned ones must pair up (as G0 = 1 arranges).
static unsigned ntt_pass0_prune(unsigned lr, unsigned prune) {
    if (!prune) return 0;
    const bool big = lr > NTT_MAX_LOG_R_MULTI;
    const unsigned lg = big ? (unsigned)ntt_lg(NTT_EPT_BIG) : 2u;
    const unsigned g0 = (big && (lr % lg)) ? lr % lg : std::min(lr, lg);
    unsigned pr = std::min(prune, lr);
    while (big && pr > 0 && ((lr - pr) % lg)) pr--;
    return (pr >= g0 && pr < lr) ? pr : 0u;
}

template <class F>
static int get_twiddles(DeviceState* st, int field, unsigned logn, int inverse, DeviceState::Twiddles** out,
                        hipStream_t s) {
    for (auto& t : st->tw)
        if (t->field == field && t->logn == (int)logn && t->inverse == inverse) {
            *out = t.get();
            return HALO_OK;
        }
    auto t = std::make_unique<DeviceState::Twiddles>();
    t->field = field;
    t->logn = (int)logn;
    t->inverse = inverse;
    t->lo_bits = (int)((logn + 1) / 2);
    const size_t nlo = (size_t)1 << t->lo_bits, nhi = (size_t)1 << (logn - t->lo_bits);
    HALO_CHECK(t->lo.reserve(nlo * 32));
    HALO_CHECK(t->hi.reserve(nhi * 32));
    const Fe<F> w = host_fe<F>(inverse ? F::OMEGA_INV[logn] : F::OMEGA[logn]);
    HALO_CHECK(launch_pow_table<F>(t->lo.as<uint4>(), nlo, w, 1, s));
    HALO_CHECK(launch_pow_table<F>(t->hi.as<uint4>(), nhi, w, (uint64_t)nlo, s));
    // stage twiddles omega_{2^(s+1)}^k (the same for every N; kept per table for simplicity)
    HALO_CHECK(t->stage.reserve(NTT_TW_MAX * 32));
    for (unsigned sg = 0; sg < NTT_MAX_LOG_R_BIG; sg++) {
        const Fe<F> ws = host_fe<F>(inverse ? F::OMEGA_INV[sg + 1] : F::OMEGA[sg + 1]);
        HALO_CHECK(launch_pow_table<F>(t->stage.as<uint4>() + 2 * (((size_t)1 << sg) - 1), (size_t)1 << sg, ws, 1, s));
    }
    // per-pass pre-twiddle tables (one multiplication per element instead of two)
    if (logn <= NTT_FULL_TABLE_MAX_LOG) {
        const std::vector<unsigned> rad = ntt_radices(logn);
        unsigned log_ns = 0;
        for (size_t p = 0; p < rad.size(); p++) {
            if (p > 0) {
                const size_t cnt = (size_t)1 << (rad[p] + log_ns);
                HALO_CHECK(t->pass[p].reserve(cnt * 32));
                const unsigned thr = 256, blocks = (unsigned)((cnt + thr - 1) / thr);
                // the last pass's table is pre-scaled by the output constant (NttPassArgs::out_scaled)
                Fe<F> oc;
                for (int l = 0; l < NLIMB; l++) oc.v[l] = inverse ? F::NINV_ARK[logn][l] : F::ONE[l];
                hipLaunchKernelGGL(k_pass_twiddles<F>, dim3(blocks), dim3(thr), 0, s, t->pass[p].as<uint4>(), rad[p],
                                   log_ns, logn, t->lo.as<const uint4>(), t->hi.as<const uint4>(),
                                   (uint32_t)t->lo_bits, oc, (int)(p + 1 == rad.size()));
                HALO_HIP(hipGetLastError());
            }
            log_ns += rad[p];
        }
        t->has_pass = true;
    }
    *out = t.get();
    st->tw.push_back(std::move(t));
    return HALO_OK;
}

// Device NTT over `batch` transforms: reads d_in (ark format), writes d_out (ark format).
// The passes ping-pong between d_out and d_tmp; when d_in == d_out and the first pass would write
// d_in, d_tmp2 (same size) takes that pass's output instead.  Buffers hold batch * N elements.
template <class F>
static int ntt_device(DeviceState* st, int field, const void* d_in, void* d_out, void* d_tmp, void* d_tmp2,
                      unsigned logn, size_t batch, int inverse, hipStream_t s, unsigned prune = 0) {
    if (logn > 30) return set_error(HALO_EINVAL, "NTT domain 2^%u too large", logn);
    const size_t N = (size_t)1 << logn;
    if (logn == 0) {
        if (d_in != d_out) HALO_HIP(hipMemcpyAsync(d_out, d_in, batch * 32, hipMemcpyDeviceToDevice, s));
        return HALO_OK;
    }
    DeviceState::Twiddles* tw = nullptr;
    HALO_CHECK(get_twiddles<F>(st, field, logn, inverse, &tw, s));
    const std::vector<unsigned> rad = ntt_radices(logn);
    const int P = (int)rad.size();
    std::vector<const void*> srcs(P);
    std::vector<void*> dsts(P);
    dsts[P - 1] = d_out;
    for (int p = P - 2; p >= 0; p--) dsts[p] = (dsts[p + 1] == d_out) ? d_tmp : d_out;
    if (P > 1 && dsts[0] == d_in) {
        if (!d_tmp2) return set_error(HALO_EINVAL, "internal: NTT buffer aliasing");
        dsts[0] = d_tmp2;
    }
    for (int p = 0; p < P; p++) srcs[p] = (p == 0) ? d_in : dsts[p - 1];
    unsigned log_ns = 0;
    for (int p = 0; p < P; p++) {
        const unsigned lr = rad[p];
        NttPassArgs a;
        a.in = (const uint4*)srcs[p];
        a.out = (uint4*)dsts[p];
        a.tw = (tw->has_pass && p > 0) ? tw->pass[p].as<const uint4>() : nullptr;
        a.tw_hi = tw->hi.as<const uint4>();
        a.tw_lo = tw->lo.as<const uint4>();
        a.stage_tw = tw->stage.as<const uint4>();
        a.logn = logn;
        a.log_r = lr;
        a.log_ns = log_ns;
        a.lo_bits = (uint32_t)tw->lo_bits;
        a.in_ark = (p == 0);
        a.out_ark = (p == P - 1);
        a.prune = (p == 0 && !inverse) ? ntt_pass0_prune(lr, prune) : 0u;
        for (int l = 0; l < NLIMB; l++) a.out_const[l] = inverse ? F::NINV_ARK[logn][l] : F::ONE[l];
        a.out_scaled = (a.out_ark && a.tw) ? 1u : 0u;  // (get_twiddles pre-scales the last pass's table)
        a.stride = N;
        const size_t NJ = N >> lr;
        const size_t NE = lr > NTT_MAX_LOG_R_MULTI ? NTT_E_BIG : NTT_E;
        const size_t T = std::min(NJ, NE >> lr);
        const size_t lds = NE * NLIMB * 4;
        dim3 grid((unsigned)(NJ / T), (unsigned)batch);
        ProfScope prof("ntt_pass", s);
        if (NE == NTT_E_BIG)
            HALO_LAUNCH(prof, (k_ntt_pass<F, NTT_E_BIG, NTT_EPT_BIG>), grid, dim3(NTT_E_BIG / NTT_EPT_BIG), lds, s, a);
        else
            HALO_LAUNCH(prof, (k_ntt_pass<F, NTT_E, NTT_EPT>), grid, dim3(NTT_E / NTT_EPT), lds, s, a);
        HALO_HIP(hipGetLastError());
        log_ns += lr;
    }
    return HALO_OK;
}

int ntt_device_dispatch(DeviceState* st, int field, const void* d_in, void* d_out, void* d_tmp, unsigned logn,
                        size_t batch, int inverse, hipStream_t s, void* d_tmp2, unsigned prune) {
    int rc;
    DISPATCH_FIELD(field, F, {
        rc = ntt_device<F>(st, field, d_in, d_out, d_tmp, d_tmp2, logn, batch, inverse, s, prune);
    });
    return rc;
}

int fold_device_dispatch(int field, const void* d_in, size_t len, void* d_out, size_t N, hipStream_t s) {
    const unsigned thr = 256, blocks = (unsigned)((N + thr - 1) / thr);
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_fold<F>, dim3(blocks), dim3(thr), 0, s, (const uint4*)d_in, len, (uint4*)d_out, N);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

}  // namespace halo

using namespace halo;

static int check_field(halo_field_t f) {
    if (f != HALO_FP && f != HALO_FQ) return set_error(HALO_EINVAL, "unknown field id %d", (int)f);
    return HALO_OK;
}

// host -> device NTT helper: in/out host arrays of N elements (in may be longer: folded)
static int ntt_host(halo_field_t field, const halo_fe_t* in, size_t len, unsigned logn, int inverse, halo_fe_t* out) {
    const size_t N = (size_t)1 << logn;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(std::max(len, N) * 32));
    HALO_CHECK(st->scratch[1].reserve(N * 32));
    HALO_CHECK(st->scratch[2].reserve(N * 32));
    void* a = st->scratch[0].ptr;
    void* b = st->scratch[1].ptr;
    void* c = st->scratch[2].ptr;
    if (len >= N) {
        HALO_CHECK(copy_h2d(a, in, len * 32, s));
        if (len > N) {
            HALO_CHECK(fold_device_dispatch(field, a, len, b, N, s));
            std::swap(a, b);
        }
    } else {
        HALO_HIP(hipMemsetAsync(a, 0, N * 32, s));
        HALO_CHECK(copy_h2d(a, in, len * 32, s));
    }
    // passes ping-pong between b and c, reading a
    HALO_CHECK(ntt_device_dispatch(st, field, a, b, c, logn, 1, inverse, s, nullptr));
    return copy_d2h(out, b, N * 32, s);
}

extern "C" int halo_ntt(halo_field_t field, halo_fe_t* inout, unsigned log_n, int inverse) {
    clear_error();
    HALO_CHECK(check_field(field));
    if (!inout) return set_error(HALO_EINVAL, "halo_ntt: null buffer");
    if (log_n > 28) return set_error(HALO_EINVAL, "halo_ntt: log_n %u too large", log_n);
    return ntt_host(field, inout, (size_t)1 << log_n, log_n, inverse, inout);
}

extern "C" int halo_evaluate_over_domain(halo_field_t field, const halo_fe_t* coeffs, size_t len, unsigned log_n,
                                         halo_fe_t* evals) {
    clear_error();
    HALO_CHECK(check_field(field));
    if ((!coeffs && len) || !evals) return set_error(HALO_EINVAL, "halo_evaluate_over_domain: null buffer");
    if (log_n > 28) return set_error(HALO_EINVAL, "log_n %u too large", log_n);
    return ntt_host(field, coeffs, len, log_n, 0, evals);
}

extern "C" int halo_interpolate(halo_field_t field, const halo_fe_t* evals, unsigned log_n, halo_fe_t* coeffs,
                                size_t* out_len) {
    clear_error();
    HALO_CHECK(check_field(field));
    if (!evals || !coeffs) return set_error(HALO_EINVAL, "halo_interpolate: null buffer");
    if (log_n > 28) return set_error(HALO_EINVAL, "log_n %u too large", log_n);
    const size_t N = (size_t)1 << log_n;
    HALO_CHECK(ntt_host(field, evals, N, log_n, 1, coeffs));
    // DensePolynomial::from_coefficients_vec trims trailing zeros
    size_t n = N;
    while (n > 0 && !(coeffs[n - 1].l[0] | coeffs[n - 1].l[1] | coeffs[n - 1].l[2] | coeffs[n - 1].l[3])) n--;
    if (out_len) *out_len = n;
    return HALO_OK;
}

extern "C" int halo_ntt_dev(halo_field_t field, void* d_data, unsigned log_n, size_t batch, int inverse, void* stream) {
    clear_error();
    HALO_CHECK(check_field(field));
    if (!d_data) return set_error(HALO_EINVAL, "halo_ntt_dev: null buffer");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    const size_t N = (size_t)1 << log_n;
    hipStream_t s = (hipStream_t)stream;
    ScratchUse su(st, s);
    // in place: the passes ping-pong through scratch (a second scratch buffer takes the first pass
    // when the pass count is odd, so no pass reads and writes one buffer)
    HALO_CHECK(st->scratch[4].reserve(batch * N * 32));
    HALO_CHECK(st->scratch[5].reserve(batch * N * 32));
    return ntt_device_dispatch(st, field, d_data, d_data, st->scratch[4].ptr, log_n, batch, inverse, s,
                               st->scratch[5].ptr);
}

// Forward device NTT of data whose elements at index >= nonzero_len are zero (the prover's
// evaluate_over_domain of a degree < n polynomial on the 8n domain): those elements are not read,
// and the first pass skips the lg(N / 2^ceil(lg nonzero_len)) stages that only replicate values.
extern "C" int halo_ntt_dev_zero_tail(halo_field_t field, void* d_data, unsigned log_n, size_t batch,
                                      size_t nonzero_len, void* stream) {
    clear_error();
    HALO_CHECK(check_field(field));
    if (!d_data) return set_error(HALO_EINVAL, "halo_ntt_dev_zero_tail: null buffer");
    const size_t N = (size_t)1 << log_n;
    if (nonzero_len > N) return set_error(HALO_EINVAL, "halo_ntt_dev_zero_tail: nonzero_len > N");
    unsigned lg_nz = 0;
    while (((size_t)1 << lg_nz) < std::max<size_t>(nonzero_len, 1)) lg_nz++;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = (hipStream_t)stream;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[4].reserve(batch * N * 32));
    HALO_CHECK(st->scratch[5].reserve(batch * N * 32));
    // the tail's contents are ignored: zero exactly what pass 0 will read beyond nonzero_len (up to
    // 2^ceil(lg nonzero_len) when it prunes, the whole tail otherwise)
    const unsigned pr = log_n ? ntt_pass0_prune(ntt_radices(log_n)[0], log_n - lg_nz) : 0u;
    const size_t read_end = pr ? (N >> pr) : N;
    if (read_end > nonzero_len)
        for (size_t b = 0; b < batch; b++)
            HALO_HIP(hipMemsetAsync((char*)d_data + (b * N + nonzero_len) * 32, 0, (read_end - nonzero_len) * 32, s));
    return ntt_device_dispatch(st, field, d_data, d_data, st->scratch[4].ptr, log_n, batch, 0, s, st->scratch[5].ptr,
                               log_n - lg_nz);
}

extern "C" int halo_ntt_twiddle_dev(halo_field_t field, void* d_data, unsigned log_n, size_t rows, size_t cols,
                                    size_t row0, size_t col0, int inverse, void* stream) {
    clear_error();
    HALO_CHECK(check_field(field));
    if (!d_data && rows * cols) return set_error(HALO_EINVAL, "halo_ntt_twiddle_dev: null buffer");
    if (log_n == 0 || log_n > 30) return set_error(HALO_EINVAL, "halo_ntt_twiddle_dev: log_n %u out of range", log_n);
    if (!rows || !cols) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = (hipStream_t)stream;
    const size_t cnt = rows * cols;
    const unsigned thr = 256, blocks = (unsigned)((cnt + thr - 1) / thr);
    DISPATCH_FIELD(field, F, {
        DeviceState::Twiddles* tw = nullptr;
        HALO_CHECK(get_twiddles<F>(st, field, log_n, inverse ? 1 : 0, &tw, s));
        hipLaunchKernelGGL(k_twiddle_mat<F>, dim3(blocks), dim3(thr), 0, s, (uint4*)d_data, rows, cols, row0, col0,
                           log_n, tw->lo.as<const uint4>(), tw->hi.as<const uint4>(), (uint32_t)tw->lo_bits);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_transpose_dev(const void* d_src, void* d_dst, size_t batch, size_t rows, size_t cols, size_t run,
                                  void* stream) {
    clear_error();
    if (!batch || !rows || !cols || !run) return HALO_OK;
    if (!d_src || !d_dst || d_src == d_dst) return set_error(HALO_EINVAL, "halo_transpose_dev: bad buffers");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    if (run == 1 && batch <= 65535 && (rows + 31) / 32 <= 65535) {
        dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32), (unsigned)batch);
        hipLaunchKernelGGL(k_transpose32, grid, dim3(256), 0, (hipStream_t)stream, (const uint4*)d_src,
                           (uint4*)d_dst, rows, cols);
    } else {
        const size_t total = batch * rows * cols * run;
        hipLaunchKernelGGL(k_transpose_runs, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           (const uint4*)d_src, (uint4*)d_dst, batch, rows, cols, run);
    }
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}
