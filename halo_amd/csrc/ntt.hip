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
// Elements per thread: radix-4 register groups, two stages per LDS round trip.  (Round 3 measured radix-8
// groups on the 2048-element blocks -- 4 LDS round trips per 11-bit pass instead of 6 -- slower: 192 VGPRs
// leave 2 waves per SIMD and the barrier waits were hidden worse than they were saved.)
constexpr int NTT_EPT = 4;
constexpr int NTT_MAX_LOG_R_MULTI = 8;
constexpr int NTT_TW_MAX = 2048;  // stage-twiddle table entries (stages 0..10), read through L1/L2
constexpr int NTT_TW_U4 = 3;      // one stage twiddle: its 9 limbs in a 48-B entry (no unpacking in the groups)
constexpr unsigned NTT_FULL_TABLE_MAX_LOG = 24;  // per-pass twiddle tables up to 2^24

struct NttPassArgs {
    const uint4* in;
    uint4* out;
    const uint4* tw;        // per-pass pre-twiddle table tw[rho * Ns + jj] (internal packed), or null
    const uint4* tw_hi;     // 2-level fallback (logn > NTT_FULL_TABLE_MAX_LOG)
    const uint4* tw_lo;
    const uint4* stage_tw;  // entry 2^s - 1 + k = omega_{2^(s+1)}^k (s < 11, k < 2^s), NTT_TW_U4 uint4 each
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
// bits with a linear function of p >> 5, chosen so that every ds_read_b32 / ds_write_b32 of the load,
// group and store phases is conflict-free (each half-wave's 32 positions on 32 banks): for NE = 1024
// over r = 1..8, for NE = 2048 over r = 9..11, including the unit groups' thread order (ntt_unit_tau).
// tools/ntt_swizzle.py enumerates the access patterns and checks / searches the constants.  (A
// 4096-element variant for 2 x 12-bit passes at 2^24 was measured 47 % slower than 3 x 8 bits: one
// 1024-thread block per CU and 32-byte strided column loads; not kept.)
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
    static constexpr uint32_t C[6] = {29, 22, 20, 23, 9, 19};
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

// ---- signed lazy butterflies (round 5) ----------------------------------------------------------
// Inside a pass a value is 9 signed int32 limbs (value = sum l_i 2^(29 i), congruent mod p to the
// element; its magnitude stays below ~20 p).  A butterfly is one limb-wise add and one limb-wise
// subtract (18 instructions: no carries, no multiple of p added), and the twiddle product fs_mul takes
// the signed operand through v_mad_i64_i32 (gen_field_asm.py fe_muls_asm) and returns low limbs in
// [0, 2^29) with a signed top limb.  Limb bounds, in units of 2^29 (low limbs; the top limb is bounded
// by the value): a product or a normalized value lies in (-eps, 1 + eps), and u +- t widens the
// interval by one, so three butterflies from normalized values leave (-3, 4) -- still int32 -- and a
// product operand in (-2, 3) keeps every column below 9 x 3 x 2^58 (products) + 5 x 2^58 (reduction
// terms) < 2^63.  So fs_norm (parallel carries, 3 instructions per limb) runs once per radix-4 group,
// and the stage from the loads (G0 = 1) needs none.  Round 4's unsigned form spent a signed carry chain
// with a 2p / 4p offset per subtraction and a carry chain per addition pair.
template <class F>
HALO_DEV Fe<F> fs_add(const Fe<F>& a, const Fe<F>& b) {
    Fe<F> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = a.v[i] + b.v[i];
    return r;
}
template <class F>
HALO_DEV Fe<F> fs_sub(const Fe<F>& a, const Fe<F>& b) {
    Fe<F> r;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) r.v[i] = a.v[i] - b.v[i];
    return r;
}
// a w with a signed-limb a (limbs in (-2, 3) x 2^29) and a normalized twiddle w (< 2p)
template <class F>
HALO_DEV Fe<F> fs_mul(const Fe<F>& a, const Fe<F>& w) {
    Fe<F> r;
    fe_muls_asm(a.v, w.v, NegP<F>::v, r.v);
    return r;
}
// limbs (-3, 4) x 2^29 -> [-3, 2^29 + 3): each limb keeps its low 29 bits plus the carry of the limb
// below (independent per limb, no chain); the top limb absorbs limb 7's carry
template <class F>
HALO_DEV Fe<F> fs_norm(const Fe<F>& a) {
    Fe<F> r;
    r.v[0] = a.v[0] & LIMB_MASK;
#pragma unroll
    for (int i = 1; i < NLIMB; i++) {
        const uint32_t c = (uint32_t)((int32_t)a.v[i - 1] >> LIMB_BITS);
        r.v[i] = ((i == NLIMB - 1) ? a.v[i] : (a.v[i] & LIMB_MASK)) + c;
    }
    return r;
}
// limbs (-4, 4) x 2^29 -> exactly normalized low limbs [0, 2^29) (one signed carry chain; the top limb
// takes the final carry)
template <class F>
HALO_DEV Fe<F> fs_carry(const Fe<F>& a) {
    Fe<F> r;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB - 1; i++) {
        const int32_t x = (int32_t)a.v[i] + c;
        r.v[i] = (uint32_t)x & LIMB_MASK;
        c = x >> LIMB_BITS;
    }
    r.v[NLIMB - 1] = a.v[NLIMB - 1] + (uint32_t)c;
    return r;
}
// signed lazy value (limbs in (-3, 4) x 2^29) -> the same residue, non-negative with normalized limbs
// and below 2^255 + 2^235 (< 4p, so it packs into 32 B): subtract (q - 1) p with q = floor(top limb /
// 2^22), within one of floor(value / 2^254) (p = 2^254 + delta, delta < 2^126), in one signed carry chain
template <class F>
HALO_DEV Fe<F> fs_settle(const Fe<F>& x) {
    const int32_t qm = 1 - ((int32_t)x.v[NLIMB - 1] >> 22);
    Fe<F> r;
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < NLIMB; i++) {
        int64_t d = (int64_t)(int32_t)x.v[i] + c;
        if (F::P[i] != 0) d += (int64_t)qm * (int64_t)F::P[i];
        r.v[i] = (i == NLIMB - 1) ? (uint32_t)d : ((uint32_t)d & LIMB_MASK);
        c = d >> LIMB_BITS;
    }
    return r;
}

// The pass's first G0 <= 2 stages on the thread's EPT consecutive positions, straight from the loads:
// stage 0's twiddles are 1; stage 1 pairs (0, 2) with twiddle 1 and (1, 3) with omega_4 (w4).  With
// G0 = 2 the results are normalized (two more stages follow before the next fs_norm); with G0 = 1 not.
template <class F>
HALO_DEV void ntt_first(Fe<F> (&v)[NTT_EPT], uint32_t G0, const uint4* twg) {
#pragma unroll
    for (int m = 0; m < NTT_EPT; m += 2) {
        const Fe<F> t = v[m + 1];
        v[m + 1] = fs_sub(v[m], t);
        v[m] = fs_add(v[m], t);
    }
    if (G0 > 1) {
        Fe<F> w4;
        const uint32_t* e = (const uint32_t*)(twg + NTT_TW_U4 * 2);
#pragma unroll
        for (int l = 0; l < NLIMB; l++) w4.v[l] = e[l];
        Fe<F> t = v[2];
        v[2] = fs_sub(v[0], t);
        v[0] = fs_add(v[0], t);
        t = fs_mul(v[3], w4);
        v[3] = fs_sub(v[1], t);
        v[1] = fs_add(v[1], t);
#pragma unroll
        for (int m = 0; m < NTT_EPT; m++) v[m] = fs_norm(v[m]);
    }
}

// The stage twiddles one thread needs for a radix-4 group at stages s, s + 1: stage s uses
// omega_{2^(s+1)}^k0 for both of its butterflies, stage s + 1 omega_{2^(s+2)}^(k0) and ^(k0 + 2^s).
// Loaded (9 limbs each) BEFORE the barrier that precedes the group's LDS reads, so the L2 round trip of
// the table overlaps the barrier wait instead of following it.
struct NttGroupTw {
    uint32_t w[3][NLIMB];
};
HALO_DEV void ntt_group_tw_load(NttGroupTw& t, uint32_t s, uint32_t G, uint32_t k0, const uint4* twg) {
#pragma unroll
    for (int g = 0; g < 2; g++) {
        if ((uint32_t)g >= G) break;
#pragma unroll
        for (int j = 0; j < (1 << g); j++) {
            const uint32_t i = ((1u << (s + g)) - 1u) + k0 + ((uint32_t)j << s);
            const uint4* e = twg + NTT_TW_U4 * i;
            const uint4 x = e[0], y = e[1];
            uint32_t* w = t.w[(1 << g) - 1 + j];
            w[0] = x.x, w[1] = x.y, w[2] = x.z, w[3] = x.w;
            w[4] = y.x, w[5] = y.y, w[6] = y.z, w[7] = y.w;
            w[8] = ((const uint32_t*)e)[8];
        }
    }
}
template <class F>
HALO_DEV Fe<F> ntt_tw(const uint32_t (&w)[NLIMB]) {
    Fe<F> r;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) r.v[l] = w[l];
    return r;
}

// Radix-4 group at stages s, s + 1 (s >= 1) with the twiddles already loaded.  UNIT: k0 = 0, so the
// twiddles of stage s and of stage s + 1's first pair are 1 (the wave-uniform unit group of
// ntt_unit_tau: three of the four multiplications skipped).  An unmultiplied butterfly operand keeps
// its own limb interval instead of a product's [0, 1), so the unit group first carries its inputs
// exactly: v0 + v1 + v2 + v3 then stays below 4 (2^29 - 1) < 2^31.
// norm: 0 none (the pass's last group when the output path multiplies nothing: fs_settle takes limbs in
// (-4, 4)), 1 partial, 2 full.  From normalized inputs a group leaves v0 in [0, 3), v1, v2 in (-1, 2)
// and v3 in (-2, 1) (units of 2^29): normalizing v0 alone leaves every output within (-2, 2), and a
// group from such inputs stays mult-safe (operands within (-3, 3)) and ends within (-4, 4), where
// every output is normalized.  So groups alternate partial / full: 5 fs_norm per 8 outputs, not 8.
template <class F, bool UNIT>
HALO_DEV void ntt_group4(Fe<F> (&v)[NTT_EPT], uint32_t G, const NttGroupTw& t, uint32_t norm) {
    if (UNIT) {
#pragma unroll
        for (int m = 0; m < NTT_EPT; m++) v[m] = fs_carry(v[m]);
    }
#pragma unroll
    for (int m = 0; m < NTT_EPT; m += 2) {
        const Fe<F> x = UNIT ? v[m + 1] : fs_mul(v[m + 1], ntt_tw<F>(t.w[0]));
        v[m + 1] = fs_sub(v[m], x);
        v[m] = fs_add(v[m], x);
    }
    if (G > 1) {
        Fe<F> x = UNIT ? v[2] : fs_mul(v[2], ntt_tw<F>(t.w[1]));
        v[2] = fs_sub(v[0], x);
        v[0] = fs_add(v[0], x);
        x = fs_mul(v[3], ntt_tw<F>(t.w[2]));
        v[3] = fs_sub(v[1], x);
        v[1] = fs_add(v[1], x);
    }
    // (written as two independent conditions: an if / else-if form made the compiler hold 144 VGPRs,
    // one wave per SIMD fewer)
    if (norm != 0) v[0] = fs_norm(v[0]);
    if (norm == 2) {
#pragma unroll
        for (int m = 1; m < NTT_EPT; m++) v[m] = fs_norm(v[m]);
    }
}

// Wave-uniform unit twiddles.  The group at stage US has twiddle index k0 = position mod 2^US; in its
// thread order ntt_unit_tau the position's low US bits come from the wave's thread bits (the top US
// bits of the thread index), so k0 is the same on a whole wave and the k0 = 0 waves skip the
// multiplications by 1 (stage US, and stage US + 1's first pair: three of four).  1024-element blocks
// (the <= 8-bit passes: 2^23, 2^24, ...): US = 2, wave 0 of the block's four is unit (with four blocks
// per CU starting on varying SIMDs the skips spread over the SIMDs): 0.19 per element per pass.
// 2048-element blocks: none (below).
// (round 6: the 2048-element blocks no longer use it -- their unit group at stage 1 spans the block, so
// it cost two full barriers per pass; without it the groups up to stage 6 stay wave-local: 2^22 pair
// 0.968-0.976 -> 0.949-0.957 ms interleaved, against 3 % more multiplications.  On 1024-element blocks
// the same change lost 1 % at 2^23 / 2^24, so they keep it.)
template <int NE>
HALO_DEV uint32_t ntt_unit_stage(uint32_t T) {
    (void)T;
    return NE == NTT_E_BIG ? 0u : 2u;
}
template <int NE>
HALO_DEV uint32_t ntt_unit_tau(uint32_t tau, uint32_t us) {
    constexpr uint32_t LG_TH = NE == NTT_E_BIG ? 9u : 8u;
    return ((tau << us) | (tau >> (LG_TH - us))) & ((1u << LG_TH) - 1u);
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
// owns T = NE / R consecutive columns.  Each thread holds EPT elements in registers; the first
// G0 stages are done straight from the global loads, the rest in radix-4 groups through LDS, and a
// final coalesced store phase writes y[(j / Ns) Ns R + (j mod Ns) + k Ns].
// FULL: the block's T R positions fill all NE (every transform of at least NE elements), so no phase
// tests a position against EB -- without the tests the compiler also drops the register copies that
// the conditional LDS reads and writes cost (36 v_mov per group and thread in the 2048-element kernel)
template <class F, int NE, bool FULL>
__global__ __launch_bounds__(NE / NTT_EPT, 4) void k_ntt_pass(NttPassArgs a) {
    constexpr int EPT = NTT_EPT;
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

    // ---- load + pre-twiddle + first G0 stages (positions base + m)
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
        if (FULL || pos < EB) {
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
                x = fs_mul(x, oc);
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
                x = fs_mul(x, w);
            }
            v[m] = x;
        } else {
            v[m] = fe_zero<F>();
        }
    }
    // on the wide blocks the short group goes first (r mod 2 stages), so later groups stay in range
    const uint32_t G0 = (NE >= NTT_E_BIG && (r & 1)) ? 1u : (r < 2u ? r : 2u);
    if (!a.prune) ntt_first<F>(v, G0, a.stage_tw);  // (pruned: host guarantees prune >= G0)
    {
        const uint32_t pb = ntt_swz<NE>(base);
#pragma unroll
        for (int m = 0; m < EPT; m++)
            if (FULL || base + m < EB) lds_put_soa(data, pb ^ (uint32_t)m, NE, v[m]);
    }
    // ---- remaining stages in radix-4 groups through LDS; each group's twiddles are loaded before the
    // barrier that precedes its LDS reads
    const uint32_t US = ntt_unit_stage<NE>(T);
    constexpr uint32_t LG_TH = NE == NTT_E_BIG ? 9u : 8u;
    // wave-uniform: the top US thread bits (the wave's) are zero
    const bool unit_wave = US != 0u && (__builtin_amdgcn_readfirstlane(tau) >> (LG_TH - US)) == 0u;
    // the output path multiplies unless the last pass's pre-twiddle table carries out_const
    const bool out_mul = a.out_ark && !a.out_scaled;
    uint32_t s = a.prune ? a.prune : G0;
    // the next group's inputs are normalized: loaded values (pruned pass) or ntt_first's G0 = 2 output;
    // G0 = 1 leaves (-1, 2)
    bool in_norm = a.prune != 0 || G0 != 1;
    NttGroupTw tw;
    {
        const uint32_t tt = (US != 0u && s == US) ? ntt_unit_tau<NE>(tau, US) : tau;
        if (s < r) ntt_group_tw_load(tw, s, (r - s) < 2u ? (r - s) : 2u, tt & ((1u << s) - 1), a.stage_tw);
    }
    // Wave-local exchanges: a group at stage s <= 6 (2^s <= 64) reads and writes exactly its wave's
    // chunk of EPT * 64 consecutive positions [EPT 64 w, EPT 64 (w + 1)), and so does the load phase
    // of a one-column block (base = EPT tau); between two such phases the wave only waits for its own
    // LDS writes.  (The unit group's order of ntt_unit_tau spans the block: full barriers around it.)
    auto wave_local = [&](uint32_t sg) { return sg <= 6u && !(US != 0u && sg == US); };
    ntt_lds_barrier((T == 1u || R < (uint32_t)EPT) && s < r && wave_local(s));
    for (; s < r; s += 2) {
        const uint32_t G = (r - s) < 2u ? (r - s) : 2u;
        const uint32_t h = 1u << s;
        const bool unit_grp = US != 0u && s == US;
        const uint32_t tt = unit_grp ? ntt_unit_tau<NE>(tau, US) : tau;
        const uint32_t gb = (tt & (h - 1)) | ((tt >> s) << (s + 2));
        const uint32_t shb = ntt_swz_hi<NE>(gb >> 5);
#pragma unroll
        for (int m = 0; m < EPT; m++) {
            const uint32_t pos = gb + (uint32_t)m * h;
            const uint32_t ph = (pos ^ shb) ^ ntt_swz_hi<NE>(((uint32_t)m * h) >> 5);
            if (FULL || pos < EB) v[m] = lds_get_soa<F>(data, ph, NE);
        }
        // partial after normalized inputs, full otherwise.  The choice is block-uniform: the next group
        // reads positions other waves wrote (the unit group's thread order crosses waves), so the unit
        // waves -- whose carried inputs would allow a partial normalization -- follow the same rule as
        // the others (a one-stage group, G = 1, stays within the partial bound too)
        const uint32_t norm = (s + 2 >= r && !out_mul) ? 0u : (in_norm ? 1u : 2u);
        if (unit_grp && unit_wave)
            ntt_group4<F, true>(v, G, tw, norm);
        else
            ntt_group4<F, false>(v, G, tw, norm);
        in_norm = norm == 2;
        // (no barrier here: a thread writes back exactly the positions it read)
#pragma unroll
        for (int m = 0; m < EPT; m++) {
            const uint32_t pos = gb + (uint32_t)m * h;
            const uint32_t ph = (pos ^ shb) ^ ntt_swz_hi<NE>(((uint32_t)m * h) >> 5);
            if (FULL || pos < EB) lds_put_soa(data, ph, NE, v[m]);
        }
        const uint32_t sn = s + 2;
        if (sn < r) {
            const uint32_t tn = (US != 0u && sn == US) ? ntt_unit_tau<NE>(tau, US) : tau;
            ntt_group_tw_load(tw, sn, (r - sn) < 2u ? (r - sn) : 2u, tn & ((1u << sn) - 1), a.stage_tw);
        }
        ntt_lds_barrier(wave_local(s) && sn < r && wave_local(sn));
    }

    // ---- store y[(j / Ns) Ns R + (j mod Ns) + k Ns]
#pragma unroll
    for (int i = 0; i < EPT; i++) {
        const uint32_t idx = tau + TH * (uint32_t)i;
        if (!FULL && idx >= EB) continue;
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
        if (out_mul) {
            Fe<F> oc;
#pragma unroll
            for (int l = 0; l < NLIMB; l++) oc.v[l] = a.out_const[l];
            x = fs_mul(x, oc);
        }
        x = fs_settle(x);
        if (a.out_ark) x = fe_canon(fe_reduce_2p(x));
        // one store statement: with a store on each branch the compiler merged their common words into
        // four stores per element (dword, dword, misaligned dwordx4, dwordx3) instead of two dwordx4
        fe_store(out + 2 * dst, x);
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

// Stage twiddles omega^k, k < count, as 9 limbs in NTT_TW_U4 uint4 (limbs 0..8, then zero padding)
template <class F>
__global__ void k_stage_twiddles(uint4* out, size_t count, Fe<F> base) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint64_t e = i;
    Fe<F> r = fe_one<F>();
    Fe<F> b = base;
    while (e) {
        if (e & 1) r = fe_mul(r, b);
        b = fe_sqr(b);
        e >>= 1;
    }
    uint4* o = out + NTT_TW_U4 * i;
    o[0] = make_uint4(r.v[0], r.v[1], r.v[2], r.v[3]);
    o[1] = make_uint4(r.v[4], r.v[5], r.v[6], r.v[7]);
    o[2] = make_uint4(r.v[8], 0u, 0u, 0u);
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
    if (logn >= 17 && logn <= std::min<long long>(2 * NTT_MAX_LOG_R_BIG, tuning(TUNE_NTT_BIG_MAX_LOG))) {
        r.push_back((logn + 1) / 2);
        r.push_back(logn / 2);
        return r;
    }
    const unsigned passes = (logn + NTT_MAX_LOG_R_MULTI - 1) / NTT_MAX_LOG_R_MULTI;
    if (tuning(TUNE_NTT_EVEN_SPLIT)) {
        // even radices where possible (an odd pass ends in a one-stage group: a whole LDS round trip
        // and normalization for half a group's butterflies): 8s, trimmed by 2 from the back, at most
        // one odd pass (2^22 = 8 + 8 + 6, 2^23 = 8 + 8 + 7)
        r.assign(passes, (unsigned)NTT_MAX_LOG_R_MULTI);
        unsigned excess = passes * NTT_MAX_LOG_R_MULTI - logn;
        for (unsigned k = passes; excess >= 2; k = (k == 1 ? passes : k - 1)) {
            r[k - 1] -= 2;
            excess -= 2;
        }
        if (excess) r[passes - 1] -= 1;
        return r;
    }
    unsigned left = logn;
    for (unsigned p = 0; p < passes; p++) {
        unsigned take = (left + (passes - p) - 1) / (passes - p);
        r.push_back(take);
        left -= take;
    }
    return r;
}

// the split as one key (5 bits per pass) for the twiddle-table cache
static uint64_t ntt_split_key(const std::vector<unsigned>& rad) {
    uint64_t k = 0;
    for (unsigned x : rad) k = (k << 5) | x;
    return k;
}

// Stages of pass 0 (radix 2^lr) that a zero tail lets the pass skip (NttPassArgs::prune): only when
// they cover its first register group; on one-column wide blocks a trailing single-stage group would
// reach past the column, so the stages left after the pruned ones must pair up (as G0 = 1 arranges).
static unsigned ntt_pass0_prune(unsigned lr, unsigned prune) {
    if (!prune) return 0;
    const bool big = lr > NTT_MAX_LOG_R_MULTI;
    const unsigned lg = 2u;
    const unsigned g0 = (big && (lr % lg)) ? lr % lg : std::min(lr, lg);
    unsigned pr = std::min(prune, lr);
    while (big && pr > 0 && ((lr - pr) % lg)) pr--;
    return (pr >= g0 && pr < lr) ? pr : 0u;
}

// `rad`: the pass split the caller launches with (ntt_radices read once per transform, so a concurrent
// halo_set_tuning of the split keys cannot pair tables built for one split with passes of another)
template <class F>
static int get_twiddles(DeviceState* st, int field, unsigned logn, int inverse, const std::vector<unsigned>& rad,
                        DeviceState::Twiddles** out, hipStream_t s) {
    const uint64_t split = ntt_split_key(rad);
    for (auto& t : st->tw)
        if (t->field == field && t->logn == (int)logn && t->inverse == inverse && t->split == split) {
            *out = t.get();
            return HALO_OK;
        }
    auto t = std::make_unique<DeviceState::Twiddles>();
    t->field = field;
    t->logn = (int)logn;
    t->inverse = inverse;
    t->split = split;
    t->lo_bits = (int)((logn + 1) / 2);
    const size_t nlo = (size_t)1 << t->lo_bits, nhi = (size_t)1 << (logn - t->lo_bits);
    HALO_CHECK(t->lo.reserve(nlo * 32));
    HALO_CHECK(t->hi.reserve(nhi * 32));
    const Fe<F> w = host_fe<F>(inverse ? F::OMEGA_INV[logn] : F::OMEGA[logn]);
    HALO_CHECK(launch_pow_table<F>(t->lo.as<uint4>(), nlo, w, 1, s));
    HALO_CHECK(launch_pow_table<F>(t->hi.as<uint4>(), nhi, w, (uint64_t)nlo, s));
    // stage twiddles omega_{2^(s+1)}^k (the same for every N; kept per table for simplicity)
    HALO_CHECK(t->stage.reserve(NTT_TW_MAX * NTT_TW_U4 * 16));
    for (unsigned sg = 0; sg < NTT_MAX_LOG_R_BIG; sg++) {
        const Fe<F> ws = host_fe<F>(inverse ? F::OMEGA_INV[sg + 1] : F::OMEGA[sg + 1]);
        const size_t cnt = (size_t)1 << sg;
        hipLaunchKernelGGL(k_stage_twiddles<F>, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s,
                           t->stage.as<uint4>() + NTT_TW_U4 * (cnt - 1), cnt, ws);
        HALO_HIP(hipGetLastError());
    }
    // per-pass pre-twiddle tables (one multiplication per element instead of two)
    if (logn <= NTT_FULL_TABLE_MAX_LOG) {
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
                      unsigned logn, size_t batch, int inverse, hipStream_t s, unsigned prune,
                      const std::vector<unsigned>* rad_in) {
    if (logn > 30) return set_error(HALO_EINVAL, "NTT domain 2^%u too large", logn);
    const size_t N = (size_t)1 << logn;
    if (logn == 0) {
        if (d_in != d_out) HALO_HIP(hipMemcpyAsync(d_out, d_in, batch * 32, hipMemcpyDeviceToDevice, s));
        return HALO_OK;
    }
    const std::vector<unsigned> rad = rad_in ? *rad_in : ntt_radices(logn);
    DeviceState::Twiddles* tw = nullptr;
    HALO_CHECK(get_twiddles<F>(st, field, logn, inverse, rad, &tw, s));
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
        const bool full = (T << lr) == NE;
        if (NE == NTT_E_BIG && full)
            HALO_LAUNCH(prof, (k_ntt_pass<F, NTT_E_BIG, true>), grid, dim3(NTT_E_BIG / NTT_EPT), lds, s, a);
        else if (NE == NTT_E_BIG)
            HALO_LAUNCH(prof, (k_ntt_pass<F, NTT_E_BIG, false>), grid, dim3(NTT_E_BIG / NTT_EPT), lds, s, a);
        else if (full)
            HALO_LAUNCH(prof, (k_ntt_pass<F, NTT_E, true>), grid, dim3(NTT_E / NTT_EPT), lds, s, a);
        else
            HALO_LAUNCH(prof, (k_ntt_pass<F, NTT_E, false>), grid, dim3(NTT_E / NTT_EPT), lds, s, a);
        HALO_HIP(hipGetLastError());
        log_ns += lr;
    }
    return HALO_OK;
}

int ntt_device_dispatch(DeviceState* st, int field, const void* d_in, void* d_out, void* d_tmp, unsigned logn,
                        size_t batch, int inverse, hipStream_t s, void* d_tmp2, unsigned prune,
                        const std::vector<unsigned>* rad) {
    int rc;
    DISPATCH_FIELD(field, F, {
        rc = ntt_device<F>(st, field, d_in, d_out, d_tmp, d_tmp2, logn, batch, inverse, s, prune, rad);
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
    const std::vector<unsigned> rad = ntt_radices(log_n);  // one read: the zeroed span and the passes agree
    const unsigned pr = log_n ? ntt_pass0_prune(rad[0], log_n - lg_nz) : 0u;
    const size_t read_end = pr ? (N >> pr) : N;
    if (read_end > nonzero_len)
        for (size_t b = 0; b < batch; b++)
            HALO_HIP(hipMemsetAsync((char*)d_data + (b * N + nonzero_len) * 32, 0, (read_end - nonzero_len) * 32, s));
    return ntt_device_dispatch(st, field, d_data, d_data, st->scratch[4].ptr, log_n, batch, 0, s, st->scratch[5].ptr,
                               log_n - lg_nz, &rad);
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
        HALO_CHECK(get_twiddles<F>(st, field, log_n, inverse ? 1 : 0, ntt_radices(log_n), &tw, s));
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
