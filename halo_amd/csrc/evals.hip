// SURVEY §8f row f1 (first slice): the prover's elementwise polynomial-evaluation algebra and the
// vanishing-polynomial division, device-resident.
//
//   Evals ops (crates/group/src/poly.rs:90-327): pointwise add / sub / mul of two evaluation
//   vectors, scale / add_scalar / sub_scalar by one scalar, and x^e (the Poseidon S-box x^7 of the
//   gate evaluation, protocol.rs:591-1011).
//   DensePolynomial::divide_by_vanishing_poly (ark-poly 0.5.0, called at protocol.rs:256): for
//   Z_H = X^n - 1, quotient q[j] = sum_{k >= 1} c[j + k n] and remainder r[j] = c[j] + q[j] (j < n),
//   both trimmed.
//
// These are HBM-streaming kernels (one read per operand, one write): every lane handles whole
// 32-byte elements with two dwordx4 accesses, consecutive lanes consecutive elements.  Values stay
// in the ark format (Montgomery R = 2^256): additions are format-agnostic; a product of two ark
// values through the R' = 2^261 multiplier carries 2^-5 too many, fixed by one multiplication by
// 2^266 mod p (ARK_MUL_FIX, computed on the host side of the launch).
#include <algorithm>

#include "dispatch.hpp"
#include "runtime.hpp"

namespace halo {

enum EvalsOp { EV_ADD = 0, EV_SUB = 1, EV_MUL = 2, EV_SCALE = 3, EV_ADD_SCALAR = 4, EV_SUB_SCALAR = 5, EV_POW = 6 };

template <class F>
__global__ __launch_bounds__(256) void k_evals_op(int op, const uint4* a, const uint4* b, Fe<F> s, uint32_t e,
                                                  Fe<F> fix, uint4* out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Fe<F> x = fe_load<F>(a + 2 * i);
    Fe<F> r;
    switch (op) {
        case EV_ADD: r = fe_add(x, fe_load<F>(b + 2 * i)); break;
        case EV_SUB: r = fe_sub(x, fe_load<F>(b + 2 * i)); break;
        case EV_MUL: r = fe_mul(fe_mul(x, fe_load<F>(b + 2 * i)), fix); break;
        case EV_SCALE: r = fe_mul(fe_mul(x, s), fix); break;
        case EV_ADD_SCALAR: r = fe_add(x, s); break;
        case EV_SUB_SCALAR: r = fe_sub(x, s); break;
        default: {  // EV_POW: internal domain, square-and-multiply
            const Fe<F> xi = fe_mul(x, fe_from_const<F>(F::ARK2INT));
            Fe<F> acc = fe_one<F>();
            for (int bit = 31; bit >= 0; bit--) {
                acc = fe_sqr(acc);
                if ((e >> bit) & 1u) acc = fe_mul(acc, xi);
            }
            r = fe_mul(acc, fe_from_const<F>(F::INT2ARK));
        }
    }
    fe_store(out + 2 * i, fe_canon(r));
}

// q[j] = sum_{k >= 1, j + k n < len} c[j + k n]  (j < len - n);  r[j] = c[j] + q[j]  (j < n)
template <class F>
__global__ __launch_bounds__(256) void k_div_vanishing(const uint4* c, size_t len, size_t n, uint4* q, uint4* r) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t qn = len - n;
    if (j < qn) {
        Fe<F> acc = fe_zero<F>();
        for (size_t k = j + n; k < len; k += n) acc = fe_add(acc, fe_load<F>(c + 2 * k));
        fe_store(q + 2 * j, fe_canon(acc));
    }
    if (j < n) {
        Fe<F> acc = fe_load<F>(c + 2 * j);
        for (size_t k = j + n; k < len; k += n) acc = fe_add(acc, fe_load<F>(c + 2 * k));
        fe_store(r + 2 * j, fe_canon(acc));
    }
}

// Running product (protocol.rs:143-154, the permutation accumulator z): inclusive prefix product
// out[i] = prod_{j <= i} in[j] (reverse: suffix product prod_{j >= i} in[j]), ark in / out.  Three
// phases: per-block scan (SCAN_EPT elements per thread, then a Hillis-Steele scan of the thread
// products in LDS), a one-block scan of the block totals, and a multiply by each block's exclusive
// prefix.  Internal Montgomery form inside (one conversion in, one out).
constexpr int SCAN_THREADS = 256, SCAN_EPT = 8, SCAN_BLOCK = SCAN_THREADS * SCAN_EPT;

HALO_DEV size_t scan_idx(size_t i, size_t n, int reverse) { return reverse ? n - 1 - i : i; }

template <class F>
HALO_DEV void lds_scan_mul(uint4* red, uint32_t tid, Fe<F>& v) {  // inclusive scan of v over the block
    fe_store(red + 2 * tid, v);
    __syncthreads();
    for (uint32_t off = 1; off < SCAN_THREADS; off <<= 1) {
        Fe<F> t = v;
        if (tid >= off) t = fe_mul(fe_load<F>(red + 2 * (tid - off)), v);
        __syncthreads();
        v = t;
        fe_store(red + 2 * tid, v);
        __syncthreads();
    }
}

template <class F>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_block(const uint4* in, uint4* out, size_t n, int reverse,
                                                             uint4* totals) {
    __shared__ uint4 red[SCAN_THREADS * 2];
    const uint32_t tid = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * SCAN_BLOCK + (size_t)tid * SCAN_EPT;
    Fe<F> x[SCAN_EPT];
    Fe<F> run = fe_one<F>();
#pragma unroll
    for (int e = 0; e < SCAN_EPT; e++) {
        x[e] = fe_one<F>();
        if (base + e < n) x[e] = fe_from_ark<F>(in + 2 * scan_idx(base + e, n, reverse));
        run = fe_mul(run, x[e]);
    }
    Fe<F> incl = run;
    lds_scan_mul<F>(red, tid, incl);
    Fe<F> p = fe_one<F>();  // exclusive prefix of this thread inside the block
    if (tid > 0) p = fe_load<F>(red + 2 * (tid - 1));
#pragma unroll
    for (int e = 0; e < SCAN_EPT; e++) {
        p = fe_mul(p, x[e]);
        if (base + e < n) fe_to_ark(out + 2 * scan_idx(base + e, n, reverse), p);
    }
    if (tid == SCAN_THREADS - 1) fe_store(totals + 2 * blockIdx.x, fe_reduce_2p(incl));
}

// one block: totals[b] <- exclusive prefix product of the block totals (internal form)
template <class F>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_totals(uint4* totals, uint32_t nb) {
    __shared__ uint4 red[SCAN_THREADS * 2];
    const uint32_t tid = threadIdx.x;
    const uint32_t per = (nb + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint32_t b0 = tid * per;
    Fe<F> run = fe_one<F>();
    for (uint32_t b = b0; b < min(nb, b0 + per); b++) run = fe_mul(run, fe_load<F>(totals + 2 * b));
    Fe<F> incl = run;
    lds_scan_mul<F>(red, tid, incl);
    Fe<F> p = fe_one<F>();
    if (tid > 0) p = fe_load<F>(red + 2 * (tid - 1));
    for (uint32_t b = b0; b < min(nb, b0 + per); b++) {
        const Fe<F> t = fe_load<F>(totals + 2 * b);
        fe_store(totals + 2 * b, fe_reduce_2p(p));
        p = fe_mul(p, t);
    }
}

template <class F>
__global__ __launch_bounds__(256) void k_scan_apply(uint4* out, size_t n, int reverse, const uint4* totals) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x + SCAN_BLOCK;  // block 0 is final
    if (i >= n) return;
    const size_t j = scan_idx(i, n, reverse);
    const Fe<F> t = fe_load<F>(totals + 2 * (i / SCAN_BLOCK));
    fe_to_ark(out + 2 * j, fe_mul(fe_from_ark<F>(out + 2 * j), t));
}

// ---------------------------------------------------------------------------------------------
// Fused gate-constraint evaluation over the 8n domain (protocol.rs:170-191 with the constraint
// polynomials of protocol.rs:591-1011, written from their *_generic forms): one pass reads the 16
// w, 3 shifted w (w_omega = w shifted by the domain ratio), 15 r, 10 q and the public-input
// evaluations of element i and writes f_gc[i] -- instead of ~250 separate Evals kernels, each a
// full read/write of 256 MiB at n = 2^20.  Internal Montgomery form inside.
// ---------------------------------------------------------------------------------------------
struct GateArgs {
    const uint4* w[16];
    const uint4* r[15];
    const uint4* q[10];
    const uint4* pi;
    uint4 mds[9][2];  // ark words of the Poseidon MDS matrix (row-major)
};

template <class F>
HALO_DEV Fe<F> fe_from_ark_words(const uint4 (&a)[2]) {
    return fe_mul(fe_load<F>(a), fe_from_const<F>(F::ARK2INT));
}

template <class F>
HALO_DEV Fe<F> pow7(const Fe<F>& x) {
    const Fe<F> x2 = fe_sqr(x), x3 = fe_mul(x2, x), x6 = fe_sqr(x3);
    return fe_mul(x6, x);
}

// Three passes keep the live register set of each kernel small (one fused kernel needed 512 VGPRs and
// spilled): poseidon -> t0; q6 aa + q7 am + q8 eq -> t1; then the range check and the f_gc sum.
#define GATE_PROLOGUE                                                        \
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;         \
    if (i >= N) return;                                                      \
    const size_t in = (i + shift) & (N - 1);                                 \
    auto W = [&](int k) { return fe_from_ark<F>(a.w[k] + 2 * i); };          \
    auto NW = [&](int k) { return fe_from_ark<F>(a.w[k] + 2 * in); };        \
    auto R = [&](int k) { return fe_from_ark<F>(a.r[k] + 2 * i); };          \
    auto Q = [&](int k) { return fe_from_ark<F>(a.q[k] + 2 * i); };          \
    const Fe<F> one = fe_one<F>();                                           \
    (void)NW; (void)R; (void)Q; (void)one;

// poseidon_constraints_generic (protocol.rs:623-648) -> t (internal packed)
template <class F>
__global__ __launch_bounds__(256) void k_gate_poseidon(const GateArgs a, size_t N, uint32_t shift, uint4* t) {
    // the 9 MDS entries converted to the internal form once per workgroup (LDS), not at each of their
    // 45 uses (one multiplication each)
    __shared__ uint4 mds[9][2];
    if (threadIdx.x < 9) fe_store(mds[threadIdx.x], fe_from_ark_words<F>(a.mds[threadIdx.x]));
    __syncthreads();
    GATE_PROLOGUE
    Fe<F> pos = fe_zero<F>();
#pragma unroll 1
    for (int rd = 0; rd < 5; rd++) {
        const int b = 3 * rd;
        const Fe<F> s0 = pow7(W(b)), s1 = pow7(W(b + 1)), s2 = pow7(W(b + 2));
#pragma unroll 1
        for (int row = 0; row < 3; row++) {
            const Fe<F> nxt = (rd < 4) ? W(b + 3 + row) : NW(row);
            Fe<F> u = fe_add(R(b + row), fe_mul(s0, fe_load<F>(mds[3 * row + 0])));
            u = fe_add(u, fe_mul(s1, fe_load<F>(mds[3 * row + 1])));
            u = fe_add(u, fe_mul(s2, fe_load<F>(mds[3 * row + 2])));
            pos = fe_add(pos, fe_sub(nxt, u));
        }
    }
    fe_store(t + 2 * i, pos);
}

// q6 * affine_add + q7 * affine_mul + q8 * eq  -> t (internal packed)
template <class F>
__global__ __launch_bounds__(256) void k_gate_affine(const GateArgs a, size_t N, uint32_t shift, uint4* t) {
    GATE_PROLOGUE
    // affine_add_constraints_generic (protocol.rs:705-761)
    Fe<F> aa;
    {
        const Fe<F> xp = W(0), yp = W(1), xq = W(2), yq = W(3), xr = W(4), yr = W(5);
        const Fe<F> al = W(6), be = W(7), ga = W(8), de = W(9), lam = W(10);
        const Fe<F> xq_xp = fe_sub(xq, xp), yq_yp = fe_sub(yq, yp);
        aa = fe_mul(xq_xp, fe_sub(fe_mul(xq_xp, lam), yq_yp));
        const Fe<F> yp2 = fe_add(yp, yp), xpxp = fe_mul(xp, xp);
        const Fe<F> xpxp3 = fe_add(fe_add(xpxp, xpxp), xpxp);
        aa = fe_add(aa, fe_mul(fe_sub(one, fe_mul(xq_xp, al)), fe_sub(fe_mul(yp2, lam), xpxp3)));
        const Fe<F> xpxq = fe_mul(xp, xq), xpxq_d = fe_mul(xpxq, fe_sub(xq, xp));
        const Fe<F> ll_x = fe_sub(fe_sub(fe_sub(fe_mul(lam, lam), xp), xq), xr);
        aa = fe_add(aa, fe_mul(xpxq_d, ll_x));
        const Fe<F> l_y = fe_sub(fe_sub(fe_mul(lam, fe_sub(xp, xr)), yp), yr);
        aa = fe_add(aa, fe_mul(xpxq_d, l_y));
        const Fe<F> xpxq_s = fe_mul(xpxq, fe_add(yq, yp));
        aa = fe_add(aa, fe_mul(xpxq_s, ll_x));
        aa = fe_add(aa, fe_mul(xpxq_s, l_y));
        const Fe<F> l_xpb = fe_sub(one, fe_mul(xp, be));
        aa = fe_add(aa, fe_mul(l_xpb, fe_sub(xr, xq)));
        aa = fe_add(aa, fe_mul(l_xpb, fe_sub(yr, yq)));
        const Fe<F> l_xqg = fe_sub(one, fe_mul(xq, ga));
        aa = fe_add(aa, fe_mul(l_xqg, fe_sub(xr, xp)));
        aa = fe_add(aa, fe_mul(l_xqg, fe_sub(yr, yp)));
        const Fe<F> l_ad = fe_sub(fe_sub(one, fe_mul(fe_sub(xq, xp), al)), fe_mul(fe_add(yq, yp), de));
        aa = fe_add(aa, fe_mul(l_ad, xr));
        aa = fe_add(aa, fe_mul(l_ad, yr));
    }

    // (the three constraint groups one after another: their loads are not hoisted above the previous
    // group's products, so the kernel's live set is one group's, not all three -- 256 VGPRs and one
    // wave per SIMD otherwise)
    Fe<F> acc = fe_mul(Q(6), aa);
    asm volatile("" ::: "memory");
    // affine_mul_constraints_generic (protocol.rs:851-937), two_pow_i = r[0]
    Fe<F> am;
    {
        const Fe<F> xp = W(0), yp = W(1), av = W(2), xg = W(3), yg = W(4), bv = W(5), xq = W(6), yq = W(7);
        const Fe<F> xr = W(8), yr = W(9), bq = W(10), lq = W(11), ar = W(12), gr = W(13), dr = W(14), lr = W(15);
        const Fe<F> xpxp = fe_mul(xp, xp), xp2 = fe_add(xp, xp), llq = fe_mul(lq, lq);
        const Fe<F> xpxp3 = fe_add(fe_add(xpxp, xpxp), xpxp), yp2 = fe_add(yp, yp);
        const Fe<F> l_xpb = fe_sub(one, fe_mul(xp, bq));
        am = fe_mul(l_xpb, xq);
        am = fe_add(am, fe_mul(l_xpb, yq));
        am = fe_add(am, fe_sub(fe_mul(yp2, lq), xpxp3));
        am = fe_add(am, fe_sub(fe_sub(llq, xp2), xq));
        am = fe_add(am, fe_sub(fe_sub(fe_mul(lq, fe_sub(xp, xq)), yp), yq));
        const Fe<F> xg_xq = fe_sub(xg, xq), yg_yq = fe_sub(yg, yq);
        am = fe_add(am, fe_mul(xg_xq, fe_sub(fe_mul(xg_xq, lr), yg_yq)));
        const Fe<F> yq2 = fe_add(yq, yq), xqxq = fe_mul(xq, xq);
        const Fe<F> xqxq3 = fe_add(fe_add(xqxq, xqxq), xqxq);
        am = fe_add(am, fe_mul(fe_sub(one, fe_mul(xg_xq, ar)), fe_sub(fe_mul(yq2, lr), xqxq3)));
        const Fe<F> xqxg = fe_mul(xq, xg), xqxg_d = fe_mul(xqxg, fe_sub(xg, xq));
        const Fe<F> ll_x = fe_sub(fe_sub(fe_sub(fe_mul(lr, lr), xq), xg), xr);
        am = fe_add(am, fe_mul(xqxg_d, ll_x));
        const Fe<F> l_y = fe_sub(fe_sub(fe_mul(lr, fe_sub(xq, xr)), yq), yr);
        am = fe_add(am, fe_mul(xqxg_d, l_y));
        const Fe<F> xqxg_s = fe_mul(xqxg, fe_add(yg, yq));
        am = fe_add(am, fe_mul(xqxg_s, ll_x));
        am = fe_add(am, fe_mul(xqxg_s, l_y));
        am = fe_add(am, fe_mul(l_xpb, fe_sub(xr, xg)));
        am = fe_add(am, fe_mul(l_xpb, fe_sub(yr, yg)));
        const Fe<F> l_xgg = fe_sub(one, fe_mul(xg, gr));
        am = fe_add(am, fe_mul(l_xgg, fe_sub(xr, xq)));
        am = fe_add(am, fe_mul(l_xgg, fe_sub(yr, yq)));
        const Fe<F> l_ad = fe_sub(fe_sub(one, fe_mul(fe_sub(xg, xq), ar)), fe_mul(fe_add(yg, yq), dr));
        am = fe_add(am, fe_mul(l_ad, xr));
        am = fe_add(am, fe_mul(l_ad, yr));
        am = fe_add(am, fe_mul(bv, fe_sub(bv, one)));
        const Fe<F> one_b = fe_sub(one, bv);
        am = fe_add(am, fe_sub(NW(0), fe_add(fe_mul(bv, xr), fe_mul(one_b, xq))));
        am = fe_add(am, fe_sub(NW(1), fe_add(fe_mul(bv, yr), fe_mul(one_b, yq))));
        am = fe_sub(fe_add(am, NW(2)), fe_add(av, fe_mul(bv, R(0))));
    }

    acc = fe_add(acc, fe_mul(Q(7), am));
    asm volatile("" ::: "memory");
    // eq_generic (protocol.rs:1001-1011)
    Fe<F> eq;
    {
        const Fe<F> ab = fe_sub(W(0), W(1)), e = W(3);
        eq = fe_add(fe_mul(ab, e), fe_sub(fe_add(fe_mul(ab, W(4)), e), W(2)));
    }

    acc = fe_add(acc, fe_mul(Q(8), eq));
    fe_store(t + 2 * i, acc);
}

// range check and f_gc (protocol.rs:179-190) with the two partial vectors
template <class F>
__global__ __launch_bounds__(256) void k_gate_final(const GateArgs a, size_t N, uint32_t shift, const uint4* t0,
                                                    const uint4* t1, uint4* out) {
    GATE_PROLOGUE
    // range_check_generic (protocol.rs:966-990)
    Fe<F> rc = fe_sub(NW(0), W(0));
    for (int k = 0; k < 15; k++) rc = fe_sub(rc, fe_mul(W(1 + k), R(k)));

    // f_gc (protocol.rs:179-190)
    const Fe<F> w0 = W(0), w1 = W(1);
    Fe<F> f = fe_mul(w0, Q(0));
    f = fe_add(f, fe_mul(Q(1), w1));
    f = fe_add(f, fe_mul(Q(2), W(2)));
    f = fe_add(f, fe_mul(fe_mul(Q(3), w0), w1));
    f = fe_add(f, Q(4));
    f = fe_add(f, fe_mul(Q(5), fe_load<F>(t0 + 2 * i)));
    f = fe_add(f, fe_load<F>(t1 + 2 * i));
    f = fe_add(f, fe_mul(Q(9), rc));
    f = fe_add(f, fe_from_ark<F>(a.pi + 2 * i));
    fe_to_ark(out + 2 * i, f);
}

template <class F>
static Fe<F> host_fe_raw(const uint32_t (&k)[NLIMB]) {
    Fe<F> r;
    for (int i = 0; i < NLIMB; i++) r.v[i] = k[i];
    return r;
}

// host: packs an ark scalar (4 x u64) into the 9 x 29-bit limb form (ark words used as-is)
template <class F>
static Fe<F> host_fe_from_words(const halo_fe_t& w) {
    Fe<F> r;
    for (int i = 0; i < NLIMB; i++) {
        const int bit = 29 * i;
        const int q = bit / 64, s = bit % 64;
        uint64_t v = w.l[q] >> s;
        if (s > 35 && q + 1 < 4) v |= w.l[q + 1] << (64 - s);
        r.v[i] = (uint32_t)v & ((i == NLIMB - 1) ? 0xffffffffu : LIMB_MASK);
    }
    return r;
}

static int evals_launch(int field, int op, const void* a, const void* b, const halo_fe_t* scalar, uint32_t e,
                        void* out, size_t n, hipStream_t s) {
    if (!n) return HALO_OK;
    const unsigned thr = 256, blocks = (unsigned)((n + thr - 1) / thr);
    DISPATCH_FIELD(field, F, {
        halo_fe_t zero = {{0, 0, 0, 0}};
        const Fe<F> sv = host_fe_from_words<F>(scalar ? *scalar : zero);
        const Fe<F> fix = host_fe_raw<F>(F::ARK_MUL_FIX);
        hipLaunchKernelGGL(k_evals_op<F>, dim3(blocks), dim3(thr), 0, s, op, (const uint4*)a, (const uint4*)b, sv, e,
                           fix, (uint4*)out, n);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

static int check_evals_args(halo_field_t field, int op, const void* a, const void* b, const halo_fe_t* scalar,
                            const void* out, size_t n) {
    if (field != HALO_FP && field != HALO_FQ) return set_error(HALO_EINVAL, "unknown field id %d", (int)field);
    if (op < EV_ADD || op > EV_POW) return set_error(HALO_EINVAL, "unknown evals op %d", op);
    if (n && (!a || !out)) return set_error(HALO_EINVAL, "halo_evals_op: null buffer");
    if (n && op <= EV_MUL && !b) return set_error(HALO_EINVAL, "halo_evals_op: op %d needs a second operand", op);
    if (op >= EV_SCALE && op <= EV_SUB_SCALAR && !scalar) return set_error(HALO_EINVAL, "halo_evals_op: null scalar");
    return HALO_OK;
}

// sum_i zeta^i p_i over k <= LINCOMB_MAX coefficient vectors of lengths len_i (missing coefficients
// are zero): per element a Horner pass over the k inputs in the raw ark domain -- fe_mul by an
// internal-form constant is value-preserving on ark words -- so each input is read once and the
// result written once (protocol.rs:542-548's geometric combinations: one launch instead of 2k
// elementwise scale / add launches and k temporaries).
constexpr int LINCOMB_MAX = 64;
struct LincombArgs {
    const uint4* p[LINCOMB_MAX];
    uint32_t len[LINCOMB_MAX];
};
template <class F>
__global__ __launch_bounds__(256) void k_lincomb(const LincombArgs a, uint32_t k, uint4 z0, uint4 z1, size_t n_out,
                                                 uint4* out) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_out) return;
    const uint4 zw[2] = {z0, z1};
    const Fe<F> z = fe_from_ark<F>(zw);
    Fe<F> acc = fe_zero<F>();
    for (int j = (int)k - 1; j >= 0; j--) {
        acc = fe_mul(acc, z);
        if (e < a.len[j]) acc = fe_add(acc, fe_load<F>(a.p[j] + 2 * e));  // raw ark words (< p)
    }
    fe_store(out + 2 * e, fe_canon(acc));
}

}  // namespace halo

using namespace halo;

extern "C" int halo_poly_lincomb_dev(halo_field_t field, const void* const* d_polys, const size_t* lens, size_t k,
                                     const halo_fe_t* zeta, void* d_out, size_t n_out, void* stream) {
    clear_error();
    if (field != HALO_FP && field != HALO_FQ) return set_error(HALO_EINVAL, "unknown field id %d", (int)field);
    if (k > LINCOMB_MAX) return set_error(HALO_EINVAL, "halo_poly_lincomb_dev: k = %zu > %d", k, LINCOMB_MAX);
    if (!zeta || (n_out && !d_out) || (k && (!d_polys || !lens)))
        return set_error(HALO_EINVAL, "halo_poly_lincomb_dev: null argument");
    if (!n_out) return HALO_OK;
    LincombArgs a;
    for (size_t j = 0; j < k; j++) {
        if (lens[j] > 0xffffffffu || (lens[j] && !d_polys[j]))
            return set_error(HALO_EINVAL, "halo_poly_lincomb_dev: bad polynomial %zu", j);
        a.p[j] = (const uint4*)d_polys[j];
        a.len[j] = (uint32_t)lens[j];
    }
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    const uint4 z0 = make_uint4((uint32_t)zeta->l[0], (uint32_t)(zeta->l[0] >> 32), (uint32_t)zeta->l[1],
                                (uint32_t)(zeta->l[1] >> 32));
    const uint4 z1 = make_uint4((uint32_t)zeta->l[2], (uint32_t)(zeta->l[2] >> 32), (uint32_t)zeta->l[3],
                                (uint32_t)(zeta->l[3] >> 32));
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_lincomb<F>, dim3((unsigned)((n_out + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a,
                           (uint32_t)k, z0, z1, n_out, (uint4*)d_out);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_evals_op_dev(halo_field_t field, int op, const void* d_a, const void* d_b, const halo_fe_t* scalar,
                                 uint32_t exponent, void* d_out, size_t n, void* stream) {
    clear_error();
    HALO_CHECK(check_evals_args(field, op, d_a, d_b, scalar, d_out, n));
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    return evals_launch(field, op, d_a, d_b, scalar, exponent, d_out, n, (hipStream_t)stream);
}

extern "C" int halo_evals_op(halo_field_t field, int op, const halo_fe_t* a, const halo_fe_t* b, const halo_fe_t* scalar,
                             uint32_t exponent, halo_fe_t* out, size_t n) {
    clear_error();
    HALO_CHECK(check_evals_args(field, op, a, b, scalar, out, n));
    if (!n) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(n * 32));
    HALO_CHECK(st->scratch[1].reserve(n * 32));
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, a, n * 32, s));
    if (op <= EV_MUL) HALO_CHECK(copy_h2d(st->scratch[1].ptr, b, n * 32, s));
    HALO_CHECK(evals_launch(field, op, st->scratch[0].ptr, st->scratch[1].ptr, scalar, exponent, st->scratch[0].ptr, n, s));
    return copy_d2h(out, st->scratch[0].ptr, n * 32, s);
}

static size_t trimmed(const halo_fe_t* c, size_t len) {
    while (len > 0 && !(c[len - 1].l[0] | c[len - 1].l[1] | c[len - 1].l[2] | c[len - 1].l[3])) len--;
    return len;
}

extern "C" int halo_divide_by_vanishing(halo_field_t field, const halo_fe_t* coeffs, size_t len, size_t n,
                                        halo_fe_t* quotient, size_t* q_len, halo_fe_t* remainder, size_t* r_len) {
    clear_error();
    if (field != HALO_FP && field != HALO_FQ) return set_error(HALO_EINVAL, "unknown field id %d", (int)field);
    if (!n || (len && !coeffs) || !quotient || !remainder || !q_len || !r_len)
        return set_error(HALO_EINVAL, "halo_divide_by_vanishing: null argument");
    len = trimmed(coeffs, len);
    if (len < n) {  // quotient zero, remainder = self
        for (size_t j = 0; j < len; j++) remainder[j] = coeffs[j];
        *q_len = 0;
        *r_len = len;
        return HALO_OK;
    }
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    const size_t qn = len - n;
    HALO_CHECK(st->scratch[0].reserve(len * 32));
    HALO_CHECK(st->scratch[1].reserve(std::max<size_t>(qn, 1) * 32));
    HALO_CHECK(st->scratch[2].reserve(n * 32));
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, coeffs, len * 32, s));
    const size_t threads = std::max(qn, n);
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_div_vanishing<F>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                           st->scratch[0].as<const uint4>(), len, n, st->scratch[1].as<uint4>(),
                           st->scratch[2].as<uint4>());
    });
    HALO_HIP(hipGetLastError());
    if (qn) HALO_CHECK(copy_d2h(quotient, st->scratch[1].ptr, qn * 32, s));
    HALO_CHECK(copy_d2h(remainder, st->scratch[2].ptr, n * 32, s));
    *q_len = trimmed(quotient, qn);
    *r_len = trimmed(remainder, n);
    return HALO_OK;
}

extern "C" int halo_evals_scan_dev(halo_field_t field, int reverse, const void* d_in, void* d_out, size_t n,
                                   void* stream) {
    clear_error();
    if (field != HALO_FP && field != HALO_FQ) return set_error(HALO_EINVAL, "unknown field id %d", (int)field);
    if (n && (!d_in || !d_out)) return set_error(HALO_EINVAL, "halo_evals_scan_dev: null buffer");
    if (!n) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    const size_t nb = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
    if (nb > (size_t)SCAN_THREADS * 4096) return set_error(HALO_EINVAL, "halo_evals_scan_dev: n too large");
    hipStream_t s = (hipStream_t)stream;
    ScratchUse su(st, s);
    DevBuf* tot;
    {
        std::lock_guard<std::mutex> g(st->mu);
        tot = &st->scan_tmp;
        HALO_CHECK(tot->reserve(nb * 32));
    }
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_scan_block<F>, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, s, (const uint4*)d_in,
                           (uint4*)d_out, n, reverse, tot->as<uint4>());
        if (nb > 1) {
            hipLaunchKernelGGL(k_scan_totals<F>, dim3(1), dim3(SCAN_THREADS), 0, s, tot->as<uint4>(), (uint32_t)nb);
            hipLaunchKernelGGL(k_scan_apply<F>, dim3((unsigned)((n - SCAN_BLOCK + 255) / 256)), dim3(256), 0, s,
                               (uint4*)d_out, n, reverse, tot->as<const uint4>());
        }
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_divide_by_vanishing_dev(halo_field_t field, const void* d_coeffs, size_t len, size_t n,
                                            void* d_quotient, void* d_remainder, void* stream) {
    clear_error();
    if (field != HALO_FP && field != HALO_FQ) return set_error(HALO_EINVAL, "unknown field id %d", (int)field);
    if (!n || len < n || !d_coeffs || !d_remainder || (len > n && !d_quotient))
        return set_error(HALO_EINVAL, "halo_divide_by_vanishing_dev: bad argument (len %zu, n %zu)", len, n);
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    const size_t threads = std::max(len - n, n);
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_div_vanishing<F>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, (const uint4*)d_coeffs, len, n, (uint4*)d_quotient,
                           (uint4*)d_remainder);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

extern "C" int halo_gate_constraints_dev(halo_field_t field, const void* const* d_w, const void* const* d_r,
                                         const void* const* d_q, const void* d_pi, const halo_fe_t* mds, size_t n,
                                         unsigned shift, void* d_out, void* stream) {
    clear_error();
    if (field != HALO_FP && field != HALO_FQ) return set_error(HALO_EINVAL, "unknown field id %d", (int)field);
    if (!d_w || !d_r || !d_q || !d_pi || !mds || !d_out || !is_pow2(n))
        return set_error(HALO_EINVAL, "halo_gate_constraints_dev: bad argument");
    GateArgs a;
    for (int k = 0; k < 16; k++) a.w[k] = (const uint4*)d_w[k];
    for (int k = 0; k < 15; k++) a.r[k] = (const uint4*)d_r[k];
    for (int k = 0; k < 10; k++) a.q[k] = (const uint4*)d_q[k];
    a.pi = (const uint4*)d_pi;
    for (int k = 0; k < 9; k++) {
        a.mds[k][0] = make_uint4((uint32_t)mds[k].l[0], (uint32_t)(mds[k].l[0] >> 32), (uint32_t)mds[k].l[1],
                                 (uint32_t)(mds[k].l[1] >> 32));
        a.mds[k][1] = make_uint4((uint32_t)mds[k].l[2], (uint32_t)(mds[k].l[2] >> 32), (uint32_t)mds[k].l[3],
                                 (uint32_t)(mds[k].l[3] >> 32));
    }
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    DevBuf* tmp;
    {
        std::lock_guard<std::mutex> g(st->mu);
        tmp = &st->gate_tmp;
        HALO_CHECK(tmp->reserve(2 * n * 32));
    }
    uint4* t0 = tmp->as<uint4>();
    uint4* t1 = t0 + 2 * n;
    const dim3 grid((unsigned)((n + 255) / 256));
    hipStream_t s = (hipStream_t)stream;
    ScratchUse su(st, s);
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_gate_poseidon<F>, grid, dim3(256), 0, s, a, n, (uint32_t)shift, t0);
        hipLaunchKernelGGL(k_gate_affine<F>, grid, dim3(256), 0, s, a, n, (uint32_t)shift, t1);
        hipLaunchKernelGGL(k_gate_final<F>, grid, dim3(256), 0, s, a, n, (uint32_t)shift, (const uint4*)t0,
                           (const uint4*)t1, (uint4*)d_out);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}
