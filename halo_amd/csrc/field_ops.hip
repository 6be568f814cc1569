// Elementwise field / curve kernels behind halo_field_op / halo_curve_op (parity surface for the
// field library).
#include "curve.hpp"
#include "dispatch.hpp"
#include "glv.hpp"
#include "runtime.hpp"
#include "msm.hpp"
#include "tree.hpp"

namespace halo {

template <class F>
__global__ __launch_bounds__(256) void k_field_op(int op, const uint4* a, const uint4* b, uint4* out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fe<F> x = fe_from_ark<F>(a + 2 * i);
    Fe<F> r;
    if (op == 0) {
        r = fe_mul(x, fe_from_ark<F>(b + 2 * i));
    } else if (op == 1) {
        r = fe_add(x, fe_from_ark<F>(b + 2 * i));
    } else if (op == 2) {
        r = fe_sub(x, fe_from_ark<F>(b + 2 * i));
    } else if (op == 3) {
        r = fe_sqr(x);
    } else if (op == 4) {
        r = fe_inv(x);
    } else {
        r = fe_neg(x);
    }
    fe_to_ark(out + 2 * i, r);
}

// k P for one lane: GLV split k = k1 + lambda k2 (|k1|, |k2| < 2^128, glv.hpp) and a joint 4-bit
// fixed window over k1 (table d P, d < 16, in LDS) and k2 (the same entries through
// phi(X, Y, ZZ, ZZZ) = (beta X, Y, ZZ, ZZZ)): ~132 doublings + ~66 additions on the lane's dependent
// chain instead of 256 + ~128 (a lone scalar multiplication is latency-bound: H' = xi_0 H, the
// accumulator's combination).
constexpr int CURVE_OP_SMUL_THREADS = 8;
template <class Cv>
HALO_DEV XYZZ<typename Cv::Base> scalar_mul_glv(const Affine<typename Cv::Base>& P, const uint32_t (&k)[8],
                                               uint4* tab /* 16 XYZZ of this lane */) {
    using F = typename Cv::Base;
    bool n1, n2;
    uint32_t k1[5], k2[5];
    glv::decompose<typename Cv::K>(k, n1, k1, n2, k2);
    const XYZZ<F> p1 = xyzz_from_aff(P);
    xyzz_store(tab, xyzz_id<F>());
    xyzz_store(tab + 8, p1);
    for (int d = 2; d < 16; d++)
        xyzz_store(tab + 8 * d, (d & 1) ? xyzz_madd(xyzz_load<F>(tab + 8 * (d - 1)), P) : xyzz_dbl(xyzz_load<F>(tab + 8 * (d / 2))));
    const Fe<F> beta = fe_from_const<F>(Cv::K::BETA);
    XYZZ<F> acc = xyzz_id<F>();
    for (int w = 32; w >= 0; w--) {  // 33 windows cover 132 bits
        if (w != 32)
            for (int b = 0; b < 4; b++) acc = xyzz_dbl(acc);
        const int q = (4 * w) >> 5, sh = (4 * w) & 31;
        const uint32_t d1 = (k1[q] >> sh) & 15u, d2 = (k2[q] >> sh) & 15u;
        if (d1) {
            XYZZ<F> t = xyzz_load<F>(tab + 8 * d1);
            if (n1) t.Y = fe_neg(t.Y);
            acc = xyzz_add(acc, t);
        }
        if (d2) {
            XYZZ<F> t = xyzz_load<F>(tab + 8 * d2);
            t.X = fe_mul(t.X, beta);
            if (n2) t.Y = fe_neg(t.Y);
            acc = xyzz_add(acc, t);
        }
    }
    return acc;
}

// The same scalar multiplication by an aligned quad of lanes (every lane holds P, k and the running
// sum): the doublings are xyzz_dbl_quad (three product rounds instead of nine) and the additions
// xyzz_add_quad (four instead of fourteen).  tab: 32 XYZZ of this quad in LDS, d P for d < 16 and
// phi(d P) at 16 + d.  Quads of one wave that take different digits stay in lockstep: an addition
// is skipped only when it is trivial for every quad.
template <class Cv>
HALO_DEV XYZZ<typename Cv::Base> scalar_mul_glv_quad(const Affine<typename Cv::Base>& P, const uint32_t (&k)[8],
                                                    uint4* tab) {
    using F = typename Cv::Base;
    const uint32_t lane = threadIdx.x & 63u, role = lane & 3u, s1 = lane & ~3u;
    bool n1, n2;
    uint32_t k1[5], k2[5];
    glv::decompose<typename Cv::K>(k, n1, k1, n2, k2);
    const XYZZ<F> p1 = xyzz_from_aff(P);
    // acc + t (t the same in every lane of the quad; trivial when either is the identity)
    auto add = [&](const XYZZ<F>& acc, const XYZZ<F>& t, bool tid) -> XYZZ<F> {
        const bool idp = xyzz_is_id(acc), idq = tid || xyzz_is_id(t);
        XYZZ<F> r = xyzz_id<F>();
        if (!__all(idp || idq)) r = xyzz_add_quad(role == 1 ? t : acc, s1, s1 + 1, idp, idq);
        const XYZZ<F> sum = xyzz_shfl(r, (int)(s1 + 2));
        return idq ? acc : (idp ? t : sum);
    };
    if (role == 0) {
        xyzz_store(tab, xyzz_id<F>());
        xyzz_store(tab + 8, p1);
    }
    XYZZ<F> prev = p1;  // d P for the previous d
    for (int d = 2; d < 16; d++) {
        const XYZZ<F> v = (d & 1) ? add(prev, p1, false) : xyzz_dbl_quad(xyzz_load<F>(tab + 8 * (d / 2)));
        if (role == 0) xyzz_store(tab + 8 * d, v);
        __syncthreads();  // (one wave per block: the quad's other lanes read entry d / 2 next)
        prev = v;
    }
    // phi(d P) = (beta X, Y, ZZ, ZZZ): lane r of the quad forms d = r, r + 4, r + 8, r + 12
    const Fe<F> beta = fe_from_const<F>(Cv::K::BETA);
    for (int j = 0; j < 4; j++) {
        const int d = (int)role + 4 * j;
        XYZZ<F> t = xyzz_load<F>(tab + 8 * d);
        t.X = fe_mul(t.X, beta);
        xyzz_store(tab + 8 * (16 + d), t);
    }
    __syncthreads();
    XYZZ<F> acc = xyzz_id<F>();
    for (int w = 32; w >= 0; w--) {  // 33 windows cover 132 bits
        if (w != 32)
            for (int b = 0; b < 4; b++) acc = xyzz_dbl_quad(acc);
        const int q = (4 * w) >> 5, sh = (4 * w) & 31;
        const uint32_t d1 = (k1[q] >> sh) & 15u, d2 = (k2[q] >> sh) & 15u;
        XYZZ<F> t = xyzz_load<F>(tab + 8 * d1);
        if (n1) t.Y = fe_neg(t.Y);
        acc = add(acc, t, d1 == 0);
        t = xyzz_load<F>(tab + 8 * (16 + d2));
        if (n2) t.Y = fe_neg(t.Y);
        acc = add(acc, t, d2 == 0);
    }
    return acc;
}

template <class Cv>
__global__ __launch_bounds__(64) void k_curve_op(int op, const uint4* a, const uint4* b, const uint4* k, uint4* out, size_t n) {
    using F = typename Cv::Base;
    using S = typename Cv::Scalar;
    extern __shared__ uint4 smul_tab[];  // op 2: 32 XYZZ (128 B) per quad
    if (op == 2) {  // one quad per scalar multiplication; quads past n repeat the last one (no store), so
                    // every lane reaches the table build's barriers
        const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
        const size_t ic = i < n ? i : n - 1;
        uint32_t w[8];
        fe_ark_to_canonical_words<S>(k + 2 * ic, w);
        const XYZZ<F> r = scalar_mul_glv_quad<Cv>(aff_from_wrapped<F>(a + 4 * ic), w, smul_tab + 32 * 8 * (threadIdx.x >> 2));
        if (i < n && (threadIdx.x & 3u) == 0) aff_to_wrapped(out + 4 * i, xyzz_to_aff(r));
        return;
    }
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Affine<F> p = aff_from_wrapped<F>(a + 4 * i);
    XYZZ<F> r;
    if (op == 0) {
        r = xyzz_madd(xyzz_from_aff(p), aff_from_wrapped<F>(b + 4 * i));
    } else if (op == 1) {
        r = xyzz_dbl(xyzz_from_aff(p));
    } else {
        uint32_t w[8];
        fe_ark_to_canonical_words<S>(k + 2 * i, w);
        r = scalar_mul_glv<Cv>(p, w, smul_tab + 16 * 8 * threadIdx.x);
    }
    aff_to_wrapped(out + 4 * i, xyzz_to_aff(r));
}

}  // namespace halo

using namespace halo;

extern "C" int halo_field_op(halo_field_t field, int op, const halo_fe_t* a, const halo_fe_t* b, size_t n,
                             halo_fe_t* out) {
    clear_error();
    if (!a || !out || (op <= 2 && !b) || op < 0 || op > 5 || (field != HALO_FP && field != HALO_FQ))
        return set_error(HALO_EINVAL, "halo_field_op: invalid argument");
    if (n == 0) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    const size_t bytes = n * sizeof(halo_fe_t);
    HALO_CHECK(st->scratch[0].reserve(bytes));
    HALO_CHECK(st->scratch[1].reserve(bytes));
    HALO_CHECK(st->scratch[2].reserve(bytes));
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, a, bytes, s));
    if (b) HALO_CHECK(copy_h2d(st->scratch[1].ptr, b, bytes, s));
    const unsigned threads = 256, blocks = (unsigned)((n + threads - 1) / threads);
    DISPATCH_FIELD(field, F, {
        hipLaunchKernelGGL(k_field_op<F>, dim3(blocks), dim3(threads), 0, s, op, st->scratch[0].as<const uint4>(),
                           st->scratch[1].as<const uint4>(), st->scratch[2].as<uint4>(), n);
    });
    HALO_HIP(hipGetLastError());
    return copy_d2h(out, st->scratch[2].ptr, bytes, s);
}

extern "C" int halo_curve_op(halo_curve_t curve, int op, const halo_wrapped_point_t* a, const halo_wrapped_point_t* b,
                             const halo_fe_t* k, size_t n, halo_wrapped_point_t* out) {
    clear_error();
    if (!a || !out || (op == 0 && !b) || (op == 2 && !k) || op < 0 || op > 2 ||
        (curve != HALO_PALLAS && curve != HALO_VESTA))
        return set_error(HALO_EINVAL, "halo_curve_op: invalid argument");
    if (n == 0) return HALO_OK;
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    const size_t pb = n * sizeof(halo_wrapped_point_t), kb = n * sizeof(halo_fe_t);
    HALO_CHECK(st->scratch[0].reserve(pb));
    HALO_CHECK(st->scratch[1].reserve(pb));
    HALO_CHECK(st->scratch[2].reserve(kb));
    HALO_CHECK(st->scratch[3].reserve(pb));
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, a, pb, s));
    if (b) HALO_CHECK(copy_h2d(st->scratch[1].ptr, b, pb, s));
    if (k) HALO_CHECK(copy_h2d(st->scratch[2].ptr, k, kb, s));
    // op 2: a quad per scalar multiplication, 32 table entries of 128 B per quad
    const size_t lanes = op == 2 ? 4 * n : n;
    const unsigned threads = op == 2 ? 4 * CURVE_OP_SMUL_THREADS : 64, blocks = (unsigned)((lanes + threads - 1) / threads);
    const size_t smem = op == 2 ? (size_t)(threads / 4) * 32 * 128 : 0;
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_curve_op<Cv>, dim3(blocks), dim3(threads), smem, s, op, st->scratch[0].as<const uint4>(),
                           st->scratch[1].as<const uint4>(), st->scratch[2].as<const uint4>(),
                           st->scratch[3].as<uint4>(), n);
    });
    HALO_HIP(hipGetLastError());
    return copy_d2h(out, st->scratch[3].ptr, pb, s);
}

// ---------------------------------------------------------------------------------------------
// The hiding branch of pcdl::open_without_eval (crates/accumulation/src/pcdl.rs:344-371):
//   p_bar = (X - z) q, C_bar = commit(p_bar, d, w_bar)         -> halo_pcdl_hiding_blind
//   (the caller's transcript: alpha = rho(C, C_bar, z, v))
//   p' = p + alpha p_bar, w' = w + alpha w_bar, C' = C + alpha C_bar - w' S  -> halo_pcdl_hiding_combine
// q (d coefficients) and w_bar are the caller's random draws (the reference samples them from its rng).
// ---------------------------------------------------------------------------------------------
namespace halo {

template <class S>
__global__ void k_pbar(const uint4* q, size_t d, const uint4* z, uint4* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > d) return;
    const Fe<S> a = i >= 1 ? fe_from_ark<S>(q + 2 * (i - 1)) : fe_zero<S>();
    const Fe<S> b = i < d ? fe_from_ark<S>(q + 2 * i) : fe_zero<S>();
    fe_to_ark(out + 2 * i, fe_sub(a, fe_mul(fe_from_ark<S>(z), b)));
}

template <class S>
__global__ void k_axpy_pad(const uint4* p, size_t len, const uint4* pb, size_t n, const uint4* alpha, uint4* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Fe<S> x = i < len ? fe_from_ark<S>(p + 2 * i) : fe_zero<S>();
    fe_to_ark(out + 2 * i, fe_add(x, fe_mul(fe_from_ark<S>(alpha), fe_from_ark<S>(pb + 2 * i))));
}

// lane 0: alpha C_bar, lane 1: w' S (both GLV scalar multiplications run side by side); lane 0 then
// forms C + alpha C_bar - w' S.  w' = w + alpha w_bar is computed by both lanes.
template <class Cv>
__global__ __launch_bounds__(64) void k_hiding_point(const uint4* C, const uint4* C_bar, const uint4* S_int,
                                                     const uint4* alpha, const uint4* w, const uint4* w_bar,
                                                     uint4* C_out, uint4* w_out) {
    using F = typename Cv::Base;
    using Sc = typename Cv::Scalar;
    __shared__ uint4 tab[2][16 * 8];
    __shared__ uint4 res[8];
    const int lane = threadIdx.x;
    if (lane >= 2) return;
    const Fe<Sc> wp = fe_add(fe_from_ark<Sc>(w), fe_mul(fe_from_ark<Sc>(alpha), fe_from_ark<Sc>(w_bar)));
    uint32_t kw[8];
    if (lane == 0) {
        fe_ark_to_canonical_words<Sc>(alpha, kw);
    } else {
        uint4 tmp[2];
        fe_to_ark(tmp, wp);
        fe_ark_to_canonical_words<Sc>(tmp, kw);
    }
    const Affine<F> base = lane == 0 ? aff_from_wrapped<F>(C_bar) : aff_load<F>(S_int);
    XYZZ<F> r = scalar_mul_glv<Cv>(base, kw, tab[lane]);
    if (lane == 1) xyzz_store(res, xyzz_neg(r));
    __syncthreads();
    if (lane == 0) {
        XYZZ<F> acc = xyzz_madd(r, aff_from_wrapped<F>(C));
        acc = xyzz_add(acc, xyzz_load<F>(res));
        aff_to_wrapped(C_out, xyzz_to_aff(acc));
        fe_to_ark(w_out, wp);
    }
}

template <class Sc>
__global__ void k_combine_scalars(uint4* p, uint4* pb, size_t n, const uint4* alpha, const uint4* w, const uint4* w_bar,
                                  uint4* w_prime, uint4* negw) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const Fe<Sc> a = fe_from_ark<Sc>(alpha);
    if (i < n) {
        const Fe<Sc> t = fe_mul(a, fe_from_ark<Sc>(pb + 2 * i));
        fe_to_ark(p + 2 * i, fe_add(fe_from_ark<Sc>(p + 2 * i), t));
        fe_to_ark(pb + 2 * i, t);
    }
    if (i == 0) {
        const Fe<Sc> wv = fe_from_ark<Sc>(w);
        fe_to_ark(w_prime, fe_add(wv, fe_mul(a, fe_from_ark<Sc>(w_bar))));
        fe_to_ark(negw, fe_neg(wv));
    }
}

template <class Cv>
__global__ void k_xyzz_add_wrapped(uint4* xyzz, const uint4* wrapped, const uint4* first_wrapped) {
    using F = typename Cv::Base;
    if (threadIdx.x != 0) return;
    const XYZZ<F> a = first_wrapped ? xyzz_from_aff(aff_from_wrapped<F>(first_wrapped)) : xyzz_load<F>(xyzz);
    xyzz_store(xyzz, xyzz_madd(a, aff_from_wrapped<F>(wrapped)));
}

}  // namespace halo

int halo::pcdl_combine_scalars_device(int curve, void* p, void* p_bar, size_t n, const void* alpha, const void* w,
                                      const void* w_bar, void* w_prime, void* negw, hipStream_t s) {
    DISPATCH_FIELD(curve == HALO_PALLAS ? HALO_FP : HALO_FQ, Fs, {
        hipLaunchKernelGGL(k_combine_scalars<Fs>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (uint4*)p,
                           (uint4*)p_bar, n, (const uint4*)alpha, (const uint4*)w, (const uint4*)w_bar, (uint4*)w_prime,
                           (uint4*)negw);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

int halo::xyzz_add_wrapped_device(int curve, void* xyzz, const void* wrapped, hipStream_t s, bool from_wrapped,
                                  const void* first_wrapped) {
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_xyzz_add_wrapped<Cv>, dim3(1), dim3(64), 0, s, (uint4*)xyzz, (const uint4*)wrapped,
                           from_wrapped ? (const uint4*)first_wrapped : (const uint4*)nullptr);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

int halo::pcdl_pbar_device(int curve, const void* q, size_t d, const void* z, void* p_bar, hipStream_t s) {
    const size_t n = d + 1;
    DISPATCH_FIELD(curve == HALO_PALLAS ? HALO_FP : HALO_FQ, Fs, {
        hipLaunchKernelGGL(k_pbar<Fs>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const uint4*)q, d,
                           (const uint4*)z, (uint4*)p_bar);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

int halo::pcdl_combine_device(int curve, const void* p, size_t len, const void* p_bar, size_t n, const void* alpha,
                              const void* w, const void* w_bar, const void* C, const void* C_bar, const void* S_int,
                              void* p_prime, void* C_prime, void* w_prime, hipStream_t s) {
    DISPATCH_FIELD(curve == HALO_PALLAS ? HALO_FP : HALO_FQ, Fs, {
        hipLaunchKernelGGL(k_axpy_pad<Fs>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const uint4*)p, len,
                           (const uint4*)p_bar, n, (const uint4*)alpha, (uint4*)p_prime);
    });
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_hiding_point<Cv>, dim3(1), dim3(64), 0, s, (const uint4*)C, (const uint4*)C_bar,
                           (const uint4*)S_int, (const uint4*)alpha, (const uint4*)w, (const uint4*)w_bar, (uint4*)C_prime,
                           (uint4*)w_prime);
    });
    HALO_HIP(hipGetLastError());
    return HALO_OK;
}

static int hiding_checks(DeviceState* st, halo_curve_t curve, size_t d) {
    SrsState& srs = st->srs[curve];
    if (!srs.n) return set_error(HALO_ESRSRANGE, "no resident SRS: call halo_srs_upload first");
    if (!srs.has_sh) return set_error(HALO_ESRSRANGE, "hiding commitment needs S: upload the SRS (S, H) first");
    const size_t n = d + 1;
    if (n <= 1) return set_error(HALO_EINVAL, "assertion failed: n > 1");
    if (!is_pow2(n)) return set_error(HALO_ENOTPOW2, "n (%zu) is not a power of two", n);
    if (d > srs.n - 1) return set_error(HALO_ESRSRANGE, "assertion failed: d <= pp.D");
    return HALO_OK;
}

extern "C" int halo_pcdl_hiding_blind(halo_curve_t curve, const halo_fe_t* q, size_t d, const halo_fe_t* z,
                                      const halo_fe_t* w_bar, halo_fe_t* p_bar_out, halo_wrapped_point_t* C_bar_out) {
    clear_error();
    if ((curve != HALO_PALLAS && curve != HALO_VESTA) || !q || !z || !w_bar || !C_bar_out)
        return set_error(HALO_EINVAL, "halo_pcdl_hiding_blind: invalid argument");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    HALO_CHECK(hiding_checks(st, curve, d));
    hipStream_t s = 0;
    ScratchUse su(st, s);
    const size_t n = d + 1;
    HALO_CHECK(st->scratch[0].reserve(d * 32 + 64));
    HALO_CHECK(st->scratch[1].reserve(n * 32));
    HALO_CHECK(st->scratch[2].reserve(64 + 128));
    char* small = st->scratch[2].as<char>();
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, q, d * 32, s));
    HALO_CHECK(copy_h2d(small, z, 32, s));
    HALO_CHECK(copy_h2d(small + 32, w_bar, 32, s));
    HALO_CHECK(pcdl_pbar_device(curve, st->scratch[0].ptr, d, small, st->scratch[1].ptr, s));
    // C_bar as packed XYZZ, converted on the host (no inversion on the MSM's last lane)
    HALO_CHECK(msm_srs_device(st, curve, st->scratch[1].ptr, n, small + 32, small + 64, s, false, true));
    if (p_bar_out) HALO_CHECK(copy_d2h(p_bar_out, st->scratch[1].ptr, n * 32, s));
    alignas(16) uint64_t buf[16];
    HALO_CHECK(copy_d2h(buf, small + 64, 128, s));
    HALO_HIP(hipStreamSynchronize(s));
    host_xyzz_to_wrapped(curve, buf, C_bar_out);
    return HALO_OK;
}

extern "C" int halo_pcdl_hiding_combine(halo_curve_t curve, const halo_fe_t* p, size_t len, const halo_fe_t* p_bar,
                                        size_t d, const halo_fe_t* alpha, const halo_wrapped_point_t* C,
                                        const halo_wrapped_point_t* C_bar, const halo_fe_t* w, const halo_fe_t* w_bar,
                                        halo_fe_t* p_prime_out, halo_fe_t* w_prime_out,
                                        halo_wrapped_point_t* C_prime_out) {
    clear_error();
    if ((curve != HALO_PALLAS && curve != HALO_VESTA) || (len && !p) || !p_bar || !alpha || !C || !C_bar || !w ||
        !w_bar || !p_prime_out || !w_prime_out || !C_prime_out)
        return set_error(HALO_EINVAL, "halo_pcdl_hiding_combine: invalid argument");
    DeviceState* st = current_state();
    if (!st) return HALO_EDEVICE;
    std::lock_guard<std::mutex> g(st->mu);
    HALO_CHECK(hiding_checks(st, curve, d));
    const size_t n = d + 1;
    if (len > n) return set_error(HALO_EDEGREE, "p has %zu coefficients for d = %zu", len, d);
    hipStream_t s = 0;
    ScratchUse su(st, s);
    HALO_CHECK(st->scratch[0].reserve(std::max<size_t>(len, 1) * 32));
    HALO_CHECK(st->scratch[1].reserve(n * 32));
    HALO_CHECK(st->scratch[3].reserve(n * 32));
    HALO_CHECK(st->scratch[2].reserve(512));
    char* sm = st->scratch[2].as<char>();  // alpha, w, w_bar | C, C_bar, S | C', w'
    HALO_CHECK(copy_h2d(st->scratch[0].ptr, p, len * 32, s));
    HALO_CHECK(copy_h2d(st->scratch[1].ptr, p_bar, n * 32, s));
    HALO_CHECK(copy_h2d(sm, alpha, 32, s));
    HALO_CHECK(copy_h2d(sm + 32, w, 32, s));
    HALO_CHECK(copy_h2d(sm + 64, w_bar, 32, s));
    HALO_CHECK(copy_h2d(sm + 128, C, 64, s));
    HALO_CHECK(copy_h2d(sm + 192, C_bar, 64, s));
    HALO_CHECK(copy_h2d(sm + 256, st->srs[curve].S, 64, s));
    HALO_CHECK(pcdl_combine_device(curve, st->scratch[0].ptr, len, st->scratch[1].ptr, n, sm, sm + 32, sm + 64, sm + 128,
                                   sm + 192, sm + 256, st->scratch[3].ptr, sm + 320, sm + 384, s));
    HALO_CHECK(copy_d2h(p_prime_out, st->scratch[3].ptr, n * 32, s));
    HALO_CHECK(copy_d2h(w_prime_out, sm + 384, 32, s));
    return copy_d2h(C_prime_out, sm + 320, 64, s);
}
