// Elementwise field / curve kernels behind halo_field_op / halo_curve_op (parity surface for the
// field library).
#include "curve.hpp"
#include "dispatch.hpp"
#include "glv.hpp"
#include "runtime.hpp"

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

template <class Cv>
__global__ __launch_bounds__(64) void k_curve_op(int op, const uint4* a, const uint4* b, const uint4* k, uint4* out, size_t n) {
    using F = typename Cv::Base;
    using S = typename Cv::Scalar;
    extern __shared__ uint4 smul_tab[];  // op 2: 16 XYZZ (128 B) per lane
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
    const unsigned threads = op == 2 ? CURVE_OP_SMUL_THREADS : 64, blocks = (unsigned)((n + threads - 1) / threads);
    const size_t smem = op == 2 ? (size_t)threads * 16 * 128 : 0;
    DISPATCH_CURVE(curve, Cv, {
        hipLaunchKernelGGL(k_curve_op<Cv>, dim3(blocks), dim3(threads), smem, s, op, st->scratch[0].as<const uint4>(),
                           st->scratch[1].as<const uint4>(), st->scratch[2].as<const uint4>(),
                           st->scratch[3].as<uint4>(), n);
    });
    HALO_HIP(hipGetLastError());
    return copy_d2h(out, st->scratch[3].ptr, pb, s);
}
