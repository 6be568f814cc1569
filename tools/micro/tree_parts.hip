// Cycle counts (s_memtime, one wave) of the pieces of a tree level (tree.hpp): the per-lane xyzz_add,
// the quad-cooperative addition, a 36-dword lane gather, one fe_mul, 9 DPP quad broadcasts.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../halo_amd/csrc -o tree_parts tree_parts.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "tree.hpp"
using namespace halo;

// (the round-4 Jacobian quad doubling, measured here against xyzz_dbl_quad; the library no longer uses it)
// 2p in Jacobian coordinates by the quad (dbl-2009-l as jac_dbl; every lane of an aligned quad holds p
// and gets 2p): A = X^2, B = Y^2, Y Z | C = B^2, (X + B)^2, F = E^2 | E (D - X3), one product per lane
// per round, the first two rounds exchanged by DPP quad broadcasts (the last product every lane forms
// itself).
template <class F>
__device__ __forceinline__ Jac<F> jac_dbl_quad(const Jac<F>& p) {
    const uint32_t role = threadIdx.x & 3u;
    const uint32_t r1 = role == 1 ? ~0u : 0u, r2 = role == 2 ? ~0u : 0u;
    // lane 0 (and 3): A = X^2; 1: B = Y^2; 2: Y Z
    const Fe<F> t1 = fe_mul(pick(r1 | r2, p.Y, p.X), pick(r2, p.Z, pick(r1, p.Y, p.X)));
    const Fe<F> A = qperm<qp(0, 0, 0, 0)>(t1), B = qperm<qp(1, 1, 1, 1)>(t1), YZ = qperm<qp(2, 2, 2, 2)>(t1);
    const Fe<F> E = fe_add(A, fe_dbl(A));
    // lane 0 (and 3): C = B^2; 1: (X + B)^2; 2: F = E^2
    const Fe<F> t2 = fe_sqr(pick(r1, fe_add(p.X, B), pick(r2, E, B)));
    const Fe<F> C = qperm<qp(0, 0, 0, 0)>(t2), XB2 = qperm<qp(1, 1, 1, 1)>(t2), Fv = qperm<qp(2, 2, 2, 2)>(t2);
    const Fe<F> D = fe_dbl(fe_sub(fe_sub(XB2, A), C));
    Jac<F> r;
    r.X = fe_sub(Fv, fe_dbl(D));
    const Fe<F> C8 = fe_dbl(fe_dbl(fe_dbl(C)));
    r.Y = fe_sub(fe_mul(E, fe_sub(D, r.X)), C8);
    r.Z = fe_dbl(YZ);
    return r;
}

using F = FqCfg;

constexpr int REP = 64;

template <class Cv>
__global__ void k_points(uint4* out, uint32_t n) {
    using Fb = typename Cv::Base;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Affine<Fb> g;
    g.x = fe_neg(fe_one<Fb>());
    g.y = fe_add(fe_one<Fb>(), fe_one<Fb>());
    XYZZ<Fb> acc = xyzz_id<Fb>();
    uint32_t k = (i * 2654435761u + 17) | 1u;
    for (int b = 31; b >= 0; b--) {
        acc = xyzz_dbl(acc);
        if ((k >> b) & 1u) acc = xyzz_madd(acc, g);
    }
    xyzz_store(out + 8 * i, acc);
}

__global__ __launch_bounds__(64) void k_parts(const uint4* pts, unsigned long long* cyc, uint4* sink) {
    XYZZ<F> v = xyzz_load<F>(pts + 8 * threadIdx.x);
    const uint32_t lane = threadIdx.x;
    unsigned long long t0, t1;
    // 1. per-lane xyzz_add with the xor-1 partner (one old tree level)
    t0 = clock64();
    for (int r = 0; r < REP; r++) v = xyzz_add(v, xyzz_shfl_xor(v, 1));
    t1 = clock64();
    if (lane == 0) cyc[0] = t1 - t0;
    // 2. quad-cooperative addition of lanes (4 q, 4 q + 1) -> every lane
    t0 = clock64();
    for (int r = 0; r < REP; r++) {
        const uint32_t s1 = (lane >> 2) & 63u, s2 = (s1 + 16) & 63u;
        const XYZZ<F> s = xyzz_add_quad(v, s1, s2, false, false);
        v = s;
    }
    t1 = clock64();
    if (lane == 0) cyc[1] = t1 - t0;
    // 3. a 36-dword gather
    t0 = clock64();
    for (int r = 0; r < REP; r++) v = xyzz_shfl(v, (int)((lane + 5) & 63u));
    t1 = clock64();
    if (lane == 0) cyc[2] = t1 - t0;
    // 4. one fe_mul (dependent chain)
    Fe<F> a = v.X;
    t0 = clock64();
    for (int r = 0; r < REP; r++) a = fe_mul(a, v.Y);
    t1 = clock64();
    if (lane == 0) cyc[3] = t1 - t0;
    // 5. four independent fe_muls per step
    Fe<F> b = v.ZZ, c = v.ZZZ, d = v.Y;
    t0 = clock64();
    for (int r = 0; r < REP; r++) {
        a = fe_mul(a, v.Y);
        b = fe_mul(b, v.X);
        c = fe_mul(c, v.X);
        d = fe_mul(d, v.ZZ);
    }
    t1 = clock64();
    if (lane == 0) cyc[4] = t1 - t0;
    // 6. 9 DPP quad broadcasts
    t0 = clock64();
    for (int r = 0; r < REP; r++) a = qperm<qp(1, 1, 1, 1)>(fe_add(a, b));
    t1 = clock64();
    if (lane == 0) cyc[5] = t1 - t0;
    // 7. jac_dbl_quad chain (k_tail_table's doubling step)
    Jac<F> j = jac_from_xyzz(v);
    t0 = clock64();
    for (int r = 0; r < REP; r++) j = jac_dbl_quad(j);
    t1 = clock64();
    if (lane == 0) cyc[6] = t1 - t0;
    // 8. xyzz_dbl_quad chain
    XYZZ<F> u = v;
    t0 = clock64();
    for (int r = 0; r < REP; r++) u = xyzz_dbl_quad(u);
    t1 = clock64();
    if (lane == 0) cyc[7] = t1 - t0;
    v.X = fe_add(fe_add(a, b), fe_add(c, d));
    v.Y = fe_add(j.X, u.X);
    xyzz_store(sink + 8 * lane, v);
}

int main() {
    uint4 *pts, *sink;
    unsigned long long* cyc;
    hipMalloc(&pts, 64 * 128);
    hipMalloc(&sink, 64 * 128);
    hipMalloc(&cyc, 64);
    hipLaunchKernelGGL(k_points<PallasCurve>, dim3(1), dim3(64), 0, 0, pts, 64);
    for (int i = 0; i < 2; i++) hipLaunchKernelGGL(k_parts, dim3(1), dim3(64), 0, 0, pts, cyc, sink);
    hipDeviceSynchronize();
    unsigned long long h[8];
    hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
    const char* nm[] = {"xyzz_add + shfl_xor (old level)", "xyzz_add_quad", "36-dword gather", "fe_mul (dependent)",
                        "4 independent fe_mul", "fe_add + 9 DPP bcast", "jac_dbl_quad (dependent)",
                        "xyzz_dbl_quad (dependent)"};
    for (int i = 0; i < 8; i++) printf("%-34s %8.0f cycles\n", nm[i], (double)h[i] / REP);
    return 0;
}
