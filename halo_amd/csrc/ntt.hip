// Radix-2 NTT / iNTT over the Pasta scalar fields.
//
// Replaces ark-poly 0.5.0 `Radix2EvaluationDomain::{fft, ifft}` as reached from
// `Evals::from_poly(_ref)` / `Evals::interpolate(_by_ref)` (crates/group/src/poly.rs:56-64,133-139),
// `DensePolynomial::evaluate_over_domain_by_ref` (crates/plonk/src/plonk/protocol.rs:89-106,140-141)
// and FFT polynomial multiplication (`&Poly * &Poly`, protocol.rs:132-139, pcdl.rs:215).
//
// Algorithm: Stockham auto-sort, radix R = 2^r per pass (r <= 8, Σ r = log N), natural order in
// and out, out-of-place ping-pong.  One workgroup owns T = E / R consecutive columns j of a pass
// (E = elements per workgroup): it loads x[j + r N/R] (T-element contiguous runs), multiplies by the
// Stockham twiddle omega_{Ns R}^(r (j mod Ns)) (two-level table, L2 resident), performs the R-point
// DFT as r radix-2 DIT stages in LDS (bit-reversed placement on load, omega_R table in LDS), and
// writes y[(j / Ns) Ns R + (j mod Ns) + k Ns].  Field elements live in LDS in the 9 x 29-bit limb
// form (stride 9 dwords: conflict-free for consecutive lanes).  The first pass converts from the
// ark ABI format and the last pass converts back (with the N^-1 scaling for the inverse); the
// intermediate buffers hold the internal packed format.
#include <algorithm>

#include "dispatch.hpp"
#include "runtime.hpp"

namespace halo {

constexpr int NTT_E = 1024;       // elements per workgroup
constexpr int NTT_THREADS = 256;  // threads per workgroup
constexpr int NTT_MAX_LOG_R_MULTI = 8;

struct NttPassArgs {
    const uint4* in;
    uint4* out;
    const uint4* tw_hi;
    const uint4* tw_lo;
    const uint4* rtab;
    uint32_t logn, log_r, log_ns, lo_bits;
    uint32_t in_ark, out_ark, scale;
    uint32_t ninv[NLIMB];  // N^-1 (internal form) applied at the output when scale != 0
    size_t stride;         // elements between consecutive transforms of a batch
};

template <class F>
HALO_DEV Fe<F> lds_get(const uint32_t* s, int idx) {
    Fe<F> r;
#pragma unroll
    for (int l = 0; l < NLIMB; l++) r.v[l] = s[idx * NLIMB + l];
    return r;
}
template <class F>
HALO_DEV void lds_put(uint32_t* s, int idx, const Fe<F>& a) {
#pragma unroll
    for (int l = 0; l < NLIMB; l++) s[idx * NLIMB + l] = a.v[l];
}

template <class F>
__global__ __launch_bounds__(NTT_THREADS) void k_ntt_pass(NttPassArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t R = 1u << a.log_r;
    const size_t N = (size_t)1 << a.logn;
    const size_t NJ = N >> a.log_r;  // columns per transform
    const uint32_t T = (uint32_t)((NJ < (size_t)(NTT_E >> a.log_r)) ? NJ : (NTT_E >> a.log_r));
    const uint32_t E = T * R;
    const size_t Ns = (size_t)1 << a.log_ns;
    uint32_t* data = smem;
    uint32_t* rt = smem + NTT_E * NLIMB;
    const size_t j0 = (size_t)blockIdx.x * T;
    const uint4* in = a.in + (size_t)blockIdx.y * a.stride * 2;
    uint4* out = a.out + (size_t)blockIdx.y * a.stride * 2;

    // omega_R table (x < R/2) into LDS
    for (uint32_t x = threadIdx.x; x < R / 2; x += NTT_THREADS) lds_put(rt, x, fe_load<F>(a.rtab + 2 * x));

    // load + Stockham twiddle, bit-reversed placement for the DIT stages
    const size_t tw_step = N >> (a.log_ns + a.log_r);  // N / (Ns R)
    const uint32_t lo_mask = (1u << a.lo_bits) - 1;
    for (uint32_t idx = threadIdx.x; idx < E; idx += NTT_THREADS) {
        const uint32_t r = idx / T, t = idx % T;
        const size_t j = j0 + t;
        const uint4* src = in + 2 * (j + (size_t)r * NJ);
        Fe<F> v = a.in_ark ? fe_from_ark<F>(src) : fe_load<F>(src);
        if (a.log_ns != 0 && r != 0) {
            const size_t x = (size_t)r * ((j & (Ns - 1)) * tw_step);
            if (x != 0) {
                Fe<F> w = fe_load<F>(a.tw_lo + 2 * (x & lo_mask));
                const size_t xh = x >> a.lo_bits;
                if (xh != 0) w = fe_mul(w, fe_load<F>(a.tw_hi + 2 * xh));
                v = fe_mul(v, w);
            }
        }
        const uint32_t rb = a.log_r ? (__brev(r) >> (32 - a.log_r)) : 0;
        lds_put(data, t * R + rb, v);
    }
    __syncthreads();

    // radix-2 DIT stages inside each column's R-point DFT
    for (uint32_t s = 0; s < a.log_r; s++) {
        const uint32_t h = 1u << s;
        for (uint32_t b = threadIdx.x; b < E / 2; b += NTT_THREADS) {
            const uint32_t t = b >> (a.log_r - 1);
            const uint32_t q = b & ((R >> 1) - 1);
            const uint32_t k = q & (h - 1);
            const uint32_t i0 = t * R + ((q >> s) << (s + 1)) + k;
            const uint32_t i1 = i0 + h;
            const Fe<F> u = lds_get<F>(data, i0);
            Fe<F> v = lds_get<F>(data, i1);
            if (k != 0) v = fe_mul(v, lds_get<F>(rt, k << (a.log_r - 1 - s)));
            lds_put(data, i0, fe_add(u, v));
            lds_put(data, i1, fe_sub(u, v));
        }
        __syncthreads();
    }

    // store y[(j / Ns) Ns R + (j mod Ns) + k Ns]
    for (uint32_t idx = threadIdx.x; idx < E; idx += NTT_THREADS) {
        uint32_t k, t;
        if (a.log_ns == 0) {
            t = idx / R;
            k = idx % R;
        } else {
            k = idx / T;
            t = idx % T;
        }
        const size_t j = j0 + t;
        const size_t dst = ((j >> a.log_ns) << (a.log_ns + a.log_r)) + (j & (Ns - 1)) + (size_t)k * Ns;
        Fe<F> v = lds_get<F>(data, t * R + k);
        if (a.out_ark) {
            if (a.scale) {
                Fe<F> ni;
#pragma unroll
                for (int l = 0; l < NLIMB; l++) ni.v[l] = a.ninv[l];
                v = fe_mul(v, ni);
            }
            fe_to_ark(out + 2 * dst, v);
        } else {
            fe_store(out + 2 * dst, v);
        }
    }
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
    *out = t.get();
    st->tw.push_back(std::move(t));
    return HALO_OK;
}

template <class F>
static int get_rtable(DeviceState* st, int field, unsigned logr, int inverse, const uint4** out, hipStream_t s) {
    for (auto& t : st->rt)
        if (t->field == field && t->logr == (int)logr && t->inverse == inverse) {
            *out = t->t.as<const uint4>();
            return HALO_OK;
        }
    auto t = std::make_unique<DeviceState::RTable>();
    t->field = field;
    t->logr = (int)logr;
    t->inverse = inverse;
    const size_t cnt = logr ? ((size_t)1 << (logr - 1)) : 1;
    HALO_CHECK(t->t.reserve(cnt * 32));
    const Fe<F> w = host_fe<F>(inverse ? F::OMEGA_INV[logr] : F::OMEGA[logr]);
    HALO_CHECK(launch_pow_table<F>(t->t.as<uint4>(), cnt, w, 1, s));
    *out = t->t.as<const uint4>();
    st->rt.push_back(std::move(t));
    return HALO_OK;
}

static std::vector<unsigned> ntt_radices(unsigned logn) {
    std::vector<unsigned> r;
    const unsigned loge = 10;  // log2(NTT_E)
    if (logn <= loge) {
        r.push_back(logn);
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

// Device NTT over `batch` transforms: reads d_in (ark format), writes d_out (ark format).
// d_tmp must hold batch * N elements (32 B) when more than one pass is needed; d_in may equal d_out.
template <class F>
static int ntt_device(DeviceState* st, int field, const void* d_in, void* d_out, void* d_tmp, unsigned logn,
                      size_t batch, int inverse, hipStream_t s) {
    if (logn > 30) return set_error(HALO_EINVAL, "NTT domain 2^%u too large", logn);
    const size_t N = (size_t)1 << logn;
    if (logn == 0) {
        if (d_in != d_out) HALO_HIP(hipMemcpyAsync(d_out, d_in, batch * 32, hipMemcpyDeviceToDevice, s));
        return HALO_OK;
    }
    DeviceState::Twiddles* tw = nullptr;
    HALO_CHECK(get_twiddles<F>(st, field, logn, inverse, &tw, s));
    const std::vector<unsigned> rad = ntt_radices(logn);
    // ping-pong: pass p reads src, writes dst; final pass must write d_out.
    // Choose buffers so that the last pass lands in d_out and no pass reads and writes one buffer.
    const int P = (int)rad.size();
    std::vector<const void*> srcs(P);
    std::vector<void*> dsts(P);
    {
        void* bufs[2] = {d_out, d_tmp};
        // walk backwards: last dst = d_out
        int cur = 0;  // index in bufs for dst of pass p
        for (int p = P - 1; p >= 0; p--) {
            dsts[p] = bufs[cur];
            cur ^= 1;
        }
        for (int p = 0; p < P; p++) srcs[p] = (p == 0) ? d_in : dsts[p - 1];
        if (P > 1 && d_in == dsts[0]) {
            // first pass would read and write the same buffer: stage through the other buffer
            return set_error(HALO_EINVAL, "internal: NTT buffer aliasing");
        }
    }
    unsigned log_ns = 0;
    for (int p = 0; p < P; p++) {
        const unsigned lr = rad[p];
        const uint4* rtab = nullptr;
        HALO_CHECK(get_rtable<F>(st, field, lr, inverse, &rtab, s));
        NttPassArgs a;
        a.in = (const uint4*)srcs[p];
        a.out = (uint4*)dsts[p];
        a.tw_hi = tw->hi.as<const uint4>();
        a.tw_lo = tw->lo.as<const uint4>();
        a.rtab = rtab;
        a.logn = logn;
        a.log_r = lr;
        a.log_ns = log_ns;
        a.lo_bits = (uint32_t)tw->lo_bits;
        a.in_ark = (p == 0);
        a.out_ark = (p == P - 1);
        a.scale = (p == P - 1) && inverse;
        for (int l = 0; l < NLIMB; l++) a.ninv[l] = F::N_INV[logn][l];
        a.stride = N;
        const size_t NJ = N >> lr;
        const size_t T = std::min(NJ, (size_t)(NTT_E >> lr));
        const size_t rt_entries = lr ? ((size_t)1 << (lr - 1)) : 1;
        const size_t lds = (NTT_E + rt_entries) * NLIMB * 4;
        dim3 grid((unsigned)(NJ / T), (unsigned)batch);
        ProfScope prof("ntt_pass", s);
        HALO_LAUNCH(prof, k_ntt_pass<F>, grid, dim3(NTT_THREADS), lds, s, a);
        HALO_HIP(hipGetLastError());
        log_ns += lr;
    }
    return HALO_OK;
}

int ntt_device_dispatch(DeviceState* st, int field, const void* d_in, void* d_out, void* d_tmp, unsigned logn,
                        size_t batch, int inverse, hipStream_t s) {
    int rc;
    DISPATCH_FIELD(field, F, { rc = ntt_device<F>(st, field, d_in, d_out, d_tmp, logn, batch, inverse, s); });
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
    HALO_CHECK(ntt_device_dispatch(st, field, a, b, c, logn, 1, inverse, s));
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
    // in place: the passes ping-pong through a scratch buffer; with an odd pass count the first
    // pass must not write d_data, so stage the input in scratch[5] first in that case.
    const size_t P = ntt_radices(log_n).size();
    HALO_CHECK(st->scratch[4].reserve(batch * N * 32));
    if (P % 2 == 1 && P > 1) {
        HALO_CHECK(st->scratch[5].reserve(batch * N * 32));
        HALO_HIP(hipMemcpyAsync(st->scratch[5].ptr, d_data, batch * N * 32, hipMemcpyDeviceToDevice, s));
        return ntt_device_dispatch(st, field, st->scratch[5].ptr, d_data, st->scratch[4].ptr, log_n, batch, inverse, s);
    }
    return ntt_device_dispatch(st, field, d_data, d_data, st->scratch[4].ptr, log_n, batch, inverse, s);
}
