/*
 * CPU restatement of the halo hot path in plain C.  TEST INFRASTRUCTURE ONLY.
 *
 * This is the parity oracle for sizes the Python oracle (oracle/pasta.py) cannot reach, and the
 * timed CPU baseline ("kind": "port") in bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it; the product library (halo_amd/lib/libhalo_gpu.so) never
 * links or calls it.
 *
 * Algorithms restated (citations relative to the reference root, rasmus-kirk/halo):
 *  - ark-ff 0.5.0 Montgomery Fp256 arithmetic (4 x u64 limbs, R = 2^256) for ark_pallas::{Fr,Fq}
 *    (crates/group/src/lib.rs:8-9; Cargo.lock:137-138).
 *  - ark-ec 0.5.0 short-Weierstrass Jacobian `Projective` add / mixed add / double for Pallas and
 *    Vesta (crates/group/src/group.rs:28-29).
 *  - `VariableBaseMSM::msm_unchecked` as called at crates/accumulation/src/pedersen.rs:21 and
 *    crates/group/src/group.rs:49: ark-ec's signed-digit bucket Pippenger with window
 *    c = (size < 32) ? 3 : ln_without_floats(size) + 2, buckets accumulated in Jacobian with mixed
 *    additions, running-sum bucket reduction, window combination by c doublings; parallel over
 *    windows (rayon in the reference, OpenMP here).
 *  - ark-poly 0.5.0 radix-2 FFT used by Evals::from_poly(_ref)/interpolate
 *    (crates/group/src/poly.rs:56-64,133-139): in-place DIF butterflies + bit-reversal permutation
 *    (forward), the same with omega^-1 and a final N^-1 scaling (inverse).
 *  - The IPA folding loop body of crates/accumulation/src/pcdl.rs:427-435: per element
 *    G_l[j] = (G_l[j] + xi * G_r[j]).into_affine(), c_l[j] += xi^-1 c_r[j], z_l[j] += xi z_r[j].
 *  - Horner evaluation (DensePolynomial::evaluate, pcdl.rs:49,471), scalar_dot and
 *    construct_powers (crates/group/src/group.rs:43-45,58-66).
 *  - The SRS generator of crates/group/src/main.rs:55-67,97-121 (SHA3-256 + from_le_bytes_mod_order
 *    + scalar multiplication of (-1, 2)).
 *
 * All field elements crossing this ABI are 4 x u64 little-endian limbs in Montgomery form; points
 * are WrappedPoint {x[4], y[4]} Montgomery affine with (0,0) = identity
 * (crates/group/src/wrappers.rs:91-93,592-597).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t l[4]; } fe;

typedef struct {
    uint64_t p[4];
    uint64_t inv;   /* -p^-1 mod 2^64 */
    uint64_t r2[4]; /* R^2 mod p */
    uint64_t one[4];
} field_t;

static const field_t FP = {
    {0x8c46eb2100000001ULL, 0x224698fc0994a8ddULL, 0x0ULL, 0x4000000000000000ULL},
    0x8c46eb20ffffffffULL,
    {0xfc9678ff0000000fULL, 0x67bb433d891a16e3ULL, 0x7fae231004ccf590ULL, 0x096d41af7ccfdaa9ULL},
    {0x5b2b3e9cfffffffdULL, 0x992c350be3420567ULL, 0xffffffffffffffffULL, 0x3fffffffffffffffULL},
};
static const field_t FQ = {
    {0x992d30ed00000001ULL, 0x224698fc094cf91bULL, 0x0ULL, 0x4000000000000000ULL},
    0x992d30ecffffffffULL,
    {0x8c78ecb30000000fULL, 0xd7d30dbd8b0de0e7ULL, 0x7797a99bc3c95d18ULL, 0x096d41af7b9cb714ULL},
    {0x34786d38fffffffdULL, 0x992c350be41914adULL, 0xffffffffffffffffULL, 0x3fffffffffffffffULL},
};

static inline const field_t *field_of(int fid) { return fid == 0 ? &FP : &FQ; }
/* curve 0 = Pallas (base Fq, scalar Fp); 1 = Vesta (base Fp, scalar Fq) */
static inline const field_t *base_of(int curve) { return curve == 0 ? &FQ : &FP; }
static inline const field_t *scalar_of(int curve) { return curve == 0 ? &FP : &FQ; }

static inline int fe_geq(const uint64_t *a, const uint64_t *b) {
    for (int i = 3; i >= 0; i--) {
        if (a[i] > b[i]) return 1;
        if (a[i] < b[i]) return 0;
    }
    return 1;
}
static inline void sub_nored(uint64_t *r, const uint64_t *a, const uint64_t *b) {
    u128 borrow = 0;
    for (int i = 0; i < 4; i++) {
        u128 t = (u128)a[i] - b[i] - borrow;
        r[i] = (uint64_t)t;
        borrow = (t >> 64) & 1;
    }
}
static inline int fe_is_zero(const fe *a) { return (a->l[0] | a->l[1] | a->l[2] | a->l[3]) == 0; }
static inline int fe_eq(const fe *a, const fe *b) { return memcmp(a, b, sizeof(fe)) == 0; }

static inline fe f_add(const field_t *F, fe a, fe b) {
    fe r;
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (u128)a.l[i] + b.l[i];
        r.l[i] = (uint64_t)c;
        c >>= 64;
    }
    if (c || fe_geq(r.l, F->p)) sub_nored(r.l, r.l, F->p);
    return r;
}
static inline fe f_sub(const field_t *F, fe a, fe b) {
    fe r;
    if (fe_geq(a.l, b.l)) {
        sub_nored(r.l, a.l, b.l);
    } else {
        fe t;
        sub_nored(t.l, F->p, b.l);
        r = f_add(F, a, t);
    }
    return r;
}
static inline fe f_neg(const field_t *F, fe a) {
    if (fe_is_zero(&a)) return a;
    fe r;
    sub_nored(r.l, F->p, a.l);
    return r;
}
/* CIOS Montgomery multiplication */
static inline fe f_mul(const field_t *F, fe a, fe b) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)a.l[j] * b.l[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[4] = (uint64_t)c;
        t[5] = (uint64_t)(c >> 64);
        uint64_t m = t[0] * F->inv;
        c = (u128)m * F->p[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 4; j++) {
            c += (u128)m * F->p[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[3] = (uint64_t)c;
        t[4] = t[5] + (uint64_t)(c >> 64);
    }
    fe r = {{t[0], t[1], t[2], t[3]}};
    if (t[4] || fe_geq(r.l, F->p)) sub_nored(r.l, r.l, F->p);
    return r;
}
static inline fe f_sqr(const field_t *F, fe a) { return f_mul(F, a, a); }
static inline fe f_one(const field_t *F) { fe r; memcpy(r.l, F->one, 32); return r; }
static inline fe f_zero(void) { fe r = {{0, 0, 0, 0}}; return r; }
static inline fe f_to_mont(const field_t *F, fe a) { fe r2; memcpy(r2.l, F->r2, 32); return f_mul(F, a, r2); }
static inline fe f_from_mont(const field_t *F, fe a) { fe one = {{1, 0, 0, 0}}; return f_mul(F, a, one); }
static fe f_pow(const field_t *F, fe a, const uint64_t *e) {
    fe r = f_one(F);
    for (int i = 3; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            r = f_sqr(F, r);
            if ((e[i] >> b) & 1) r = f_mul(F, r, a);
        }
    return r;
}
static fe f_inv(const field_t *F, fe a) {
    uint64_t e[4];
    uint64_t two[4] = {2, 0, 0, 0};
    sub_nored(e, F->p, two);
    return f_pow(F, a, e);
}

/* ----------------------------------------------------------------------------- curves */
typedef struct { fe x, y; } aff;       /* (0,0) = identity */
typedef struct { fe x, y, z; } jac;    /* z = 0 = identity */

static inline int aff_is_id(const aff *a) { return fe_is_zero(&a->x) && fe_is_zero(&a->y); }
static inline jac jac_id(void) { jac r; r.x = f_zero(); r.y = f_zero(); r.z = f_zero(); return r; }

static jac jac_dbl(const field_t *F, jac p) {
    if (fe_is_zero(&p.z)) return p;
    /* dbl-2009-l (a = 0) */
    fe A = f_sqr(F, p.x), B = f_sqr(F, p.y), C = f_sqr(F, B);
    fe t = f_add(F, p.x, B);
    fe D = f_sub(F, f_sub(F, f_sqr(F, t), A), C);
    D = f_add(F, D, D);
    fe E = f_add(F, f_add(F, A, A), A);
    fe Fv = f_sqr(F, E);
    jac r;
    r.x = f_sub(F, Fv, f_add(F, D, D));
    fe C8 = f_add(F, C, C);
    C8 = f_add(F, C8, C8);
    C8 = f_add(F, C8, C8);
    r.y = f_sub(F, f_mul(F, E, f_sub(F, D, r.x)), C8);
    fe yz = f_mul(F, p.y, p.z);
    r.z = f_add(F, yz, yz);
    return r;
}
static jac jac_add_aff(const field_t *F, jac p, const aff *q) {
    if (aff_is_id(q)) return p;
    if (fe_is_zero(&p.z)) { jac r; r.x = q->x; r.y = q->y; r.z = f_one(F); return r; }
    /* madd-2007-bl */
    fe Z1Z1 = f_sqr(F, p.z);
    fe U2 = f_mul(F, q->x, Z1Z1);
    fe S2 = f_mul(F, f_mul(F, q->y, p.z), Z1Z1);
    fe H = f_sub(F, U2, p.x);
    fe rr = f_sub(F, S2, p.y);
    if (fe_is_zero(&H)) {
        if (fe_is_zero(&rr)) return jac_dbl(F, p);
        return jac_id();
    }
    fe HH = f_sqr(F, H);
    fe I = f_add(F, HH, HH); I = f_add(F, I, I);
    fe J = f_mul(F, H, I);
    rr = f_add(F, rr, rr);
    fe V = f_mul(F, p.x, I);
    jac r;
    r.x = f_sub(F, f_sub(F, f_sqr(F, rr), J), f_add(F, V, V));
    fe YJ = f_mul(F, p.y, J);
    r.y = f_sub(F, f_mul(F, rr, f_sub(F, V, r.x)), f_add(F, YJ, YJ));
    fe zh = f_add(F, p.z, H);
    r.z = f_sub(F, f_sub(F, f_sqr(F, zh), Z1Z1), HH);
    return r;
}
static jac jac_add(const field_t *F, jac p, jac q) {
    if (fe_is_zero(&p.z)) return q;
    if (fe_is_zero(&q.z)) return p;
    /* add-2007-bl */
    fe Z1Z1 = f_sqr(F, p.z), Z2Z2 = f_sqr(F, q.z);
    fe U1 = f_mul(F, p.x, Z2Z2), U2 = f_mul(F, q.x, Z1Z1);
    fe S1 = f_mul(F, f_mul(F, p.y, q.z), Z2Z2);
    fe S2 = f_mul(F, f_mul(F, q.y, p.z), Z1Z1);
    fe H = f_sub(F, U2, U1);
    fe rr = f_sub(F, S2, S1);
    if (fe_is_zero(&H)) {
        if (fe_is_zero(&rr)) return jac_dbl(F, p);
        return jac_id();
    }
    fe I = f_add(F, H, H); I = f_sqr(F, I);
    fe J = f_mul(F, H, I);
    rr = f_add(F, rr, rr);
    fe V = f_mul(F, U1, I);
    jac r;
    r.x = f_sub(F, f_sub(F, f_sqr(F, rr), J), f_add(F, V, V));
    fe SJ = f_mul(F, S1, J);
    r.y = f_sub(F, f_mul(F, rr, f_sub(F, V, r.x)), f_add(F, SJ, SJ));
    fe zz = f_add(F, p.z, q.z);
    r.z = f_mul(F, f_sub(F, f_sub(F, f_sqr(F, zz), Z1Z1), Z2Z2), H);
    return r;
}
static aff jac_to_aff(const field_t *F, jac p) {
    aff r;
    if (fe_is_zero(&p.z)) { r.x = f_zero(); r.y = f_zero(); return r; }
    fe zi = f_inv(F, p.z);
    fe zi2 = f_sqr(F, zi);
    r.x = f_mul(F, p.x, zi2);
    r.y = f_mul(F, p.y, f_mul(F, zi2, zi));
    return r;
}
/* k canonical (not Montgomery) */
static jac scalar_mul(const field_t *F, const aff *P, const uint64_t *k) {
    jac r = jac_id();
    for (int i = 3; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            r = jac_dbl(F, r);
            if ((k[i] >> b) & 1) r = jac_add_aff(F, r, P);
        }
    return r;
}

/* ----------------------------------------------------------------------------- MSM */
static int log2_ceil(size_t a) { int r = 0; while (((size_t)1 << r) < a) r++; return r; }

/* ark-ec 0.5.0 `make_digits`: signed radix-2^w digits of a canonical scalar */
static void make_digits(const uint64_t *s, int w, int num_bits, int64_t *digits, int digits_count) {
    const uint64_t radix = 1ULL << w;
    const uint64_t window_mask = radix - 1;
    uint64_t carry = 0;
    for (int i = 0; i < digits_count; i++) {
        int bit_offset = i * w;
        int u64_idx = bit_offset / 64;
        int bit_idx = bit_offset % 64;
        uint64_t bit_buf;
        if (bit_idx < 64 - w || u64_idx == 3) {
            bit_buf = s[u64_idx] >> bit_idx;
        } else {
            bit_buf = (s[u64_idx] >> bit_idx) | (s[1 + u64_idx] << (64 - bit_idx));
        }
        uint64_t coef = carry + (bit_buf & window_mask);
        carry = (coef + radix / 2) >> w;
        int64_t digit = (int64_t)coef - (int64_t)(carry << w);
        digits[i] = digit;
    }
    (void)num_bits;
    if (digits_count > 0) digits[digits_count - 1] += (int64_t)(carry << w);
}

int orc_msm_window_size(size_t n) {
    if (n < 32) return 3;
    return (log2_ceil(n) * 69 / 100) + 2;
}

/* bases: WrappedPoint (x,y Montgomery, (0,0)=id); scalars: Montgomery (mont=1) or canonical.
 * out: affine WrappedPoint of the result. */
void orc_msm(int curve, const uint64_t *bases, const uint64_t *scalars, size_t n, int scalars_mont,
             int threads, uint64_t *out) {
    const field_t *F = base_of(curve);
    const field_t *S = scalar_of(curve);
    if (threads > 0) omp_set_num_threads(threads);
    const int c = orc_msm_window_size(n);
    const int num_bits = 255;
    const int digits_count = (num_bits + c - 1) / c;
    int64_t *digits = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1) * digits_count);
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) {
        fe s;
        memcpy(s.l, scalars + 4 * i, 32);
        if (scalars_mont) s = f_from_mont(S, s);
        make_digits(s.l, c, num_bits, digits + i * digits_count, digits_count);
    }
    jac *window_sums = (jac *)malloc(sizeof(jac) * digits_count);
#pragma omp parallel for schedule(dynamic, 1)
    for (int w = 0; w < digits_count; w++) {
        size_t nb = (size_t)1 << c;
        jac *buckets = (jac *)malloc(sizeof(jac) * nb);
        for (size_t b = 0; b < nb; b++) buckets[b] = jac_id();
        for (size_t i = 0; i < n; i++) {
            int64_t d = digits[i * digits_count + w];
            if (d == 0) continue;
            aff P;
            memcpy(&P, bases + 8 * i, 64);
            if (d > 0) {
                buckets[d - 1] = jac_add_aff(F, buckets[d - 1], &P);
            } else {
                if (!aff_is_id(&P)) P.y = f_neg(F, P.y);
                buckets[-d - 1] = jac_add_aff(F, buckets[-d - 1], &P);
            }
        }
        jac running = jac_id(), res = jac_id();
        for (size_t b = nb; b-- > 0;) {
            running = jac_add(F, running, buckets[b]);
            res = jac_add(F, res, running);
        }
        window_sums[w] = res;
        free(buckets);
    }
    jac total = jac_id();
    for (int w = digits_count - 1; w >= 1; w--) {
        total = jac_add(F, total, window_sums[w]);
        for (int k = 0; k < c; k++) total = jac_dbl(F, total);
    }
    total = jac_add(F, total, window_sums[0]);
    aff r = jac_to_aff(F, total);
    memcpy(out, &r, 64);
    free(window_sums);
    free(digits);
}

/* ----------------------------------------------------------------------------- NTT */
static size_t bitrev(size_t x, int logn) {
    size_t r = 0;
    for (int i = 0; i < logn; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

/* omega_N = 5^((p-1)/N) in Montgomery form */
static fe root_of_unity(const field_t *F, int logn) {
    uint64_t e[4];
    uint64_t one[4] = {1, 0, 0, 0};
    sub_nored(e, F->p, one);
    for (int k = 0; k < logn; k++) { /* e >>= 1 */
        for (int i = 0; i < 4; i++) e[i] = (e[i] >> 1) | (i < 3 ? (e[i + 1] << 63) : 0);
    }
    fe g = {{5, 0, 0, 0}};
    g = f_to_mont(F, g);
    return f_pow(F, g, e);
}

/* In-place natural-order transform of a[0..2^logn).  DIF butterflies + bit reversal
 * (ark-poly Radix2EvaluationDomain::in_order_fft_in_place). */
void orc_ntt(int fid, uint64_t *data, int logn, int inverse, int threads) {
    const field_t *F = field_of(fid);
    if (threads > 0) omp_set_num_threads(threads);
    const size_t n = (size_t)1 << logn;
    fe *a = (fe *)data;
    fe w = root_of_unity(F, logn);
    if (inverse) w = f_inv(F, w);
    /* twiddle table w^0..w^(n/2-1) */
    size_t half = n / 2 ? n / 2 : 1;
    fe *tw = (fe *)malloc(sizeof(fe) * half);
    tw[0] = f_one(F);
    for (size_t i = 1; i < half; i++) tw[i] = f_mul(F, tw[i - 1], w);
    for (size_t gap = n / 2, step = 1; gap >= 1; gap >>= 1, step <<= 1) {
        /* blocks of size 2*gap; twiddle for index k within block = w^(k*step) */
#pragma omp parallel for schedule(static)
        for (size_t idx = 0; idx < n / 2; idx++) {
            size_t blk = idx / gap, k = idx % gap;
            size_t i0 = blk * 2 * gap + k, i1 = i0 + gap;
            fe u = a[i0], v = a[i1];
            a[i0] = f_add(F, u, v);
            a[i1] = f_mul(F, f_sub(F, u, v), tw[k * step]);
        }
        if (gap == 1) break;
    }
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) {
        size_t j = bitrev(i, logn);
        if (i < j) { fe t = a[i]; a[i] = a[j]; a[j] = t; }
    }
    if (inverse) {
        fe ninv = {{n, 0, 0, 0}};
        ninv = f_inv(F, f_to_mont(F, ninv));
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < n; i++) a[i] = f_mul(F, a[i], ninv);
    }
    free(tw);
}

/* ----------------------------------------------------------------------------- poly / dots */
void orc_poly_eval(int fid, const uint64_t *coeffs, size_t n, const uint64_t *z, uint64_t *out) {
    const field_t *F = field_of(fid);
    fe zz; memcpy(zz.l, z, 32);
    fe v = f_zero();
    for (size_t i = n; i-- > 0;) {
        fe c; memcpy(c.l, coeffs + 4 * i, 32);
        v = f_add(F, f_mul(F, v, zz), c);
    }
    memcpy(out, v.l, 32);
}

void orc_scalar_dot(int fid, const uint64_t *xs, const uint64_t *ys, size_t n, uint64_t *out) {
    const field_t *F = field_of(fid);
    fe acc = f_zero();
    for (size_t i = 0; i < n; i++) {
        fe a, b;
        memcpy(a.l, xs + 4 * i, 32);
        memcpy(b.l, ys + 4 * i, 32);
        acc = f_add(F, acc, f_mul(F, a, b));
    }
    memcpy(out, acc.l, 32);
}

void orc_field_mul(int fid, const uint64_t *a, const uint64_t *b, uint64_t *out) {
    fe x, y; memcpy(x.l, a, 32); memcpy(y.l, b, 32);
    fe r = f_mul(field_of(fid), x, y);
    memcpy(out, r.l, 32);
}
void orc_field_inv(int fid, const uint64_t *a, uint64_t *out) {
    fe x; memcpy(x.l, a, 32);
    fe r = f_inv(field_of(fid), x);
    memcpy(out, r.l, 32);
}

/* ----------------------------------------------------------------------------- IPA fold */
/* One fold (pcdl.rs:427-435) over m pairs; gs is 2m WrappedPoints, cs/zs 2m scalars (Montgomery).
 * xi, xi_inv Montgomery.  Updates the left halves in place. */
void orc_ipa_fold(int curve, uint64_t *gs, uint64_t *cs, uint64_t *zs, size_t m, const uint64_t *xi,
                  const uint64_t *xi_inv, int threads) {
    const field_t *F = base_of(curve);
    const field_t *S = scalar_of(curve);
    if (threads > 0) omp_set_num_threads(threads);
    fe x, xinv;
    memcpy(x.l, xi, 32);
    memcpy(xinv.l, xi_inv, 32);
    fe xc = f_from_mont(S, x);
#pragma omp parallel for schedule(static)
    for (size_t j = 0; j < m; j++) {
        aff gl, gr;
        memcpy(&gl, gs + 8 * j, 64);
        memcpy(&gr, gs + 8 * (j + m), 64);
        jac t = scalar_mul(F, &gr, xc.l);
        t = jac_add_aff(F, t, &gl);
        aff r = jac_to_aff(F, t);
        memcpy(gs + 8 * j, &r, 64);
        fe cl, cr, zl, zr;
        memcpy(cl.l, cs + 4 * j, 32); memcpy(cr.l, cs + 4 * (j + m), 32);
        memcpy(zl.l, zs + 4 * j, 32); memcpy(zr.l, zs + 4 * (j + m), 32);
        cl = f_add(S, cl, f_mul(S, cr, xinv));
        zl = f_add(S, zl, f_mul(S, zr, x));
        memcpy(cs + 4 * j, cl.l, 32);
        memcpy(zs + 4 * j, zl.l, 32);
    }
}

/* ----------------------------------------------------------------------------- SRS recipe */
/* Keccak-f[1600] / SHA3-256 (FIPS 202), for the SRS hash of crates/group/src/main.rs:55-67 */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
static inline uint64_t rol(uint64_t x, int r) { return r ? (x << r) | (x >> (64 - r)) : x; }
static void keccakf(uint64_t s[25]) {
    for (int round = 0; round < 24; round++) {
        uint64_t C[5], D[5], B[25];
        for (int x = 0; x < 5; x++) C[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
        for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rol(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; i++) s[i] ^= D[i % 5];
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rol(s[x + 5 * y], KROT[x + 5 * y]);
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) s[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        s[0] ^= KRC[round];
    }
}
void orc_sha3_256(const uint8_t *msg, size_t len, uint8_t *out) {
    uint64_t s[25];
    memset(s, 0, sizeof(s));
    const size_t rate = 136;
    uint8_t block[136];
    while (len >= rate) {
        for (size_t i = 0; i < rate / 8; i++) { uint64_t w; memcpy(&w, msg + 8 * i, 8); s[i] ^= w; }
        keccakf(s);
        msg += rate; len -= rate;
    }
    memset(block, 0, rate);
    memcpy(block, msg, len);
    block[len] ^= 0x06;
    block[rate - 1] ^= 0x80;
    for (size_t i = 0; i < rate / 8; i++) { uint64_t w; memcpy(&w, block + 8 * i, 8); s[i] ^= w; }
    keccakf(s);
    memcpy(out, s, 32);
}

static const char GENESIS[] = "To understand recursion, one must first understand recursion";

/* canonical scalar h(j) = from_le_bytes_mod_order(SHA3-256(u64le(j) || GENESIS)) */
void orc_srs_hash_scalar(int curve, uint64_t j, uint64_t *out) {
    const field_t *S = scalar_of(curve);
    uint8_t msg[8 + sizeof(GENESIS) - 1];
    for (int i = 0; i < 8; i++) msg[i] = (uint8_t)(j >> (8 * i));
    memcpy(msg + 8, GENESIS, sizeof(GENESIS) - 1);
    uint8_t h[32];
    orc_sha3_256(msg, sizeof(msg), h);
    fe v;
    memcpy(v.l, h, 32);
    /* reduce a 256-bit integer mod p (< 4p since p > 2^254) */
    while (fe_geq(v.l, S->p)) sub_nored(v.l, v.l, S->p);
    memcpy(out, v.l, 32);
}

/* affine k * (-1, 2) for canonical k */
void orc_generator_mul(int curve, const uint64_t *k, uint64_t *out) {
    const field_t *F = base_of(curve);
    aff G;
    G.x = f_neg(F, f_one(F));
    fe two = f_add(F, f_one(F), f_one(F));
    G.y = two;
    jac r = scalar_mul(F, &G, k);
    aff a = jac_to_aff(F, r);
    memcpy(out, &a, 64);
}

/* The reference SRS prefix G[0..n) (n <= 2^20 as the reference ships; any n accepted): entry j is
 * H((j >> 14) + (j & 16383) + 2).  Distinct hash indices are computed once. */
void orc_srs_generate(int curve, size_t n, int threads, uint64_t *out) {
    if (threads > 0) omp_set_num_threads(threads);
    if (n == 0) return;
    size_t max_idx = ((n - 1) >> 14) + ((n - 1) < 16384 ? (n - 1) : 16383) + 2;
    uint64_t *pts = (uint64_t *)malloc(64 * (max_idx + 1));
#pragma omp parallel for schedule(dynamic, 16)
    for (size_t t = 2; t <= max_idx; t++) {
        uint64_t k[4];
        orc_srs_hash_scalar(curve, t, k);
        orc_generator_mul(curve, k, pts + 8 * t);
    }
#pragma omp parallel for schedule(static)
    for (size_t j = 0; j < n; j++) {
        size_t t = (j >> 14) + (j & 16383) + 2;
        memcpy(out + 8 * j, pts + 8 * t, 64);
    }
    free(pts);
}

int orc_max_threads(void) { return omp_get_max_threads(); }

/* ----------------------------------------------------------------------------- prover helpers
 * Vectorised Evals ops for the CPU restatement of the prover pipeline (oracle/prover_ref.py,
 * CRefBackend), on Montgomery words: op 0 a+b, 1 a-b, 2 a*b, 3 a*s, 4 a+s, 5 a-s, 6 a^e. */
void orc_evals_op(int fid, int op, const uint64_t *a, const uint64_t *b, const uint64_t *s, uint32_t e, size_t n,
                  uint64_t *out, int threads) {
    const field_t *F = field_of(fid);
    if (threads > 0) omp_set_num_threads(threads);
    fe sv = f_zero();
    if (s) memcpy(sv.l, s, 32);
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) {
        fe x, y, r;
        memcpy(x.l, a + 4 * i, 32);
        if (op <= 2) memcpy(y.l, b + 4 * i, 32);
        switch (op) {
            case 0: r = f_add(F, x, y); break;
            case 1: r = f_sub(F, x, y); break;
            case 2: r = f_mul(F, x, y); break;
            case 3: r = f_mul(F, x, sv); break;
            case 4: r = f_add(F, x, sv); break;
            case 5: r = f_sub(F, x, sv); break;
            default: /* x^e as e - 1 multiplications, like the reference's sbox closure w*w*...*w */
                r = x;
                for (uint32_t k = 1; k < e; k++) r = f_mul(F, r, x);
                if (e == 0) r = f_one(F);
        }
        memcpy(out + 4 * i, r.l, 32);
    }
}

/* z[0] = 1, z[i] = z[i-1] * f[i] / g[i] (protocol.rs:143-154, sequential, one inversion each) */
void orc_perm_acc(int fid, const uint64_t *f, const uint64_t *g, size_t n, uint64_t *z) {
    const field_t *F = field_of(fid);
    fe acc = f_one(F);
    for (size_t i = 0; i < n; i++) {
        if (i) {
            fe fi, gi;
            memcpy(fi.l, f + 4 * i, 32);
            memcpy(gi.l, g + 4 * i, 32);
            acc = f_mul(F, f_mul(F, acc, fi), f_inv(F, gi));
        }
        memcpy(z + 4 * i, acc.l, 32);
    }
}
