/*
 * halo_gpu.h -- C ABI of the MI355X (gfx950) backend for the rasmus-kirk/halo proving hot path.
 *
 * Every entry point replaces one reference function (or the arkworks call inside it) on the path
 * named by BASELINE.json's north_star; the reference interface each one stands in for is cited
 * next to it (paths relative to the reference root).  A Rust `extern "C"` shim that binds these
 * symbols is given in INTEGRATION.md.
 *
 * Conventions
 *  - Field elements (`halo_fe_t`): 4 x u64 little-endian limbs in arkworks Montgomery form
 *    (R = 2^256), canonical in [0, p) -- the in-memory layout of `ark_ff::Fp256` / `BigInt<4>`,
 *    so `&[Fr]` can be passed zero-copy.
 *  - Points (`halo_wrapped_point_t`): `WrappedPoint { x: [u64; 4], y: [u64; 4] }`
 *    (crates/group/src/wrappers.rs:592-597, #[repr(C)]), affine, Montgomery limbs; the identity is
 *    (0, 0) (`PastaAffine::identity`, wrappers.rs:91-93).  Every point-valued result is returned in
 *    this canonical affine form, so results compare bit-exactly.
 *  - Curves: HALO_PALLAS (base field Fq, scalars Fp = ark_pallas::Fr), HALO_VESTA (base Fp,
 *    scalars Fq).  Fields: HALO_FP (ark_pallas::Fr), HALO_FQ (ark_pallas::Fq)
 *    (crates/group/src/lib.rs:8-9).
 *  - Host-pointer entry points take caller-owned host buffers, borrowed for the call only.
 *    `_dev` entry points take device pointers (hipMalloc'd on the current device) plus a
 *    `hipStream_t` passed as `void*` (NULL = default stream) and are asynchronous with respect to
 *    the host unless stated otherwise.
 *  - Errors: the reference panics (`assert!`) on contract violations; this ABI never aborts and
 *    returns a nonzero `halo_status_t` instead, with the reference's panic message available from
 *    `halo_last_error()` (thread-local).
 *  - Thread safety: every call is re-entrant.  Device-resident state (SRS, twiddles, scratch) is
 *    per (device, curve/field), created once under a mutex (mirrors the `OnceLock<PublicParams>`
 *    of crates/group/src/pp.rs:63-94 and wrappers.rs:28-29).
 */
#ifndef HALO_GPU_H
#define HALO_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { uint64_t l[4]; } halo_fe_t;
typedef struct { uint64_t x[4]; uint64_t y[4]; } halo_wrapped_point_t;

typedef enum { HALO_PALLAS = 0, HALO_VESTA = 1 } halo_curve_t;
typedef enum { HALO_FP = 0, HALO_FQ = 1 } halo_field_t;

typedef enum {
    HALO_OK = 0,
    HALO_EINVAL = 1,     /* bad argument (null pointer, unknown curve/field, length mismatch) */
    HALO_ENOMEM = 2,     /* device allocation failed */
    HALO_EDEVICE = 3,    /* HIP runtime / kernel error, or no GPU */
    HALO_ENOTPOW2 = 4,   /* "n ({n}) is not a power of two"  (pcdl.rs:282, pp.rs:32) */
    HALO_ESRSRANGE = 5,  /* "d ({d}) <= D ({D})" / SRS too short (pcdl.rs:284, pp.rs:33) */
    HALO_EDEGREE = 6,    /* "p_deg ({p_deg}) <= d ({d})" (pcdl.rs:283) */
    HALO_ELENGTH = 7     /* "ms must be larger than Gs" (pedersen.rs:14-19) */
} halo_status_t;

/* ------------------------------------------------------------------ runtime */
/* Selects the HIP device used by subsequent calls from this thread and creates its context. */
int halo_init(int device);
/* Number of visible GPUs (0 when no GPU is present). */
int halo_device_count(void);
/* Message of the last failed call on this thread ("" if none). */
const char* halo_last_error(void);
/* ABI version (major * 100 + minor). */
int halo_abi_version(void);
/* Releases the library's streams, events and pending profiling events while the HIP runtime is
 * alive (call before process exit; the Python mirror registers it with atexit).  Idempotent; the
 * library remains usable afterwards. */
int halo_shutdown(void);
/* Blocks until all work queued by this library on `stream` is complete. */
int halo_stream_sync(void* stream);
/* Path-selection tuning (library-wide, read by every later call; value -1 restores the default).
 * Keys: "ipa_weighted" (1: IPA rounds over the resident window-shifted SRS without folding G; 0:
 * GLV-fold G every round), "ipa_tail" (1: switch to the direct-sum tail rounds at length 2048),
 * "ipa_srs_tail_n" (SRS openings of n <= this run tail rounds from round 1; default 4096),
 * "ipa_mat_n" (weighted rounds materialise G at this length; 0 = never; default 2048),
 * "msm_multi_max" (commitment batches of polynomials up to this length run as one MSM; default
 * 2^18), "ipa_pool_keep_bytes" (an idle pooled IPA session keeps at most this many bytes of device
 * buffers; default 2^30), "ipa_pair_max" (weighted rounds up to this half-length form L and R as one
 * MSM; default 2^19), "ntt_big_max_log" (NTTs up to 2^this use 11-bit passes; default 22),
 * "ntt_even_split" (1: stages split evenly over the passes; default 0).  Every setting yields the same results; the parity tests pin each path with it.  The
 * reference has no counterpart (host-side knob of this backend only).  HALO_EINVAL on an unknown key. */
int halo_set_tuning(const char* key, long long value);
int halo_get_tuning(const char* key, long long* value);

/* ------------------------------------------------------------------ a10: SRS provider
 * Replaces PublicParams::{new, set_pp, get_pp} (crates/group/src/pp.rs:26-94): the SRS bases Gs,
 * S and H become device-resident once per (device, curve).  `gs` is the decoded
 * `Vec<WrappedPoint>` of crates/group/.precompute/<curve>/gs-XX.bin (or any prefix of it). */
int halo_srs_upload(halo_curve_t curve, const halo_wrapped_point_t* gs, size_t n,
                    const halo_wrapped_point_t* S, const halo_wrapped_point_t* H);
/* f3: PublicParams::new(n) from the wire format (pp.rs:26-61): `blocks` are the gs-XX.bin files
 * (bincode-v2 standard() Vec<WrappedPoint>, decoded in order until n points), `sh` is sh.bin
 * ((S, H); may be NULL).  Decoded and curve-checked on the device; the reference's panics map to
 * HALO_ENOTPOW2 ("assertion failed: n.is_power_of_two()"), HALO_ESRSRANGE (n > available points),
 * HALO_EINVAL ("Failed to decode G_BLOCKS_NO i", "assertion failed: affine.is_on_curve()"). */
int halo_srs_load_bincode(halo_curve_t curve, const uint8_t* const* blocks, const size_t* block_lens, size_t nblocks,
                          const uint8_t* sh, size_t sh_len, size_t n);
/* Current resident SRS length (0 if none). */
int halo_srs_len(halo_curve_t curve, size_t* n);
/* The resident PublicParams' (S, H) (crates/group/src/pp.rs:26-61) as WrappedPoints. */
int halo_srs_sh(halo_curve_t curve, halo_wrapped_point_t* S, halo_wrapped_point_t* H);
/* Synthetic SRS for sizes beyond the reference's N = 2^20 (crates/group/src/consts.rs:1):
 * G_j = k_j * (-1, 2) with k_j from halo_synth_scalar(seed, j), generated on the device.
 * S, H as in the reference are left unchanged if already uploaded. */
int halo_srs_synthesize(halo_curve_t curve, size_t n, uint64_t seed);
/* The canonical (non-Montgomery) discrete log k_j used by halo_srs_synthesize (host function; lets
 * a verifier check MSM results over synthetic bases in O(n) field operations). */
void halo_synth_scalar(halo_curve_t curve, uint64_t seed, uint64_t j, uint64_t out_canonical[4]);
/* Precomputes the window-shifted copies 2^(c*w) * G_i of the resident SRS used by the
 * single-bucket-set MSM (trades HBM capacity for the per-window combination); optional. */
int halo_srs_precompute_windows(halo_curve_t curve);
/* The copies of windows [w_lo, w_hi) only, of width c bits (c = 0: the default width for the SRS
 * length; w_hi = 0: every window): one rank of a window-partitioned MSM holds just its own windows
 * (BASELINE configs[4]); such a partial set serves halo_msm_srs_windows_dev over that range only (the
 * other SRS MSMs then run without shifted copies). */
int halo_srs_precompute_window_range(halo_curve_t curve, int c, int w_lo, int w_hi);

/* Copies resident SRS points Gs[offset .. offset + n) back to the host as WrappedPoints. */
int halo_srs_read(halo_curve_t curve, size_t offset, size_t n, halo_wrapped_point_t* out);

/* ------------------------------------------------------------------ a3/a4: MSM
 * sum_{i < min(n_bases, n_scalars)} scalars[i] * bases[i]
 * Replaces `Projective::msm_unchecked` as called by group::point_dot_affine
 * (crates/group/src/group.rs:48-50) and pedersen::commit (crates/accumulation/src/pedersen.rs:21).
 * Empty input -> identity (0, 0). */
int halo_msm(halo_curve_t curve, const halo_wrapped_point_t* bases, size_t n_bases,
             const halo_fe_t* scalars, size_t n_scalars, halo_wrapped_point_t* out);
/* Same over the resident SRS prefix Gs[0..n) (the pcdl::commit path, pcdl.rs:286). */
int halo_msm_srs(halo_curve_t curve, const halo_fe_t* scalars, size_t n, halo_wrapped_point_t* out);
/* pedersen::commit(w, Gs, ms) (crates/accumulation/src/pedersen.rs:7-27): asserts
 * Gs.len() >= ms.len(), MSM, then + S*w when `w` is non-NULL. */
int halo_pedersen_commit(halo_curve_t curve, const halo_fe_t* w, const halo_wrapped_point_t* gs,
                         size_t n_gs, const halo_fe_t* ms, size_t n_ms, halo_wrapped_point_t* out);
/* pcdl::commit(p, d, w) (crates/accumulation/src/pcdl.rs:275-287): n = d + 1 must be a power of
 * two, deg(p) <= d <= D, then pedersen::commit(w, Gs[0..n], p.coeffs) over the resident SRS.
 * `coeffs` has `len` entries (trailing zeros allowed). */
int halo_pcdl_commit(halo_curve_t curve, const halo_fe_t* coeffs, size_t len, size_t d,
                     const halo_fe_t* w, halo_wrapped_point_t* out);
/* The hiding branch of pcdl::open_without_eval (crates/accumulation/src/pcdl.rs:344-371), in the
 * two steps around the caller's transcript challenge alpha = rho(C, C_bar, z, v):
 *   blind:   p_bar = (X - z) q (q: d coefficients, the reference's random q of degree d - 1) and the
 *            hiding commitment C_bar = pcdl::commit(p_bar, d, w_bar); p_bar_out (d + 1, optional).
 *   combine: p' = p + alpha p_bar (d + 1 coefficients; p has len <= d + 1), w' = w + alpha w_bar,
 *            C' = C + alpha C_bar - w' S, over the resident SRS's S.
 * Same assertions as the reference (n = d + 1 > 1 a power of two, d <= D); needs (S, H) uploaded. */
int halo_pcdl_hiding_blind(halo_curve_t curve, const halo_fe_t* q, size_t d, const halo_fe_t* z,
                           const halo_fe_t* w_bar, halo_fe_t* p_bar_out, halo_wrapped_point_t* C_bar_out);
int halo_pcdl_hiding_combine(halo_curve_t curve, const halo_fe_t* p, size_t len, const halo_fe_t* p_bar, size_t d,
                             const halo_fe_t* alpha, const halo_wrapped_point_t* C, const halo_wrapped_point_t* C_bar,
                             const halo_fe_t* w, const halo_fe_t* w_bar, halo_fe_t* p_prime_out,
                             halo_fe_t* w_prime_out, halo_wrapped_point_t* C_prime_out);
/* group::point_dot(xs, &[Projective]) (crates/group/src/group.rs:53-56, called at
 * crates/accumulation/src/acc.rs:166): bases are ark Projective points -- Jacobian (X, Y, Z), each
 * coordinate 4 x u64 Montgomery, 96 B per point, Z = 0 the identity -- normalised on the device
 * (Projective::normalize_batch), then the MSM; length = min(n_bases, n_scalars). */
int halo_point_dot_projective(halo_curve_t curve, const halo_fe_t* scalars, size_t n_scalars,
                              const uint64_t (*bases)[12], size_t n_bases, halo_wrapped_point_t* out);
/* Device-pointer MSM: d_bases (n WrappedPoints, or NULL to use the resident SRS prefix) and
 * d_scalars (n halo_fe_t) in HBM; result written to host `out`.  Synchronous on `stream`. */
int halo_msm_dev(halo_curve_t curve, const void* d_bases, const void* d_scalars, size_t n,
                 halo_wrapped_point_t* out, void* stream);
/* Asynchronous device MSM for batches of commitments: enqueues the MSM on `stream` and returns;
 * the 64-B result lands in device memory d_out.  Consecutive calls pipeline: the reduction tail
 * of MSM k overlaps the accumulation of MSM k+1 (two scratch sets, a per-device tail stream).
 * Buffers must stay valid until halo_msm_join(stream) has been ordered before their reuse. */
int halo_msm_dev_async(halo_curve_t curve, const void* d_bases, const void* d_scalars, size_t n,
                       void* d_out, void* stream);
/* Makes `stream` wait (device-side, no host sync) for every asynchronous MSM still in flight. */
int halo_msm_join(void* stream);
/* Batched commitments over the resident SRS prefix: k independent MSMs, MSM i over d_scalars[i]
 * (device pointer, lens[i] <= SRS length ark scalars), result i (64-B WrappedPoint) at
 * d_out + 64 i.  Replaces a loop of pcdl::commit / pedersen::commit calls over one SRS -- the
 * reference's commitment batches (crates/plonk/src/plonk/protocol.rs:114,263 -- 16 commits each;
 * crates/plonk/src/plonk/trace.rs:188-192).  All inputs must be ready on `stream` at the call;
 * asynchronous like halo_msm_dev_async (halo_msm_join before reading d_out).  Polynomials of up to
 * 2^18 coefficients (HALO_MSM_MULTI_MAX) form ONE MSM whose sort keys are (polynomial, bucket); longer
 * ones run as back-to-back pipelined MSMs. */
int halo_msm_batch_dev(halo_curve_t curve, const void* const* d_scalars, const size_t* lens, size_t k, void* d_out,
                       void* stream);
/* Window-partitioned MSM (BASELINE configs[4]): one rank's share -- the signed digits of windows
 * [w_lo, w_hi) of the n scalars against the resident window-shifted copies 2^(c w) G_i -- as a 64-B
 * partial sum at d_out (asynchronous, halo_msm_join).  Partials of a partition of [0, W) add up to
 * the full MSM (pedersen.rs:21).  halo_srs_windows gives W (0 without the shifted copies); the range
 * must lie inside the resident copies (all of them, or halo_srs_precompute_window_range's range). */
int halo_msm_srs_windows_dev(halo_curve_t curve, const void* d_scalars, size_t n, int w_lo, int w_hi, void* d_out,
                             void* stream);
int halo_srs_windows(halo_curve_t curve);
/* Sum of k points (host arrays) on the device: the combine step after an RCCL all-gather of
 * per-rank partial MSMs (RCCL has no elliptic-curve reduction operator). */
int halo_point_sum(halo_curve_t curve, const halo_wrapped_point_t* pts, size_t k, halo_wrapped_point_t* out);
/* Device variant: k WrappedPoints at d_pts (stride_bytes = 64) summed into d_out, on `stream`. */
int halo_point_sum_dev(halo_curve_t curve, const void* d_pts, size_t k, size_t stride_bytes, void* d_out,
                       void* stream);
/* rows independent sums at once (one launch): row b sums the k WrappedPoints d_pts[b k .. b k + k) into
 * d_out[b] -- the combine of `rows` point-partitioned MSMs after one all-gather (bench.py --gpus N). */
int halo_point_sum_rows_dev(halo_curve_t curve, const void* d_pts, size_t rows, size_t k, void* d_out, void* stream);
/* The same sum over packed XYZZ points (128 B each: X, Y, ZZ, ZZZ in the library's internal Montgomery
 * form, as halo_ipa_round_lr_dev writes them), stride_bytes apart, into one packed XYZZ point: no
 * affine conversion (and no inversion) on the device.  A distributed opening sums its ranks' L_r, R_r
 * with it and converts the one sum on the host (halo_xyzz_to_wrapped). */
int halo_point_sum_xyzz_dev(halo_curve_t curve, const void* d_pts, size_t k, size_t stride_bytes, void* d_out,
                            void* stream);
/* k packed XYZZ points (host memory) -> affine WrappedPoints (host binary extended Euclid). */
int halo_xyzz_to_wrapped(halo_curve_t curve, const void* xyzz, size_t k, halo_wrapped_point_t* out);
/* Window size the device MSM uses for n points. */
int halo_msm_window_bits(size_t n);
/* Window size of the resident SRS's window-shifted copies (halo_srs_precompute_windows), or 0 when
 * they are not built (MSMs against the resident SRS then use halo_msm_window_bits). */
int halo_srs_window_bits(halo_curve_t curve);

/* ------------------------------------------------------------------ a5/a6/a7: NTT
 * Radix-2 domain of size N = 2^log_n, omega = 5^((p-1)/N) (ark-poly Radix2EvaluationDomain,
 * crates/group/src/poly.rs:11).  Natural order in and out. */
/* In-place forward (evals[i] = p(omega^i)) or inverse (includes the N^-1 scaling). */
int halo_ntt(halo_field_t field, halo_fe_t* inout, unsigned log_n, int inverse);
/* Evals::from_poly(_ref) / DensePolynomial::evaluate_over_domain(_by_ref) (poly.rs:56-64):
 * `len` coefficients (len may exceed N: reduced mod X^N - 1 first) -> N evaluations. */
int halo_evaluate_over_domain(halo_field_t field, const halo_fe_t* coeffs, size_t len,
                              unsigned log_n, halo_fe_t* evals);
/* Evals::interpolate(_by_ref) (poly.rs:133-139): N evaluations -> coefficients with trailing
 * zeros trimmed (`*out_len` = trimmed length, <= N). */
int halo_interpolate(halo_field_t field, const halo_fe_t* evals, unsigned log_n, halo_fe_t* coeffs,
                     size_t* out_len);
/* &DensePolynomial * &DensePolynomial (FFT multiply; protocol.rs:132-139, pcdl.rs:215):
 * out has room for la + lb - 1 entries; *out_len = trimmed length. */
int halo_poly_mul(halo_field_t field, const halo_fe_t* a, size_t la, const halo_fe_t* b, size_t lb,
                  halo_fe_t* out, size_t* out_len);
/* Batched device NTT: `batch` contiguous transforms of size 2^log_n at d_data, in place. */
int halo_ntt_dev(halo_field_t field, void* d_data, unsigned log_n, size_t batch, int inverse,
                 void* stream);
/* Forward halo_ntt_dev for inputs that are zero from index nonzero_len on (a polynomial of degree
 * < nonzero_len evaluated over a larger domain, protocol.rs:89-106): the tail's contents are ignored
 * (the caller need not clear it) and the first pass skips the stages that only replicate values. */
int halo_ntt_dev_zero_tail(halo_field_t field, void* d_data, unsigned log_n, size_t batch,
                           size_t nonzero_len, void* stream);
/* Distributed-NTT building blocks (four-step decomposition, halo_amd/dist.py sharded_ntt; SURVEY
 * §8e).  halo_ntt_twiddle_dev: element (a, b) of the rows x cols matrix at d_data (ark format) is
 * multiplied by omega_N^((row0 + a)(col0 + b)) (omega^-1 when inverse), N = 2^log_n.
 * halo_transpose_dev: for `batch` consecutive rows x cols matrices whose elements are runs of `run`
 * 32-byte field elements: dst[s][b][a] = src[s][a][b]. */
int halo_ntt_twiddle_dev(halo_field_t field, void* d_data, unsigned log_n, size_t rows, size_t cols, size_t row0,
                         size_t col0, int inverse, void* stream);
int halo_transpose_dev(const void* d_src, void* d_dst, size_t batch, size_t rows, size_t cols, size_t run,
                       void* stream);

/* ------------------------------------------------------------------ f4: h(X) and the decider MSM
 * HPoly::get_poly (pcdl.rs:198-219): coefficients of h(X) = prod_{i<lg n} (1 + xi_{lg n-i} X^(2^i)),
 * lg n = n_xis - 1, generated directly (coef[j] = product of xi_{lg n-b} over the set bits b of j). */
int halo_hpoly_coeffs(halo_field_t field, const halo_fe_t* xis, size_t n_xis, halo_fe_t* out);
/* sum_i alphas[i] * h_i(X) over k h-polynomials (xis: k rows of n_xis; acc.rs:89); alphas NULL = 1;
 * *out_len (if not NULL) = trimmed length. */
int halo_hpoly_combine(halo_field_t field, const halo_fe_t* xis, size_t k, size_t n_xis, const halo_fe_t* alphas,
                       halo_fe_t* out, size_t* out_len);
/* The same combination into a device buffer d_out (2^(n_xis - 1) ark coefficients, untrimmed), stream-
 * ordered on `stream` (acc::prover's h(X) stays on the device for its commitment and opening). */
int halo_hpoly_combine_dev(halo_field_t field, const halo_fe_t* xis, size_t k, size_t n_xis,
                           const halo_fe_t* alphas, void* d_out, void* stream);
/* pcdl::check step 5 (pcdl.rs:579): pedersen::commit(None, &pp.Gs[0..d+1], &h.get_poly().coeffs)
 * against the resident SRS, the coefficients never leaving the device. */
int halo_pcdl_decider_commit(halo_curve_t curve, const halo_fe_t* xis, size_t n_xis, size_t d,
                             halo_wrapped_point_t* out);

/* ------------------------------------------------------------------ f2: Trace::new batch
 * trace.rs:165-192: k evaluation vectors (k x 2^log_n, row-major) -> Evals::from_vec_and_domain
 * (rotate right by one) -> interpolate (iNTT) -> pcdl::commit(poly, d, None) each; the pcdl::commit
 * assertions and messages apply per row.  coeffs_out (k x 2^log_n, untrimmed) and lens_out (trimmed
 * lengths) are optional. */
int halo_trace_commit_batch(halo_curve_t curve, const halo_fe_t* evals, size_t k, unsigned log_n, size_t d,
                            halo_fe_t* coeffs_out, size_t* lens_out, halo_wrapped_point_t* commits_out);

/* ------------------------------------------------------------------ f1: evaluation algebra
 * Evals ops (crates/group/src/poly.rs:90-327), elementwise over n ark scalars:
 *   op 0 add (a + b), 1 sub (a - b), 2 mul (a * b), 3 scale (a * scalar), 4 add_scalar, 5 sub_scalar,
 *   6 pow (a^exponent, e.g. the Poseidon S-box x^7).  out may alias a or b. */
int halo_evals_op(halo_field_t field, int op, const halo_fe_t* a, const halo_fe_t* b, const halo_fe_t* scalar,
                  uint32_t exponent, halo_fe_t* out, size_t n);
int halo_evals_op_dev(halo_field_t field, int op, const void* d_a, const void* d_b, const halo_fe_t* scalar,
                      uint32_t exponent, void* d_out, size_t n, void* stream);
/* DensePolynomial::divide_by_vanishing_poly (ark-poly 0.5.0; protocol.rs:256): division by
 * X^n - 1; quotient (room for len - n) and remainder (room for n), both trimmed. */
int halo_divide_by_vanishing(halo_field_t field, const halo_fe_t* coeffs, size_t len, size_t n, halo_fe_t* quotient,
                             size_t* q_len, halo_fe_t* remainder, size_t* r_len);
/* Device-resident variant (no trimming): d_coeffs has len >= n entries; quotient len - n entries
 * (may be null when len == n), remainder n entries. */
int halo_divide_by_vanishing_dev(halo_field_t field, const void* d_coeffs, size_t len, size_t n,
                                 void* d_quotient, void* d_remainder, void* stream);
/* Gate-constraint evaluation of naive_prover round 4 (protocol.rs:170-191 with the constraint
 * polynomials of protocol.rs:591-1011), fused into one pass over the n-point (8x) domain: d_w (16),
 * d_r (15), d_q (10) device evaluation vectors, d_pi the public-input evaluations, w_omega = d_w[0..3]
 * shifted left by `shift`; mds = the 3 x 3 Poseidon MDS matrix (row-major, ark).  d_out = f_gc. */
int halo_gate_constraints_dev(halo_field_t field, const void* const* d_w, const void* const* d_r,
                              const void* const* d_q, const void* d_pi, const halo_fe_t* mds, size_t n,
                              unsigned shift, void* d_out, void* stream);
/* Running product of the permutation argument (protocol.rs:143-154): inclusive prefix product
 * out[i] = prod_{j<=i} in[j] over n device elements (reverse != 0: suffix product prod_{j>=i}). */
int halo_evals_scan_dev(halo_field_t field, int reverse, const void* d_in, void* d_out, size_t n, void* stream);
/* sum_i zeta^i p_i (protocol.rs:542-548, the geometric combinations of round 5) over k <= 64 device
 * coefficient vectors d_polys[i] of lens[i] ark elements (shorter ones zero-extended) into d_out
 * (n_out elements, n_out >= max lens[i]), one launch on `stream`. */
int halo_poly_lincomb_dev(halo_field_t field, const void* const* d_polys, const size_t* lens, size_t k,
                          const halo_fe_t* zeta, void* d_out, size_t n_out, void* stream);

/* ------------------------------------------------------------------ a8: evaluation / dots */
/* DensePolynomial::evaluate (Horner; pcdl.rs:49,471), k polynomials at one point z. */
int halo_poly_eval_batch(halo_field_t field, const halo_fe_t* const* polys, const size_t* lens,
                         size_t k, const halo_fe_t* z, halo_fe_t* out);
/* Device-resident variant: d_polys is a host array of k device pointers (ark coefficients);
 * d_out receives k device field elements.  Stream-ordered. */
int halo_poly_eval_batch_dev(halo_field_t field, const void* const* d_polys, const size_t* lens, size_t k,
                             const halo_fe_t* z, void* d_out, void* stream);
/* group::scalar_dot (crates/group/src/group.rs:43-45). */
int halo_scalar_dot(halo_field_t field, const halo_fe_t* xs, const halo_fe_t* ys, size_t n,
                    halo_fe_t* out);
/* group::construct_powers (crates/group/src/group.rs:58-66): out[i] = z^i, i < n. */
int halo_construct_powers(halo_field_t field, const halo_fe_t* z, size_t n, halo_fe_t* out);

/* ------------------------------------------------------------------ a9: IPA folding
 * The round loop of pcdl::open_without_eval (crates/accumulation/src/pcdl.rs:404-438) with the
 * vectors device-resident across rounds; the caller keeps the Fiat-Shamir transcript and
 * supplies xi each round.  Session lifecycle:
 *   begin(cs = p'.coeffs resized to n, z, H') -> per round: round_lr -> (transcript) -> fold
 *   -> end(U = G[0], c = c[0]).  gs starts as the resident SRS prefix Gs[0..n) (pcdl.rs:393). */
typedef struct halo_ipa_session halo_ipa_session;
int halo_ipa_begin(halo_curve_t curve, const halo_fe_t* cs, size_t n, const halo_fe_t* z,
                   const halo_wrapped_point_t* H_prime, halo_ipa_session** out);
/* As halo_ipa_begin with the n coefficients already on the device (ark format; null stream order). */
int halo_ipa_begin_dev(halo_curve_t curve, const void* d_cs, size_t n, const halo_fe_t* z,
                       const halo_wrapped_point_t* H_prime, halo_ipa_session** out);
/* The same sessions with pcdl::open_without_eval's H' = xi_0 H (pcdl.rs:390-391) formed inside:
 * the caller passes H (WrappedPoint) and xi_0 (ark) instead of H'; the hiding terms <c, z> H' of
 * every round use a 2^i H table (built once per H and kept) with the dots scaled by xi_0, so a
 * session needs neither the scalar multiplication for H' nor its own 2^i H' doubling chain. */
int halo_ipa_begin_xi(halo_curve_t curve, const halo_fe_t* cs, size_t n, const halo_fe_t* z,
                      const halo_wrapped_point_t* H, const halo_fe_t* xi0, halo_ipa_session** out);
int halo_ipa_begin_dev_xi(halo_curve_t curve, const void* d_cs, size_t n, const halo_fe_t* z,
                          const halo_wrapped_point_t* H, const halo_fe_t* xi0, halo_ipa_session** out);
/* Session over explicit vectors G (WrappedPoints), c, z of length n (power of two >= 2) instead of
 * the SRS prefix and the powers of z: one rank's shard of a distributed opening (the
 * strided split G[i P + r] keeps every fold pair on one rank) and its collapsed final rounds. */
int halo_ipa_begin_vectors(halo_curve_t curve, const halo_wrapped_point_t* gs, const halo_fe_t* cs,
                           const halo_fe_t* zs, size_t n, const halo_wrapped_point_t* H_prime,
                           halo_ipa_session** out);
/* pcdl::open_without_eval (crates/accumulation/src/pcdl.rs:326-392) as one session whose p, p_bar
 * and p' never leave the device; the caller keeps the transcript between the steps, as the
 * reference does:
 *   halo_pcdl_open_begin(p: len coefficients, d, z)    n = d + 1 > 1 a power of two, p.degree() <= d,
 *                                                      d <= D (pcdl.rs:338-341); c = p padded to n;
 *                                                      v_out (optional) = p(z), pcdl::open's evaluation (pcdl.rs:471)
 *   hiding (w = Some):
 *     halo_pcdl_open_blind(q: d coefficients, w_bar) -> C_bar       p_bar = (X - z) q,
 *                                                      C_bar = pcdl::commit(p_bar, d, w_bar) (pcdl.rs:344-355)
 *     (transcript: absorb_g(C, C_bar), absorb_fr(z, v), alpha = challenge)
 *     halo_pcdl_open_combine(alpha, C, w) -> w', C'  c = p + alpha p_bar, w' = w + alpha w_bar,
 *                                                      C' = C + alpha C_bar - w' S (pcdl.rs:366-371)
 *   (transcript: absorb_g(C'), absorb_fr(z, v), xi_0 = challenge)
 *   halo_pcdl_open_start(H, xi_0)                     H' = xi_0 H (pcdl.rs:390; H = NULL: the resident
 *                                                      SRS's pp.H), then the rounds
 * followed by halo_ipa_round_lr / halo_ipa_fold / halo_ipa_end as for the other sessions.  The
 * rounds refuse a session that was not started. */
int halo_pcdl_open_begin(halo_curve_t curve, const halo_fe_t* p, size_t len, size_t d, const halo_fe_t* z,
                         halo_fe_t* v_out, halo_ipa_session** out);
int halo_pcdl_open_blind(halo_ipa_session* s, const halo_fe_t* q, const halo_fe_t* w_bar, halo_wrapped_point_t* C_bar);
int halo_pcdl_open_combine(halo_ipa_session* s, const halo_fe_t* alpha, const halo_wrapped_point_t* C,
                           const halo_fe_t* w, halo_fe_t* w_prime, halo_wrapped_point_t* C_prime);
int halo_pcdl_open_start(halo_ipa_session* s, const halo_wrapped_point_t* H, const halo_fe_t* xi0);
/* L = <c_r, G_l> + H' <c_r, z_l>,  R = <c_l, G_r> + H' <c_l, z_r>  (pcdl.rs:412-418) */
int halo_ipa_round_lr(halo_ipa_session* s, halo_wrapped_point_t* L, halo_wrapped_point_t* R);
/* G_l[j] = G_l[j] + xi G_r[j] (affine), c_l[j] += xi^-1 c_r[j], z_l[j] += xi z_r[j]; m /= 2
 * (pcdl.rs:427-437).  xi_inv may be NULL: the library forms xi^-1 on the host (binary extended
 * Euclid), as the reference's fold does itself; xi = 0 is HALO_EINVAL. */
int halo_ipa_fold(halo_ipa_session* s, const halo_fe_t* xi, const halo_fe_t* xi_inv);
/* k independent openings advanced in lockstep (each session has its own stream; all k rounds /
 * folds are enqueued before any is waited for, so the openings overlap on the device): L[i], R[i]
 * of session i; xi[i], xi_inv[i] for session i (xi_inv NULL: formed on the host).  The fold checks
 * every session and xi before it enqueues any fold: an argument error (a null, closed or repeated
 * session, xi = 0) leaves all k sessions unfolded. */
int halo_ipa_round_lr_multi(halo_ipa_session* const* ses, size_t k, halo_wrapped_point_t* L,
                            halo_wrapped_point_t* R);
int halo_ipa_fold_multi(halo_ipa_session* const* ses, size_t k, const halo_fe_t* xi, const halo_fe_t* xi_inv);
/* One round whose L, R stay on the device: d_lr (256 B of device memory) receives L then R as packed XYZZ
 * (halo_point_sum_xyzz_dev's format), ordered before later work on `stream`; no host wait.  The
 * distributed opening's per-round reduce (pcdl.rs:412-418 summed over the ranks' shards):
 * round_lr_dev -> all-gather -> halo_point_sum_xyzz_dev -> one D2H -> halo_xyzz_to_wrapped. */
int halo_ipa_round_lr_dev(halo_ipa_session* s, void* d_lr, void* stream);
/* Current half-length m, and the folded vectors (length 2m) copied back to the host (any of the
 * output pointers may be NULL).  Sessions over the resident SRS do not materialise G in their
 * weighted / tail rounds (the default; HALO_IPA_WEIGHTED=0 and HALO_IPA_TAIL=0 keep G folded every
 * round): asking for gs there is HALO_EINVAL. */
int halo_ipa_state(halo_ipa_session* s, size_t* m, halo_wrapped_point_t* gs, halo_fe_t* cs,
                   halo_fe_t* zs);
/* U = G_0 and c_0 after the last round (in weighted / tail rounds U is only defined then).  The
 * session's streams and device buffers go back to a per-device pool (reused by the next opening;
 * released by halo_shutdown), so a warm opening allocates nothing.  After its end a handle must not
 * be used again: every entry point refuses (HALO_EINVAL) a handle whose session was destroyed or is
 * idle in the pool, but once the pool hands that session to a later opening the old handle names the
 * new opening. */
int halo_ipa_end(halo_ipa_session* s, halo_wrapped_point_t* U, halo_fe_t* c);
/* halo_ipa_end of k lockstep sessions (U[i], c[i] of session i; U or c may be NULL): every session's
 * final U sum is enqueued on its own stream before any is waited for.  Argument errors (a null,
 * closed or repeated session) release nothing; otherwise every listed session is released, also on
 * an error. */
int halo_ipa_end_multi(halo_ipa_session* const* ses, size_t k, halo_wrapped_point_t* U, halo_fe_t* c);
/* One stateless fold over host vectors of length 2m (the loop body of pcdl.rs:427-435), in place
 * on the left halves. */
int halo_ipa_fold_host(halo_curve_t curve, halo_wrapped_point_t* gs, halo_fe_t* cs, halo_fe_t* zs,
                       size_t m, const halo_fe_t* xi, const halo_fe_t* xi_inv);

/* ------------------------------------------------------------------ measurement hooks
 * When enabled, the library brackets its dominant kernels (MSM bucket accumulation, NTT passes)
 * with hipEvents on the stream they run on; halo_profile_read returns the number of launches and
 * the summed kernel time in ms for a kernel name ("msm_acc", "ntt_pass") since the last reset. */
int halo_profile_enable(int on);
int halo_profile_read(const char* name, size_t* launches, double* total_ms);
int halo_profile_reset(void);

/* ------------------------------------------------------------------ field self-test helpers
 * Elementwise device field ops over host arrays (used by the parity tests of a1):
 * op 0 = mul, 1 = add, 2 = sub, 3 = sqr(a), 4 = inverse(a) (0 -> 0), 5 = neg(a). */
int halo_field_op(halo_field_t field, int op, const halo_fe_t* a, const halo_fe_t* b, size_t n,
                  halo_fe_t* out);
/* Elementwise device curve ops over host arrays (parity tests of a2):
 * op 0 = a + b, 1 = 2a, 2 = k * a (k = scalars, Montgomery). */
int halo_curve_op(halo_curve_t curve, int op, const halo_wrapped_point_t* a,
                  const halo_wrapped_point_t* b, const halo_fe_t* k, size_t n,
                  halo_wrapped_point_t* out);

#ifdef __cplusplus
}
#endif
#endif /* HALO_GPU_H */
