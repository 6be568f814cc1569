// Internal interfaces shared between msm.hip, ipa.hip and the multi-GPU glue.
#pragma once
#include <vector>
#include "runtime.hpp"

namespace halo {

int msm_window_bits(size_t n);
// MSM over device-resident internal-format affine bases (64 B each) and ark-format scalars.
// Writes one ark WrappedPoint (64 B) to d_out_wrapped (device).  Optional hiding term
// hide_scalar * P where hide_table = {2^i P : i < 256} (internal affine; both device pointers), or
// with hide_glv {2^i P : i < 128} and the GLV split of the scalar (k_hide_term).  out_xyzz: the
// result is written as 128 B packed XYZZ instead of an affine WrappedPoint (host_xyzz_to_wrapped).
// hide_ready: event after which the hiding table is complete (built on another stream).
int msm_device(DeviceState* st, int curve, const void* bases_int, const void* scalars_ark, size_t n,
               const void* hide_table, const void* hide_scalar, void* d_out_wrapped, hipStream_t s,
               bool async = false, bool hide_glv = false, bool out_xyzz = false, hipEvent_t hide_ready = nullptr,
               int preset = -1);
// Claims the scratch set the next MSM on stream s will use (s waits for its previous tail) and
// returns its base-conversion buffer; pass the set to msm_device as `preset`.
int msm_claim_set(DeviceState* st, hipStream_t s, int* set, DevBuf** conv);
// k commitments over the resident SRS prefix, MSM i over lens[i] ark scalars at d_scalars[i] (device),
// result i (WrappedPoint) at d_out + 64 i; asynchronous on s like msm_device(async) (msm_join).
int msm_batch_device(DeviceState* st, int curve, const void* const* d_scalars, const size_t* lens, size_t k, void* d_out,
                     hipStream_t s);
// Destroys the MSM pipeline's streams and events (halo_shutdown).
void msm_shutdown();
// Releases the pooled IPA sessions (halo_shutdown, ipa.hip).
void ipa_shutdown();
// Makes stream s wait for the reduction tails of the async MSMs enqueued on s.
int msm_join(DeviceState* st, hipStream_t s);
// Restarts the scratch-set slot assignment (no owners, first sets) when no MSM tail is running.
void msm_slots_reset(DeviceState* st);
// MSM over the resident SRS prefix (window-shifted copies when precomputed); optional hiding
// scalar (ark, device pointer) times S.
int msm_srs_device(DeviceState* st, int curve, const void* scalars_ark, size_t n, const void* hide_scalar,
                   void* d_out_wrapped, hipStream_t s, bool async = false, bool out_xyzz = false);
// MSM over the resident SRS range [offset, offset + n) with a caller hiding table (2^i P, i < 256,
// internal affine) and scalar; uses the window-shifted copies (returns HALO_EINVAL without them).
// blk_lg < 32: scalar i goes with point offset + i + ((i >> blk_lg) << blk_lg), i.e. the blocks
// [2b B, 2b B + B) (B = 2^blk_lg) of the range -- the even half-blocks an IPA round's G_l / G_r
// occupy in the unfolded SRS.
int msm_srs_range_device(DeviceState* st, int curve, size_t offset, const void* scalars_ark, size_t n,
                         const void* hide_table, const void* hide_scalar, void* d_out_wrapped, hipStream_t s,
                         bool async, uint32_t blk_lg = 32, bool hide_glv = false, bool out_xyzz = false,
                         hipEvent_t hide_ready = nullptr);
// Batched MSM with shared scalars: out[i] = sum_{u < T} w[u] bases[i + u len] for i < len
// (internal affine bases, ark scalars; outputs internal affine, or XYZZ (128 B) when xyzz_out;
// stream-ordered on s).
struct BatchScratch {
    DevBuf digits, lists, keys, vals, bstart, partials, bucket_sums, window_sums;
};
// The IPA weighted rounds' L and R (sum_i sl[i] G[map(i)], sum_i sr[i] G[m + map(i)], map(i) =
// i + (i >> lgm) << lgm, m = 2^lgm) each plus dot H' (hide_l / hide_r ark scalars, GLV table), for
// np <= 4 sessions with the same geometry, as one MSM over the window-shifted SRS; packed XYZZ
// outputs; asynchronous on s (msm_join).
struct MsmPairIO {
    const void *sl, *sr, *hide_l, *hide_r;
    void *out_l, *out_r;
};
// pre_hide (optional): enqueued on the MSM's tail stream right before the hiding terms, after the MSM
// start (the caller's prior work on s) -- the IPA's weighted rounds form the hiding terms' dots there,
// beside the digit / sort / accumulation phase instead of ahead of it.
struct MsmPreHide {
    void (*fn)(hipStream_t ts, void* ctx);
    void* ctx;
};
// host_emit (np == 1 only): L and R also go to pinned host memory with flags = seq (MsmTailArgs::pair_host)
int msm_srs_pairs_device(DeviceState* st, int curve, size_t np, const MsmPairIO* io, size_t half, uint32_t lgm,
                         const void* hide_table, hipStream_t s, hipEvent_t hide_ready, const MsmPreHide* pre_hide = nullptr,
                         uint32_t* host_emit = nullptr, uint32_t seq = 0);
// shift_stride > 0: bases are the resident window-shifted SRS (copy w = 2^(c_s w) G at w shift_stride):
// every c_s-bit digit of w[u] is split into three unsigned sub-digits, so the final Horner runs
// over three windows (~2 c_s / 3 doublings) instead of ~255 / c windows (~255 doublings).
int msm_shared_batch(DeviceState* st, int curve, const void* bases_int, const void* w_ark, size_t T, size_t len,
                     void* out, bool xyzz_out, BatchScratch& S, hipStream_t s, size_t shift_stride = 0, int c_s = 0);
int srs_precompute_windows(DeviceState* st, int curve, hipStream_t s, int c = 0, int w_lo = 0, int w_hi = 0);
// Small MSM over the resident SRS prefix (1 <= n <= srs_small_max(), ipa.hip): every (point, 4-bit GLV
// window) term is one entry of a per-SRS multiples table, then block trees with the hiding term
// hide_scalar * S from the 2^i S table -- no sort, buckets or bucket reduction.  Stream-ordered on s;
// writes one ark WrappedPoint to d_out_wrapped.
size_t srs_tab_n();      // points covered by the SRS multiples table (HALO_SRS_TAB_N, default 8192)
size_t srs_small_max();  // largest MSM on the table path (HALO_SRS_SMALL_N, default srs_tab_n())
// The multiples table of the SRS prefix (SrsState::small_tab, built on first use over
// min(srs_tab_n(), srs.n) points); stream s waits for its completion.  Shared by the small MSMs and
// by IPA sessions whose tail rounds start on the unfolded SRS prefix.
int srs_small_table(DeviceState* st, int curve, hipStream_t s);
// MSM of n <= msm_tiny_max() caller points (internal affine) by GLV windows and one Horner (ipa.hip):
// packed XYZZ to out_xyzz (device); scratch >= 4 KiB of device memory.  Stream-ordered on s.
int msm_tiny(int curve, const void* bases_int, const void* scalars_ark, size_t n, void* scratch, void* out_xyzz,
             hipStream_t s);
size_t msm_tiny_max();
// out_xyzz: the result as 128 B packed XYZZ (host_xyzz_to_wrapped) instead of a WrappedPoint.
// plus_wrapped (device WrappedPoint, or null): added to the result.
int msm_srs_small(DeviceState* st, int curve, const void* scalars_ark, size_t n, const void* hide_scalar,
                  void* d_out_wrapped, hipStream_t s, bool out_xyzz = false, const void* plus_wrapped = nullptr);
// The hiding branch of pcdl::open_without_eval on device buffers (field_ops.hip), stream-ordered on s:
// p_bar = (X - z) q (q: d ark coefficients, z: ark scalar) -> d + 1 ark coefficients;
// p' = p (len coefficients, zero-padded to n) + alpha p_bar (p' may alias p), w' = w + alpha w_bar,
// C' = C + alpha C_bar - w' S (C, C_bar, C' WrappedPoints; S internal affine).
int pcdl_pbar_device(int curve, const void* q, size_t d, const void* z, void* p_bar, hipStream_t s);
int pcdl_combine_device(int curve, const void* p, size_t len, const void* p_bar, size_t n, const void* alpha,
                        const void* w, const void* w_bar, const void* C, const void* C_bar, const void* S_int,
                        void* p_prime, void* C_prime, void* w_prime, hipStream_t s);
// p[i] += alpha p_bar[i] and p_bar[i] = alpha p_bar[i] in place (i < n); w' = w + alpha w_bar, negw = -w.
int pcdl_combine_scalars_device(int curve, void* p, void* p_bar, size_t n, const void* alpha, const void* w,
                                const void* w_bar, void* w_prime, void* negw, hipStream_t s);
// xyzz (128 B packed XYZZ) = xyzz (or, from_wrapped, the WrappedPoint first_wrapped) + the WrappedPoint
// at wrapped (one lane).
int xyzz_add_wrapped_device(int curve, void* xyzz, const void* wrapped, hipStream_t s, bool from_wrapped = false,
                            const void* first_wrapped = nullptr);
// Host conversion of a 128-B packed XYZZ point (internal format, each coordinate < 2p) to an ark
// WrappedPoint: one inversion in 4 x 64-bit Montgomery arithmetic on the CPU (identity -> (0, 0)).
void host_xyzz_to_wrapped(int curve, const void* xyzz, void* wrapped);
// x^-1 of an ark (Montgomery) scalar of the curve's scalar field, on the host (binary extended Euclid);
// false for x = 0
bool host_scalar_inverse(int curve, const void* x_ark, void* out_ark);
// k <= 16 points at once with one inversion (Montgomery's trick)
void host_xyzz_to_wrapped2(int curve, const void* const* xyzz, void* const* wrapped, int k);
int convert_wrapped_to_internal(int curve, const void* in, void* out, size_t n, hipStream_t s);
int convert_internal_to_wrapped(int curve, const void* in, void* out, size_t n, hipStream_t s);
// rad: the pass split to launch (null: ntt_radices(logn)); a caller that sized anything by the split
// (the zero-tail prune) passes the vector it used
int ntt_device_dispatch(DeviceState* st, int field, const void* d_in, void* d_out, void* d_tmp, unsigned logn,
                        size_t batch, int inverse, hipStream_t s, void* d_tmp2 = nullptr, unsigned prune = 0,
                        const std::vector<unsigned>* rad = nullptr);

// chunk-partial group size of the skew guard (msm_tail.hip k_group_sums)
constexpr uint32_t MSM_GROUP = 64;

// Inputs of the MSM's reduction tail (msm_tail.hip), launched on the tail stream.
struct MsmOuts8 {
    uint4* o[8];
};
struct MsmTailArgs {
    size_t n, NB, E, ng1, ng2;
    const uint32_t* skeys;
    const uint32_t* scount;
    uint32_t K;
    uint4 *first, *last, *g1, *g2;
    uint32_t* bstart;
    uint4 *bucket_sums, *rows, *cols, *terms, *window_sums;
    uint32_t L, H, logH, logL, NT;
    int SW, c;
    const uint4* hide_table;
    const uint4* hide_scalar;
    uint4* out_wrapped;
    bool batch_windows = false;  // SW windows of 128 buckets: k_batch_window_sums instead of the grid reduction
    // SW == 1 only: k_bitcombine also does k_final's work (+ final_hide, -> final_out as an ark
    // WrappedPoint (1) or packed XYZZ (2)); 0: it writes window_sums and k_final follows
    int final_mode = 0;
    const uint4* final_hide = nullptr;
    uint4* final_out = nullptr;
    uint32_t num_cu = 256;  // the device's CUs: sizes k_rowcol's entries per lane
    // pair MSMs (msm_srs_pairs): k_bitcombine's block w writes pair_outs.o[w] = its window sum +
    // pair_hide[w] (packed XYZZ) instead of window_sums -- no separate output launch
    const uint4* pair_hide = nullptr;
    MsmOuts8 pair_outs{};
    // optional: outputs 0 and 1 also stored straight into pinned host memory (32 words each) with
    // release flags = pair_seq at pair_host + 64 words (the IPA's polled L / R, as its tail rounds)
    uint32_t* pair_host = nullptr;
    uint32_t pair_seq = 0;
};
int msm_tail_launch(int curve, const MsmTailArgs& a, hipStream_t ts);
// Horner over W window sums (+ the hiding term) -> ark WrappedPoint, or packed XYZZ (xyzz_out)
int msm_final_launch(int curve, const uint4* window_sums, int W, int c, const uint4* hide, uint4* out, int xyzz_out,
                     hipStream_t s);

}  // namespace halo
