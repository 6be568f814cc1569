// Host-side runtime shared by every translation unit of libhalo_gpu.so: error reporting,
// per-device state, device memory helpers.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/halo_gpu.h"

namespace halo {

// ---- errors ---------------------------------------------------------------------------------
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();

#define HALO_HIP(expr)                                                                      \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return ::halo::set_error(HALO_EDEVICE, "%s failed: %s (%s:%d)", #expr,          \
                                     hipGetErrorString(_e), __FILE__, __LINE__);            \
    } while (0)

#define HALO_CHECK(expr)              \
    do {                              \
        int _rc = (expr);             \
        if (_rc != HALO_OK) return _rc; \
    } while (0)

// ---- tuning (halo_set_tuning): path selections the parity tests pin; read on every use
enum TuneKey { TUNE_IPA_WEIGHTED, TUNE_IPA_TAIL, TUNE_IPA_SRS_TAIL_N, TUNE_IPA_MAT_N, TUNE_MSM_MULTI_MAX, TUNE_IPA_POOL_KEEP,
               TUNE_NTT_BIG_MAX_LOG, TUNE_NTT_EVEN_SPLIT, TUNE_IPA_PAIR_MAX, TUNE_COUNT };
long long tuning(TuneKey k);

// ---- device buffers ---------------------------------------------------------------------------
// Grow-only device buffer (no shrinking; reused across calls so that timed regions never allocate).
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    int reserve(size_t n);  // ensures capacity >= n bytes
    void release();         // hipFree now (the caller has ordered every user of the buffer before it)
    template <class T>
    T* as() const { return static_cast<T*>(ptr); }
    ~DevBuf();
};

// Per-device, per-curve state (the OnceLock<PublicParams> analogue, crates/group/src/pp.rs:63-94)
struct SrsState {
    DevBuf gs;          // n internal-format affine points (64 B each)
    size_t n = 0;
    bool has_sh = false;
    uint32_t S[16];     // internal packed (x, y)
    uint32_t H[16];
    halo_wrapped_point_t H_wrapped;  // H as uploaded (the key of its 2^i H table)
    DevBuf s_table;     // 2^i S (i < 256), internal affine: hiding term of pedersen::commit
    // 2^i H (i < 128), internal affine: the IPA's H' = xi_0 H terms (halo_ipa_begin_xi), one table per
    // distinct H, never rewritten while the library lives (open sessions keep pointers into them)
    struct HTable {
        uint64_t key[8];  // the WrappedPoint H the table was built from
        DevBuf t;
    };
    std::vector<std::unique_ptr<HTable>> h_tables;
    // d 2^(4 w) G_k (k < small_n0, w < 32, 1 <= d <= 8), XYZZ: small SRS MSMs, IPA tails (ipa.hip); shared
    // with the open IPA sessions that read it, so a rebuild never overwrites a buffer in use
    std::shared_ptr<DevBuf> small_tab;
    size_t small_n0 = 0;             // 0 = not built for the current SRS
    hipEvent_t small_tab_ev = nullptr;  // small_tab's build completed
    DevBuf small_scr;                // GLV digits, block partials of a small MSM
    hipEvent_t small_ev = nullptr;   // last small MSM's completion (orders reuse of small_scr)
    DevBuf shifted;     // optional window-shifted copies
    int shifted_c = 0;  // window bits of `shifted` when it holds every window (0: not built)
    int part_c = 0, part_w0 = 0, part_w1 = 0;  // ... or only the windows [part_w0, part_w1) of width part_c
    bool shifted_has_id = true;  // some SRS point is the identity (k_acc then tests every base)
    int shifted_windows = 0;
    // Every writer of `gs` calls this: the tables derived from the old points (window-shifted copies,
    // the small-MSM / tail multiples table) are rebuilt on next use.  (a synthesize after
    // a small commit used to keep the old SRS's table.)
    void invalidate_derived() {
        shifted_c = part_c = 0;
        shifted_windows = 0;
        shifted_has_id = true;
        small_n0 = 0;
    }
};

struct DeviceState {
    int device = -1;
    int num_cu = 256;              // compute units (MI355X: 256), sizes one-round launches
    std::mutex mu;                 // serialises API calls on this device
    SrsState srs[2];               // per curve
    // scratch
    DevBuf scratch[8];
    DevBuf scan_tmp;     // halo_evals_scan_dev block totals
    DevBuf gate_tmp;     // halo_gate_constraints_dev partial vectors
    DevBuf eval_meta[2]; // halo_poly_eval_batch_dev: pointer/length tables, partial sums
    // NTT twiddle caches: key (field, log, inverse)
    struct Twiddles {
        int field, logn, inverse;
        DevBuf hi, lo;
        int lo_bits;
        DevBuf stage;    // stage twiddles: entry 2^s - 1 + k = omega_{2^(s+1)}^k, s < 11 (9 limbs, 48 B each)
        DevBuf pass[4];  // per-pass pre-twiddle tables (logn <= 24), see ntt.hip
        bool has_pass = false;
        uint64_t split = 0;  // the pass split the tables were built for (ntt_radices, tuning-dependent)
    };
    std::vector<std::unique_ptr<Twiddles>> tw;
    struct RTable {
        int field, logr, inverse;
        DevBuf t;
    };
    std::vector<std::unique_ptr<RTable>> rt;
    // ScratchUse state: completion event of the last scratch user and its stream
    hipEvent_t scratch_ev = nullptr;
    hipStream_t scratch_last = nullptr;
    bool scratch_used = false;
};

// Shared-scratch fence: the device-global scratch buffers (scratch[], scan_tmp, gate_tmp, eval_meta)
// are used by calls on different streams (the caller's torch stream, IPA session streams, the null
// stream of the host-array calls).  Every call that touches them holds a ScratchUse for its stream:
// the stream first waits for the last other-stream user's completion event, and the call records a
// new one when it ends, so the uses are ordered on the device whatever the streams.  (The API mutex
// only orders the enqueueing.)
struct ScratchUse {
    DeviceState* st;
    hipStream_t s;
    ScratchUse(DeviceState* st, hipStream_t s);
    ~ScratchUse();
};

// Current device's state (calls halo_init(current device) lazily).  Returns nullptr on failure
// (with the error set).
DeviceState* current_state();

// Pinned staging helpers
int copy_h2d(void* dst, const void* src, size_t bytes, hipStream_t s);
int copy_d2h(void* dst, const void* src, size_t bytes, hipStream_t s);

// ---- measurement hooks (halo_profile_*) ----------------------------------------------------
// ProfScope owns a start/stop hipEvent pair for one launch when profiling is enabled; the launch
// goes through hipExtLaunchKernelGGL, which records the kernel's own start/stop on its stream
// (HALO_LAUNCH), so the measured time is the kernel's execution only.
bool prof_enabled();
struct ProfScope {
    int slot = -1;
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s = nullptr;
    ProfScope(const char* name, hipStream_t stream);
    ~ProfScope();
};

#define HALO_LAUNCH(prof, kern, grid, block, shmem, stream, ...)                                       \
    do {                                                                                              \
        if ((prof).slot >= 0)                                                                         \
            hipExtLaunchKernelGGL(kern, grid, block, shmem, stream, (prof).a, (prof).b, 0, __VA_ARGS__); \
        else                                                                                          \
            hipLaunchKernelGGL(kern, grid, block, shmem, stream, __VA_ARGS__);                        \
    } while (0)

inline bool is_pow2(size_t n) { return n && !(n & (n - 1)); }
inline unsigned ilog2(size_t n) {
    unsigned r = 0;
    while ((size_t(1) << (r + 1)) <= n) r++;
    return r;
}

}  // namespace halo
