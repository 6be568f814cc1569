"""ctypes binding of libhalo_gpu.so (the C ABI declared in include/halo_gpu.h).

This is the product path: it loads only halo_amd/lib/libhalo_gpu.so (hand-written HIP for gfx950)
and fails loudly if that library is missing or no GPU is present.  There is no CPU fallback.
"""
from __future__ import annotations

import atexit
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HALO_LIB") or os.path.join(_HERE, "lib", "libhalo_gpu.so")  # HALO_LIB: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "halo_gpu.h")

PALLAS, VESTA = 0, 1
FP, FQ = 0, 1
CURVES = {"pallas": PALLAS, "vesta": VESTA}
FIELDS = {"fp": FP, "fq": FQ}
# scalar field of each curve (Pallas scalars are Fp = ark_pallas::Fr)
SCALAR_FIELD = {PALLAS: FP, VESTA: FQ}
BASE_FIELD = {PALLAS: FQ, VESTA: FP}

HALO_OK = 0
STATUS_NAMES = {
    1: "EINVAL", 2: "ENOMEM", 3: "EDEVICE", 4: "ENOTPOW2", 5: "ESRSRANGE", 6: "EDEGREE", 7: "ELENGTH",
}


class HaloError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{STATUS_NAMES.get(code, code)}] {msg}")
        self.code = code


class HaloAssertion(HaloError, AssertionError):
    """Contract violation: the reference panics with this message (assert!)."""


_lib = None
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t

# (name, argtypes) for every exported symbol of include/halo_gpu.h
SIGNATURES = {
    "halo_init": [ctypes.c_int],
    "halo_device_count": [],
    "halo_last_error": [],
    "halo_abi_version": [],
    "halo_stream_sync": [_vp],
    "halo_set_tuning": [ctypes.c_char_p, ctypes.c_longlong],
    "halo_get_tuning": [ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong)],
    "halo_srs_upload": [ctypes.c_int, _vp, _sz, _vp, _vp],
    "halo_srs_len": [ctypes.c_int, ctypes.POINTER(_sz)],
    "halo_srs_synthesize": [ctypes.c_int, _sz, ctypes.c_uint64],
    "halo_synth_scalar": [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, _vp],
    "halo_srs_precompute_windows": [ctypes.c_int],
    "halo_srs_precompute_window_range": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int],
    "halo_msm": [ctypes.c_int, _vp, _sz, _vp, _sz, _vp],
    "halo_msm_srs": [ctypes.c_int, _vp, _sz, _vp],
    "halo_pedersen_commit": [ctypes.c_int, _vp, _vp, _sz, _vp, _sz, _vp],
    "halo_pcdl_commit": [ctypes.c_int, _vp, _sz, _sz, _vp, _vp],
    "halo_msm_dev": [ctypes.c_int, _vp, _vp, _sz, _vp, _vp],
    "halo_msm_window_bits": [_sz],
    "halo_srs_window_bits": [ctypes.c_int],
    "halo_msm_dev_async": [ctypes.c_int, _vp, _vp, _sz, _vp, _vp],
    "halo_msm_batch_dev": [ctypes.c_int, _vp, _vp, _sz, _vp, _vp],
    "halo_shutdown": [],
    "halo_srs_sh": [ctypes.c_int, _vp, _vp],
    "halo_msm_srs_windows_dev": [ctypes.c_int, _vp, _sz, ctypes.c_int, ctypes.c_int, _vp, _vp],
    "halo_srs_windows": [ctypes.c_int],
    "halo_point_dot_projective": [ctypes.c_int, _vp, _sz, _vp, _sz, _vp],
    "halo_pcdl_hiding_blind": [ctypes.c_int, _vp, _sz, _vp, _vp, _vp, _vp],
    "halo_pcdl_hiding_combine": [ctypes.c_int, _vp, _sz, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "halo_msm_join": [_vp],
    "halo_srs_read": [ctypes.c_int, _sz, _sz, _vp],
    "halo_point_sum": [ctypes.c_int, _vp, _sz, _vp],
    "halo_point_sum_dev": [ctypes.c_int, _vp, _sz, _sz, _vp, _vp],
    "halo_point_sum_xyzz_dev": [ctypes.c_int, _vp, _sz, _sz, _vp, _vp],
    "halo_point_sum_rows_dev": [ctypes.c_int, _vp, _sz, _sz, _vp, _vp],
    "halo_xyzz_to_wrapped": [ctypes.c_int, _vp, _sz, _vp],
    "halo_profile_enable": [ctypes.c_int],
    "halo_profile_read": [ctypes.c_char_p, ctypes.POINTER(_sz), ctypes.POINTER(ctypes.c_double)],
    "halo_profile_reset": [],
    "halo_ntt": [ctypes.c_int, _vp, ctypes.c_uint, ctypes.c_int],
    "halo_evaluate_over_domain": [ctypes.c_int, _vp, _sz, ctypes.c_uint, _vp],
    "halo_interpolate": [ctypes.c_int, _vp, ctypes.c_uint, _vp, ctypes.POINTER(_sz)],
    "halo_poly_mul": [ctypes.c_int, _vp, _sz, _vp, _sz, _vp, ctypes.POINTER(_sz)],
    "halo_ntt_dev": [ctypes.c_int, _vp, ctypes.c_uint, _sz, ctypes.c_int, _vp],
    "halo_ntt_dev_zero_tail": [ctypes.c_int, _vp, ctypes.c_uint, _sz, _sz, _vp],
    "halo_hpoly_coeffs": [ctypes.c_int, _vp, _sz, _vp],
    "halo_hpoly_combine": [ctypes.c_int, _vp, _sz, _sz, _vp, _vp, ctypes.POINTER(_sz)],
    "halo_hpoly_combine_dev": [ctypes.c_int, _vp, _sz, _sz, _vp, _vp, _vp],
    "halo_pcdl_decider_commit": [ctypes.c_int, _vp, _sz, _sz, _vp],
    "halo_trace_commit_batch": [ctypes.c_int, _vp, _sz, ctypes.c_uint, _sz, _vp, _vp, _vp],
    "halo_srs_load_bincode": [ctypes.c_int, _vp, _vp, _sz, _vp, _sz, _sz],
    "halo_evals_op": [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, ctypes.c_uint32, _vp, _sz],
    "halo_evals_op_dev": [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, ctypes.c_uint32, _vp, _sz, _vp],
    "halo_divide_by_vanishing": [ctypes.c_int, _vp, _sz, _sz, _vp, ctypes.POINTER(_sz), _vp, ctypes.POINTER(_sz)],
    "halo_divide_by_vanishing_dev": [ctypes.c_int, _vp, _sz, _sz, _vp, _vp, _vp],
    "halo_evals_scan_dev": [ctypes.c_int, ctypes.c_int, _vp, _vp, _sz, _vp],
    "halo_poly_lincomb_dev": [ctypes.c_int, _vp, _vp, _sz, _vp, _vp, _sz, _vp],
    "halo_gate_constraints_dev": [ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_uint, _vp, _vp],
    "halo_ntt_twiddle_dev": [ctypes.c_int, _vp, ctypes.c_uint, _sz, _sz, _sz, _sz, ctypes.c_int, _vp],
    "halo_transpose_dev": [_vp, _vp, _sz, _sz, _sz, _sz, _vp],
    "halo_poly_eval_batch": [ctypes.c_int, _vp, _vp, _sz, _vp, _vp],
    "halo_poly_eval_batch_dev": [ctypes.c_int, _vp, _vp, _sz, _vp, _vp, _vp],
    "halo_scalar_dot": [ctypes.c_int, _vp, _vp, _sz, _vp],
    "halo_construct_powers": [ctypes.c_int, _vp, _sz, _vp],
    "halo_ipa_begin": [ctypes.c_int, _vp, _sz, _vp, _vp, ctypes.POINTER(_vp)],
    "halo_ipa_begin_dev": [ctypes.c_int, _vp, _sz, _vp, _vp, ctypes.POINTER(_vp)],
    "halo_ipa_begin_xi": [ctypes.c_int, _vp, _sz, _vp, _vp, _vp, ctypes.POINTER(_vp)],
    "halo_ipa_begin_dev_xi": [ctypes.c_int, _vp, _sz, _vp, _vp, _vp, ctypes.POINTER(_vp)],
    "halo_ipa_round_lr_multi": [_vp, _sz, _vp, _vp],
    "halo_ipa_fold_multi": [_vp, _sz, _vp, _vp],
    "halo_ipa_round_lr_dev": [_vp, _vp, _vp],
    "halo_ipa_begin_vectors": [ctypes.c_int, _vp, _vp, _vp, _sz, _vp, ctypes.POINTER(_vp)],
    "halo_pcdl_open_begin": [ctypes.c_int, _vp, _sz, _sz, _vp, _vp, ctypes.POINTER(_vp)],
    "halo_pcdl_open_blind": [_vp, _vp, _vp, _vp],
    "halo_pcdl_open_combine": [_vp, _vp, _vp, _vp, _vp, _vp],
    "halo_pcdl_open_start": [_vp, _vp, _vp],
    "halo_ipa_round_lr": [_vp, _vp, _vp],
    "halo_ipa_fold": [_vp, _vp, _vp],
    "halo_ipa_state": [_vp, ctypes.POINTER(_sz), _vp, _vp, _vp],
    "halo_ipa_end": [_vp, _vp, _vp],
    "halo_ipa_end_multi": [_vp, _sz, _vp, _vp],
    "halo_ipa_fold_host": [ctypes.c_int, _vp, _vp, _vp, _sz, _vp, _vp],
    "halo_field_op": [ctypes.c_int, ctypes.c_int, _vp, _vp, _sz, _vp],
    "halo_curve_op": [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _sz, _vp],
}
RESTYPES = {"halo_last_error": ctypes.c_char_p, "halo_synth_scalar": None}


def load(path: str = LIB_PATH):
    """Load libhalo_gpu.so.  Raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: build it with `make -C halo_amd/csrc` (or __graft_entry__.build()); "
            "halo_amd has no CPU fallback")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7.  Load it first so
    # that this library's NEEDED libamdhip64.so.7 binds to the same runtime (otherwise two HIP
    # runtimes end up in the process and the second one sees no devices).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    for name, args in SIGNATURES.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            continue  # reported by missing_symbols(); tests/test_abi.py requires none missing
        fn.argtypes = args
        fn.restype = RESTYPES.get(name, ctypes.c_int)
    _lib = L
    if hasattr(L, "halo_shutdown"):
        # release streams/events before the HIP runtime tears down (registered after torch's own
        # handlers, so it runs before them)
        atexit.register(L.halo_shutdown)
    return L


def missing_symbols(path: str = LIB_PATH) -> list[str]:
    L = ctypes.CDLL(path)
    out = []
    for name in SIGNATURES:
        try:
            getattr(L, name)
        except AttributeError:
            out.append(name)
    return out


def last_error() -> str:
    return load().halo_last_error().decode()


_ASSERT_CODES = {4, 5, 6, 7}


def check(rc: int) -> None:
    if rc != HALO_OK:
        msg = last_error()
        if rc in _ASSERT_CODES:
            raise HaloAssertion(rc, msg)
        raise HaloError(rc, msg)


_initialized = set()


def ensure_device(device: int | None = None) -> None:
    """halo_init on first use (device from HALO_DEVICE / LOCAL_RANK, default 0)."""
    if device is None:
        if _initialized:  # the process already chose its device (e.g. bench.py's explicit one)
            return
        device = int(os.environ.get("HALO_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    if device in _initialized:
        return
    L = load()
    if L.halo_device_count() <= 0:
        raise HaloError(3, "no GPU visible: halo_amd runs only on the MI355X backend (no CPU fallback)")
    check(L.halo_init(device))
    _initialized.add(device)


def ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed to libhalo_gpu must be C-contiguous"
    # data_as keeps a reference to the array in the returned pointer object, so a temporary
    # (e.g. ``ptr(fe(x))`` inside a call's argument list) stays alive until the call returns
    return a.ctypes.data_as(ctypes.c_void_p)


def fe_array(a, n: int | None = None) -> np.ndarray:
    """Coerce to a C-contiguous (n, 4) uint64 array of field elements."""
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.uint64).reshape(-1, 4))
    if n is not None:
        assert arr.shape[0] == n
    return arr


def point_array(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64).reshape(-1, 8))


def set_tuning(key: str, value: int) -> None:
    """halo_set_tuning: a library-wide path selection (value -1 restores the default)."""
    check(load().halo_set_tuning(key.encode(), int(value)))


def get_tuning(key: str) -> int:
    v = ctypes.c_longlong(0)
    check(load().halo_get_tuning(key.encode(), ctypes.byref(v)))
    return v.value


class tuning:
    """Context manager: ``with tuning(ipa_weighted=0): ...`` sets the keys and restores the previous
    values on exit (the parity tests pin the IPA / commitment paths with it)."""

    def __init__(self, **kv):
        self.kv = kv
        self.prev = {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.prev[k] = get_tuning(k)
            set_tuning(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.prev.items():
            set_tuning(k, v)
        return False
