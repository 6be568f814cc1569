"""ctypes binding of the C oracle (oracle/oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
Arrays are numpy uint64 arrays of shape (n, 4) (field elements, Montgomery) or (n, 8)
(WrappedPoint affine, Montgomery, (0,0) = identity).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

CURVE_ID = {"pallas": 0, "vesta": 1}
FIELD_ID = {"fp": 0, "fq": 1}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.orc_msm.argtypes = [ctypes.c_int, u64p, u64p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, u64p]
        L.orc_ntt.argtypes = [ctypes.c_int, u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_poly_eval.argtypes = [ctypes.c_int, u64p, ctypes.c_size_t, u64p, u64p]
        L.orc_scalar_dot.argtypes = [ctypes.c_int, u64p, u64p, ctypes.c_size_t, u64p]
        L.orc_field_mul.argtypes = [ctypes.c_int, u64p, u64p, u64p]
        L.orc_field_inv.argtypes = [ctypes.c_int, u64p, u64p]
        L.orc_ipa_fold.argtypes = [ctypes.c_int, u64p, u64p, u64p, ctypes.c_size_t, u64p, u64p, ctypes.c_int]
        L.orc_srs_hash_scalar.argtypes = [ctypes.c_int, ctypes.c_uint64, u64p]
        L.orc_generator_mul.argtypes = [ctypes.c_int, u64p, u64p]
        L.orc_srs_generate.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, u64p]
        L.orc_msm_window_size.argtypes = [ctypes.c_size_t]
        L.orc_msm_window_size.restype = ctypes.c_int
        L.orc_max_threads.restype = ctypes.c_int
        L.orc_evals_op.argtypes = [ctypes.c_int, ctypes.c_int, u64p, u64p, u64p, ctypes.c_uint32, ctypes.c_size_t,
                                   u64p, ctypes.c_int]
        L.orc_perm_acc.argtypes = [ctypes.c_int, u64p, u64p, ctypes.c_size_t, u64p]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def max_threads() -> int:
    return lib().orc_max_threads()


def msm(curve: str, bases: np.ndarray, scalars: np.ndarray, scalars_mont: bool = True, threads: int = 0) -> np.ndarray:
    n = min(len(bases), len(scalars))
    bases = np.ascontiguousarray(bases[:n])
    scalars = np.ascontiguousarray(scalars[:n])
    out = np.zeros(8, dtype=np.uint64)
    lib().orc_msm(CURVE_ID[curve], _p(bases), _p(scalars), n, int(scalars_mont), threads, _p(out))
    return out


def ntt(field: str, data: np.ndarray, inverse: bool = False, threads: int = 0) -> np.ndarray:
    a = np.ascontiguousarray(data.copy())
    n = len(a)
    logn = n.bit_length() - 1
    assert 1 << logn == n
    lib().orc_ntt(FIELD_ID[field], _p(a), logn, int(inverse), threads)
    return a


def poly_eval(field: str, coeffs: np.ndarray, z: np.ndarray) -> np.ndarray:
    coeffs = np.ascontiguousarray(coeffs)
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_poly_eval(FIELD_ID[field], _p(coeffs), len(coeffs), _p(np.ascontiguousarray(z)), _p(out))
    return out


def scalar_dot(field: str, xs: np.ndarray, ys: np.ndarray) -> np.ndarray:
    n = min(len(xs), len(ys))
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_scalar_dot(FIELD_ID[field], _p(np.ascontiguousarray(xs[:n])), _p(np.ascontiguousarray(ys[:n])), n, _p(out))
    return out


def field_mul(field: str, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_field_mul(FIELD_ID[field], _p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), _p(out))
    return out


def field_inv(field: str, a: np.ndarray) -> np.ndarray:
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_field_inv(FIELD_ID[field], _p(np.ascontiguousarray(a)), _p(out))
    return out


def ipa_fold(curve: str, gs: np.ndarray, cs: np.ndarray, zs: np.ndarray, xi: np.ndarray, xi_inv: np.ndarray, threads: int = 0):
    gs = np.ascontiguousarray(gs.copy())
    cs = np.ascontiguousarray(cs.copy())
    zs = np.ascontiguousarray(zs.copy())
    m = len(gs) // 2
    lib().orc_ipa_fold(CURVE_ID[curve], _p(gs), _p(cs), _p(zs), m, _p(np.ascontiguousarray(xi)),
                       _p(np.ascontiguousarray(xi_inv)), threads)
    return gs[:m], cs[:m], zs[:m]


def evals_op(field: str, op: int, a: np.ndarray, b=None, s=None, e: int = 0, threads: int = 0) -> np.ndarray:
    """Elementwise Evals op over Montgomery words (0 add, 1 sub, 2 mul, 3 scale, 4 add_scalar,
    5 sub_scalar, 6 pow)."""
    a = np.ascontiguousarray(a)
    out = np.empty_like(a)
    bp = _p(np.ascontiguousarray(b)) if b is not None else None
    sp = _p(np.ascontiguousarray(s)) if s is not None else None
    lib().orc_evals_op(FIELD_ID[field], op, _p(a), bp, sp, e, len(a), _p(out), threads)
    return out


def perm_acc(field: str, f: np.ndarray, g: np.ndarray) -> np.ndarray:
    """z[0] = 1, z[i] = z[i-1] f[i] / g[i] (sequential; protocol.rs:143-154)."""
    f, g = np.ascontiguousarray(f), np.ascontiguousarray(g)
    out = np.empty_like(f)
    lib().orc_perm_acc(FIELD_ID[field], _p(f), _p(g), len(f), _p(out))
    return out


def srs_generate(curve: str, n: int, threads: int = 0) -> np.ndarray:
    out = np.zeros((n, 8), dtype=np.uint64)
    lib().orc_srs_generate(CURVE_ID[curve], n, threads, _p(out))
    return out


def srs_hash_scalar(curve: str, j: int) -> np.ndarray:
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_srs_hash_scalar(CURVE_ID[curve], j, _p(out))
    return out


def generator_mul(curve: str, k_canonical: np.ndarray) -> np.ndarray:
    out = np.zeros(8, dtype=np.uint64)
    lib().orc_generator_mul(CURVE_ID[curve], _p(np.ascontiguousarray(k_canonical)), _p(out))
    return out


def msm_window_size(n: int) -> int:
    return lib().orc_msm_window_size(n)


def synth_scalars(seed: int, n: int) -> np.ndarray:
    """numpy restatement of halo_synth_scalar (msm.hip synth_scalar: a splitmix64 stream per index,
    top word masked below 2^253, zero replaced by 1): the known discrete logs k_j of the synthetic
    SRS G_j = k_j G, canonical (not Montgomery)."""
    j = np.arange(n, dtype=np.uint64)
    st = np.uint64(seed) ^ (j * np.uint64(0xD1B54A32D192ED03))
    out = np.zeros((n, 4), dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in range(4):
            st = st + np.uint64(0x9E3779B97F4A7C15)
            z = st.copy()
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out[:, i] = z ^ (z >> np.uint64(31))
    out[:, 3] &= np.uint64(0x1FFFFFFFFFFFFFFF)
    zero = (out == 0).all(axis=1)
    out[zero, 0] = 1
    return out


def known_log_msm(curve: str, scalars_mont: np.ndarray, logs_canonical: np.ndarray) -> np.ndarray:
    """MSM(G_j = k_j G, s) = (sum_j s_j k_j) G for bases with known discrete logs: one Montgomery dot
    product (S_j k_j R^-1 = s_j k_j) and one scalar multiplication of the generator."""
    acc = scalar_dot("fp" if curve == "pallas" else "fq", scalars_mont, logs_canonical)
    return generator_mul(curve, acc)


def window_scalars(curve: str, scalars_mont: np.ndarray, c: int, lo: int, hi: int) -> np.ndarray:
    """The part of each scalar carried by the signed c-bit windows [lo, hi) of the device's digit
    recoding (msm.hip k_digits: s > r/2 is replaced by r - s with every digit negated; digits in
    [-2^(c-1), 2^(c-1)] with a carry), as Montgomery scalars: sum_{w in [lo, hi)} d_w 2^(c w) mod r.
    The window-partitioned MSM's partial of rank r is MSM(G, window_scalars(...)) (checker only)."""
    import pasta as P
    r = P.CURVES[curve].scalar
    out = np.zeros_like(scalars_mont)
    W = -(-255 // c)
    for j, row in enumerate(np.asarray(scalars_mont).reshape(-1, 4)):
        s = P.from_mont(P.limbs_to_int(row), r)
        neg = (r - s) < s
        if neg:
            s = r - s
        carry, acc = 0, 0
        for w in range(W):
            v = ((s >> (c * w)) & ((1 << c) - 1)) + carry
            if v > (1 << (c - 1)):
                d, carry = v - (1 << c), 1
            else:
                d, carry = v, 0
            if lo <= w < hi:
                acc += d << (c * w)
        if neg:
            acc = -acc
        out[j] = P.int_to_limbs(P.to_mont(acc % r, r))
    return out
