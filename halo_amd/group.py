"""Mirror of crates/group/src/group.rs and crates/group/src/pp.rs on the MI355X backend."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as H


def _curve(curve) -> int:
    return H.CURVES[curve] if isinstance(curve, str) else int(curve)


def _field(field) -> int:
    return H.FIELDS[field] if isinstance(field, str) else int(field)


def scalar_dot(xs, ys, field="fp") -> np.ndarray:
    """group.rs:43-45 ``scalar_dot``: sum_i xs[i] * ys[i] over the zipped length."""
    H.ensure_device()
    xs, ys = H.fe_array(xs), H.fe_array(ys)
    n = min(len(xs), len(ys))
    out = np.zeros(4, dtype=np.uint64)
    H.check(H.load().halo_scalar_dot(_field(field), H.ptr(np.ascontiguousarray(xs[:n])),
                                     H.ptr(np.ascontiguousarray(ys[:n])), n, H.ptr(out)))
    return out


def point_dot_affine(xs, Gs, curve="pallas") -> np.ndarray:
    """group.rs:48-50 ``point_dot_affine`` = ``Projective::msm_unchecked(Gs, xs)``; returns the
    canonical affine WrappedPoint (8 limbs)."""
    H.ensure_device()
    xs, Gs = H.fe_array(xs), H.point_array(Gs)
    out = np.zeros(8, dtype=np.uint64)
    H.check(H.load().halo_msm(_curve(curve), H.ptr(Gs), len(Gs), H.ptr(xs), len(xs), H.ptr(out)))
    return out


def point_dot(xs, Gs_projective, curve="pallas") -> np.ndarray:
    """group.rs:53-56: sum_i xs[i] Gs[i] over ark Projective (Jacobian) bases, (n, 12) u64 Montgomery."""
    H.ensure_device()
    x = H.fe_array(xs)
    g = np.ascontiguousarray(np.asarray(Gs_projective, dtype=np.uint64).reshape(-1, 12))
    out = np.zeros(8, dtype=np.uint64)
    H.check(H.load().halo_point_dot_projective(_curve(curve), H.ptr(x), len(x), H.ptr(g), len(g), H.ptr(out)))
    return out


def construct_powers(z, n: int, field="fp") -> np.ndarray:
    """group.rs:58-66 ``construct_powers``: [1, z, z^2, ..., z^(n-1)]."""
    H.ensure_device()
    z = H.fe_array(z, 1)
    out = np.zeros((n, 4), dtype=np.uint64)
    H.check(H.load().halo_construct_powers(_field(field), H.ptr(z), n, H.ptr(out)))
    return out


def point_sum(points, curve="pallas") -> np.ndarray:
    """Sum of WrappedPoints on the device (combine step of the multi-GPU MSM)."""
    H.ensure_device()
    pts = H.point_array(points)
    out = np.zeros(8, dtype=np.uint64)
    H.check(H.load().halo_point_sum(_curve(curve), H.ptr(pts), len(pts), H.ptr(out)))
    return out


class PublicParams:
    """pp.rs:10-94 ``PublicParams``: the SRS made device-resident once per (device, curve)."""

    @staticmethod
    def upload(curve, Gs, S=None, Hp=None, precompute_windows: bool = True) -> None:
        H.ensure_device()
        Gs = H.point_array(Gs)
        Sa = H.point_array(S) if S is not None else None
        Ha = H.point_array(Hp) if Hp is not None else None
        L = H.load()
        H.check(L.halo_srs_upload(_curve(curve), H.ptr(Gs), len(Gs), H.ptr(Sa), H.ptr(Ha)))
        if precompute_windows:
            H.check(L.halo_srs_precompute_windows(_curve(curve)))

    @staticmethod
    def synthesize(curve, n: int, seed: int, precompute_windows: bool = True) -> None:
        H.ensure_device()
        L = H.load()
        H.check(L.halo_srs_synthesize(_curve(curve), n, seed))
        if precompute_windows:
            H.check(L.halo_srs_precompute_windows(_curve(curve)))

    @staticmethod
    def load_bincode(curve, blocks, sh=None, n: int | None = None, precompute_windows: bool = True) -> None:
        """PublicParams::new(n) from the wire format (pp.rs:26-61): `blocks` = the gs-XX.bin byte
        strings in order, `sh` = sh.bin; decoded and curve-checked on the device."""
        H.ensure_device()
        bl = [bytes(b) for b in blocks]
        k = len(bl)
        arrs = [np.frombuffer(b, dtype=np.uint8) for b in bl]
        ptrs = (ctypes.c_void_p * max(k, 1))(*[a.ctypes.data for a in arrs])
        lens = (ctypes.c_size_t * max(k, 1))(*[len(b) for b in bl])
        sha = np.frombuffer(bytes(sh), dtype=np.uint8) if sh is not None else None
        if n is None:
            n = 0
            for b in bl:  # count prefix of each block (bincode varint)
                t = b[0]
                n += t if t < 251 else int.from_bytes(b[1:1 + {251: 2, 252: 4, 253: 8}[t]], "little")
        L = H.load()
        H.check(L.halo_srs_load_bincode(_curve(curve), ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(lens, ctypes.c_void_p),
                                        k, H.ptr(sha) if sha is not None else None, len(sha) if sha is not None else 0, n))
        if precompute_windows:
            H.check(L.halo_srs_precompute_windows(_curve(curve)))

    @staticmethod
    def sh(curve):
        """(S, H) of the resident PublicParams (pp.rs:26-61), WrappedPoints."""
        H.ensure_device()
        S = np.zeros(8, dtype=np.uint64)
        Hp = np.zeros(8, dtype=np.uint64)
        H.check(H.load().halo_srs_sh(_curve(curve), H.ptr(S), H.ptr(Hp)))
        return S, Hp

    @staticmethod
    def len(curve) -> int:
        H.ensure_device()
        n = ctypes.c_size_t(0)
        H.check(H.load().halo_srs_len(_curve(curve), ctypes.byref(n)))
        return n.value

    @staticmethod
    def read(curve, offset: int, n: int) -> np.ndarray:
        H.ensure_device()
        out = np.zeros((n, 8), dtype=np.uint64)
        H.check(H.load().halo_srs_read(_curve(curve), offset, n, H.ptr(out)))
        return out


def synth_scalar(seed: int, j: int, curve="pallas") -> int:
    """Canonical discrete log of synthetic SRS point j (host function, no GPU needed)."""
    out = (ctypes.c_uint64 * 4)()
    H.load().halo_synth_scalar(_curve(curve), seed, j, out)
    return sum(int(out[i]) << (64 * i) for i in range(4))
