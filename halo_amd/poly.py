"""Mirror of crates/group/src/poly.rs (Domain / Evals) on the MI355X backend.

``Evals`` wraps ark-poly ``Evaluations``; its NTT entry points (``from_poly``, ``from_poly_ref``,
``interpolate``, ``interpolate_by_ref``) run on the GPU.  ``from_vec_and_domain`` keeps the
reference's rotate-right-by-one convention (poly.rs:21-31).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as H
from .group import _field


class Domain:
    """``GeneralEvaluationDomain`` of size N = 2^k (radix-2; poly.rs:11)."""

    def __init__(self, size: int, field="fp"):
        if size <= 0 or size & (size - 1):
            raise AssertionError(f"domain size ({size}) is not a power of two")
        self.n = size
        self.log_n = size.bit_length() - 1
        self.field = _field(field)

    def size(self) -> int:
        return self.n


class Evals:
    def __init__(self, evals: np.ndarray, domain: Domain):
        self.evals = H.fe_array(evals)
        self.domain = domain

    @classmethod
    def from_vec_and_domain(cls, evals, domain: Domain) -> "Evals":
        """poly.rs:21-24: wraps then ``shift_right`` (last element moves to the front)."""
        e = H.fe_array(evals)
        assert len(e) > 0
        return cls(np.ascontiguousarray(np.roll(e, 1, axis=0)), domain)

    @classmethod
    def from_poly_ref(cls, coeffs, domain: Domain) -> "Evals":
        """poly.rs:56-59 ``evaluate_over_domain_by_ref``: coefficients (any length; reduced mod
        X^N - 1 when longer than N) -> N evaluations p(omega^i)."""
        H.ensure_device()
        c = H.fe_array(coeffs) if len(coeffs) else np.zeros((0, 4), dtype=np.uint64)
        out = np.zeros((domain.n, 4), dtype=np.uint64)
        H.check(H.load().halo_evaluate_over_domain(domain.field, H.ptr(c) if len(c) else None, len(c), domain.log_n,
                                                   H.ptr(out)))
        return cls(out, domain)

    from_poly = from_poly_ref

    def interpolate_by_ref(self) -> np.ndarray:
        """poly.rs:137-139 -> ``Evaluations::interpolate``: iNTT, trailing zeros trimmed."""
        H.ensure_device()
        out = np.zeros((self.domain.n, 4), dtype=np.uint64)
        n = ctypes.c_size_t(0)
        H.check(H.load().halo_interpolate(self.domain.field, H.ptr(self.evals), self.domain.log_n, H.ptr(out),
                                          ctypes.byref(n)))
        return out[: n.value].copy()

    interpolate = interpolate_by_ref

    # ---- elementwise algebra (poly.rs:90-327), on the device (halo_evals_op) ----
    def _op(self, op: int, other=None, scalar=None, e: int = 0) -> "Evals":
        H.ensure_device()
        n = len(self.evals)
        b = None
        if other is not None:
            b = other.evals if isinstance(other, Evals) else H.fe_array(other)
            assert len(b) == n, "evaluation vectors of different lengths"
        sc = H.fe_array(scalar, 1) if scalar is not None else None
        out = np.zeros((n, 4), dtype=np.uint64)
        H.check(H.load().halo_evals_op(self.domain.field, op, H.ptr(self.evals), H.ptr(b), H.ptr(sc), e, H.ptr(out), n))
        return Evals(out, self.domain)

    def __add__(self, other):
        return self._op(0, other)

    def __sub__(self, other):
        return self._op(1, other)

    def __mul__(self, other):
        return self._op(2, other)

    def scale(self, s):
        return self._op(3, scalar=s)

    def add_scalar(self, s):
        return self._op(4, scalar=s)

    def sub_scalar(self, s):
        return self._op(5, scalar=s)

    def pow(self, e: int):
        return self._op(6, e=e)


def divide_by_vanishing_poly(coeffs, domain: Domain):
    """``DensePolynomial::divide_by_vanishing_poly`` (ark-poly 0.5.0, protocol.rs:256): division by
    X^n - 1 -> (quotient, remainder), both trimmed."""
    H.ensure_device()
    c = H.fe_array(coeffs) if len(coeffs) else np.zeros((0, 4), dtype=np.uint64)
    n = domain.n
    q = np.zeros((max(len(c) - n, 0) + 1, 4), dtype=np.uint64)
    r = np.zeros((n, 4), dtype=np.uint64)
    ql, rl = ctypes.c_size_t(0), ctypes.c_size_t(0)
    H.check(H.load().halo_divide_by_vanishing(domain.field, H.ptr(c) if len(c) else None, len(c), n, H.ptr(q),
                                              ctypes.byref(ql), H.ptr(r), ctypes.byref(rl)))
    return q[: ql.value].copy(), r[: rl.value].copy()


def t_split(t, n: int, parts: int):
    """protocol.rs:509-517: t (degree < parts * n) zero-padded and cut into `parts` chunks of n."""
    t = H.fe_array(t) if len(t) else np.zeros((0, 4), dtype=np.uint64)
    deg = max(len(t) - 1, 0)
    if not deg < parts * n:
        raise AssertionError(f"{deg} < {parts * n}")
    pad = np.zeros((parts * n, 4), dtype=np.uint64)
    pad[: len(t)] = t
    out = []
    for i in range(parts):
        chunk = pad[i * n:(i + 1) * n]
        m = len(chunk)
        while m > 0 and not chunk[m - 1].any():
            m -= 1
        out.append(chunk[:m].copy())
    return out


def poly_mul(a, b, field="fp") -> np.ndarray:
    """``&DensePolynomial * &DensePolynomial`` (FFT multiplication), trimmed."""
    H.ensure_device()
    a, b = H.fe_array(a), H.fe_array(b)
    if len(a) == 0 or len(b) == 0:
        return np.zeros((0, 4), dtype=np.uint64)
    out = np.zeros((len(a) + len(b) - 1, 4), dtype=np.uint64)
    n = ctypes.c_size_t(0)
    H.check(H.load().halo_poly_mul(_field(field), H.ptr(a), len(a), H.ptr(b), len(b), H.ptr(out), ctypes.byref(n)))
    return out[: n.value].copy()


def evaluate_batch(polys, z, field="fp") -> np.ndarray:
    """``DensePolynomial::evaluate`` (Horner) for several polynomials at one point."""
    H.ensure_device()
    arrs = [H.fe_array(p) if len(p) else np.zeros((0, 4), dtype=np.uint64) for p in polys]
    k = len(arrs)
    ptrs = (ctypes.c_void_p * k)(*[a.ctypes.data if len(a) else None for a in arrs])
    lens = (ctypes.c_size_t * k)(*[len(a) for a in arrs])
    zz = H.fe_array(z, 1)
    out = np.zeros((k, 4), dtype=np.uint64)
    H.check(H.load().halo_poly_eval_batch(_field(field), ctypes.cast(ptrs, ctypes.c_void_p),
                                          ctypes.cast(lens, ctypes.c_void_p), k, H.ptr(zz), H.ptr(out)))
    return out
