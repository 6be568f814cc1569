"""GPU parity: field and curve (a2) arithmetic through the C ABI vs the oracle."""
import random

import numpy as np
import pytest

import pasta as P

pytestmark = pytest.mark.gpu

OPS = {
    0: lambda x, y, m: x * y % m,
    1: lambda x, y, m: (x + y) % m,
    2: lambda x, y, m: (x - y) % m,
    3: lambda x, y, m: x * x % m,
    4: lambda x, y, m: pow(x, -1, m) if x else 0,
    5: lambda x, y, m: (-x) % m,
}


def fe(vals, m):
    return np.array([P.int_to_limbs(P.to_mont(v % m, m)) for v in vals], dtype=np.uint64).reshape(-1, 4)


@pytest.mark.parametrize("fname,fid", [("fp", 0), ("fq", 1)])
def test_field_ops(hal, fname, fid):
    m = P.FIELDS[fname]
    rng = random.Random(fid)
    n = 2000
    a = [rng.randrange(m) for _ in range(n)]
    b = [rng.randrange(m) for _ in range(n)]
    # edge values: 0, 1, p-1, 2^k boundaries of the 29-bit limbs, values just below p
    edge = [0, 1, m - 1, m - 2, (1 << 29) - 1, 1 << 29, (1 << 232) - 1, 1 << 232, (1 << 254) - 1, m >> 1]
    a[: len(edge)] = edge
    b[: len(edge)] = edge[::-1]
    A, B = fe(a, m), fe(b, m)
    L = hal.load()
    for op, fn in OPS.items():
        out = np.zeros_like(A)
        hal.check(L.halo_field_op(fid, op, hal.ptr(A), hal.ptr(B), n, hal.ptr(out)))
        assert np.array_equal(out, fe([fn(x, y, m) for x, y in zip(a, b)], m)), f"op {op}"


@pytest.mark.parametrize("cname,cid", [("pallas", 0), ("vesta", 1)])
def test_curve_ops(hal, corc, cname, cid):
    c = P.CURVES[cname]
    n = 96
    g = corc.srs_generate(cname, 400)
    A = np.ascontiguousarray(g[:n])
    B = np.ascontiguousarray(g[200:200 + n])
    B[5] = A[5]                                   # P + P -> doubling branch
    B[6] = 0                                      # P + O
    A[8] = 0                                      # O + Q
    B[7] = P.point_to_wrapped(c, P.neg(c, P.wrapped_to_point(c, list(A[7]))))  # P + (-P) = O
    L = hal.load()
    out = np.zeros_like(A)
    pa = [P.wrapped_to_point(c, list(x)) for x in A]
    pb = [P.wrapped_to_point(c, list(x)) for x in B]
    hal.check(L.halo_curve_op(cid, 0, hal.ptr(A), hal.ptr(B), None, n, hal.ptr(out)))
    assert np.array_equal(out, np.array([P.point_to_wrapped(c, P.add(c, x, y)) for x, y in zip(pa, pb)], dtype=np.uint64))
    hal.check(L.halo_curve_op(cid, 1, hal.ptr(A), None, None, n, hal.ptr(out)))
    assert np.array_equal(out, np.array([P.point_to_wrapped(c, P.add(c, x, x)) for x in pa], dtype=np.uint64))
    rng = random.Random(4)
    ks = [rng.randrange(c.scalar) for _ in range(n)]
    ks[0], ks[1], ks[2] = 0, 1, c.scalar - 1
    K = fe(ks, c.scalar)
    hal.check(L.halo_curve_op(cid, 2, hal.ptr(A), None, hal.ptr(K), n, hal.ptr(out)))
    assert np.array_equal(out, np.array([P.point_to_wrapped(c, P.mul_fast(c, k, x)) for k, x in zip(ks, pa)],
                                        dtype=np.uint64))


def test_invalid_arguments(hal):
    L = hal.load()
    x = np.zeros((4, 4), dtype=np.uint64)
    assert L.halo_field_op(7, 0, hal.ptr(x), hal.ptr(x), 4, hal.ptr(x)) == 1
    assert L.halo_ntt(0, None, 3, 0) == 1
