"""GPU parity: NTT / iNTT / evaluate_over_domain / interpolate / poly_mul.

Small sizes are checked against the committed golden vectors and the C oracle bit-for-bit; the
BASELINE size 2^22 (configs[2]) and the prover's 2^23 transforms against the C oracle element by
element too (forward and inverse, both fields, the zero-tail path with a 2^20 prefix), and 2^20 /
2^22 also through size-independent properties: iNTT(NTT(x)) == x, linearity, and spot evaluations
p(omega^i) by Horner on the CPU oracle.
"""
import ctypes
import random

import numpy as np
import pytest

import pasta as P
from halo_amd import poly

pytestmark = pytest.mark.gpu


def rand_fe(n, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * 2 + rng.integers(0, 2, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)  # < 2^254 < p
    return np.ascontiguousarray(a)


def fe(vals, m):
    return np.array([P.int_to_limbs(P.to_mont(v % m, m)) for v in vals], dtype=np.uint64).reshape(-1, 4)


def unfe(a, m):
    return [P.from_mont(P.limbs_to_int(r), m) for r in np.asarray(a).reshape(-1, 4)]


@pytest.mark.parametrize("tag,fid", [("fp", 0), ("fq", 1)])
def test_ntt_golden(hal, golden, tag, fid):
    L = hal.load()
    for logn in range(0, 9):
        x = np.ascontiguousarray(golden[f"ntt_{tag}_log{logn}_in"].copy())
        hal.check(L.halo_ntt(fid, hal.ptr(x), logn, 0))
        assert np.array_equal(x, golden[f"ntt_{tag}_log{logn}_out"]), logn
        hal.check(L.halo_ntt(fid, hal.ptr(x), logn, 1))
        assert np.array_equal(x, golden[f"ntt_{tag}_log{logn}_in"]), logn


@pytest.mark.parametrize("tag,fid", [("fp", 0), ("fq", 1)])
def test_ntt_vs_c_oracle(hal, corc, tag, fid):
    L = hal.load()
    for logn in (9, 10, 11, 12, 13, 15, 16, 17, 18):
        x = rand_fe(1 << logn, logn)
        exp = corc.ntt(tag, x)
        got = x.copy()
        hal.check(L.halo_ntt(fid, hal.ptr(got), logn, 0))
        assert np.array_equal(got, exp), logn
        hal.check(L.halo_ntt(fid, hal.ptr(got), logn, 1))
        assert np.array_equal(got, x), logn


@pytest.mark.parametrize("tag,fid", [("fp", 0), ("fq", 1)])
def test_ntt_2p22_vs_c_oracle(hal, corc, tag, fid):
    """configs[2] at its own size (two 11-bit passes over 2048-element blocks): the forward and the
    inverse transform of independent random inputs, each against the oracle element by element."""
    L = hal.load()
    logn = 22
    x = rand_fe(1 << logn, 2200 + fid)
    got = x.copy()
    hal.check(L.halo_ntt(fid, hal.ptr(got), logn, 0))
    assert np.array_equal(got, corc.ntt(tag, x))
    got = x.copy()
    hal.check(L.halo_ntt(fid, hal.ptr(got), logn, 1))
    assert np.array_equal(got, corc.ntt(tag, x, inverse=True))


@pytest.mark.parametrize("tag,fid", [("fp", 0), ("fq", 1)])
def test_ntt_2p23_prover_shapes_vs_c_oracle(hal, corc, tag, fid):
    """The prover's 8n transforms at n = 2^20 (protocol.rs:88-106; three 8-bit passes over 1024-element
    blocks) against the oracle element by element: halo_ntt_dev_zero_tail of a 2^20-coefficient
    polynomial (the 42 NTT(8n) of round 0; the tail holds garbage the transform must ignore), a ragged
    prefix, and the full forward / inverse device transforms of a random 2^23 vector."""
    import torch

    L = hal.load()
    logn = 23
    N = 1 << logn
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for nz in (1 << 20, (1 << 20) - 3):
        x = np.zeros((N, 4), dtype=np.uint64)
        x[:nz] = rand_fe(nz, 2300 + fid)
        exp = corc.ntt(tag, x)
        junk = rand_fe(N, 2310 + fid)
        junk[:nz] = x[:nz]
        d = torch.from_numpy(junk.view(np.int64)).cuda()
        hal.check(L.halo_ntt_dev_zero_tail(fid, ctypes.c_void_p(d.data_ptr()), logn, 1, nz, s))
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy().view(np.uint64), exp), nz
    x = rand_fe(N, 2320 + fid)
    for inverse in (0, 1):
        d = torch.from_numpy(x.view(np.int64).copy()).cuda()
        hal.check(L.halo_ntt_dev(fid, ctypes.c_void_p(d.data_ptr()), logn, 1, inverse, s))
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy().view(np.uint64), corc.ntt(tag, x, inverse=bool(inverse))), inverse


@pytest.mark.parametrize("logn", [20, 22])
def test_ntt_full_size_properties(hal, corc, logn):
    """BASELINE config 3 sizes: round trip, linearity, and Horner spot checks."""
    L = hal.load()
    m = P.FP_MODULUS
    n = 1 << logn
    x = rand_fe(n, 100 + logn)
    ev = x.copy()
    hal.check(L.halo_ntt(0, hal.ptr(ev), logn, 0))
    back = ev.copy()
    hal.check(L.halo_ntt(0, hal.ptr(back), logn, 1))
    assert np.array_equal(back, x)
    w = P.root_of_unity(m, n)
    for i in (0, 1, 12345 % n, n - 1):
        z = fe([pow(w, i, m)], m)[0]
        assert np.array_equal(corc.poly_eval("fp", x, z), ev[i]), i
    # linearity: NTT(x + y) == NTT(x) + NTT(y), checked on a window of outputs
    y = rand_fe(n, 7)
    ey = y.copy()
    hal.check(L.halo_ntt(0, hal.ptr(ey), logn, 0))
    s = np.ascontiguousarray(fe([(a + b) % m for a, b in zip(unfe(x[:n], m), unfe(y[:n], m))], m)) if logn <= 16 else None
    if s is None:
        # sum on the device via field_op (add), then transform
        s = np.zeros_like(x)
        hal.check(L.halo_field_op(0, 1, hal.ptr(x), hal.ptr(y), n, hal.ptr(s)))
    es = s.copy()
    hal.check(L.halo_ntt(0, hal.ptr(es), logn, 0))
    idx = slice(n // 2, n // 2 + 256)
    chk = np.zeros((256, 4), dtype=np.uint64)
    hal.check(L.halo_field_op(0, 1, hal.ptr(np.ascontiguousarray(ev[idx])), hal.ptr(np.ascontiguousarray(ey[idx])), 256,
                              hal.ptr(chk)))
    assert np.array_equal(chk, es[idx])


def test_ntt_batched_device(hal, corc):
    import torch
    L = hal.load()
    for logn, batch in ((12, 5), (17, 3), (8, 7)):
        n = 1 << logn
        x = rand_fe(batch * n, logn)
        d = torch.from_numpy(x.view(np.int64)).cuda()
        hal.check(L.halo_ntt_dev(1, ctypes.c_void_p(d.data_ptr()), logn, batch, 0, None))
        torch.cuda.synchronize()
        got = d.cpu().numpy().view(np.uint64)
        for b in range(batch):
            assert np.array_equal(got[b * n:(b + 1) * n], corc.ntt("fq", x[b * n:(b + 1) * n])), (logn, b)


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_evaluate_over_domain_and_interpolate(hal, golden, tag):
    """poly.rs:56-64,133-139: longer-than-domain input is reduced mod X^N - 1; short input is
    zero-padded; interpolate trims trailing zeros (DensePolynomial::from_coefficients_vec)."""
    m = P.FIELDS[tag]
    d16 = poly.Domain(16, tag)
    ev = poly.Evals.from_poly_ref(golden[f"fold_{tag}_in40"], d16)
    assert np.array_equal(ev.evals, golden[f"fold_{tag}_out16"])
    rng = random.Random(9)
    coeffs = [rng.randrange(m) for _ in range(10)]
    d64 = poly.Domain(64, tag)
    ev = poly.Evals.from_poly(fe(coeffs, m), d64)
    assert unfe(ev.evals, m) == P.ntt(coeffs, 64, m)
    back = ev.interpolate()
    assert back.shape == (10, 4) and unfe(back, m) == coeffs
    zero = poly.Evals(np.zeros((8, 4), dtype=np.uint64), poly.Domain(8, tag))
    assert zero.interpolate().shape == (0, 4)
    # from_vec_and_domain rotates right by one (poly.rs:21-31)
    e = poly.Evals.from_vec_and_domain(fe([1, 2, 3, 4], m), poly.Domain(4, tag))
    assert unfe(e.evals, m) == [4, 1, 2, 3]


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_evals_add_sub_mul_scale(hal, tag):
    """protocol.rs:1037-1118 evals_add / evals_sub / evals_mul / evals_scale on the GPU NTT."""
    m = P.FIELDS[tag]
    rng = random.Random(21)
    for n in (32, 1024):
        a = [rng.randrange(m) for _ in range(n)]
        b = [rng.randrange(m) for _ in range(n)]
        dom = poly.Domain(n, tag)
        ea = unfe(poly.Evals.from_poly_ref(fe(a, m), dom).evals, m)
        eb = unfe(poly.Evals.from_poly_ref(fe(b, m), dom).evals, m)
        s = poly.Evals(fe([x + y for x, y in zip(ea, eb)], m), dom).interpolate()
        assert unfe(s, m) == P.trim([(x + y) % m for x, y in zip(a, b)])
        d = poly.Evals(fe([x - y for x, y in zip(ea, eb)], m), dom).interpolate()
        assert unfe(d, m) == P.trim([(x - y) % m for x, y in zip(a, b)])
        k = rng.randrange(m)
        sc = poly.Evals(fe([x * k for x in ea], m), dom).interpolate()
        assert unfe(sc, m) == P.trim([x * k % m for x in a])
        big = poly.Domain(2 * n, tag)
        ea2 = unfe(poly.Evals.from_poly_ref(fe(a, m), big).evals, m)
        eb2 = unfe(poly.Evals.from_poly_ref(fe(b, m), big).evals, m)
        prod = unfe(poly.Evals(fe([x * y for x, y in zip(ea2, eb2)], m), big).interpolate(), m)
        if n == 32:
            assert prod == P.poly_mul(a, b, m)
        assert unfe(poly.poly_mul(fe(a, m), fe(b, m), tag), m) == prod


def test_poly_mul_edge(hal):
    m = P.FP_MODULUS
    assert poly.poly_mul(np.zeros((0, 4), dtype=np.uint64), fe([1, 2], m)).shape == (0, 4)
    assert unfe(poly.poly_mul(fe([3], m), fe([5], m)), m) == [15]
    assert unfe(poly.poly_mul(fe([m - 1, 1], m), fe([1, 1], m)), m) == [m - 1, 0, 1]  # (X-1)(X+1) = X^2 - 1


def test_sharded_ntt_virtual_ranks(hal, corc):
    """The distributed four-step NTT (halo_amd.dist) with the device primitives (batched NTT,
    twiddle, transposes) and P virtual ranks on one GPU, bit-exact vs the oracle NTT."""
    import torch

    from halo_amd import _lib as H
    from halo_amd.dist import GpuNttOps, sharded_ntt_virtual

    ops = GpuNttOps(H.FP)
    rng = np.random.default_rng(11)
    for logn, world in ((6, 2), (9, 4), (12, 8), (16, 4)):
        N = 1 << logn
        x = rng.integers(0, 2**62, size=(N, 4), dtype=np.uint64)
        xd = torch.from_numpy(x.view(np.int64).copy()).cuda()
        y = sharded_ntt_virtual(xd, logn, False, ops, world)
        assert np.array_equal(y.cpu().numpy().view(np.uint64), corc.ntt("fp", x)), (logn, world)
        z = sharded_ntt_virtual(y, logn, True, ops, world)
        assert np.array_equal(z.cpu().numpy().view(np.uint64), x), (logn, world)


def test_transpose_and_twiddle_dev(hal, corc):
    import ctypes

    import pasta as P
    import torch

    from halo_amd import _lib as H
    L = H.load()
    rng = np.random.default_rng(3)
    for (b, r, c, run) in ((1, 37, 45, 1), (3, 64, 33, 1), (2, 5, 7, 3)):
        x = torch.from_numpy(rng.integers(0, 2**62, size=(b * r * c * run, 4), dtype=np.int64)).cuda()
        y = torch.empty_like(x)
        H.check(L.halo_transpose_dev(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), b, r, c, run, None))
        exp = x.view(b, r, c, run, 4).permute(0, 2, 1, 3, 4).reshape(-1, 4)
        assert torch.equal(y, exp)
    m = P.FP_MODULUS
    logn, rows, cols, row0, col0 = 10, 6, 9, 5, 3
    x = rng.integers(0, 2**62, size=(rows * cols, 4), dtype=np.uint64)
    for inv in (0, 1):
        d = torch.from_numpy(x.view(np.int64).copy()).cuda()
        H.check(L.halo_ntt_twiddle_dev(H.FP, ctypes.c_void_p(d.data_ptr()), logn, rows, cols, row0, col0, inv, None))
        w = pow(5, (m - 1) >> logn, m)
        if inv:
            w = pow(w, -1, m)
        got = d.cpu().numpy().view(np.uint64)
        for i in range(rows * cols):
            a, bb = divmod(i, cols)
            v = P.from_mont(P.limbs_to_int(x[i]), m) * pow(w, (row0 + a) * (col0 + bb), m) % m
            assert P.from_mont(P.limbs_to_int(got[i]), m) == v


# ---- evaluation algebra and vanishing division ---------------------------------------
@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_evals_ops_vs_python(hal, tag):
    m = P.FIELDS[tag]
    dom = poly.Domain(1 << 10, tag)
    rnd = random.Random(3)
    a = [rnd.randrange(m) for _ in range(dom.n)]
    b = [rnd.randrange(m) for _ in range(dom.n)]
    a[0], b[1] = m - 1, 0
    A = poly.Evals(fe(a, m), dom)
    B = poly.Evals(fe(b, m), dom)
    s = rnd.randrange(m)
    chk = {
        "add": ((A + B), [(x + y) % m for x, y in zip(a, b)]),
        "sub": ((A - B), [(x - y) % m for x, y in zip(a, b)]),
        "mul": ((A * B), [(x * y) % m for x, y in zip(a, b)]),
        "scale": (A.scale(fe([s], m)[0]), [(x * s) % m for x in a]),
        "add_scalar": (A.add_scalar(fe([s], m)[0]), [(x + s) % m for x in a]),
        "sub_scalar": (A.sub_scalar(fe([s], m)[0]), [(x - s) % m for x in a]),
        "pow7": (A.pow(7), [pow(x, 7, m) for x in a]),
    }
    for name, (got, exp) in chk.items():
        assert [P.from_mont(P.limbs_to_int(r), m) for r in got.evals] == exp, name


@pytest.mark.parametrize("tag", ["fp", "fq"])
def test_divide_by_vanishing_poly(hal, tag):
    """ark-poly divide_by_vanishing_poly (protocol.rs:256): p = q (X^n - 1) + r with deg r < n,
    checked against Python long division, incl. len < n, len = n, len > 2n, trailing zeros."""
    m = P.FIELDS[tag]
    rnd = random.Random(9)
    n = 64
    dom = poly.Domain(n, tag)
    for ln in (0, 5, n, n + 1, 2 * n + 3, 8 * n, 8 * n - 7):
        c = [rnd.randrange(m) for _ in range(ln)]
        if ln > 3:
            c[-1] = rnd.randrange(1, m)
        q, r = poly.divide_by_vanishing_poly(fe(c, m) if ln else [], dom)
        # Python: quotient q[j] = sum_{k>=1} c[j + k n], remainder c[j] + q[j]
        qe = [sum(c[j + k * n] for k in range(1, (ln - j - 1) // n + 1)) % m for j in range(max(ln - n, 0))]
        re = [(c[j] + (qe[j] if j < len(qe) else 0)) % m for j in range(min(ln, n))] if ln >= n else c[:]
        while qe and qe[-1] == 0:
            qe.pop()
        while re and re[-1] == 0:
            re.pop()
        assert [P.from_mont(P.limbs_to_int(x), m) for x in q] == qe, ln
        assert [P.from_mont(P.limbs_to_int(x), m) for x in r] == re, ln
        # and the defining identity at a random point
        if ln:
            z = rnd.randrange(m)
            ev = lambda cs: sum(v * pow(z, i, m) for i, v in enumerate(cs)) % m
            assert ev(c) == (ev(qe) * (pow(z, n, m) - 1) + ev(re)) % m
    ts = poly.t_split(fe([rnd.randrange(m) for _ in range(3 * n - 2)], m), n, 3)
    assert [len(t) for t in ts] == [n, n, n - 2]


@pytest.mark.parametrize("logn,nz", [(8, 32), (8, 33), (12, 100), (18, 1 << 15), (20, 1 << 17), (20, 5),
                                     (23, 1 << 20), (23, (1 << 20) - 3), (22, 1 << 20)])
def test_ntt_zero_tail_matches_full(hal, corc, logn, nz):
    """halo_ntt_dev_zero_tail (first pass skips the stages that only replicate the nonzero prefix; the
    tail's contents are ignored, here garbage) equals halo_ntt_dev on the zero-padded input: 1-, 2- and
    3-pass sizes, power-of-two and ragged prefixes -- and both equal the C oracle's NTT of the
    zero-padded input (corc, ark-poly's radix-2 FFT restated)."""
    import torch

    N = 1 << logn
    L = hal.load()
    x = torch.zeros((N, 4), dtype=torch.int64, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(logn * 1000 + nz)
    v = torch.randint(0, 2**62, (nz, 4), dtype=torch.int64, device="cuda", generator=g)
    x[:nz] = v
    y = x.clone()
    y[nz:] = torch.randint(0, 2**62, (N - nz, 4), dtype=torch.int64, device="cuda", generator=g)  # ignored tail
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    x0 = x.cpu().numpy().view(np.uint64).copy()  # the zero-padded input, before the in-place transform
    hal.check(L.halo_ntt_dev(0, ctypes.c_void_p(x.data_ptr()), logn, 1, 0, s))
    hal.check(L.halo_ntt_dev_zero_tail(0, ctypes.c_void_p(y.data_ptr()), logn, 1, nz, s))
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    assert np.array_equal(y.cpu().numpy().view(np.uint64), corc.ntt("fp", x0))


def test_ntt_dev_concurrent_streams(hal, corc):
    """halo_ntt_dev on two torch streams at once plus host-array NTTs (null stream) in between: the
    device-global NTT scratch is fenced per stream (ScratchUse), so every transform is bit-exact."""
    import torch
    L = hal.load()
    logn = 18
    n = 1 << logn
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    xs = [rand_fe(n, 900 + i) for i in range(6)]
    exps = [corc.ntt("fp", x) for x in xs]
    ds = [torch.from_numpy(x.view(np.int64)).cuda() for x in xs]
    torch.cuda.synchronize()
    for i, d in enumerate(ds):
        st = s1 if i % 2 == 0 else s2
        hal.check(L.halo_ntt_dev(0, ctypes.c_void_p(d.data_ptr()), logn, 1, 0, ctypes.c_void_p(st.cuda_stream)))
        if i == 2:  # a host-array transform on the null stream while the others are in flight
            h = xs[0].copy()
            hal.check(L.halo_ntt(0, hal.ptr(h), logn, 0))
            assert np.array_equal(h, exps[0])
    torch.cuda.synchronize()
    for i, d in enumerate(ds):
        assert np.array_equal(d.cpu().numpy().view(np.uint64), exps[i]), i
