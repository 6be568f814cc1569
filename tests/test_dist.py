"""N > 1 path on CPU: world_size-2 gloo run of halo_amd.dist.sharded_msm (the protocol bench.py
uses with RCCL on GPUs).  The per-rank partial MSM and the final point sum are computed by the C
oracle here (no GPU in this container); the test checks the partition, the all-gather and the
combine give the unsharded result on every rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist

    import corc
    import pasta as P
    from halo_amd.dist import shard_range, sharded_msm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = corc.srs_generate("pallas", n)
    rng = np.random.default_rng(42)
    sc = rng.integers(0, 2**62, size=(n, 4), dtype=np.uint64)
    c = P.PALLAS

    def partial(lo, hi):
        return corc.msm("pallas", g[lo:hi], sc[lo:hi]) if hi > lo else np.zeros(8, dtype=np.uint64)

    def psum(parts):
        acc = None
        for p in parts:
            acc = P.add(c, acc, P.wrapped_to_point(c, list(p)))
        return np.array(P.point_to_wrapped(c, acc), dtype=np.uint64)

    res = sharded_msm(partial, psum, n, dist)
    lo, hi = shard_range(n, rank, world)
    q.put((rank, res.tolist(), (lo, hi)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_msm_gloo(corc, world):
    n = 3000
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = corc.srs_generate("pallas", n)
    rng = np.random.default_rng(42)
    sc = rng.integers(0, 2**62, size=(n, 4), dtype=np.uint64)
    exp = corc.msm("pallas", g, sc).tolist()
    ranges = sorted(r[2] for r in out)
    assert ranges[0][0] == 0 and ranges[-1][1] == n and ranges[0][1] == ranges[1][0]
    for _, res, _ in out:
        assert res == exp


# ---------------------------------------------------------------------------------------------
# distributed NTT (four-step, three all-to-alls): oracle-backed primitives on CPU, gloo world 2
# ---------------------------------------------------------------------------------------------
class OracleNttOps:
    """halo_amd.dist.NttOps on the CPU: C-oracle NTTs, Python big-int twiddles, numpy transposes."""

    def __init__(self, field):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import corc
        import pasta as P
        self.corc, self.P, self.field = corc, P, field
        self.m = P.FIELDS[field]

    def ntt_batch(self, t, log_len, batch, inverse):
        a = t.numpy().view(np.uint64).reshape(batch, 1 << log_len, 4)
        for b in range(batch):
            a[b] = self.corc.ntt(self.field, np.ascontiguousarray(a[b]), inverse=inverse)

    def twiddle(self, t, logn, rows, cols, row0, col0, inverse):
        P, m = self.P, self.m
        w = pow(5, (m - 1) >> logn, m)
        if inverse:
            w = pow(w, -1, m)
        a = t.numpy().view(np.uint64).reshape(rows * cols, 4)
        for i in range(rows * cols):
            r, c = divmod(i, cols)
            x = P.from_mont(P.limbs_to_int(a[i]), m) * pow(w, (row0 + r) * (col0 + c), m) % m
            a[i] = P.int_to_limbs(P.to_mont(x, m))

    def transpose(self, src, batch, rows, cols, run=1):
        import torch
        v = src.view(batch, rows, cols, run, 4).permute(0, 2, 1, 3, 4).contiguous()
        return v.view(src.shape)


def _ntt_worker(rank, world, port, logn, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from halo_amd.dist import sharded_ntt, torch_alltoall

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N = 1 << logn
    rng = np.random.default_rng(7)
    x = rng.integers(0, 2**62, size=(N, 4), dtype=np.uint64)
    per = N // world
    loc = torch.from_numpy(x[rank * per:(rank + 1) * per].view(np.int64).copy())
    ops = OracleNttOps("fp")
    y = sharded_ntt(loc, logn, False, ops, rank, world, torch_alltoall(dist))
    z = sharded_ntt(y.clone(), logn, True, ops, rank, world, torch_alltoall(dist))
    q.put((rank, y.numpy().view(np.uint64).tolist(), z.numpy().view(np.uint64).tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,logn", [(2, 6), (2, 7)])
def test_sharded_ntt_gloo(corc, world, logn):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ntt_worker, args=(r, world, port, logn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=180) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    N = 1 << logn
    rng = np.random.default_rng(7)
    x = rng.integers(0, 2**62, size=(N, 4), dtype=np.uint64)
    exp = corc.ntt("fp", x)
    got = np.array([v for _, y, _ in out for v in y], dtype=np.uint64).reshape(N, 4)
    back = np.array([v for _, _, z in out for v in z], dtype=np.uint64).reshape(N, 4)
    assert np.array_equal(got, exp)
    assert np.array_equal(back, x)


# ---------------------------------------------------------------------------------------------
# distributed IPA opening (strided shards, per-round all-gather of 2 points): oracle-backed
# session primitives on CPU, gloo world 2 and 4, against the single-session oracle loop
# ---------------------------------------------------------------------------------------------
def _oracle_mods():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pasta as P
    return P


from halo_amd.dist import IpaOps  # noqa: E402


class OracleIpaOps(IpaOps):
    """halo_amd.dist.IpaOps on the CPU: pure-Python restatement of pcdl.rs:404-438."""

    def __init__(self, cname):
        self.P = P = _oracle_mods()
        self.c = P.CURVES[cname]

    def _ints(self, a):
        P, r = self.P, self.c.scalar
        return [P.from_mont(P.limbs_to_int(x), r) for x in np.asarray(a, dtype=np.uint64).reshape(-1, 4)]

    def _fe(self, xs):
        P, r = self.P, self.c.scalar
        return np.array([P.int_to_limbs(P.to_mont(x % r, r)) for x in xs], dtype=np.uint64).reshape(-1, 4)

    def begin(self, shard, H_prime):
        P, c = self.P, self.c
        gs, cs, zs = shard
        G = [P.wrapped_to_point(c, list(g)) for g in np.asarray(gs, dtype=np.uint64).reshape(-1, 8)]
        return {"G": G, "C": self._ints(cs), "Z": self._ints(zs),
                "H": P.wrapped_to_point(c, list(np.asarray(H_prime, dtype=np.uint64)))}

    def round_lr(self, s):
        P, c, r = self.P, self.c, self.c.scalar
        G, C, Z, Hp = s["G"], s["C"], s["Z"], s["H"]
        m = len(G) // 2
        L = P.add(c, P.msm(c, G[:m], C[m:]), P.mul_fast(c, P.scalar_dot(C[m:], Z[:m], r), Hp))
        R = P.add(c, P.msm(c, G[m:], C[:m]), P.mul_fast(c, P.scalar_dot(C[:m], Z[m:], r), Hp))
        return (np.array(P.point_to_wrapped(c, L), dtype=np.uint64), np.array(P.point_to_wrapped(c, R), dtype=np.uint64))

    def fold(self, s, xi, xi_inv):
        x = self._ints(xi)[0]
        _, _, _, _, s["G"], s["C"], s["Z"] = self.P.ipa_round(self.c, s["G"], s["C"], s["Z"], x)

    def final(self, s):
        P, c = self.P, self.c
        return (np.array([P.point_to_wrapped(c, s["G"][0])], dtype=np.uint64), self._fe(s["C"][:1]),
                self._fe(s["Z"][:1]))

    def round_lr_dev(self, s):  # (the CPU stand-in of a device-resident pair: the plumbing of device_lr)
        return self.round_lr(s)

    def point_sum(self, pts):
        P, c = self.P, self.c
        acc = None
        for p in pts:
            acc = P.add(c, acc, P.wrapped_to_point(c, list(p)))
        return np.array(P.point_to_wrapped(c, acc), dtype=np.uint64)


def ipa_transcript(cname):
    """Deterministic stand-in for the Poseidon transcript (the distributed loop only needs every
    rank to derive the same xi from (xi_prev, L, R))."""
    import hashlib
    P = _oracle_mods()
    r = P.CURVES[cname].scalar

    def challenge(xi_prev, L, R):
        h = hashlib.sha3_256((b"" if xi_prev is None else np.asarray(xi_prev).tobytes()) + L.tobytes() + R.tobytes())
        v = int.from_bytes(h.digest(), "little") % r or 1
        return np.array(P.int_to_limbs(P.to_mont(v, r)), dtype=np.uint64)

    def inverse(x):
        v = P.from_mont(P.limbs_to_int(x), r)
        return np.array(P.int_to_limbs(P.to_mont(P.inv(v, r), r)), dtype=np.uint64)

    return challenge, inverse


def ipa_instance(cname, n, seed=5):
    """(G, c, z-powers, H') of an opening of length n: G from the reference SRS recipe (C oracle)."""
    import random
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import corc
    P = _oracle_mods()
    c = P.CURVES[cname]
    r = c.scalar
    rng = random.Random(seed)
    g = corc.srs_generate(cname, n)
    cs = [rng.randrange(r) for _ in range(n)]
    z = rng.randrange(r)
    zs = P.construct_powers(z, n, r)
    Hp = P.mul_fast(c, rng.randrange(r), c.generator)
    fe = lambda xs: np.array([P.int_to_limbs(P.to_mont(x, r)) for x in xs], dtype=np.uint64).reshape(-1, 4)
    return g, fe(cs), fe(zs), np.array(P.point_to_wrapped(c, Hp), dtype=np.uint64)


def _ipa_worker(rank, world, port, cname, n, q, device_lr=False):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from halo_amd.dist import ipa_shard, sharded_ipa_rounds, torch_gather_arrays

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g, cs, zs, Hp = ipa_instance(cname, n)
    shard = (ipa_shard(g, rank, world), ipa_shard(cs, rank, world), ipa_shard(zs, rank, world))
    ch, inv = ipa_transcript(cname)
    Ls, Rs, U, c = sharded_ipa_rounds([shard], Hp, ch, inv, OracleIpaOps(cname), world, torch_gather_arrays(dist),
                                      device_lr=device_lr)
    q.put((rank, [x.tolist() for x in Ls], [x.tolist() for x in Rs], U.tolist(), c.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def single_session_ipa(cname, g, cs, zs, Hp):
    """The unsharded round loop (world 1 of the same code path, oracle primitives)."""
    sys.path.insert(0, ROOT)
    from halo_amd.dist import sharded_ipa_rounds
    ch, inv = ipa_transcript(cname)
    return sharded_ipa_rounds([(g, cs, zs)], Hp, ch, inv, OracleIpaOps(cname), 1, lambda objs: objs)


@pytest.mark.parametrize("world,n,cname,device_lr", [(2, 16, "pallas", False), (4, 16, "vesta", False),
                                                     (4, 4, "pallas", False), (2, 16, "vesta", True)])
def test_sharded_ipa_gloo(corc, world, n, cname, device_lr):
    """device_lr: the shard rounds go through ops.round_lr_dev (the device-resident per-round reduce's
    plumbing; its device half is tests/test_gpu_ipa_eval.py::test_sharded_ipa_weighted_virtual_ranks)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ipa_worker, args=(r, world, port, cname, n, q, device_lr)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g, cs, zs, Hp = ipa_instance(cname, n)
    Ls, Rs, U, c = single_session_ipa(cname, g, cs, zs, Hp)
    assert len(Ls) == n.bit_length() - 1
    for _, ls, rs, u, cc in out:  # every rank returns the unsharded proof
        assert ls == [x.tolist() for x in Ls]
        assert rs == [x.tolist() for x in Rs]
        assert u == U.tolist() and cc == c.tolist()
    # and the unsharded loop itself is the reference round loop (the restatement of pcdl.rs:404-438)
    P = _oracle_mods()
    cv = P.CURVES[cname]
    G = [P.wrapped_to_point(cv, list(x)) for x in g]
    Cs = OracleIpaOps(cname)._ints(cs)
    Zs = OracleIpaOps(cname)._ints(zs)
    Hpt = P.wrapped_to_point(cv, list(Hp))
    challenge, _ = ipa_transcript(cname)
    xi = None
    for k in range(n.bit_length() - 1):
        m = len(G) // 2
        L = P.add(cv, P.msm(cv, G[:m], Cs[m:]), P.mul_fast(cv, P.scalar_dot(Cs[m:], Zs[:m], cv.scalar), Hpt))
        assert Ls[k].tolist() == P.point_to_wrapped(cv, L)
        xi = challenge(xi, Ls[k], Rs[k])
        _, _, _, _, G, Cs, Zs = P.ipa_round(cv, G, Cs, Zs, OracleIpaOps(cname)._ints(xi)[0])
    assert U.tolist() == P.point_to_wrapped(cv, G[0])


# ---------------------------------------------------------------------------------------------
# distributed polynomial evaluation: block partials + combine at z^per, gloo world 2 and 3
# ---------------------------------------------------------------------------------------------
class OraclePolyOps:
    def __init__(self, field):
        self.P = _oracle_mods()
        self.m = self.P.FIELDS[field]

    def _i(self, x):
        return self.P.from_mont(self.P.limbs_to_int(np.asarray(x, dtype=np.uint64).reshape(4)), self.m)

    def _f(self, v):
        return np.array(self.P.int_to_limbs(self.P.to_mont(v, self.m)), dtype=np.uint64)

    def eval_batch(self, polys, z):
        zi = self._i(z)
        return [self._f(self.P.horner([self._i(c) for c in np.asarray(p).reshape(-1, 4)], zi, self.m)) for p in polys]

    def pow(self, z, e):
        return self._f(pow(self._i(z), e, self.m))


def _eval_worker(rank, world, port, n, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from halo_amd.dist import shard_range, sharded_poly_eval

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(11)
    coeffs = rng.integers(0, 2**62, size=(n, 4), dtype=np.uint64)
    z = rng.integers(0, 2**62, size=4, dtype=np.uint64)
    lo, hi = shard_range(n, rank, world)
    v = sharded_poly_eval(coeffs[lo:hi], n, z, dist, OraclePolyOps("fp"))
    q.put((rank, v.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 37), (3, 100)])
def test_sharded_poly_eval_gloo(world, n):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_eval_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(11)
    coeffs = rng.integers(0, 2**62, size=(n, 4), dtype=np.uint64)
    z = rng.integers(0, 2**62, size=4, dtype=np.uint64)
    exp = OraclePolyOps("fp").eval_batch([coeffs], z)[0].tolist()
    for _, v in out:
        assert v == exp


def _wworker(rank, world, port, n, c, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist

    import corc
    import pasta as P
    from halo_amd.dist import window_partitioned_msm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = corc.srs_generate("pallas", n)
    rng = np.random.default_rng(43)
    sc = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
    sc[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    cv = P.PALLAS
    W = -(-255 // c)

    def partial(lo, hi):  # oracle restatement of halo_msm_srs_windows_dev's share
        return corc.msm("pallas", g, corc.window_scalars("pallas", sc, c, lo, hi))

    def psum(parts):
        acc = None
        for p in parts:
            acc = P.add(cv, acc, P.wrapped_to_point(cv, list(p)))
        return np.array(P.point_to_wrapped(cv, acc), dtype=np.uint64)

    res = window_partitioned_msm(partial, psum, W, dist)
    q.put((rank, res.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_window_partitioned_msm_gloo(corc, world):
    """BASELINE configs[4]'s protocol over gloo: windows split across ranks (replicated scalars),
    partials all-gathered and summed == the unsharded MSM on every rank; window_range covers [0, W)."""
    from halo_amd.dist import window_range
    for W in (13, 15, 16):
        for P_ in (1, 2, 3, 8):
            rs = [window_range(W, r, P_) for r in range(P_)]
            assert rs[0][0] == 0 and rs[-1][1] == W and all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    n, c = 500, 17
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_wworker, args=(r, world, port, n, c, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = corc.srs_generate("pallas", n)
    rng = np.random.default_rng(43)
    sc = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
    sc[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    exp = corc.msm("pallas", g, sc).tolist()
    assert all(o[1] == exp for o in out)


def test_partition_window_bits_balanced():
    """configs[4]: the window width chosen for a window partition splits W evenly over the ranks
    (16 windows of 16 bits over 2 / 4 / 8 / 16 ranks, the default 15 x 17 bits over 3 / 5)."""
    from halo_amd.dist import partition_window_bits, window_range
    for world, c in ((1, 17), (2, 16), (3, 17), (4, 16), (5, 17), (8, 16), (16, 16)):
        assert partition_window_bits(world) == c
        W = -(-255 // c)
        spans = [window_range(W, r, world) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == W
        assert len({hi - lo for lo, hi in spans}) == 1


def _rows_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from halo_amd.dist import allgather_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # a rank's (L_r, R_r) as 16 words, as torch_reduce_lr gathers them ahead of halo_point_sum_dev
    t = torch.arange(16, dtype=torch.int64) + 100 * rank
    got = allgather_rows(t, dist)
    q.put((rank, list(got.shape), got.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_rows_gloo(world):
    """The distributed opening's per-round L/R gather (dist.torch_reduce_lr -> allgather_rows): one
    flat all_gather_into_tensor, (world, 16) rows in rank order.  gloo rejects a (world, k) output
    for a (k,) input, so the gather runs flat (found by the two-rank bench rehearsal on one GPU)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = [[w + 100 * r for w in range(16)] for r in range(world)]
    for _, shape, rows in out:
        assert shape == [world, 16] and rows == exp
