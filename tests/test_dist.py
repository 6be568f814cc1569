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
