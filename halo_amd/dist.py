"""Multi-GPU sharding of the MSM: point-partition across ranks, all-gather of the
per-rank partial sums (one 64-B WrappedPoint each), combine by elliptic-curve addition.

RCCL (torch.distributed "nccl") has no EC-point reduction operator, so the collective is an
all-gather of the partials followed by a device-side sum (halo_point_sum).  There is no data-path
collective: every rank reads only its own resident SRS block and scalars.
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of points owned by `rank` (SRS block r, scalars r)."""
    per = (n_total + world - 1) // world
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


def allgather_points(partial: np.ndarray, dist, device=None) -> np.ndarray:
    """All-gather one WrappedPoint (8 x u64) per rank -> (world, 8) uint64 array."""
    import torch

    world = dist.get_world_size()
    t = torch.from_numpy(np.ascontiguousarray(partial, dtype=np.uint64).view(np.int64).copy())
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.stack([p.cpu().numpy().view(np.uint64) for p in parts])


def sharded_msm(partial_msm: Callable[[int, int], np.ndarray], point_sum: Callable[[np.ndarray], np.ndarray],
                n_total: int, dist, device=None) -> np.ndarray:
    """MSM over n_total points split across ranks: each rank computes partial_msm(lo, hi) over its
    block, partials are all-gathered and summed with point_sum (identical result on every rank)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = shard_range(n_total, rank, world)
    part = partial_msm(lo, hi)
    if world == 1:
        return part
    return point_sum(allgather_points(part, dist, device))


# ---------------------------------------------------------------------------------------------
# Distributed NTT: one transform of N = n1 n2 elements, natural order, rank r holding
# the contiguous block x[r N/P, (r+1) N/P) in and X[r N/P, (r+1) N/P) out.
#
# Four-step decomposition with i = i1 n2 + i2 and k = k1 + n1 k2:
#   X[k1 + n1 k2] = sum_i2 w_n2^(i2 k2) * w_N^(i2 k1) * sum_i1 w_n1^(i1 k1) x[i1 n2 + i2]
# Input blocks are i1-blocks; the inner DFT needs i2-blocks, the outer one k1-blocks, the output is
# k2-blocks: three all-to-alls of N/P^2 elements per rank pair.  Everything between the exchanges is
# device work: batched NTTs (halo_ntt_dev), the w_N^(i2 k1) twiddle (halo_ntt_twiddle_dev) and LDS
# transposes (halo_transpose_dev).
#
# At the BASELINE sizes a single transform fits one GPU's HBM many times over and one MI355X does a
# 2^24 NTT in ~2 ms, while each all-to-all moves 7/8 of 64 MiB per GPU over xGMI; so the prover's
# NTTs shard by transform (independent batches, no exchange) and this path exists for transforms
# beyond one GPU (and is measured in bench.py's multi-GPU extra).
# ---------------------------------------------------------------------------------------------
def ntt_dims(logn: int, world: int) -> tuple[int, int]:
    l1 = (logn + 1) // 2
    n1, n2 = 1 << l1, 1 << (logn - l1)
    if n1 % world or n2 % world:
        raise ValueError(f"2^{logn}-point distributed NTT needs world ({world}) dividing {n1} and {n2}")
    return n1, n2


class NttOps:
    """Device (or oracle) primitives the distributed NTT is built from.  Tensors are int64 views of
    (.., 4) u64 ark-format field elements."""

    def ntt_batch(self, t, log_len: int, batch: int, inverse: bool):  # in place, rows of 2^log_len
        raise NotImplementedError

    def twiddle(self, t, logn: int, rows: int, cols: int, row0: int, col0: int, inverse: bool):  # in place
        raise NotImplementedError

    def transpose(self, src, batch: int, rows: int, cols: int, run: int = 1):
        """-> new tensor: per batch, [rows][cols] of runs of `run` elements -> [cols][rows]."""
        raise NotImplementedError


class GpuNttOps(NttOps):
    def __init__(self, field: int, stream=None):
        from . import _lib
        self.H = _lib
        self.L = _lib.load()
        self.field = field
        self.stream = stream

    def _sp(self):
        import ctypes
        import torch
        s = self.stream if self.stream is not None else torch.cuda.current_stream().cuda_stream
        return ctypes.c_void_p(s)

    def ntt_batch(self, t, log_len, batch, inverse):
        import ctypes
        self.H.check(self.L.halo_ntt_dev(self.field, ctypes.c_void_p(t.data_ptr()), log_len, batch, int(inverse),
                                         self._sp()))

    def twiddle(self, t, logn, rows, cols, row0, col0, inverse):
        import ctypes
        self.H.check(self.L.halo_ntt_twiddle_dev(self.field, ctypes.c_void_p(t.data_ptr()), logn, rows, cols, row0,
                                                 col0, int(inverse), self._sp()))

    def transpose(self, src, batch, rows, cols, run=1):
        import ctypes
        import torch
        dst = torch.empty_like(src)
        self.H.check(self.L.halo_transpose_dev(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                               batch, rows, cols, run, self._sp()))
        return dst


def sharded_ntt_steps(x_local, logn: int, inverse: bool, ops: NttOps, rank: int, world: int):
    """Generator form of the rank-local distributed NTT: yields each all-to-all send buffer (P equal
    consecutive slices) and expects the received buffer back; returns this rank's output block."""
    N = 1 << logn
    P = world
    n1, n2 = ntt_dims(logn, P)
    n1p, n2p = n1 // P, n2 // P
    assert x_local.shape[0] == N // P
    l1, l2 = n1.bit_length() - 1, n2.bit_length() - 1
    # exchange 1: rows R_r as [n1p][P][n2p] -> [P][n1p][n2p] (column block C_s for rank s)
    recv = yield ops.transpose(x_local, 1, n1p, P, n2p)  # [t][a][i2_loc] = A[i1 = t n1p + a][i2_loc]
    B = ops.transpose(recv, 1, n1, n2p)  # [i2_loc][i1]
    ops.ntt_batch(B, l1, n2p, inverse)  # inner DFTs over i1 -> [i2_loc][k1]
    ops.twiddle(B, logn, n2p, n1, rank * n2p, 0, inverse)  # * w_N^(i2 k1)
    # exchange 2: [i2_loc][P][n1p] -> [P][i2_loc][n1p] (k1 block K_s for rank s)
    recv = yield ops.transpose(B, 1, n2p, P, n1p)  # [t][i2_loc(t)][k1_loc] = D[i2][k1_loc]
    E = ops.transpose(recv, 1, n2, n1p)  # [k1_loc][i2]
    ops.ntt_batch(E, l2, n1p, inverse)  # outer DFTs over i2 -> [k1_loc][k2]
    # exchange 3: [k1_loc][P][n2p] -> [P][k1_loc][n2p] (k2 block for rank s)
    recv = yield ops.transpose(E, 1, n1p, P, n2p)  # [t][k1_loc(t)][k2_loc] = F[k1][k2_loc]
    return ops.transpose(recv, 1, n1, n2p)  # [k2_loc][k1]: X[k1 + n1 (r n2p + k2_loc)]


def sharded_ntt(x_local, logn: int, inverse: bool, ops: NttOps, rank: int, world: int, alltoall):
    """Rank-local part of the distributed NTT.  x_local: (N/P, 4) int64 tensor, this rank's block of
    the input; returns this rank's block of the output.  alltoall(send) -> recv exchanges P equal
    consecutive slices (torch.distributed.all_to_all_single for real ranks)."""
    g = sharded_ntt_steps(x_local, logn, inverse, ops, rank, world)
    send = next(g)
    while True:
        try:
            send = g.send(alltoall(send))
        except StopIteration as e:
            return e.value


def sharded_ntt_virtual(x, logn: int, inverse: bool, ops: NttOps, world: int):
    """All `world` ranks of the distributed NTT in one process (lock-step, exchanges by slicing):
    exercises the device primitives and the data movement on a single GPU."""
    import torch

    per = x.shape[0] // world
    gens = [sharded_ntt_steps(x[r * per:(r + 1) * per].contiguous(), logn, inverse, ops, r, world)
            for r in range(world)]
    sends = [next(g) for g in gens]
    while True:
        sl = [s.view(world, -1, 4) for s in sends]
        recvs = [torch.cat([sl[t][r] for t in range(world)]).contiguous() for r in range(world)]
        outs = []
        done = False
        for g, rv in zip(gens, recvs):
            try:
                outs.append(g.send(rv))
            except StopIteration as e:
                outs.append(e.value)
                done = True
        if done:
            return torch.cat(outs)
        sends = outs


def torch_alltoall(dist):
    """alltoall over torch.distributed (RCCL on GPUs, gloo on CPU): P equal slices."""
    import torch

    def f(send):
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send)
        return recv
    return f
