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


def allgather_words(words: np.ndarray, dist, device=None) -> np.ndarray:
    """All-gather a fixed-shape uint64 array from every rank as one tensor collective (RCCL over xGMI
    when `device` is a GPU, gloo on the CPU; no object pickling) -> (world, *shape) uint64 array."""
    import torch

    world = dist.get_world_size()
    a = np.ascontiguousarray(words, dtype=np.uint64)
    t = torch.from_numpy(a.reshape(-1).view(np.int64).copy())
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return torch.stack(parts).cpu().numpy().view(np.uint64).reshape((world,) + a.shape)


def allgather_rows(t, dist):
    """One flat all_gather_into_tensor of a rank's 1-D tensor `t` (k words) -> (world, k) tensor on t's
    device.  The output is allocated flat (world * k), the form both RCCL and gloo accept."""
    import torch

    world = dist.get_world_size()
    flat = t.reshape(-1)
    out = torch.empty(world * flat.numel(), dtype=flat.dtype, device=flat.device)
    dist.all_gather_into_tensor(out, flat)
    return out.view(world, flat.numel())


def allgather_points(partial: np.ndarray, dist, device=None) -> np.ndarray:
    """All-gather one WrappedPoint (8 x u64) per rank -> (world, 8) uint64 array."""
    return allgather_words(np.asarray(partial, dtype=np.uint64).reshape(8), dist, device)


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
# Window partition (BASELINE configs[4]): every rank holds the SAME scalars (broadcast from rank 0)
# and the same window-shifted SRS copies; rank r takes the windows window_range(W, r, P) of every
# scalar (halo_msm_srs_windows_dev).  With the shifted copies 2^(c w) G the per-window sums are
# already weighted, so the partials simply add: the same all-gather + point sum as point-partition.
# It costs a scalar broadcast (32 B x n over xGMI) that point-partition does not need; the window
# width is chosen so that W divides the world size (partition_window_bits: 16 windows of 16 bits over
# 8 ranks) and each rank precomputes only its own windows' copies (halo_srs_precompute_window_range).
# Point-partition stays the default; this path is measured beside it in bench.py.
# ---------------------------------------------------------------------------------------------
def partition_window_bits(world: int) -> int:
    """Window width for a window partition over `world` ranks: the default 17 bits (15 windows) when
    15 splits evenly, else the nearest width whose window count W = ceil(255 / c) does (16 bits: 16
    windows for 2, 4, 8, 16 ranks), so no rank carries an extra window (15 over 8 ranks would cap the
    split at 7.5x)."""
    for c in (17, 16, 15, 18, 14):
        if (-(-255 // c)) % world == 0:
            return c
    return 17


def window_range(W: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous windows [lo, hi) of rank r: the first W % P ranks take one more."""
    base, extra = divmod(W, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def window_partitioned_msm(partial_windows: Callable[[int, int], np.ndarray],
                           point_sum: Callable[[np.ndarray], np.ndarray], W: int, dist, device=None) -> np.ndarray:
    """MSM whose W windows are split across ranks: partial_windows(lo, hi) is this rank's share (the
    scalars are replicated on every rank), partials all-gathered and summed on every rank."""
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = window_range(W, rank, world)
    part = partial_windows(lo, hi) if hi > lo else np.zeros(8, dtype=np.uint64)
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


# ---------------------------------------------------------------------------------------------
# Distributed polynomial evaluation (SURVEY §8e "Poly eval"): rank r holds the coefficient block
# [lo_r, hi_r) (shard_range) and evaluates it at z; p(z) = sum_r z^lo_r v_r.  With equal blocks
# lo_r = r * per, so the combine is the evaluation of the polynomial (v_0 .. v_{P-1}) at z^per:
# one all-gather of 32 B per rank and two tiny device calls (x^e, Horner), no host field math.
# ---------------------------------------------------------------------------------------------
class PolyOps:
    """Device primitives of the distributed evaluation: Horner of k polynomials at one point and
    z^e."""

    def __init__(self, field="fp"):
        self.field = field

    def eval_batch(self, polys, z):
        from .poly import evaluate_batch

        return evaluate_batch(polys, z, self.field)

    def pow(self, z, e: int):
        from . import _lib as H
        from .group import _field

        zz = H.fe_array(z, 1)
        w = np.zeros((1, 4), dtype=np.uint64)
        H.check(H.load().halo_evals_op(_field(self.field), 6, H.ptr(zz), None, None, e, H.ptr(w), 1))
        return w[0]


def poly_eval_partial(coeffs_local, z, ops: PolyOps) -> np.ndarray:
    """v_r = sum_i coeffs_local[i] z^i (this rank's block, unshifted)."""
    if len(coeffs_local) == 0:
        return np.zeros(4, dtype=np.uint64)
    return np.asarray(ops.eval_batch([coeffs_local], z)[0], dtype=np.uint64)


def poly_eval_combine(parts, n_total: int, z, ops: PolyOps) -> np.ndarray:
    """p(z) = sum_r (z^per)^r v_r for the equal blocks of shard_range."""
    world = len(parts)
    if world == 1:
        return np.asarray(parts[0], dtype=np.uint64)
    per = (n_total + world - 1) // world
    return np.asarray(ops.eval_batch([np.stack(parts)], ops.pow(z, per))[0], dtype=np.uint64)


def sharded_poly_eval(coeffs_local, n_total: int, z, dist, ops: PolyOps | None = None, device=None) -> np.ndarray:
    """DensePolynomial::evaluate (pcdl.rs:49,471) of a polynomial whose coefficients are split into
    contiguous blocks over the ranks (rank r holds coeffs[shard_range(n_total, r, P)]).  The 32-B
    partial values travel as one tensor all-gather (RCCL when `device` is the rank's GPU)."""
    ops = ops or PolyOps()
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = shard_range(n_total, rank, world)
    if len(coeffs_local) != hi - lo:
        raise ValueError("coefficient block does not match shard_range")
    parts = allgather_words(poly_eval_partial(coeffs_local, z, ops), dist, device)
    return poly_eval_combine(list(parts), n_total, z, ops)


# ---------------------------------------------------------------------------------------------
# Distributed IPA opening (SURVEY §8e "IPA fold ... shards by j"): the round loop of
# open_without_eval (pcdl.rs:404-438) over P ranks.  Rank r holds the strided shard
# G[i P + r], c[i P + r], z[i P + r] (i < n / P).  While the half-length m is a multiple of P the
# fold pairs j and j + m lie on the same rank (local i and i + m / P), so every fold is local and
# the local session is the single-GPU one.  L and R are linear in the shards: L = sum_r L_r with
# each L_r carrying its own <c_r, z_l>_r H' term, so a round all-gathers two points per rank and
# sums them on the device, and every rank runs the same transcript.  After lg(n / P) rounds each
# rank holds one element; the P elements are all-gathered (global order j = r) and the last lg P
# rounds run on one session, replicated on every rank (all ranks return the same proof).
#
# Two kinds of shard session (round 5):
#  * weighted (GpuWeightedIpaOps, the default on GPUs): the rank's resident SRS IS its shard
#    G[r::P] (uploaded with its window-shifted copies, as a rank of a sharded deployment holds it), so
#    the shard runs the single-GPU weighted rounds (n/2-term MSMs over the resident copies, no fold of
#    G).  Its z-vector z^(i P + r) = z^r (z^P)^i is the session's powers of z^P with the factor z^r
#    moved onto the hiding point: H'_r = z^r H' (the dots <c, z> are linear in z), and the shard's final
#    z is z^r times the session's folded one.
#  * explicit vectors (GpuIpaOps): G, c, z of the shard handed over (halo_ipa_begin_vectors), G folded
#    by GLV scalar multiplications every round -- the collapsed final rounds, and shards of an SRS that
#    is not resident.
# ---------------------------------------------------------------------------------------------
def ipa_shard(vec, rank: int, world: int):
    """Rank r's strided shard vec[r::P] of an IPA vector."""
    return np.ascontiguousarray(np.asarray(vec)[rank::world])


class IpaOps:
    """Per-rank session primitives the distributed opening is written against.  ``shard`` is the
    ops' own description of one rank's part (explicit (gs, cs, zs) vectors, or (cs, z) over a
    resident SRS shard)."""

    def begin(self, shard, H_prime):
        raise NotImplementedError

    def round_lr(self, ses):  # -> (L, R) WrappedPoints of this shard (H' terms included)
        raise NotImplementedError

    def round_lr_dev(self, ses):  # -> the same pair left on the device (sharded_ipa_rounds device_lr=True)
        raise NotImplementedError

    def fold(self, ses, xi, xi_inv):
        raise NotImplementedError

    def final(self, ses):  # -> (g (1, 8), c (1, 4), z (1, 4)) once fully folded
        raise NotImplementedError

    def point_sum(self, pts):  # (k, 8) WrappedPoints -> (8,)
        raise NotImplementedError

    def begin_vectors(self, gs, cs, zs, H_prime):  # the collapsed final rounds' session
        return self.begin((gs, cs, zs), H_prime)

    def final_vectors(self, ses):  # ... and its folded element
        return self.final(ses)

    def shard_len(self, shard) -> int:
        return len(shard[1])

    def trivial_final(self, shard):  # n / P == 1: the shard's only element, (g (1, 8), c (1, 4), z (1, 4))
        g, c, z = shard
        return (np.asarray(g, dtype=np.uint64).reshape(-1, 8)[:1], np.asarray(c, dtype=np.uint64).reshape(-1, 4)[:1],
                np.asarray(z, dtype=np.uint64).reshape(-1, 4)[:1])


class GpuIpaOps(IpaOps):
    """Shard sessions over explicit vectors: shard = (gs, cs, zs)."""

    def __init__(self, curve="pallas"):
        self.curve = curve

    def begin(self, shard, H_prime):
        from .pcdl import IpaSession

        gs, cs, zs = shard
        return IpaSession.from_vectors(gs, cs, zs, H_prime, self.curve)

    def round_lr(self, ses):
        return ses.round_lr()

    def round_lr_dev(self, ses):
        """L_r, R_r as one device tensor (32 int64 = two packed XYZZ points, halo_ipa_round_lr_dev) on the
        current torch stream: no host round trip; torch_reduce_lr_dev gathers and sums them."""
        import torch

        t = torch.empty(32, dtype=torch.int64, device="cuda")
        ses.round_lr_dev(t.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return t

    def fold(self, ses, xi, xi_inv):
        ses.fold(xi, xi_inv)

    def final(self, ses):
        _, gs, cs, zs = ses.state()
        ses.end()
        return gs[:1], cs[:1], zs[:1]

    def point_sum(self, pts):
        from .group import point_sum

        return point_sum(pts, self.curve)


class GpuWeightedIpaOps(GpuIpaOps):
    """Shard sessions over the rank's resident SRS shard G[rank::world] (weighted rounds):
    shard = (cs_shard, z) with z the opening point (ark scalar)."""

    def __init__(self, curve, rank: int, world: int):
        super().__init__(curve)
        self.rank, self.world = rank, world

    def _field(self):
        return "fp" if self.curve in ("pallas", 0) else "fq"

    def _pow(self, z, e: int):
        from . import _lib as H
        from .group import _field

        zz = H.fe_array(z, 1)
        out = np.zeros((1, 4), dtype=np.uint64)
        H.check(H.load().halo_evals_op(_field(self._field()), 6, H.ptr(zz), None, None, e, H.ptr(out), 1))
        return out[0]

    def begin(self, shard, H_prime):
        from .group import point_dot_affine
        from .pcdl import IpaSession

        cs, z = shard
        z_r = self._pow(z, self.rank)
        hp = np.asarray(H_prime, dtype=np.uint64).reshape(1, 8)
        h_r = hp[0] if self.rank == 0 else point_dot_affine(z_r.reshape(1, 4), hp, self.curve)
        ses = IpaSession(cs, self._pow(z, self.world), h_r, self.curve)
        ses._z_r = z_r
        return ses

    def final(self, ses):
        from .group import scalar_dot

        _, _, cs, zs = ses.state(with_gs=False)
        U, c = ses.end()
        z = scalar_dot(ses._z_r.reshape(1, 4), zs[:1], self._field())
        return U.reshape(1, 8), c.reshape(1, 4), np.asarray(z, dtype=np.uint64).reshape(1, 4)

    def begin_vectors(self, gs, cs, zs, H_prime):
        return GpuIpaOps.begin(self, (gs, cs, zs), H_prime)

    def final_vectors(self, ses):
        return GpuIpaOps.final(self, ses)

    def shard_len(self, shard) -> int:
        return len(shard[0])

    def trivial_final(self, shard):
        """n / P == 1: the shard is the global element j = rank -- G_rank is element 0 of the rank's
        resident SRS shard, c_rank the shard's one scalar, and z_rank = z^rank."""
        from . import _lib as H
        from .group import _curve

        cs, z = shard
        g = np.zeros((1, 8), dtype=np.uint64)
        H.check(H.load().halo_srs_read(_curve(self.curve), 0, 1, H.ptr(g)))
        return g, np.asarray(cs, dtype=np.uint64).reshape(-1, 4)[:1].copy(), self._pow(z, self.rank).reshape(1, 4)


def ipa_shard_steps(ops: IpaOps, shard, H_prime, rounds: int, device_lr: bool = False):
    """One rank's shard session as a generator: yields (L_r, R_r) each round (device_lr: the pair as a
    device tensor, ops.round_lr_dev), receives (xi, xi_inv), returns the fully folded (g, c, z) element."""
    ses = ops.begin(shard, H_prime)
    for _ in range(rounds):
        xi, xi_inv = yield (ops.round_lr_dev(ses) if device_lr else ops.round_lr(ses))
        ops.fold(ses, xi, xi_inv)
    return ops.final(ses)


def _drive(gens, reduce_lr, challenge, inverse, xi, Ls, Rs, rounds: int):
    lrs = [next(g) for g in gens]
    finals = []
    for k in range(rounds):
        L, R = reduce_lr(lrs)
        Ls.append(L)
        Rs.append(R)
        xi = challenge(xi, L, R)
        xinv = inverse(xi)
        lrs = []
        for g in gens:
            try:
                lrs.append(g.send((xi, xinv)))
            except StopIteration as e:
                finals.append(e.value)
    return xi, finals


def sharded_ipa_rounds(local_shards, H_prime, challenge: Callable, inverse: Callable, ops: IpaOps, world: int,
                       gather: Callable, reduce_lr: Callable | None = None, device_lr: bool = False):
    """Distributed pcdl round loop.  ``local_shards``: the shards this process holds (ops.begin's
    description; (gs, cs, zs) strided vectors for GpuIpaOps, (cs, z) for GpuWeightedIpaOps) -- one
    with a real communicator, all P with virtual ranks; ``gather(objs)`` returns the list of every
    rank's objs in rank order (torch_gather_arrays(dist), or identity for virtual ranks);
    ``reduce_lr(local (L_r, R_r) list) -> (L, R)`` the round's sums over every rank (default: gather,
    then ops.point_sum; torch_reduce_lr sums on the device).  device_lr: the shard rounds leave L_r, R_r
    on the device (ops.round_lr_dev) and reduce_lr is torch_reduce_lr_dev (gather, XYZZ sum and one D2H).
    Returns (Ls, Rs, U, c) exactly as the single-session ipa_rounds does."""
    if world < 1 or world & (world - 1):
        raise ValueError("world size must be a power of two")
    n_loc = ops.shard_len(local_shards[0])
    if n_loc < 1 or n_loc & (n_loc - 1):
        raise ValueError("n / P must be a power of two")
    if reduce_lr is None:
        def reduce_lr(lrs):
            parts = gather(lrs)
            return (ops.point_sum(np.stack([p[0] for p in parts])), ops.point_sum(np.stack([p[1] for p in parts])))
    Ls, Rs = [], []
    xi = None
    if n_loc >= 2:
        gens = [ipa_shard_steps(ops, sh, H_prime, n_loc.bit_length() - 1, device_lr) for sh in local_shards]
        xi, finals = _drive(gens, reduce_lr, challenge, inverse, xi, Ls, Rs, n_loc.bit_length() - 1)
        finals = gather(finals)
    else:  # one element per rank: no shard rounds
        finals = gather([ops.trivial_final(sh) for sh in local_shards])
    G = np.concatenate([f[0] for f in finals])
    C = np.concatenate([f[1] for f in finals])
    Z = np.concatenate([f[2] for f in finals])
    if world > 1:
        ses = ops.begin_vectors(G, C, Z, H_prime)
        for _ in range(world.bit_length() - 1):
            L, R = ops.round_lr(ses)
            Ls.append(L)
            Rs.append(R)
            xi = challenge(xi, L, R)
            ops.fold(ses, xi, inverse(xi))
        G, C, _ = ops.final_vectors(ses)
    return Ls, Rs, np.asarray(G[0], dtype=np.uint64), np.asarray(C[0], dtype=np.uint64)


def sharded_ipa_fixed_challenges(ops_for_rank: Callable, shard_for_rank: Callable, H_prime, xis, xi_invs, world: int,
                                 point_sum: Callable, ops_final: IpaOps, reduce_pairs: Callable | None = None):
    """Virtual ranks run ONE AT A TIME (each may need its own resident SRS shard) against a challenge
    sequence fixed in advance (xis[k] for round k, independent of L and R): rank r's generator is
    driven to the end before rank r + 1 starts, then the per-round L_r, R_r are summed and the last
    lg P rounds run on the gathered finals.  Used by the GPU test of the weighted shards on one
    device; the live transcript needs real ranks (sharded_ipa_rounds).  reduce_pairs: the shards leave
    L_r, R_r on the device (ops.round_lr_dev) and reduce_pairs((P, 32) device rows) sums them
    (xyzz_pair_reducer), as torch_reduce_lr_dev does after its all-gather.  Returns (Ls, Rs, U, c)."""
    per_rank, finals = [], []
    rounds = None
    for r in range(world):
        ops = ops_for_rank(r)
        shard = shard_for_rank(r)
        rounds = ops.shard_len(shard).bit_length() - 1
        g = ipa_shard_steps(ops, shard, H_prime, rounds, reduce_pairs is not None)
        lr = [next(g)]
        for k in range(rounds):
            try:
                lr.append(g.send((xis[k], xi_invs[k])))
            except StopIteration as e:
                finals.append(e.value)
        per_rank.append(lr[:rounds])
    if reduce_pairs is not None:
        import torch

        pairs = [reduce_pairs(torch.stack([per_rank[r][k] for r in range(world)])) for k in range(rounds)]
        Ls, Rs = [p[0] for p in pairs], [p[1] for p in pairs]
    else:
        Ls = [point_sum(np.stack([per_rank[r][k][0] for r in range(world)])) for k in range(rounds)]
        Rs = [point_sum(np.stack([per_rank[r][k][1] for r in range(world)])) for k in range(rounds)]
    G = np.concatenate([f[0] for f in finals])
    C = np.concatenate([f[1] for f in finals])
    Z = np.concatenate([f[2] for f in finals])
    ses = ops_final.begin_vectors(G, C, Z, H_prime)
    for k in range(rounds, rounds + world.bit_length() - 1):
        L, R = ops_final.round_lr(ses)
        Ls.append(L)
        Rs.append(R)
        ops_final.fold(ses, xis[k], xi_invs[k])
    G, C, _ = ops_final.final_vectors(ses)
    return Ls, Rs, np.asarray(G[0], dtype=np.uint64), np.asarray(C[0], dtype=np.uint64)


def torch_gather_arrays(dist, device=None):
    """gather() for sharded_ipa_rounds over a torch.distributed group: each rank's objs (tuples of
    uint64 arrays whose shapes are the same on every rank: (L, R) points, or the final (g, c, z)) are
    flattened into one word vector and exchanged by one tensor all-gather (RCCL when `device` is the
    rank's GPU, gloo on the CPU) -- no object pickling on the data path."""

    def f(objs):
        objs = [tuple(np.ascontiguousarray(a, dtype=np.uint64) for a in o) for o in objs]
        shapes = [[a.shape for a in o] for o in objs]
        flat = np.concatenate([a.reshape(-1) for o in objs for a in o]) if objs else np.zeros(0, np.uint64)
        got = allgather_words(flat, dist, device)
        out = []
        for r in range(got.shape[0]):
            pos = 0
            for shp in shapes:
                parts = []
                for sh in shp:
                    k = int(np.prod(sh))
                    parts.append(got[r, pos:pos + k].reshape(sh))
                    pos += k
                out.append(tuple(parts))
        return out

    return f


def torch_reduce_lr(dist, curve, device):
    """reduce_lr() for sharded_ipa_rounds with one shard per rank on a GPU: the rank's (L_r, R_r)
    (2 x 64 B) go to the device once, one all_gather_into_tensor over RCCL collects every rank's,
    and halo_point_sum_dev sums the L column and the R column on the device; only the two sums come
    back to the host, for the transcript."""
    import ctypes

    import torch

    from . import _lib as H
    from .group import _curve

    world = dist.get_world_size()
    L_ = H.load()
    cid = _curve(curve)

    # gloo (the one-GPU rehearsal) gathers host tensors; RCCL gathers on the device
    gdev = device if dist.get_backend() == "nccl" else "cpu"

    def f(lrs):
        (Lr, Rr), = lrs
        t = torch.from_numpy(np.concatenate([np.asarray(Lr, np.uint64).reshape(8),
                                             np.asarray(Rr, np.uint64).reshape(8)]).view(np.int64)).to(gdev)
        allv = allgather_rows(t, dist).to(device)
        cols = (allv[:, :8].contiguous(), allv[:, 8:].contiguous())  # every rank's L, every rank's R
        out = torch.empty(16, dtype=torch.int64, device=device)
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for k in range(2):
            H.check(L_.halo_point_sum_dev(cid, ctypes.c_void_p(cols[k].data_ptr()), world, 64,
                                          ctypes.c_void_p(out.data_ptr() + 64 * k), sp))
        o = out.cpu().numpy().view(np.uint64)
        return o[:8].copy(), o[8:].copy()

    return f


def xyzz_pair_reducer(curve, device):
    """The device half of torch_reduce_lr_dev: rows (k, 32) int64 on the device, row r = rank r's L_r | R_r
    as packed XYZZ -> (L, R) WrappedPoints: halo_point_sum_xyzz_dev over each column (no inversion on the
    device), one D2H of the two sums, host conversion (halo_xyzz_to_wrapped)."""
    import ctypes

    import torch

    from . import _lib as H
    from .group import _curve

    L_ = H.load()
    cid = _curve(curve)
    out = torch.empty(32, dtype=torch.int64, device=device)
    wrapped = np.zeros((2, 8), dtype=np.uint64)

    def f(rows):
        rows = rows.contiguous()
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for k in range(2):
            H.check(L_.halo_point_sum_xyzz_dev(cid, ctypes.c_void_p(rows.data_ptr() + 128 * k), rows.shape[0], 256,
                                               ctypes.c_void_p(out.data_ptr() + 128 * k), sp))
        host = np.ascontiguousarray(out.cpu().numpy())
        H.check(L_.halo_xyzz_to_wrapped(cid, H.ptr(host), 2, H.ptr(wrapped)))
        return wrapped[0].copy(), wrapped[1].copy()

    return f


def torch_reduce_lr_dev(dist, curve, device):
    """reduce_lr() for sharded_ipa_rounds(device_lr=True), one shard per rank: the rank's (L_r, R_r) is
    already on the device as packed XYZZ (GpuIpaOps.round_lr_dev), one all_gather_into_tensor over RCCL
    collects every rank's 256 B, and xyzz_pair_reducer sums the L and R columns on the device and brings
    the two sums home in one D2H.  Against torch_reduce_lr: no D2H + host conversion + H2D of the rank's
    own pair, and no lone-lane affine conversion in the device sums."""
    gloo = dist.get_backend() != "nccl"  # (the one-GPU rehearsal gathers host tensors)
    pair_sum = xyzz_pair_reducer(curve, device)

    def f(lrs):
        (t,) = lrs
        return pair_sum(allgather_rows(t.cpu() if gloo else t, dist).to(device))

    return f
