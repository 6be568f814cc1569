"""GPU parity: the device-resident naive_prover pipeline (halo_amd.prover; SURVEY §8f f1/f2/f4,
BASELINE configs[3]) against the same pipeline on the CPU restatement backend (oracle/prover_ref.py).

Every commitment (16 C_ws, C_z, 16 C_ts), the 91 evaluations of the proof, and the three IPA
openings (q_r, q_r_omega, acc::prover's open of h) must be bit-exact.  The device backend computes
the permutation accumulator with prefix/suffix product scans; the CPU backend by its sequential
per-element division (protocol.rs:143-154), so that formulation is checked too.
"""
import numpy as np
import pytest

from halo_amd import prover

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("curve,logn", [("pallas", 4), ("vesta", 4), ("pallas", 5)])
def test_naive_prover_matches_cpu_restatement(hal, curve, logn):
    from prover_ref import RefBackend

    n = 1 << logn
    L = hal.load()
    cid = hal.CURVES[curve]
    hal.check(L.halo_srs_synthesize(cid, n, 4242 + logn))
    srs = np.zeros((n, 8), dtype=np.uint64)
    hal.check(L.halo_srs_read(cid, 0, n, hal.ptr(srs)))

    dev = prover.DeviceBackend(curve)
    ref = RefBackend(curve, srs, srs[1])
    outs = []
    for B in (dev, ref):
        wit = prover.synthetic_witness(B, n, seed=7)
        outs.append(prover.naive_prover(B, wit, n, prover.Challenges(B.m)))
    d, r = outs

    def same_points(a, b):
        return len(a) == len(b) and all(np.array_equal(x, y) for x, y in zip(a, b))

    assert same_points(d["C_ws"], r["C_ws"])
    assert np.array_equal(d["C_z"], r["C_z"])
    assert same_points(d["C_ts"], r["C_ts"])
    assert d["vs"] == r["vs"]
    for key in ("q_r", "q_r_omega", "acc"):
        a, b = d[key], r[key]
        assert np.array_equal(a["C"], b["C"]), key
        assert a["v"] == b["v"], key
        assert same_points(a["Ls"], b["Ls"]) and same_points(a["Rs"], b["Rs"]), key
        assert np.array_equal(a["U"], b["U"]) and a["c"] == b["c"], key


@pytest.mark.parametrize("curve", ["pallas", "vesta"])
def test_naive_prover_2p16_matches_c_restatement(hal, curve):
    """The production paths inside the prover at the reference's own circuit size (the IVC circuits
    are 2^16 rows, crates/plonk/src/frontend/ivc/mod.rs:54,111): bucket MSMs over the window-shifted
    SRS, the batched commitments (protocol.rs:114,263), the 2-pass NTTs of 2^16..2^20 and the
    weighted -> materialised -> tail IPA rounds, all compared bit for bit with the same pipeline on
    the C restatement backend (oracle/prover_ref.py CRefBackend, OpenMP): 16 C_ws, C_z, 16 C_ts,
    the 91 evaluations, and the three openings (C, v, Ls, Rs, U, c)."""
    import os
    from prover_ref import CRefBackend

    logn = 16
    n = 1 << logn
    L = hal.load()
    cid = hal.CURVES[curve]
    hal.check(L.halo_srs_synthesize(cid, n, 0x505256 + logn))
    hal.check(L.halo_srs_precompute_windows(cid))
    srs = np.zeros((n, 8), dtype=np.uint64)
    hal.check(L.halo_srs_read(cid, 0, n, hal.ptr(srs)))
    dev = prover.DeviceBackend(curve)
    ref = CRefBackend(curve, srs, srs[1], threads=min(16, os.cpu_count() or 8))
    outs = []
    for B in (dev, ref):
        wit = prover.synthetic_witness(B, n, seed=1)
        outs.append(prover.naive_prover(B, wit, n, prover.Challenges(B.m)))
    d, r = outs

    def same_points(a, b):
        return len(a) == len(b) and all(np.array_equal(x, y) for x, y in zip(a, b))

    assert len(d["C_ws"]) == 16 and len(d["C_ts"]) == 16 and len(d["vs"]) >= 78
    assert same_points(d["C_ws"], r["C_ws"])
    assert np.array_equal(d["C_z"], r["C_z"])
    assert same_points(d["C_ts"], r["C_ts"])
    assert d["vs"] == r["vs"]
    for key in ("q_r", "q_r_omega", "acc"):
        a, b = d[key], r[key]
        assert len(a["Ls"]) == logn, key
        assert np.array_equal(a["C"], b["C"]), key
        assert a["v"] == b["v"], key
        assert same_points(a["Ls"], b["Ls"]) and same_points(a["Rs"], b["Rs"]), key
        assert np.array_equal(a["U"], b["U"]) and a["c"] == b["c"], key


def test_permutation_accumulator_scan_large(hal):
    """z via prefix/suffix scans at 2^18 (multi-block scan path) vs the sequential definition."""
    import torch

    dev = prover.DeviceBackend("pallas")
    n = 1 << 18
    rng = np.random.default_rng(5)
    f = prover.DevEvals(dev, dev.random_vec(n, rng))
    g = prover.DevEvals(dev, dev.random_vec(n, rng))
    z = dev.permutation_accumulator(f, g).t.cpu().numpy().view(np.uint64)
    fi = [dev.to_int(x) for x in f.t.cpu().numpy().view(np.uint64)]
    gi = [dev.to_int(x) for x in g.t.cpu().numpy().view(np.uint64)]
    m = dev.m
    # sequential definition on a sample of positions: z[i] = prod_{j=1..i} f_j / g_j
    num = den = 1
    checks = {0, 1, 2, 2047, 2048, 2049, 65535, n // 2, n - 2, n - 1}
    for i in range(n):
        if i:
            num = num * fi[i] % m
            den = den * gi[i] % m
        if i in checks:
            assert dev.to_int(z[i]) == num * pow(den, -1, m) % m, i
    torch.cuda.synchronize()


@pytest.mark.parametrize("curve,logn,mode", [
    ("pallas", 12, "fold"), ("pallas", 13, "fold"), ("pallas", 13, "fold_srs_round0"),
    ("pallas", 12, "weighted"), ("pallas", 14, "weighted"), ("vesta", 13, "weighted"),
    ("pallas", 13, "weighted_to_end"), ("pallas", 15, "weighted"), ("pallas", 12, "weighted_fold_after"),
    ("pallas", 13, "srs_tail"), ("vesta", 12, "srs_tail"),
])
def test_ipa_open_tail_switch_vs_c_restatement(hal, curve, logn, mode):
    """An SRS-based opening longer than the tail threshold (2048), against the C restatement of
    pcdl.rs:404-438 (Ls, Rs, U, c).  fold: ordinary rounds (MSM L/R + GLV fold of G) switch to the
    tail rounds (direct sums over G0 with fold weights) mid-opening; fold_srs_round0: the same with
    round 1's L / R on the resident window-shifted SRS (ranges [0, m), [m, 2m)); weighted (the default
    with the shifted SRS): G is never folded, every round's L / R are block-mapped MSMs over the
    shifted SRS with scalars c * w until the length reaches 1024, where G is materialised by one
    batched shared-scalar MSM and the tail rounds finish; weighted_to_end: no switch, U = sum w[u] G[u]
    at the end; weighted_fold_after: the materialised G continues with ordinary rounds; srs_tail:
    every round a tail round over the SRS's own multiples table (no weighted rounds, no materialised G)."""
    n = 1 << logn
    L = hal.load()
    cid = hal.CURVES[curve]
    hal.check(L.halo_srs_synthesize(cid, n, 777 + logn))
    if mode != "fold":
        hal.check(L.halo_srs_precompute_windows(cid))
    knobs = {"ipa_weighted": 1 if mode.startswith("weighted") else 0,
             # srs_tail (the default up to 2^12): tail rounds from round 1 over the SRS's multiples
             # table; the other modes pin the weighted / fold paths at these sizes
             "ipa_srs_tail_n": n if mode == "srs_tail" else 0}
    if mode == "weighted_to_end":  # no switch to the tail rounds: U = sum w[u] G[u] over the SRS
        knobs["ipa_mat_n"] = 0
    if mode == "weighted_fold_after":  # materialised G (affine) continues with L/R MSMs + GLV folds
        knobs["ipa_tail"] = 0
    with hal.tuning(**knobs):
        _ipa_open_vs_c(hal, L, cid, curve, n, logn)


def _ipa_open_vs_c(hal, L, cid, curve, n, logn):
    from prover_ref import CRefBackend

    srs = np.zeros((n, 8), dtype=np.uint64)
    hal.check(L.halo_srs_read(cid, 0, n, hal.ptr(srs)))
    dev = prover.DeviceBackend(curve)
    ref = CRefBackend(curve, srs, srs[1])
    rng = np.random.default_rng(logn)
    p_dev = dev.random_vec(n, rng)
    p_ref = p_dev.cpu().numpy().view(np.uint64).copy()
    z, xi0 = 0x1234567, 0xABCDEF
    a = dev.ipa(p_dev, n, z, dev.h_mul(xi0), prover.Challenges(dev.m, seed=5))
    b = ref.ipa(p_ref, n, z, ref.h_mul(xi0), prover.Challenges(ref.m, seed=5))
    assert all(np.array_equal(x, y) for x, y in zip(a[0], b[0]))
    assert all(np.array_equal(x, y) for x, y in zip(a[1], b[1]))
    assert np.array_equal(a[2], b[2]) and a[3] == b[3]


def test_pooled_session_releases_large_buffers(hal):
    """an idle pooled IPA session keeps at most "ipa_pool_keep_bytes" of device buffers.
    A 2^18 opening (weighted rounds, materialised G, the session's own 126 MB tail table) is run on a
    drained pool (halo_shutdown) and the device memory it leaves allocated is compared between the
    default cap (1 GB: the session keeps its buffers for the next opening) and a 64 MB cap (released
    at halo_ipa_end): the difference is the session's large buffers, the tail table at least."""
    import torch

    n = 1 << 18
    L = hal.load()
    cid = hal.CURVES["pallas"]
    hal.check(L.halo_srs_synthesize(cid, n, 4218))
    hal.check(L.halo_srs_precompute_windows(cid))
    dev = prover.DeviceBackend("pallas")
    rng = np.random.default_rng(18)
    p = dev.random_vec(n, rng)

    def opening():
        return dev.ipa(p, n, 0x1234567, dev.h_mul(0xABCDEF), prover.Challenges(dev.m, seed=5))

    ref = opening()  # warms the shared scratch (MSM sets, SRS-derived tables)
    kept = {}
    for cap in (-1, 64 << 20):
        with hal.tuning(ipa_pool_keep_bytes=cap):
            hal.check(L.halo_shutdown())  # drains the session pool (the library stays usable)
            torch.cuda.synchronize()
            free0 = torch.cuda.mem_get_info()[0]
            got = opening()
            torch.cuda.synchronize()
            kept[cap] = free0 - torch.cuda.mem_get_info()[0]
        assert np.array_equal(got[2], ref[2]) and got[3] == ref[3]
    assert kept[-1] - kept[64 << 20] > (100 << 20), {k: v / 2**20 for k, v in kept.items()}
