"""GPU parity at the north-star sizes (BASELINE.json north_star: "2^24-point MSM and 2^24-element
NTT bit-exact"; configs[3]: the full prove at n = 2^20).

* 2^24-point MSM over a synthetic SRS G_j = k_j G (beyond the reference's N = 2^20): bit-exact through
  the known-log identity MSM(G, s) = (sum_j s_j k_j) G, the dot product and the generator
  multiplication done by the C oracle (corc.known_log_msm).
* 2^24-element NTT and iNTT over Fp (and the forward NTT over Fq) against the C oracle's
  ark-poly radix-2 restatement, element by element.
* naive_prover at n = 2^20 on the device: its three openings (the two Instance::open of round 5 and
  acc::prover's open of h) pass the CPU restatement of pcdl::succinct_check (oracle/pcdl_check.py,
  pcdl.rs:483-554) and the decider identity U == commit(h) (pcdl.rs:563-583) against the oracle MSM.
"""
import numpy as np
import pytest

import pasta as P
from halo_amd import group, pcdl

pytestmark = pytest.mark.gpu


def rand_words(n, seed, top_mask=0x0FFFFFFFFFFFFFFF):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * np.uint64(2)
    a |= rng.integers(0, 2, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64(top_mask)  # < 2^252 < r: valid Montgomery words
    return np.ascontiguousarray(a)


def test_msm_2p24_synthetic_srs_known_logs(hal, corc):
    n = 1 << 24
    seed = 0x2424
    group.PublicParams.synthesize("pallas", n, seed, precompute_windows=True)
    k = corc.synth_scalars(seed, n)
    from halo_amd.group import synth_scalar
    assert [P.limbs_to_int(k[j]) for j in (0, 1, n - 1)] == [synth_scalar(seed, j) for j in (0, 1, n - 1)]
    sc = rand_words(n, 24)
    sc[0] = 0                                                                  # zero scalar
    sc[1] = P.int_to_limbs(P.to_mont(P.FP_MODULUS - 1, P.FP_MODULUS))         # r - 1
    sc[2:1026] = sc[3000]                                                      # a skewed bucket
    got = pcdl.commit(sc, n - 1, None, "pallas")
    assert np.array_equal(got, corc.known_log_msm("pallas", sc, k))
    # a ragged prefix (n_scalars < n_bases: the MSM length is the shorter one, pedersen.rs:21)
    m = (1 << 23) + 12345
    got = pcdl.commit(sc[:m], n - 1, None, "pallas")
    assert np.array_equal(got, corc.known_log_msm("pallas", sc[:m], k[:m]))


def test_msm_2p24_window_partitioned_virtual_ranks_known_logs(hal, corc):
    """BASELINE configs[4] at its size on one GPU: the 2^24-point MSM split by windows over 8 virtual
    ranks (halo_amd.dist.window_range, the ranges bench.py --gpus 8 gives its ranks), each rank's
    partial from halo_msm_srs_windows_dev, the partials summed on the device (halo_point_sum_dev, the
    RCCL leg's combine) -- checked against the known-log identity (an independent oracle, not the
    device's own one-GPU MSM); and the 3-rank partition of the same MSM."""
    import ctypes

    import torch
    from halo_amd.dist import window_range

    L = hal.load()
    n = 1 << 24
    seed = 0x57494E44
    group.PublicParams.synthesize("pallas", n, seed, precompute_windows=True)
    k = corc.synth_scalars(seed, n)
    sc = rand_words(n, 4242)
    sc[0] = P.int_to_limbs(P.to_mont(P.FP_MODULUS - 1, P.FP_MODULUS))
    sc[1:2049] = sc[7]  # one bucket per window takes 2^11 extra points
    exp = corc.known_log_msm("pallas", sc, k)
    W = L.halo_srs_windows(0)
    d_sc = torch.from_numpy(sc.view(np.int64)).cuda()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for world in (8, 3):
        outs = torch.zeros((world, 8), dtype=torch.int64, device="cuda")
        for r in range(world):
            lo, hi = window_range(W, r, world)
            assert hi > lo
            hal.check(L.halo_msm_srs_windows_dev(0, ctypes.c_void_p(d_sc.data_ptr()), n, lo, hi,
                                                 ctypes.c_void_p(outs[r].data_ptr()), sp))
        hal.check(L.halo_msm_join(sp))
        total = torch.zeros(8, dtype=torch.int64, device="cuda")
        hal.check(L.halo_point_sum_dev(0, ctypes.c_void_p(outs.data_ptr()), world, 64, ctypes.c_void_p(total.data_ptr()),
                                       sp))
        torch.cuda.synchronize()
        assert np.array_equal(total.cpu().numpy().view(np.uint64), exp), world
    del d_sc


@pytest.mark.parametrize("tag,fid,inverse", [("fp", 0, True), ("fq", 1, False)])
def test_ntt_2p24_vs_c_oracle(hal, corc, tag, fid, inverse):
    L = hal.load()
    logn = 24
    x = rand_words(1 << logn, 240 + fid)
    exp = corc.ntt(tag, x)
    got = x.copy()
    hal.check(L.halo_ntt(fid, hal.ptr(got), logn, 0))
    assert np.array_equal(got, exp)
    if inverse:
        back = exp.copy()
        hal.check(L.halo_ntt(fid, hal.ptr(back), logn, 1))
        assert np.array_equal(back, x)
        assert np.array_equal(corc.ntt(tag, exp, inverse=True), x)


def test_prove_2p20_openings_pass_succinct_check_and_decider(hal, corc):
    import pcdl_check

    from halo_amd import prover

    L = hal.load()
    n = 1 << 20
    cid = hal.CURVES["pallas"]
    hal.check(L.halo_srs_synthesize(cid, n, 0x505256 + 20))
    hal.check(L.halo_srs_precompute_windows(cid))
    B = prover.DeviceBackend("pallas")
    out = prover.naive_prover(B, prover.synthetic_witness(B, n, seed=1), n, prover.Challenges(B.m))
    srs = np.zeros((n, 8), dtype=np.uint64)
    hal.check(L.halo_srs_read(cid, 0, n, hal.ptr(srs)))
    for key in ("q_r", "q_r_omega", "acc"):
        q = out[key]
        assert len(q["Ls"]) == 20
        pcdl_check.succinct_check("pallas", q["C"], n - 1, q["z"], q["v"], q["Ls"], q["Rs"], q["U"], q["c"],
                                  q["xis"], B.H_point)
        assert pcdl_check.decider_commit_matches("pallas", q["U"], q["xis"], srs, corc.msm), key
