"""GPU parity: pcdl::open_without_eval driven by the reference's own transcript.

The device round loop (halo_amd.pcdl.open_without_eval: halo_pcdl_open_begin / _blind / _combine /
_start, the IPA session) is driven by the CPU restatement of the Poseidon PCDL sponge (oracle/poseidon.py, pinned
to the reference's Kimchi / Mina vectors in tests/test_oracle.py), so every challenge -- alpha,
xi_0 and the per-round xi -- is derived from the device's own C_bar, L and R exactly as
pcdl.rs:326-453 derives them.  The resulting EvalProof (Ls, Rs, U, c, C_bar, w') must equal the
committed fixture of tests/golden/make_transcript.py bit for bit (plain and hiding openings, n =
16..1024, Pallas and Vesta, reference-recipe SRS and the reference's (S, H)).  The n = 4096 / 2^14
cases ("big_*") run the device's SRS-table tail rounds and its weighted -> materialised -> tail
rounds under the reference's transcript order (pcdl.rs:387-425); their inputs are regenerated from
the stored seed."""
import os

import numpy as np
import pytest

import pasta as P
import poseidon
from halo_amd import group, pcdl

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(os.path.dirname(__file__), "golden", "transcript.npz"))
CASES = sorted({k[:-2] for k in G.files if k.startswith("open_") and k.endswith("_p")})
BIG = sorted({k[:-5] for k in G.files if k.startswith("big_") and k.endswith("_seed")})


class SpongeAdapter:
    """The oracle sponge behind the reference's Sponge interface, over WrappedPoints / ark scalars."""

    def __init__(self, cname):
        self.c = P.CURVES[cname]
        self.s = poseidon.Sponge(cname, poseidon.PCDL)

    def absorb_g(self, pts):
        self.s.absorb_g([P.wrapped_to_point(self.c, [int(x) for x in q]) for q in pts])

    def absorb_fr(self, xs):
        self.s.absorb_fr([P.from_mont(P.limbs_to_int(x), self.c.scalar) for x in xs])

    def challenge(self):
        return np.array(P.int_to_limbs(P.to_mont(self.s.challenge(), self.c.scalar)), dtype=np.uint64)


@pytest.mark.parametrize("key", CASES)
def test_open_without_eval_matches_transcript_fixture(hal, golden, corc, key):
    cname = key.split("_")[1]
    n = int(key.split("_")[2][1:])
    hiding = key.endswith("hiding")
    S, Hh = golden[f"ref_sh_{cname}"]
    group.PublicParams.upload(cname, corc.srs_generate(cname, n), S, Hh, precompute_windows=True)
    Sd, Hd = group.PublicParams.sh(cname)
    assert np.array_equal(Sd, S) and np.array_equal(Hd, Hh)
    z, v = G[key + "_zv"]
    w = q = w_bar = None
    if hiding:
        w, w_bar = G[key + "_w"]
        q = G[key + "_q"]
    if hiding:  # pcdl::open (pcdl.rs:463-473): v = p(z) formed on the device at the session start
        pi = pcdl.open(G[key + "_p"], G[key + "_C"][0], n - 1, z, w=w, transcript=SpongeAdapter(cname), q=q,
                       w_bar=w_bar, curve=cname)
        assert np.array_equal(pi["v"], v), key
    else:
        pi = pcdl.open_without_eval(G[key + "_p"], G[key + "_C"][0], n - 1, z, v, w=w,
                                    transcript=SpongeAdapter(cname), q=q, w_bar=w_bar, curve=cname)
    assert np.array_equal(np.stack(pi["Ls"]), G[key + "_Ls"]), key
    assert np.array_equal(np.stack(pi["Rs"]), G[key + "_Rs"]), key
    assert np.array_equal(pi["U"], G[key + "_U"][0]) and np.array_equal(pi["c"], G[key + "_c"][0]), key
    if hiding:
        assert np.array_equal(pi["C_bar"], G[key + "_Cbar"][0]), key
        assert np.array_equal(pi["w_prime"], G[key + "_wprime_alpha"][0]), key


def det_scalars(seed: int, k: int) -> np.ndarray:
    """tests/golden/make_transcript.py det_scalars: k Montgomery-form scalars < 2^254 from seed."""
    a = np.random.default_rng(seed).integers(0, 2**64 - 1, size=(k, 4), dtype=np.uint64, endpoint=True)
    a[:, 3] &= np.uint64(0x3FFFFFFFFFFFFFFF)
    return np.ascontiguousarray(a)


BIG_PATHS = [(k, "default") for k in BIG] + [(k, "weighted") for k in BIG if k.split("_")[2] == "n4096"]


@pytest.mark.parametrize("key,path", BIG_PATHS)
def test_open_without_eval_weighted_rounds_transcript(hal, golden, corc, key, path):
    """default: n = 4096 starts in the tail rounds over the SRS table (ipa_srs_tail_n = 4096), 2^14
    runs weighted -> materialised -> tail; weighted: n = 4096 pinned to the weighted -> materialised
    -> tail switch too, under the same reference transcript fixture."""
    with hal.tuning(ipa_srs_tail_n=0 if path == "weighted" else -1):
        _open_big(hal, golden, corc, key)


def _open_big(hal, golden, corc, key):
    cname = key.split("_")[1]
    n = int(key.split("_")[2][1:])
    hiding = key.endswith("hiding")
    S, Hh = golden[f"ref_sh_{cname}"]
    group.PublicParams.upload(cname, corc.srs_generate(cname, n), S, Hh, precompute_windows=True)
    ins = det_scalars(int(G[key + "_seed"][0]), 2 * n + 4)
    p = ins[: n - 1]
    z, v = G[key + "_zv"]
    assert np.array_equal(z, ins[2 * n])
    w = q = w_bar = None
    if hiding:
        q, w, w_bar = ins[n: 2 * n - 1], ins[2 * n + 1], ins[2 * n + 2]
    pi = pcdl.open_without_eval(p, G[key + "_C"][0], n - 1, z, v, w=w, transcript=SpongeAdapter(cname), q=q,
                                w_bar=w_bar, curve=cname)
    assert np.array_equal(np.stack(pi["Ls"]), G[key + "_Ls"]), key
    assert np.array_equal(np.stack(pi["Rs"]), G[key + "_Rs"]), key
    assert np.array_equal(pi["U"], G[key + "_U"][0]) and np.array_equal(pi["c"], G[key + "_c"][0]), key
    if hiding:
        assert np.array_equal(pi["C_bar"], G[key + "_Cbar"][0]), key
        assert np.array_equal(pi["w_prime"], G[key + "_wprime_alpha"][0]), key


def test_hiding_assertions(hal, golden, corc):
    S, Hh = golden["ref_sh_pallas"]
    group.PublicParams.upload("pallas", corc.srs_generate("pallas", 64), S, Hh, precompute_windows=False)
    q = np.zeros((10, 4), dtype=np.uint64)
    one = np.array([1, 0, 0, 0], dtype=np.uint64)
    with pytest.raises(AssertionError, match=r"n \(11\) is not a power of two"):
        pcdl.open_without_eval(q, np.zeros(8, dtype=np.uint64), 10, one, one, w=one, transcript=SpongeAdapter("pallas"),
                               q=q, w_bar=one)
    # p.degree() <= d and d <= pp.D (pcdl.rs:340-341); trailing zero coefficients do not count
    p = np.ones((9, 4), dtype=np.uint64)
    with pytest.raises(AssertionError, match=r"p.degree\(\) <= d"):
        pcdl.open_without_eval(p, np.zeros(8, dtype=np.uint64), 7, one, one, transcript=SpongeAdapter("pallas"))
    with pytest.raises(AssertionError, match=r"d <= pp.D"):
        pcdl.open_without_eval(p[:4], np.zeros(8, dtype=np.uint64), 127, one, one, transcript=SpongeAdapter("pallas"))
    with pytest.raises(ValueError, match="transcript"):
        pcdl.open_without_eval(p[:4], np.zeros(8, dtype=np.uint64), 7, one, one)


def test_open_session_pool_and_srs_change(hal, golden, corc):
    """Openings reuse pooled sessions (halo_ipa_end returns them): many openings in a row stay
    bit-exact, device memory stays flat, and a re-uploaded SRS (new points, same length) is seen by
    the next opening's tail table (no stale SRS-derived tables)."""
    import torch
    key = "open_pallas_n256_plain"
    S, Hh = golden["ref_sh_pallas"]
    n = 256
    z, v = G[key + "_zv"]
    g = corc.srs_generate("pallas", n)
    group.PublicParams.upload("pallas", g, S, Hh, precompute_windows=True)
    free0 = None
    for i in range(40):
        pi = pcdl.open_without_eval(G[key + "_p"], G[key + "_C"][0], n - 1, z, v, transcript=SpongeAdapter("pallas"))
        assert np.array_equal(np.stack(pi["Ls"]), G[key + "_Ls"]) and np.array_equal(pi["U"], G[key + "_U"][0]), i
        if i == 5:
            free0 = torch.cuda.mem_get_info()[0]
    assert torch.cuda.mem_get_info()[0] >= free0 - (64 << 20)
    # a different SRS of the same length: the opening must follow it (U = <h, G> changes)
    group.PublicParams.upload("pallas", np.ascontiguousarray(g[::-1]), S, Hh, precompute_windows=True)
    pi = pcdl.open_without_eval(G[key + "_p"], G[key + "_C"][0], n - 1, z, v, transcript=SpongeAdapter("pallas"))
    assert not np.array_equal(pi["U"], G[key + "_U"][0])
    group.PublicParams.upload("pallas", g, S, Hh, precompute_windows=True)
    pi = pcdl.open_without_eval(G[key + "_p"], G[key + "_C"][0], n - 1, z, v, transcript=SpongeAdapter("pallas"))
    assert np.array_equal(pi["U"], G[key + "_U"][0])


def _rounds(ses, xis, cid, k=None):
    """k rounds (all when None) of L/R + fold with the given Montgomery challenges."""
    out = []
    for xi in xis[:k]:
        out.append(ses.round_lr())
        ses.fold(xi, pcdl._ark_inverse(xi, cid))
    return out


def test_open_session_across_srs_write(hal, golden, corc):
    """a session reading the SRS's multiples table (tail rounds from round 1) stays
    correct when the SRS is rewritten mid-opening (the table is versioned: the rebuild goes to a fresh
    buffer while the session holds the old one), and a second halo_ipa_end of the same handle does not
    pool the session twice (two later concurrent sessions keep distinct resources)."""
    import ctypes

    S, Hh = golden["ref_sh_pallas"]
    n = 256
    cid = hal.CURVES["pallas"]
    g = corc.srs_generate("pallas", n)
    g2 = np.ascontiguousarray(g[::-1])
    rng = np.random.default_rng(31)
    m = P.FP_MODULUS
    cs = det_scalars(77, n)
    z = det_scalars(78, 1)[0]
    hp = g[5]
    xis = [np.array(P.int_to_limbs(P.to_mont(int(x), m)), dtype=np.uint64)
           for x in rng.integers(1, 2**62, size=8)]

    def full(srs):
        group.PublicParams.upload("pallas", srs, S, Hh, precompute_windows=True)
        ses = pcdl.IpaSession(cs, z, hp)
        lr = _rounds(ses, xis, cid)
        return lr, ses.end()

    ref_g, ref_g2 = full(g), full(g2)
    group.PublicParams.upload("pallas", g, S, Hh, precompute_windows=True)
    a = pcdl.IpaSession(cs, z, hp)
    lr_a = _rounds(a, xis, cid, 3)
    group.PublicParams.upload("pallas", g2, S, Hh, precompute_windows=True)  # SRS write under session a
    b = pcdl.IpaSession(cs, z, hp)
    lr_b = _rounds(b, xis, cid)
    Ub = b.end()
    lr_a += _rounds(a, xis[3:], cid)
    Ua = a.end()
    for (got_lr, got_U), (exp_lr, exp_U) in (((lr_a, Ua), ref_g), ((lr_b, Ub), ref_g2)):
        assert all(np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) for x, y in zip(got_lr, exp_lr))
        assert np.array_equal(got_U[0], exp_U[0]) and np.array_equal(got_U[1], exp_U[1])
    # a second end of an ended handle: reported or harmless, never a doubly pooled session
    c = pcdl.IpaSession(cs, z, hp)
    _rounds(c, xis, cid)
    handle = c._s
    c.end()
    hal.load().halo_ipa_end(handle, None, None)
    d, e = pcdl.IpaSession(cs, z, hp), pcdl.IpaSession(cs, z, hp)
    assert ctypes.cast(d._s, ctypes.c_void_p).value != ctypes.cast(e._s, ctypes.c_void_p).value
    lr_d, lr_e = [], []
    for xi in xis:  # interleaved, so shared buffers would corrupt one of them
        lr_d.append(d.round_lr())
        lr_e.append(e.round_lr())
        d.fold(xi, pcdl._ark_inverse(xi, cid))
        e.fold(xi, pcdl._ark_inverse(xi, cid))
    for got in (lr_d, lr_e):
        assert all(np.array_equal(x[0], y[0]) for x, y in zip(got, ref_g2[0]))
    assert np.array_equal(d.end()[0], ref_g2[1][0]) and np.array_equal(e.end()[0], ref_g2[1][0])
