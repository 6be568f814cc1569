"""CPU restatement of the reference's Poseidon sponge and its Fiat-Shamir wrapper.
TEST INFRASTRUCTURE ONLY: the transcript is host logic outside the GPU hot path; it
is restated here so that tests can drive the device's IPA round loop with the reference's own
challenge derivation.  Only tests/ and fixture generators import it.

* InnerSponge -- crates/poseidon/src/inner_sponge.rs:1-108: state width 3 (rate 2, capacity 1), 55
  full rounds of x^7, MDS, round constants (sbox -> MDS -> add constants), the Absorbed(n) /
  Squeezed(n) state machine of absorb() / squeeze().
* Sponge -- crates/poseidon/src/outer_sponge.rs:11-100: label absorbed first (Protocols::PCDL = 0),
  absorb_g (affine x, y; the identity as (0, 0)), absorb_fr (the scalar absorbed as one base-field
  element when r < q, else as (s >> 1, s & 1)), challenge (squeeze; >> 1 when r < q).
Constants (crates/group/src/poseidon_consts.rs, Montgomery limbs) and the Kimchi / Mina test vectors
(crates/poseidon/test-vectors/kimchi-vecs.json, inner_sponge.rs:315-368) come from
tests/golden/transcript.npz (tests/golden/make_transcript.py), checked in tests/test_oracle.py.
"""
from __future__ import annotations

import os

import numpy as np

import pasta as P

PCDL, ASDL, PLONK, SIGNATURE = 0, 1, 2, 3  # outer_sponge.rs:17-22
_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "transcript.npz")
_CONSTS = {}


def _limbs(a):
    return [P.limbs_to_int(r) for r in np.asarray(a).reshape(-1, 4)]


def constants(field: str):
    """(MDS 3x3, round constants 55x3) of the base field 'fq' (Pallas sponge) or 'fp' (Vesta), canonical."""
    if field not in _CONSTS:
        g = np.load(_GOLDEN)
        m = P.FIELDS[field]
        mds = [P.from_mont(x, m) for x in _limbs(g[f"poseidon_{field}_mds"])]
        rc = [P.from_mont(x, m) for x in _limbs(g[f"poseidon_{field}_rc"])]
        _CONSTS[field] = ([mds[3 * i:3 * i + 3] for i in range(3)], [rc[3 * i:3 * i + 3] for i in range(55)])
    return _CONSTS[field]


class InnerSponge:
    RATE = 2

    def __init__(self, field: str):
        self.m = P.FIELDS[field]
        self.mds, self.rc = constants(field)
        self.state = [0, 0, 0]
        self.mode, self.n = "absorbed", 0

    def _permute(self):
        m = self.m
        s = self.state
        for r in range(55):
            s = [pow(x, 7, m) for x in s]
            s = [sum(self.mds[i][j] * s[j] for j in range(3)) % m for i in range(3)]
            s = [(s[i] + self.rc[r][i]) % m for i in range(3)]
        self.state = s

    def absorb(self, xs):
        for x in xs:
            if self.mode == "absorbed" and self.n < self.RATE:
                self.state[self.n] = (self.state[self.n] + x) % self.m
                self.n += 1
            elif self.mode == "absorbed":  # n == RATE
                self._permute()
                self.n = 1
                self.state[0] = (self.state[0] + x) % self.m
            else:  # squeezed
                self.mode, self.n = "absorbed", 1
                self.state[0] = (self.state[0] + x) % self.m

    def squeeze(self) -> int:
        if self.mode == "squeezed" and self.n < self.RATE:
            self.n += 1
            return self.state[self.n - 1]
        self._permute()
        self.mode, self.n = "squeezed", 1
        return self.state[0]


class Sponge:
    """outer_sponge.rs Sponge<P> for curve 'pallas' (base Fq, scalar Fp) or 'vesta'."""

    def __init__(self, curve: str, label: int = PCDL):
        self.c = P.CURVES[curve]
        self.inner = InnerSponge("fq" if curve == "pallas" else "fp")
        self.inner.absorb([label])

    def absorb_g(self, points):
        """points: affine (x, y) canonical, or None for the identity."""
        for g in points:
            self.inner.absorb([0, 0] if g is None else [g[0], g[1]])

    def absorb_fr(self, xs):
        for x in xs:
            if self.c.scalar < self.c.base:
                self.inner.absorb([x])
            else:
                self.inner.absorb([x >> 1, x & 1])

    def challenge(self) -> int:
        v = self.inner.squeeze()
        if self.c.scalar < self.c.base:
            return v >> 1
        assert v < self.c.scalar
        return v
