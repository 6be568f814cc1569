"""Exact CPU model of one workgroup of ntt.hip's k_ntt_pass (round 5 signed lazy butterflies).

Emulates, thread by thread, the kernel's element positions (load phase, ntt_first, the radix-4 groups
in their thread orders -- including ntt_unit_tau's wave-uniform unit groups -- and the store phase)
with the exact limb arithmetic of fs_add / fs_sub / fs_norm / fs_carry / fs_settle and fs_mul's
result (low limbs normalized, signed top limb, value (t - M p) / R' + p with M = t p^-1 mod R'), and
asserts the bounds the kernel relies on: every limb inside int32, every fs_mul operand's low limbs
within +-3 x 2^29 (tests/test_field_bounds.py checks that range against the generated asm), every
fs_settle input within +-4 x 2^29.  The block's outputs are compared with a direct DFT of its columns.
Test infrastructure (tests/test_ntt_model.py); the GPU tests run the kernel itself.
"""
from __future__ import annotations

import random

NLIMB, B = 9, 29
MASK = (1 << B) - 1
RP = 1 << (NLIMB * B)
P_FP = 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001
MAXI32 = 1 << 31


def limbs(x):  # non-negative x < 2^256 -> normalized limbs
    return [(x >> (B * i)) & MASK for i in range(NLIMB - 1)] + [x >> (B * (NLIMB - 1))]


def value(a):
    return sum(l << (B * i) for i, l in enumerate(a))


def i32(a):
    for l in a:
        assert -MAXI32 <= l < MAXI32, f"limb {l / 2**29:.3f} x 2^29 outside int32"
    return a


class Model:
    def __init__(self, p=P_FP):
        self.p = p
        self.pinv = pow(p, -1, RP)
        self.max_mul_limb = 0
        self.max_settle_limb = 0

    def add(self, a, b):
        return i32([x + y for x, y in zip(a, b)])

    def sub(self, a, b):
        return i32([x - y for x, y in zip(a, b)])

    def norm(self, a):  # fs_norm: parallel carries
        r = [a[0] & MASK]
        for i in range(1, NLIMB):
            c = a[i - 1] >> B  # arithmetic shift
            r.append((a[i] if i == NLIMB - 1 else a[i] & MASK) + c)
        return i32(r)

    def carry(self, a):  # fs_carry: one chain
        r, c = [], 0
        for i in range(NLIMB - 1):
            x = a[i] + c
            assert -MAXI32 <= x < MAXI32
            r.append(x & MASK)
            c = x >> B
        r.append(a[-1] + c)
        return i32(r)

    def mul(self, a, w):  # fs_mul(a, w): w a normalized twiddle (< 2p)
        for l in a[:-1]:
            assert abs(l) <= 3 * (1 << B), f"fs_mul operand limb {l / 2**29:.3f} x 2^29"
        self.max_mul_limb = max(self.max_mul_limb, max(abs(l) for l in a[:-1]))
        t = value(a) * value(w)
        m = (t * self.pinv) % RP
        r = (t - m * self.p) // RP + self.p
        low = [(r >> (B * i)) & MASK for i in range(NLIMB - 1)]
        top = r >> (B * (NLIMB - 1))  # floor: the signed top limb
        return i32(low + [top])

    def settle(self, x):  # fs_settle
        for l in x[:-1]:
            assert abs(l) < 4 * (1 << B), f"fs_settle input limb {l / 2**29:.3f} x 2^29"
        self.max_settle_limb = max(self.max_settle_limb, max(abs(l) for l in x[:-1]))
        qm = 1 - (x[-1] >> 22)
        pl = limbs(self.p)
        r, c = [], 0
        for i in range(NLIMB):
            d = x[i] + c + qm * pl[i]
            r.append(d if i == NLIMB - 1 else d & MASK)
            c = d >> B
        v = value(r)
        assert 0 <= v < 1 << 256 and all(0 <= l <= MASK for l in r[:-1]), v
        return r


def bitrev(x, r):
    return int(format(x, f"0{r}b")[::-1], 2) if r else 0


def run_block(NE, r, T, loads, stage_tw, pretw, prune=0, out_mul_const=None, rng=None):
    """One workgroup: loads[t][rho] = the internal value (int) of column t's input rho; pretw(t, rho) =
    the pre-twiddle (int, normalized) or None; stage_tw(s, k) = omega_{2^(s+1)}^k (internal, < 2p).
    Returns (outputs[t][k] values, model)."""
    M = Model()
    p = M.p
    EPT = 4
    TH = NE // EPT
    LG_TH = TH.bit_length() - 1
    R = 1 << r
    EB = T * R
    lds = {}
    G0 = 1 if (NE == 2048 and r % 2) else min(r, 2)
    # load + first stages
    for tau in range(TH):
        if R >= EPT:
            base = (tau % T) * R + EPT * (tau // T)
        else:
            base = EPT * tau
        v = []
        for m in range(EPT):
            pos = base + m
            if pos >= EB:
                v.append([0] * NLIMB)
                continue
            t = pos >> r
            pl = pos & ~((1 << prune) - 1) if prune else pos
            rho = bitrev(pl & (R - 1), r)
            x = limbs(loads[t][rho])
            w = pretw(t, rho)
            if w is not None and rho != 0:
                x = M.mul(x, limbs(w))
            v.append(x)
        if not prune:
            for m in (0, 2):
                tt = v[m + 1]
                v[m + 1] = M.sub(v[m], tt)
                v[m] = M.add(v[m], tt)
            if G0 > 1:
                tt = v[2]
                v[2] = M.sub(v[0], tt)
                v[0] = M.add(v[0], tt)
                tt = M.mul(v[3], limbs(stage_tw(1, 1)))
                v[3] = M.sub(v[1], tt)
                v[1] = M.add(v[1], tt)
                v = [M.norm(x) for x in v]
        for m in range(EPT):
            if base + m < EB:
                lds[base + m] = v[m]
    US = 0 if NE == 2048 else 2  # (ntt.hip ntt_unit_stage: the 2048-element blocks have no unit group since round 6)
    out_mul = out_mul_const is not None
    in_norm = {tau: (prune != 0 or G0 != 1) for tau in range(TH)}
    s = prune if prune else G0
    while s < r:
        G = min(r - s, 2)
        h = 1 << s
        seen = set()
        new = {}
        for tau in range(TH):
            unit_grp = US != 0 and s == US
            tt = (((tau << US) | (tau >> (LG_TH - US))) & (TH - 1)) if unit_grp else tau
            unit_wave = US != 0 and (tau >> (LG_TH - US)) == 0  # (wave-uniform by construction)
            gb = (tt & (h - 1)) | ((tt >> s) << (s + 2))
            pos = [gb + m * h for m in range(EPT)]
            if any(q < EB for q in pos):
                assert all(q < EB for q in pos)
            else:
                continue
            for q in pos:
                assert q not in seen
                seen.add(q)
            v = [lds[q] for q in pos]
            k0 = tt & (h - 1)
            unit = unit_grp and unit_wave
            if unit:
                assert k0 == 0
                v = [M.carry(x) for x in v]
            w0 = limbs(stage_tw(s, k0))
            for m in (0, 2):
                x = v[m + 1] if unit else M.mul(v[m + 1], w0)
                v[m + 1] = M.sub(v[m], x)
                v[m] = M.add(v[m], x)
            if G > 1:
                x = v[2] if unit else M.mul(v[2], limbs(stage_tw(s + 1, k0)))
                v[2] = M.sub(v[0], x)
                v[0] = M.add(v[0], x)
                x = M.mul(v[3], limbs(stage_tw(s + 1, k0 + h)))
                v[3] = M.sub(v[1], x)
                v[1] = M.add(v[1], x)
            norm = 0 if (s + 2 >= r and not out_mul) else (1 if in_norm[tau] else 2)
            if norm == 2:
                v = [M.norm(x) for x in v]
            elif norm == 1:
                v[0] = M.norm(v[0])
            in_norm[tau] = norm == 2
            for q, x in zip(pos, v):
                new[q] = x
        assert len(seen) == EB, (s, len(seen), EB)
        lds.update(new)
        s += 2
    out = [[None] * R for _ in range(T)]
    for t in range(T):
        for k in range(R):
            x = lds[t * R + k]
            if out_mul:
                x = M.mul(x, limbs(out_mul_const))
            out[t][k] = value(M.settle(x)) % p
    return out, M


def dft_check(NE, r, T, seed=1, prune=0, pretwiddle=False, out_mul=False, max_in=None):
    """Runs one block on random inputs and compares every output with a direct DFT of its columns
    (internal Montgomery domain: the transform is linear there).  Returns the model (bound maxima)."""
    p = P_FP
    rng = random.Random(seed)
    R = 1 << r
    # a primitive 2^r-th root of unity: 5 generates Fp^*, (p - 1) / 2^32 odd
    g = 5
    omega = pow(g, (p - 1) >> r, p)
    assert pow(omega, R // 2, p) != 1 and pow(omega, R, p) == 1
    omegaN = pow(g, (p - 1) >> (r + 3), p) if pretwiddle else None  # a pass of a larger transform
    top = max_in or (1 << 256)
    loads = [[rng.randrange(top) for _ in range(R)] for _ in range(T)]
    if prune:
        for t in range(T):
            for rho in range(R):  # zero tail: rho's low `prune` bits select the zero inputs
                if bitrev(rho, r) % (1 << prune):
                    loads[t][rho] = 0
    RPm = RP % p

    def to_int(x):  # internal Montgomery value of x (random representative below 2p)
        return x * RPm % p + (p if rng.random() < 0.5 else 0)

    tw_cache = {}

    def stage_tw(s, k):
        key = (s, k)
        if key not in tw_cache:
            tw_cache[key] = to_int(pow(omega, (R >> (s + 1)) * k, p))
        return tw_cache[key]

    def pretw(t, rho):
        return to_int(pow(omegaN, rho * (t + 1), p)) if pretwiddle else None

    oc = to_int(rng.randrange(1, p)) if out_mul else None
    out, M = run_block(NE, r, T, loads, stage_tw, pretw, prune=prune, out_mul_const=oc)
    rinv = pow(RP, -1, p)
    for t in range(T):
        xs = [loads[t][rho] * (pow(omegaN, rho * (t + 1), p) if pretwiddle and rho else 1) % p for rho in range(R)]
        if out_mul:
            xs = [x * (oc * rinv % p) % p for x in xs]
        exp = dft(xs, omega, p)
        for k in range(R):
            assert out[t][k] == exp[k], (t, k)
    return M


def dft(xs, w, p):
    """X[k] = sum_rho xs[rho] w^(rho k) mod p (recursive radix 2, len(xs) a power of two)."""
    n = len(xs)
    if n == 1:
        return [xs[0] % p]
    ev = dft(xs[0::2], w * w % p, p)
    od = dft(xs[1::2], w * w % p, p)
    out = [0] * n
    t = 1
    for k in range(n // 2):
        a, b = ev[k], od[k] * t % p
        out[k] = (a + b) % p
        out[k + n // 2] = (a - b) % p
        t = t * w % p
    return out


if __name__ == "__main__":
    for args in ((1024, 8, 4), (1024, 7, 8), (1024, 3, 128), (2048, 11, 1), (2048, 10, 2), (2048, 9, 4)):
        M = dft_check(*args)
        print(args, f"max fs_mul limb {M.max_mul_limb / 2**29:.3f} x 2^29, max settle limb "
              f"{M.max_settle_limb / 2**29:.3f} x 2^29")
