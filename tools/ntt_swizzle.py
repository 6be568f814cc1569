"""Searches / checks the LDS bank swizzle of the NTT pass kernel (halo_amd/csrc/ntt.hip, NttSwz).

The kernel keeps a block's elements limb-major in LDS: limb l of position p at word l * NE + swz(p),
swz(p) = p ^ M(p >> 5) with M linear over GF(2) (constants C[b] = M(1 << b)).  ds_read_b32 /
ds_write_b32 serve a wave in two groups of 32 lanes, bank = word mod 32 (MI355X_MICROARCH.md, LDS), so
an access is conflict-free when the 32 positions of each half-wave land on 32 different banks.

This enumerates every LDS access pattern of the kernel (load-phase stores, each radix-4 group's reads
and writes, the output phase's reads) for the block shapes that use the swizzle, and either checks a
given C or searches for one.

    python3 tools/ntt_swizzle.py check 2048 10 29 31 20 30 17
    python3 tools/ntt_swizzle.py search 2048
"""
import random
import sys


def unit_stage(NE, T):
    """Stage of the wave-uniform unit-twiddle group (ntt.hip ntt_unit_stage): 1 on one-column
    2048-element blocks, 2 on 1024-element blocks, none (0) otherwise."""
    if NE == 2048:
        return 1 if T == 1 else 0
    return 2


def tau_remap(tau, th, us):
    """Thread -> position-bits order of the unit-twiddle group (ntt.hip ntt_unit_tau): the top `us`
    thread bits (the wave's) become the lowest, so the group at stage us has a wave-uniform k0."""
    lg = th.bit_length() - 1
    return ((tau << us) | (tau >> (lg - us))) & (th - 1)


def patterns(NE):
    """Yields lists of 32 positions accessed together by one half-wave."""
    EPT = 4
    TH = NE // EPT
    rs = range(9, 12) if NE == 2048 else range(1, 9)
    for r in rs:
        R = 1 << r
        T = max(1, NE >> r)
        EB = T * R
        G0 = (r % 2 if r % 2 else 2) if NE == 2048 else min(r, 2)
        # load phase stores
        for m in range(EPT):
            for h in range(TH // 32):
                ps = []
                for tau in range(32 * h, 32 * h + 32):
                    if R >= EPT:
                        q, t = tau // T, tau % T
                        base = t * R + EPT * q
                    else:
                        base = EPT * tau
                    ps.append(base + m)
                yield [p for p in ps if p < EB]
        # groups (any start parity the prune can give keeps r - s even on the wide blocks)
        starts = set()
        for s0 in range(G0, r):
            if NE == 2048 and (r - s0) % 2:
                continue
            starts.add(s0)
        for s0 in starts:
            for s in range(s0, r, 2):
                hh = 1 << s
                for m in range(EPT):
                    for h in range(TH // 32):
                        ps = []
                        for tau in range(32 * h, 32 * h + 32):
                            us = unit_stage(NE, T)
                            tt = tau_remap(tau, TH, us) if (us and s == us) else tau
                            gb = (tt & (hh - 1)) | ((tt >> s) << (s + 2))
                            ps.append(gb + m * hh)
                        yield [p for p in ps if p < EB]
        # output phase (log_ns == 0 and != 0)
        for ns0 in (True, False):
            for i in range(EPT):
                for h in range(TH // 32):
                    ps = []
                    for tau in range(32 * h, 32 * h + 32):
                        idx = tau + TH * i
                        if idx >= EB:
                            continue
                        if ns0:
                            t, k = idx >> r, idx & (R - 1)
                        else:
                            k, t = idx // T, idx % T
                        ps.append(t * R + k)
                    yield ps


def swz(p, C):
    m = 0
    hi = p >> 5
    for b, c in enumerate(C):
        if (hi >> b) & 1:
            m ^= c
    return p ^ m


def conflicts(C, pats):
    bad = 0
    for ps in pats:
        banks = [swz(p, C) & 31 for p in ps]
        bad += len(banks) - len(set(banks))
    return bad


def main():
    mode, NE = sys.argv[1], int(sys.argv[2])
    nb = {1024: 5, 2048: 6}[NE]
    pats = list(patterns(NE))
    if mode == "check":
        C = [int(x) for x in sys.argv[3:3 + nb]]
        print(f"NE {NE} C {C}: {len(pats)} patterns, {conflicts(C, pats)} extra bank hits")
        return
    rng = random.Random(int(sys.argv[3]) if len(sys.argv) > 3 else 1)
    # the patterns only reach bank bits through small position sets: prune with a sample first
    sample = pats[:: max(1, len(pats) // 400)]
    for it in range(2_000_000):
        C = [rng.randrange(32) for _ in range(nb)]
        if conflicts(C, sample):
            continue
        if conflicts(C, pats) == 0:
            print(f"found after {it}: C = {C}")
            return
    print("none found")


if __name__ == "__main__":
    main()
