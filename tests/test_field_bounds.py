"""CPU model of the generated Montgomery multiplications (halo_amd/csrc/gen_field_asm.py -> field_asm.hpp).

ADVICE r04: the signed reduction narrows the column headroom to 2^63, so correctness rests on operand
bounds (fields.hpp: at most one loose operand with limbs < 2^30; ntt.hip: the NTT's signed-limb operand
with limbs in [-3, 3] x 2^29).  This executes the exact instruction list the generator emits -- 64-bit
two's complement accumulators, v_mad_u64_u32 / v_mad_i64_i32 / v_ashrrev_i64 / v_alignbit_b32 -- on
limb-adversarial and random operands, asserts that every column's exact value stays inside the signed
64-bit range (the register and the integer agree), and checks the result against Python integers:
r == a b 2^-261 (mod p), low limbs in [0, 2^29), and the value range the callers rely on.
No GPU: this models the code, the GPU tests run it.
"""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "halo_amd", "csrc"))
import gen_field_asm as G  # noqa: E402

N, B = 9, 29
MASK = (1 << B) - 1
RP = 1 << (N * B)  # R' = 2^261
PRIMES = {
    "fp": 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001,
    "fq": 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001,
}


def limbs(x):
    return [(x >> (B * i)) & MASK for i in range(N - 1)] + [x >> (B * (N - 1))]


def value(ls):
    return sum(l << (B * i) for i, l in enumerate(ls))


def s32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def run(kind, p, ops):
    """Executes body(kind); ops maps operand names (a0.., b0.., c0.., d0.., a20..) to int32-range ints."""
    pl = limbs(p)
    regs = dict(ops)
    for j in G.RED_J:
        regs[f"np{j}"] = -pl[j]
    acc = {"v[0:1]": 0, "v[2:3]": 0}  # exact integers
    out = {}

    def rd(name):
        return regs[name] if name in regs else out[name]

    def check(v):
        assert -(1 << 63) <= v < (1 << 63), f"column overflow {v / 2**63:.4f} x 2^63"
        return v

    for ln in G.body(kind):
        op, rest = ln.split(" ", 1)
        args = [x.strip().strip("{}") for x in rest.split(",")]
        if op in ("v_mad_u64_u32", "v_mad_i64_i32"):
            dst, _, x, y, z = args
            xv, yv = rd(x), rd(y)
            if op == "v_mad_u64_u32":
                assert 0 <= xv < 1 << 32 and 0 <= yv < 1 << 32, (ln, xv, yv)
            else:
                xv, yv = s32(xv), s32(yv)
            zv = 0 if z == "0" else acc[z]
            acc[dst] = check(xv * yv + zv)
        elif op == "v_lshl_add_u64":
            dst, src, _, z = args
            acc[dst] = check(acc[src] + (1 if z == "1" else acc[z]))
        elif op == "v_and_b32":
            out[args[0]] = acc["v[0:1]"] & MASK
        elif op == "v_or_b32":
            out[args[0]] = s32((acc["v[0:1]"] & 0xFFFFFFFF) | 0xE0000000)
        elif op == "v_ashrrev_i64":
            acc["v[0:1]"] = acc["v[0:1]"] >> 29
        elif op == "v_alignbit_b32":
            out[args[0]] = s32(acc["v[0:1]"] >> 29)
        else:
            raise AssertionError(ln)
    return [out[f"r{k}"] for k in range(N)]


def check_result(r, expect_mod_p, p, lo, hi):
    assert all(0 <= x <= MASK for x in r[:-1])
    v = value(r)
    assert (v - expect_mod_p) % p == 0
    assert lo <= v < hi, (v / p, lo / p, hi / p)


def operand(name, ls):
    return {f"{name}{i}": l for i, l in enumerate(ls)}


@pytest.mark.parametrize("field", ["fp", "fq"])
def test_fe_mul_and_sqr_column_bounds(field):
    """fe_mul: one operand loose (limbs < 2^30), the other normalized; fe_sqr / fe_mul2: normalized.
    Limb-adversarial operands (every limb at its maximum) plus random values below 8p."""
    p = PRIMES[field]
    rinv = pow(RP, -1, p)
    rng = random.Random(1)
    loose = [(1 << 30) - 1] * (N - 1) + [(1 << 25) - 1]
    tight = [MASK] * (N - 1) + [(1 << 24) - 1]
    cases = [(loose, tight), (tight, tight)]
    for _ in range(200):
        a = rng.randrange(8 * p)
        b = rng.randrange(8 * p)
        cases.append((limbs(a), limbs(b)))
        # loose a: a sum of two normalized values, limb-wise (no carries)
        x, y = limbs(rng.randrange(2 * p)), limbs(rng.randrange(2 * p))
        cases.append(([u + w for u, w in zip(x, y)], limbs(b)))
    for a, b in cases:
        av, bv = value(a), value(b)
        r = run("mul", p, {**operand("a", a), **operand("b", b)})
        # output in [0, 2p) whenever a b < p R'
        check_result(r, av * bv * rinv, p, 0, 2 * p if av * bv < p * RP else 1 << 300)
    for _ in range(200):
        a = limbs(rng.randrange(8 * p))
        r = run("sqr", p, {**operand("a", a), **operand("a2", [2 * x for x in a])})
        check_result(r, value(a) ** 2 * rinv, p, 0, 2 * p)
    for a, b in [(tight, tight)] + [(limbs(rng.randrange(8 * p)), limbs(rng.randrange(8 * p))) for _ in range(100)]:
        r = run("sqr", p, {**operand("a", a), **operand("a2", [2 * x for x in a])})
        c, d = limbs(rng.randrange(8 * p)), limbs(rng.randrange(8 * p))
        r = run("mul2", p, {**operand("a", a), **operand("b", b), **operand("c", c), **operand("d", d)})
        t = value(a) * value(b) + value(c) * value(d)
        check_result(r, t * rinv, p, 0, 2 * p if t < p * RP else 1 << 300)


@pytest.mark.parametrize("field", ["fp", "fq"])
def test_ntt_signed_products(field):
    """ntt.hip fs_mul (fe_muls_asm): a signed-limb operand with low limbs in [-3, 3] x 2^29 -- the
    widest a butterfly operand gets between two fs_norm -- times a normalized twiddle below 2p; the
    result is a b R'^-1 mod p with low limbs in [0, 2^29) and |value| < p + |a b| / R'."""
    p = PRIMES[field]
    rinv = pow(RP, -1, p)
    rng = random.Random(2)
    # the widest operands ntt.hip feeds fs_mul: after a partially normalized group (inputs within
    # [-2^30 - 1, 2^30 + 1]) one butterfly reaches +-3 x 2^29
    hi = 3 * (1 << 29)
    lo = -3 * (1 << 29)
    top_hi = 20 * p >> (B * (N - 1))  # the value bound (|x| < ~20 p) bounds the top limb
    cases = [([hi] * (N - 1) + [top_hi], limbs(2 * p - 1)),
             ([lo] * (N - 1) + [-top_hi], limbs(2 * p - 1)),
             ([hi, lo] * 4 + [top_hi], [MASK] * (N - 1) + [(1 << 24) - 1]),
             ([hi] * (N - 1) + [top_hi], [MASK] * (N - 1) + [(1 << 24) - 1]),
             ([lo] * (N - 1) + [-top_hi], [MASK] * (N - 1) + [(1 << 24) - 1])]
    for _ in range(300):
        a = [rng.randint(lo, hi) for _ in range(N - 1)] + [rng.randint(-top_hi, top_hi)]
        cases.append((a, limbs(rng.randrange(2 * p))))
    for a, w in cases:
        av, wv = value(a), value(w)
        r = run("muls", p, {**operand("a", a), **operand("b", w)})
        assert all(0 <= x <= MASK for x in r[:-1])
        rv = value(r)
        assert (rv - av * wv * rinv) % p == 0
        bound = p + abs(av * wv) // RP + 1
        assert -bound < rv < bound + p


# ---------------------------------------------------------------------------------------------
# GLV halves for the IPA tail's signed 4-bit windows (ipa.hip tail_bias / tail_digit): a half k is
# stored as |k| + 0x8888...8 in 128 bits, so |k| must stay below 2^128 - 0x8888...8 (~0.467 x 2^128).
# ---------------------------------------------------------------------------------------------
def _glv_consts():
    import re
    src = open(os.path.join(ROOT, "halo_amd", "csrc", "consts.hpp")).read()
    out = {}
    for name in ("PallasCurveCfg", "VestaCurveCfg"):
        body = src[src.index(f"struct {name}"):]
        body = body[:body.index("\n};")]
        c = {}
        for key in ("A1", "A2", "B1", "B2", "G1", "G2"):
            words = re.search(rf"GLV_{key}\[\d+\] = \{{([^}}]*)\}}", body).group(1)
            mag = sum(int(w, 16) << (32 * i) for i, w in enumerate(words.split(",")))
            neg = int(re.search(rf"GLV_{key}_NEG = (\d)", body).group(1))
            c[key] = -mag if neg else mag
        out[name] = c
    return out


@pytest.mark.parametrize("curve,r", [("PallasCurveCfg", PRIMES["fq"]), ("VestaCurveCfg", PRIMES["fp"])])
def test_glv_halves_fit_signed_windows(curve, r):
    c = _glv_consts()[curve]
    limit = (1 << 128) - sum(8 << (4 * w) for w in range(32))
    # the rounding bound: |k1| <= (|a1| + |a2|) / 2 + 1, |k2| <= (|b1| + |b2|) / 2 + 1
    assert (abs(c["A1"]) + abs(c["A2"])) // 2 + 1 < limit
    assert (abs(c["B1"]) + abs(c["B2"])) // 2 + 1 < limit

    def decompose(k):  # glv.hpp decompose on Python integers (round_shift384 included)
        c1 = (k * abs(c["G1"]) + (1 << 383)) >> 384
        c2 = (k * abs(c["G2"]) + (1 << 383)) >> 384
        c1 = -c1 if c["G1"] < 0 else c1
        c2 = -c2 if c["G2"] < 0 else c2
        return k - c1 * c["A1"] - c2 * c["A2"], -c1 * c["B1"] - c2 * c["B2"]

    rng = random.Random(5)
    ks = [0, 1, r - 1, r // 2, r // 2 + 1, r // 3, 2 * r // 3] + [rng.randrange(r) for _ in range(20000)]
    for k in ks:
        k1, k2 = decompose(k)
        assert abs(k1) < limit and abs(k2) < limit, (k, k1, k2)
