"""Generate halo_amd/csrc/consts.hpp: field/curve constants in the device-internal representation.

Device-internal field format (see DESIGN.md "Field representation"):
  9 limbs x 29 bits (radix 2^29) in uint32 registers, Montgomery with R' = 2^261, values kept in
  [0, 2p) after every operation.  ABI buffers use the arkworks format (4 x u64, Montgomery with
  R = 2^256, canonical in [0, p)); conversion is one Montgomery multiplication by a constant.

Run:  python3 halo_amd/csrc/gen_consts.py > halo_amd/csrc/consts.hpp
"""
from __future__ import annotations

FP = 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001  # ark_pallas::Fr
FQ = 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001  # ark_pallas::Fq
W = 29
NL = 9
RP = 1 << (W * NL)  # 2^261
MAXLOG = 32


def limbs29(x: int) -> list[int]:
    assert 0 <= x < RP
    return [(x >> (W * i)) & ((1 << W) - 1) for i in range(NL)]


def arr(name: str, x: int) -> str:
    return f"    static constexpr uint32_t {name}[{NL}] = {{{', '.join(hex(v) for v in limbs29(x))}}};\n"


def u64s(x: int) -> str:
    return ", ".join(f"0x{(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF:016x}ull" for i in range(4))


def field_block(struct: str, p: int) -> str:
    out = [f"struct {struct} {{\n"]
    out.append(f"    static constexpr uint64_t MODULUS64[4] = {{{u64s(p)}}};\n")
    out.append(arr("P", p))
    out.append(arr("P2", 2 * p))
    out.append(arr("P4", 4 * p))
    out.append(arr("P6", 6 * p))
    out.append(arr("P8", 8 * p))
    out.append(arr("ONE", RP % p))                         # 1 in internal Montgomery form
    out.append(arr("R2", RP * RP % p))                     # canonical -> internal
    out.append(arr("ARK2INT", (RP * RP >> 256) % p))       # ark Montgomery -> internal
    out.append(arr("INT2ARK", (1 << 256) % p))             # internal -> ark Montgomery
    out.append(arr("ARK_MUL_FIX", (1 << 266) % p))         # ark x ark through R' = 2^261 -> ark
    out.append(arr("ARK2CANON", 32))                        # ark Montgomery -> canonical integer
    out.append(arr("INV_FIX", pow(RP, 3, p)))              # fe_inv: (x R')^-1 -> x^-1 R'
    # NTT domain constants: omega_N = 5^((p-1)/N) for N = 2^k, internal Montgomery form
    om = [pow(5, (p - 1) >> k, p) for k in range(MAXLOG + 1)]
    omi = [pow(w, -1, p) for w in om]
    ninv = [pow(1 << k, -1, p) for k in range(MAXLOG + 1)]

    def table(name, vals):
        rows = ",\n        ".join("{" + ", ".join(hex(v) for v in limbs29(x * RP % p)) + "}" for x in vals)
        return f"    static constexpr uint32_t {name}[{MAXLOG + 1}][{NL}] = {{\n        {rows}}};\n"

    out.append(table("OMEGA", om))
    out.append(table("OMEGA_INV", omi))
    out.append(table("N_INV", ninv))
    # NTT output multiplier with the inverse scaling folded in: (2^261 / N) mod p, raw limbs.  The NTT
    # passes take ark words (x 2^256) as internal values (x 2^-5 R'), so the last pass multiplies by
    # 2^261 (forward: ONE) or 2^261 / N (inverse) to land on ark words again (ntt.hip).
    rows = ",\n        ".join("{" + ", ".join(hex(v) for v in limbs29(RP * x % p)) + "}" for x in ninv)
    out.append(f"    static constexpr uint32_t NINV_ARK[{MAXLOG + 1}][{NL}] = {{\n        {rows}}};\n")
    out.append("};\n")
    return "".join(out)


# GLV endomorphism phi(x, y) = (beta x, y) = lambda (x, y) (beta: cube root of unity in the base
# field, lambda: in the scalar field; the matching pair, checked against the oracle in
# tests/test_oracle.py::test_glv_constants) and the short lattice basis (a_i, b_i) with
# a_i + b_i lambda = 0 mod r from the half extended Euclid of (r, lambda).
GLV = {
    "PallasCurveCfg": dict(
        lam=0x397E65A7D7C1AD71AEE24B27E308F0A61259527EC1D4752E619D1840AF55F1B1,
        beta=0x2D33357CB532458ED3552A23A8554E5005270D29D19FC7D27B7FD22F0201B547),
    "VestaCurveCfg": dict(
        lam=0x12CCCA834ACDBA712CAAD5DC57AAB1B01D1F8BD237AD31491DAD5EBDFDFE4AB9,
        beta=0x06819A58283E528E511DB4D81CF70F5A0FED467D47C033AF2AA9D2E050AA0E4F),
}


def glv_basis(r: int, lam: int):
    import math
    r0, t0, r1, t1 = r, 0, lam, 1
    sq = math.isqrt(r)
    seq = [(r0, t0), (r1, t1)]
    while r1 >= sq:
        qq = r0 // r1
        r0, r1 = r1, r0 - qq * r1
        t0, t1 = t1, t0 - qq * t1
        seq.append((r1, t1))
    (rl1, tl1), (rl, tl) = seq[-1], seq[-2]
    qq = r0 // r1
    r2, t2 = r0 - qq * r1, t0 - qq * t1
    v1 = (rl1, -tl1)
    v2 = min([(rl, -tl), (r2, -t2)], key=lambda v: v[0] ** 2 + v[1] ** 2)
    return v1, v2


def words32(x: int, n: int) -> str:
    assert 0 <= x < (1 << (32 * n))
    return ", ".join(hex((x >> (32 * i)) & 0xFFFFFFFF) for i in range(n))


def curve_block(struct: str, base: int, scalar: int) -> str:
    # short Weierstrass y^2 = x^3 + 5; generator (-1, 2)
    out = [f"struct {struct} {{\n"]
    out.append(arr("B", 5 * RP % base))
    out.append(arr("GX", (base - 1) * RP % base))
    out.append(arr("GY", 2 * RP % base))
    g = GLV[struct]
    lam, beta = g["lam"], g["beta"]
    assert pow(beta, 3, base) == 1 and pow(lam, 3, scalar) == 1
    out.append(arr("BETA", beta * RP % base))  # internal Montgomery form
    (a1, b1), (a2, b2) = glv_basis(scalar, lam)
    det = a1 * b2 - a2 * b1
    assert abs(det) == scalar and (a1 + b1 * lam) % scalar == 0 and (a2 + b2 * lam) % scalar == 0
    # c1 = round(b2 k / det), c2 = round(-b1 k / det) ~ (k * G) >> 384 with G = round(2^384 * num / det)
    g1 = (b2 * (1 << 384) + det // 2) // det
    g2 = (-b1 * (1 << 384) + det // 2) // det
    for name, v in (("GLV_A1", a1), ("GLV_B1", b1), ("GLV_A2", a2), ("GLV_B2", b2), ("GLV_G1", g1), ("GLV_G2", g2)):
        nw = 9 if name in ("GLV_G1", "GLV_G2") else 5
        out.append(f"    static constexpr uint32_t {name}[{nw}] = {{{words32(abs(v), nw)}}};  // magnitude\n")
        out.append(f"    static constexpr int {name}_NEG = {1 if v < 0 else 0};\n")
    out.append("};\n")
    return "".join(out)


def main() -> None:
    print("// Generated by gen_consts.py -- do not edit.")
    print("#pragma once")
    print("#include <stdint.h>")
    print("namespace halo {")
    print(f"constexpr int NLIMB = {NL};")
    print(f"constexpr int LIMB_BITS = {W};")
    print(f"constexpr uint32_t LIMB_MASK = 0x{(1 << W) - 1:x}u;")
    print(f"constexpr int MAX_LOG_DOMAIN = {MAXLOG};")
    print(field_block("FpCfg", FP))
    print(field_block("FqCfg", FQ))
    print(curve_block("PallasCurveCfg", FQ, FP))
    print(curve_block("VestaCurveCfg", FP, FQ))
    print("}  // namespace halo")


if __name__ == "__main__":
    main()
