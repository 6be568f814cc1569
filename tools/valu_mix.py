"""VALU instruction mix of a kernel in the built library, by issue class (the compute roofline's weights).

    python3 tools/valu_mix.py [--lib halo_amd/lib/libhalo_gpu.so] [--json out.json] NAME_SUBSTRING...

Extracts every gfx950 code object from the library's .hip_fatbin (one clang offload bundle per
translation unit), disassembles them (llvm-objdump), and for each kernel whose mangled name contains
the substring prints the static VALU counts of the whole function and of its innermost loop body (the
region between the largest backward branch's target and the branch), split into the issue classes
measured by tools/micro/issue_bench.hip:
  mad_u64, mad_i64 -- v_mad_u64_u32, v_mad_i64_i32;
  ashr64  -- v_ashrrev_i64;  other64 -- the other 64-bit VOP3 integer ops (v_lshl_add_u64, ...);
  vop3  -- every other VALU in a VOP3 encoding (no _e32 suffix: v_add3_u32, v_alignbit_b32,
           v_bfe_*, *_e64 forms, ...);
  vop2  -- VOP1 / VOP2 encodings (_e32 suffix: v_and_b32_e32, v_add_u32_e32, v_mov_b32_e32, ...).
The loop body's mix stands for the kernel's dynamic mix when the loop dominates (k_acc: 16 additions
per lane; k_ntt_pass: the radix-4 group loop); bench.py weights the measured per-class costs by it.
"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def code_objects(lib, tmp):
    fat = os.path.join(tmp, "fatbin.bin")
    # an explicit output file: with only an input objcopy rewrites the library in place (new sha256)
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", lib, os.path.join(tmp, "discard.so")],
                   check=True)
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    out = []
    for k in range(len(offs) - 1):
        part = os.path.join(tmp, f"b{k}.bin")
        open(part, "wb").write(data[offs[k]:offs[k + 1]])
        co = os.path.join(tmp, f"b{k}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            f"--targets={TARGET}", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co):
            out.append(co)
    return out


def functions(co):
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True, text=True,
                         check=True).stdout
    funcs, cur = {}, None
    for ln in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", ln)
        if m:
            cur = m.group(2)
            funcs[cur] = []
            continue
        if cur is None or not ln.startswith("\t"):
            continue
        body, _, cmt = ln.partition("//")
        toks = body.split()
        if not toks:
            continue
        addr = re.search(r"([0-9A-F]{8,}):", cmt)
        tgt = re.search(r"<.*\+0x([0-9a-f]+)>", cmt)
        funcs[cur].append((int(addr.group(1), 16) if addr else None, toks[0], int(tgt.group(1), 16) if tgt else None))
    return funcs


def klass(op):
    if not op.startswith("v_") or op.startswith("v_mfma"):
        return None
    if op == "v_mad_u64_u32":
        return "mad_u64"
    if op == "v_mad_i64_i32":
        return "mad_i64"
    if op.endswith("_e32") or "_dpp" in op or "_sdwa" in op:
        return "vop2"
    if op == "v_ashrrev_i64":
        return "ashr64"
    if any(t in op for t in ("_i64", "_u64", "_b64")):
        return "other64"
    return "vop3"


CLASSES = ("mad_u64", "mad_i64", "ashr64", "other64", "vop3", "vop2")
INT64 = ("mad_u64", "mad_i64", "ashr64", "other64")


def mix(insts):
    c = dict.fromkeys(CLASSES, 0)
    for _, op, _ in insts:
        k = klass(op)
        if k:
            c[k] += 1
    return c


def analyse(name, insts):
    start = insts[0][0] if insts and insts[0][0] is not None else 0
    # backward branches: target offset (relative to the function) below the branch's own offset
    loops = []
    for i, (addr, op, tgt) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            if tgt is not None and addr is not None and tgt < addr - start:
                j0 = next(k for k, x in enumerate(insts) if x[0] is not None and x[0] - start >= tgt)
                loops.append((i - j0, j0, i))
    res = {"function": mix(insts), "static_valu": sum(mix(insts).values())}
    if loops:
        loops.sort()
        _, j0, j1 = loops[0]  # innermost (shortest) loop
        big = max(loops)
        res["inner_loop"] = mix(insts[j0:j1 + 1])
        res["largest_loop"] = mix(insts[big[1]:big[2] + 1])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(__file__), "..", "halo_amd", "lib", "libhalo_gpu.so"))
    ap.add_argument("--json")
    ap.add_argument("names", nargs="+")
    a = ap.parse_args()
    lib = os.path.abspath(a.lib)
    out = {"library_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(), "kernels": {}}
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            for fn, insts in functions(co).items():
                if any(n in fn for n in a.names):
                    out["kernels"][fn] = analyse(fn, insts)
    for fn, r in out["kernels"].items():
        print(fn)
        for k, v in r.items():
            print(f"  {k}: {v}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
