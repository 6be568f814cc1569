"""Merges the VALU counter passes of tools/pmc_valu.sh into profiles/pmc_summary.json.

usage: python3 tools/pmc_valu_merge.py <acc_dir> <ntt_dir> <pmc_summary.json> [<ntt24_dir>]

Per kernel key (msm_acc: k_acc<PallasCurve> of the headline; ntt_pass: k_ntt_pass<FpCfg, 2048, true> (full blocks) of the
2^22 pair; ntt_pass_1024: k_ntt_pass<FpCfg, 1024, true> of the 2^24 pair, 8-bit passes) it stores, per dispatch: SQ_INSTS_VALU, SQ_INSTS_VALU_INT64, SQ_INSTS_VALU_INT32, SQ_WAVES
(wave-instructions), and the kernel's static class counts from tools/valu_mix.py, which split the
dynamic INT64 count into multiply-adds and other 64-bit ops and the INT32 count into VOP3 and
VOP1/VOP2 encodings.  The file must already be stamped for the current library (pmc_stamp.sh).
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from pmc_summary import load, summarise  # noqa: E402
import valu_mix  # noqa: E402

KERNELS = {"msm_acc": ("acc", "k_acc<halo::PallasCurve>", "5k_accINS_11PallasCurve"),
           "ntt_pass": ("ntt", "k_ntt_pass<halo::FpCfg, 2048, true>", "k_ntt_passINS_5FpCfgELi2048ELb1E"),
           "ntt_pass_1024": ("ntt24", "k_ntt_pass<halo::FpCfg, 1024, true>", "k_ntt_passINS_5FpCfgELi1024ELb1E")}


def main():
    acc_dir, ntt_dir, path = sys.argv[1:4]
    ntt24_dir = sys.argv[4] if len(sys.argv) > 4 else None
    summ = json.load(open(path))
    lib = os.path.join(os.path.dirname(HERE), "halo_amd", "lib", "libhalo_gpu.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    if summ.get("library_sha256") != sha:
        raise SystemExit("pmc_summary.json is stamped for another library: run tools/pmc_stamp.sh first")
    dirs = {"acc": summarise(load(acc_dir)), "ntt": summarise(load(ntt_dir)),
            "ntt24": summarise(load(ntt24_dir)) if ntt24_dir else {}}
    import tempfile
    static = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in valu_mix.code_objects(lib, tmp):
            for fn, insts in valu_mix.functions(co).items():
                for key, (_, _, mangled) in KERNELS.items():
                    if mangled in fn:
                        static[key] = valu_mix.analyse(fn, insts)["function"]
    for key, (src, name, _) in KERNELS.items():
        rows = {k: v for k, v in dirs[src].items() if name in k}
        if not rows and src == "ntt24" and not ntt24_dir:
            continue
        if not rows:
            raise SystemExit(f"no dispatches of {name}")
        k0 = max(rows, key=lambda k: rows[k]["dispatches"])
        r = rows[k0]
        summ.setdefault(key, {})["valu"] = {
            "kernel": k0.split("(")[0],
            "dispatches": r["dispatches"],
            "valu_per_dispatch": r["SQ_INSTS_VALU"],
            "int64_per_dispatch": r["SQ_INSTS_VALU_INT64"],
            "int32_per_dispatch": r["SQ_INSTS_VALU_INT32"],
            "waves_per_dispatch": r["SQ_WAVES"],
            "static_classes": static.get(key),
            "units": "wave-instructions per dispatch",
        }
    summ["valu_source"] = ("rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES over the "
                           "headline bench (k_acc), tools/ntt_time.py 22 (k_ntt_pass<2048>) and tools/ntt_time.py 24 "
                           "(k_ntt_pass<1024>); static classes from tools/valu_mix.py on the same library")
    json.dump(summ, open(path, "w"), indent=1)
    print(json.dumps({k: summ[k]["valu"] for k in KERNELS if k in summ and "valu" in summ[k]}, indent=1))


if __name__ == "__main__":
    main()
