"""Compute rooflines of the naive_prover's kernels from tools/pmc_prove.sh's passes.

usage: python3 tools/pmc_prove_merge.py <valu_pmc_dir> <kernel_stats.csv> <out.json> [library.so]

For every kernel that takes at least 1 % of the traced prove time: its calls and mean duration
(rocprofv3 --kernel-trace --stats), its counted VALU instructions per dispatch (SQ_INSTS_VALU, _INT64,
_INT32) split into issue classes by the kernel's static code (tools/valu_mix.py), and the issue-time
ceiling at the measured per-class rates (profiles/issue_rates.json; bench.py valu_ceiling): frac =
ceiling / mean duration.  Written with the library's sha256 so bench.py can attach the figures to the
build they were measured on.
"""
import csv
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from pmc_summary import load, summarise  # noqa: E402
import valu_mix  # noqa: E402
from bench import valu_ceiling  # noqa: E402


def short(name):
    return name.split("(")[0].replace("void ", "").replace("halo::", "")


def main():
    pmc_dir, stats_csv, out_path = sys.argv[1:4]
    lib = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "halo_amd", "lib", "libhalo_gpu.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    rates = json.load(open(os.path.join(ROOT, "profiles", "issue_rates.json")))["rates"]
    stats = {r["Name"]: r for r in csv.DictReader(open(stats_csv))}
    total_ns = sum(float(r["TotalDurationNs"]) for r in stats.values())
    counters = summarise(load(pmc_dir))
    # static classes by demangled kernel name
    static = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in valu_mix.code_objects(lib, tmp):
            funcs = {fn: insts for fn, insts in valu_mix.functions(co).items() if fn.startswith("_Z")}
            names = list(funcs)
            dms = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                                 check=True).stdout.splitlines()
            for fn, dm in zip(names, dms):
                static[short(dm)] = valu_mix.analyse(fn, funcs[fn])["function"]
    out = {"library_sha256": sha, "source": "tools/pmc_prove.sh: rocprofv3 --kernel-trace --stats and one --pmc pass "
           "(SQ_INSTS_VALU, SQ_INSTS_VALU_INT32, SQ_INSTS_VALU_INT64, SQ_WAVES) of tools/prove_time.py",
           "traced_total_ms": total_ns / 1e6, "kernels": {}}
    for name, r in sorted(stats.items(), key=lambda kv: -float(kv[1]["TotalDurationNs"])):
        share = float(r["TotalDurationNs"]) / total_ns
        if share < 0.01:
            continue
        k = short(name)
        entry = {"calls": int(r["Calls"]), "mean_us": float(r["AverageNs"]) / 1e3,
                 "total_ms": float(r["TotalDurationNs"]) / 1e6, "share": share}
        c = next((v for kk, v in counters.items() if short(kk) == k), None)
        if c and k in static and "SQ_INSTS_VALU" in c:
            valu = {"valu_per_dispatch": c["SQ_INSTS_VALU"], "int64_per_dispatch": c.get("SQ_INSTS_VALU_INT64", 0.0),
                    "int32_per_dispatch": c.get("SQ_INSTS_VALU_INT32", 0.0), "static_classes": static[k]}
            t, lanes, mix = valu_ceiling(valu, rates)
            entry.update({"valu_lane_instructions_per_dispatch": lanes, "ceiling_us": t * 1e6,
                          "compute_frac": t * 1e6 / entry["mean_us"], "dynamic_mix": mix,
                          "waves_per_dispatch": c.get("SQ_WAVES")})
        out["kernels"][k] = entry
    json.dump(out, open(out_path, "w"), indent=1)
    for k, e in out["kernels"].items():
        print("%-60s %5d x %9.1f us = %8.2f ms (%4.1f %%)  frac %s" % (
            k[:60], e["calls"], e["mean_us"], e["total_ms"], 100 * e["share"],
            "%.3f" % e["compute_frac"] if "compute_frac" in e else "-"))


if __name__ == "__main__":
    main()
