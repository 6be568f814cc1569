"""Summarises the SQ / GRBM counter passes of tools/pmc_valu.sh into per-launch VALU issue rates.

VALU issue rate = SQ_INSTS_VALU / (CUs x cycles of one XCD's GRBM_GUI_ACTIVE); GRBM_GUI_ACTIVE is
reported summed over the 8 XCDs.  The reference rate is the measured VOP3 issue ceiling of the
integer multiply-add (tools/micro/modmul_bench.hip): ~0.9 wave-instructions per CU
per clock.
usage: python tools/valu_summary.py <dir with a/ and b/ rocprofv3 outputs> <command description>
"""
import collections
import csv
import glob
import json
import sys

KERNELS = {"msm_acc": "k_acc<", "ntt_pass": "k_ntt_pass<"}
CUS, XCDS = 256, 8


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    out, cmd = sys.argv[1], sys.argv[2]
    a, b = load(f"{out}/a"), load(f"{out}/b")
    res = {"source": f"rocprofv3 --pmc (two passes: SQ counters; GRBM_GUI_ACTIVE) of '{cmd}'",
           "valu_issue_ceiling_wave_instr_per_cu_clk": 0.9}
    for key, sub in KERNELS.items():
        ka = [k for k in a if sub in k]
        kb = [k for k in b if sub in k]
        if not ka or not kb:
            continue
        avg = lambda agg, ks, c: sum(sum(agg[k][c]) for k in ks) / sum(len(agg[k][c]) for k in ks)
        valu = avg(a, ka, "SQ_INSTS_VALU")
        cyc = avg(b, kb, "GRBM_GUI_ACTIVE") / XCDS
        res[key] = {
            "kernel": ka[0].split("(")[0],
            "SQ_INSTS_VALU": valu,
            "SQ_INSTS_SALU": avg(a, ka, "SQ_INSTS_SALU"),
            "SQ_INSTS_LDS": avg(a, ka, "SQ_INSTS_LDS"),
            "SQ_INSTS_VMEM": avg(a, ka, "SQ_INSTS_VMEM"),
            "SQ_WAVES": avg(a, ka, "SQ_WAVES"),
            "gui_active_cycles_per_xcd": cyc,
            "valu_wave_instr_per_cu_clk": valu / (CUS * cyc),
        }
    json.dump(res, sys.stdout, indent=1)


main()
