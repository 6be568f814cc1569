"""Summarises tools/pmc_kacc.sh: per build, k_acc's VALU instructions per launch, wave-cycle split
(active / issue-stalled / parked), GUI-active cycles and the effective shader clock (cycles over the
kernel-trace duration).  SQ cycle counters count quad-cycles (MI355X_MICROARCH.md constants table).
usage: python tools/pmc_kacc_summary.py <out dir> <tag>=<lib> ...
"""
import collections
import csv
import glob
import json
import sys

import os
SUB, XCDS, CUS = os.environ.get("KSUB", "k_acc<"), 8, 256


def counters(d):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if SUB in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def durations(d):
    ds = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if SUB in r["Kernel_Name"]:
                ds.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return sum(ds) / len(ds) if ds else None


def main():
    out = {}
    for spec in sys.argv[2:]:
        tag = spec.split("=", 1)[0]
        a, b = counters(f"{sys.argv[1]}/{tag}/a"), counters(f"{sys.argv[1]}/{tag}/b")
        ms = durations(f"{sys.argv[1]}/{tag}/c")
        cyc = b.get("GRBM_GUI_ACTIVE", 0) / XCDS
        r = {"kernel_ms": ms, "kernel": SUB, **a, "gui_active_cycles_per_xcd": cyc}
        if ms and cyc:
            r["effective_clock_GHz"] = cyc / (ms * 1e6)
            r["valu_wave_instr_per_cu_clk"] = a["SQ_INSTS_VALU"] / (CUS * cyc)
        wc = a.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                r[k + "_frac_of_wave_cycles"] = a.get(k, 0) / wc
        out[tag] = r
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
