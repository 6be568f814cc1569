"""Summarises tools/pmc_kernels.sh: per kernel (name prefix up to the template arguments), mean
serialised duration, counters per launch, HBM bytes (FETCH_SIZE x 2 for streaming reads on gfx950 is
NOT applied here: raw values, MI355X_MICROARCH.md HBM section), VALU issue per CU-cycle, VALU
instructions per wave (k_acc: a wave's 64 lanes each run K = 16 additions, so / 16 = per addition)
and the GUI-active clock in MHz.
usage: python tools/pmc_kernels_summary.py <dir> [substring ...]"""
import collections
import csv
import glob
import sys

D = sys.argv[1]
SUBS = sys.argv[2:] or ["k_rs_", "k_digits", "k_acc<", "k_bucket_starts", "k_merge", "k_rowcol", "k_bitterms",
                        "k_bitcombine", "k_final", "k_group_sums"]
XCDS, CUS = 8, 256


def short(name):
    for s in SUBS:
        if s in name:
            i = name.find("(")
            return name[:i if i > 0 else 80][:70]
    return None


def counters(p):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{D}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def durations(p):
    ds = collections.defaultdict(list)
    for f in glob.glob(f"{D}/{p}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                ds[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    return {k: (sum(v) / len(v), len(v)) for k, v in ds.items()}


dur = durations("a")
c = {}
for p in "abcde":
    for k, d in counters(p).items():
        c.setdefault(k, {}).update(d)
print(f"{'kernel':70s} {'us':>8s} {'n':>4s} {'VALU/CU/clk':>11s} {'LDSi/CU/clk':>11s} {'wait%':>6s} "
      f"{'issue%':>6s} {'fetchMB':>8s} {'writeMB':>8s} {'ldsconf%':>8s} {'waves':>7s} {'VALU/wave':>10s} {'MHz':>6s}")
for k in sorted(c, key=lambda k: -dur.get(k, (0, 0))[0]):
    d = c[k]
    us, n = dur.get(k, (0.0, 0))
    cyc = d.get("GRBM_GUI_ACTIVE", 0) / XCDS
    valu = d.get("SQ_INSTS_VALU", 0) / (CUS * cyc) if cyc else 0
    ldsi = d.get("SQ_INSTS_LDS", 0) / (CUS * cyc) if cyc else 0
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    conf = d.get("SQ_LDS_BANK_CONFLICT", 0) / (d.get("SQ_LDS_IDX_ACTIVE", 0) or 1) * 100
    print(f"{k:70s} {us:8.1f} {n:4d} {valu:11.3f} {ldsi:11.3f} {100 * d.get('SQ_WAIT_ANY', 0) / wc:6.1f} "
          f"{100 * d.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} {d.get('FETCH_SIZE', 0) / 1024:8.1f} "
          f"{d.get('WRITE_SIZE', 0) / 1024:8.1f} {conf:8.1f} {d.get('SQ_WAVES', 0):7.0f} "
          f"{d.get('SQ_INSTS_VALU', 0) / (d.get('SQ_WAVES', 0) or 1):10.0f} {cyc / us if us else 0:6.0f}")
