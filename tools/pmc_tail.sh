# Per-wave instruction counts and lifetimes of the MSM reduction-tail kernels during an IPA opening
# (tools/ipa_time.py at 2^${1:-16}); one --pmc pass, run through gpurun from the repo root.
# Output: gpurun_out/pmc_tail/summary.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_tail; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $O/a -o run -- python3 tools/ipa_time.py ${1:-16} > $O/a.log 2>&1 || { tail -5 $O/a.log; exit 1; }
python3 - $O/a > $O/summary.txt <<'PY'
import collections, csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES"]
print("kernel".ljust(42) + "".join(c[3:].rjust(16) for c in cols) + "   per-wave: valu  cycles")
for k, d in sorted(agg.items()):
    avg = {c: sum(d[c]) / max(1, len(d[c])) for c in cols}
    w = max(avg["SQ_WAVES"], 1)
    print(k.ljust(42) + "".join(f"{avg[c]:16.0f}" for c in cols) + f"   {avg['SQ_INSTS_VALU']/w:10.0f} {avg['SQ_WAVE_CYCLES']/w:10.0f}")
PY
rm -rf $O/a
cat $O/summary.txt
