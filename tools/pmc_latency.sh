# Counters of the reduction-tail kernels for synchronous single MSMs at 2^${1:-15} (tools/msm_latency.py,
# serialised by --pmc), run through gpurun from the repo root.  Output: gpurun_out/pmc_lat/summary.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/pmc_lat; rm -rf $D; mkdir -p $D
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $D/a -o run -- python3 tools/msm_latency.py ${1:-15} > $D/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $D/b -o run -- python3 tools/msm_latency.py ${1:-15} > $D/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $D/e -o run -- python3 tools/msm_latency.py ${1:-15} > $D/e.log 2>&1 || exit 1
python3 tools/pmc_kernels_summary.py $D > $D/summary.txt; cat $D/summary.txt
python3 - $D <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/a/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_merge" in r["Kernel_Name"] or "k_acc<" in r["Kernel_Name"]:
            agg[(r["Kernel_Name"][:30], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, sum(v) / len(v))
PY
