# SQ counters of the NTT pass kernel (run through gpurun from the repo root)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_ntt; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $O/a -o run -- python3 tools/ntt_time.py 22 > $O/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM --output-format csv -d $O/b -o run -- python3 tools/ntt_time.py 22 > $O/b.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for sub in ('a', 'b'):
    f = glob.glob(f'{O}/{sub}/**/*counter_collection.csv', recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:40]
        agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, d in agg.items():
        if 'ntt_pass' not in k and 'k_acc' not in k: continue
        print(sub, k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
rm -rf $O/a $O/b
