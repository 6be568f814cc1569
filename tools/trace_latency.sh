# Kernel trace of synchronous single MSMs at 2^${1:-10} (tools/msm_latency.py), run through gpurun
# from the repo root: per-kernel durations and the gaps between them for the last call.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tl_lat_${1:-10}
rm -rf $O && mkdir -p $O
timeout -k 10 200 python3 tools/msm_latency.py ${1:-10} > $O/plain.log 2>&1 || { tail -5 $O/plain.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 tools/msm_latency.py ${1:-10} > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $O/timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
acc = [i for i, r in enumerate(rows) if 'k_acc<' in r['Kernel_Name']]
i0 = acc[-2] - 8
t0 = int(rows[i0]['Start_Timestamp'])
for r in rows[i0:acc[-1] - 7]:
    s = int(r['Start_Timestamp']); e = int(r['End_Timestamp'])
    print(f"{(s - t0)/1e3:9.1f} {(e - t0)/1e3:9.1f} {(e - s)/1e3:8.1f} us q{r.get('Queue_Id','?'):>3} {r['Kernel_Name'][:60]}")
PY
rm -rf $O/t
cat $O/plain.log; cat $O/timeline.txt
