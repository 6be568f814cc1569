# Kernel timeline of batched 16 x 2^16 commitments (tools/msm_batch_time.py), run through gpurun from
# the repo root.  Output: gpurun_out/tl_batch/timeline.txt (the last batch call).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tl_batch; rm -rf $O && mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 tools/msm_batch_time.py 16 16 3 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $O/timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
so = [i for i, r in enumerate(rows) if 'k_sums_out' in r['Kernel_Name']]
i1 = so[-1]; i0 = so[-2] + 1
t0 = int(rows[i0]['Start_Timestamp'])
for r in rows[i0:i1 + 1]:
    s = int(r['Start_Timestamp']); e = int(r['End_Timestamp'])
    print(f"{(s - t0)/1e3:9.1f} {(e - t0)/1e3:9.1f} {(e - s)/1e3:8.1f} us q{r.get('Queue_Id','?'):>3} {r['Kernel_Name'][:60]}")
PY
rm -rf $O/t; cat $O/log | tail -2; cat $O/timeline.txt
