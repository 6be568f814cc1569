# Kernel timeline of the pipelined 2^20 MSM bench (run through gpurun from the repo root).
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tl_${1:-a}
rm -rf $O && mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --steps 10 --warmup 2 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $O/timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
acc = [r for r in rows if 'k_acc<' in r['Kernel_Name']]
t0 = int(acc[len(acc)//2 - 3]['Start_Timestamp'])
t1 = int(acc[len(acc)//2 + 1]['Start_Timestamp'])
for r in rows:
    s = int(r['Start_Timestamp']); e = int(r['End_Timestamp'])
    if t0 - 200000 <= s <= t1:
        print(f"{(s - t0)/1e3:9.1f} {(e - t0)/1e3:9.1f} {(e - s)/1e3:8.1f} us q{r.get('Queue_Id','?'):>3} {r['Kernel_Name'][:60]}")
PY
rm -rf $O/t
head -80 $O/timeline.txt
