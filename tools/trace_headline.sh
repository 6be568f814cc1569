# Two-stream headline timeline: rocprofv3 kernel trace of the headline-only bench, then the last
# ${1:-6} k_acc launches' neighbourhood as rows (start, end, duration, queue, kernel) relative to the
# first of them.  bash tools/trace_headline.sh [steps]   (through gpurun; gpurun_out/tl_head/)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tl_head; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --steps 20 --warmup 3 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" ${1:-6} > $O/timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
k = int(sys.argv[2])
accs = [r for r in rows if 'k_acc' in r['Kernel_Name']]
# the timed region's k_acc launches are the ones before the standalone (isolated) ones: take the middle
acc = accs[len(accs) // 2 - k // 2: len(accs) // 2 + k // 2]
t0 = int(acc[0]['Start_Timestamp']) - 400000
t1 = int(acc[-1]['End_Timestamp'])
for r in rows:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if t0 <= s <= t1:
        n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('halo::', '')[:34]
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r.get('Queue_Id', '?'):>2} {n}")
PY
rm -rf $O/t
grep '^{' $O/log | tail -1 | cut -c1-200
