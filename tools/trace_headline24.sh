# Two-stream pipelined MSM timeline at 2^24 (bench.py --logn 24, 8 steps): rocprofv3 kernel trace, the
# middle k_acc launches' neighbourhood as rows (start, end, duration, queue, kernel) relative to the first
# of them, and per-kernel totals over the timed region.  Run through gpurun from the repo root.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tl_head24; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py --no-cpu --logn 24 --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --batch-ntt 0 --pcdl "" --steps 8 --warmup 4 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $O/timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
accs = [r for r in rows if 'k_acc' in r['Kernel_Name']]
acc = accs[6:12]  # after the 4 warm-up steps (each step one k_acc) and the first timed ones
t0 = int(acc[0]['Start_Timestamp']) - 4000000
t1 = int(acc[-1]['End_Timestamp'])
tot = {}
for r in rows:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if t0 <= s <= t1:
        n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('halo::', '')[:34]
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r.get('Queue_Id', '?'):>2} {n}")
        tot[n] = tot.get(n, 0) + (e - s)
print("totals (ms) over the window:", {k: round(v / 1e6, 2) for k, v in sorted(tot.items(), key=lambda kv: -kv[1])})
PY
rm -rf $O/t
grep '^{' $O/log | tail -1 | cut -c1-300
