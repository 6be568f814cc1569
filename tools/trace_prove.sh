# Kernel timeline of the prover's round 5 at 2^${1:-16} (tools/prove_time.py, second repetition): every
# kernel from the last two k_lincomb launches (the round's geometric sums) on, with a per-queue column and
# idle gaps; run through gpurun from the repo root.  Output: gpurun_out/tl_prove/timeline.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tl_prove
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 tools/prove_time.py ${1:-16} > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $O/timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
ws = [r for r in rows if 'k_lincomb' in r['Kernel_Name']]
t0 = int(ws[-2]['Start_Timestamp'])
prev_end = None
for r in rows:
    s = int(r['Start_Timestamp']); e = int(r['End_Timestamp'])
    if s >= t0:
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        name = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('halo::', '')[:60]
        print(f"{(s - t0)/1e3:9.1f} {(e - t0)/1e3:9.1f} {(e - s)/1e3:8.1f} us gap {gap:7.1f} q{r.get('Queue_Id','?'):>3} {name}")
        prev_end = max(prev_end or 0, e)
PY
rm -rf $O/t
wc -l $O/timeline.txt; cat $O/log
