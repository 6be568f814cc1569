# Kernel timeline of one weighted IPA round (tools/ipa_time.py at 2^${1:-16}, second repetition), or
# of the window after the last launch of kernel ${2} when given (e.g. k_batch_lists: the switch to
# the tail rounds); run through gpurun from the repo root.  Output: gpurun_out/tl_ipa/timeline.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tl_ipa
rm -rf $O && mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 tools/ipa_time.py ${1:-16} > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" "${2:-}" > $O/timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
if len(sys.argv) > 2 and sys.argv[2]:
    ws = [r for r in rows if sys.argv[2] in r['Kernel_Name']]
    t0 = int(ws[-1]['Start_Timestamp']); t1 = t0 + 6000000
else:
    ws = [r for r in rows if 'k_weighted_prep' in r['Kernel_Name']]
    k = len(ws) - 6
    t0 = int(ws[k]['Start_Timestamp']); t1 = int(ws[k + 2]['Start_Timestamp'])
prev_end = None
for r in rows:
    s = int(r['Start_Timestamp']); e = int(r['End_Timestamp'])
    if t0 - 100000 <= s <= t1:
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        print(f"{(s - t0)/1e3:9.1f} {(e - t0)/1e3:9.1f} {(e - s)/1e3:8.1f} us gap {gap:7.1f} q{r.get('Queue_Id','?'):>3} {r['Kernel_Name'][:70]}")
        prev_end = max(prev_end or 0, e)
PY
rm -rf $O/t
cat $O/timeline.txt
