# Device idle time of the naive_prover at 2^${1:-20} (tools/prove_time.py, second repetition): the
# union of kernel intervals against the wall span of the repetition, and the largest idle gaps with the
# kernels on either side.  Run through gpurun from the repo root.  Output: gpurun_out/prove_gaps/gaps.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/prove_gaps
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 tools/prove_time.py ${1:-20} > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" $O/log > $O/gaps.txt <<'PY'
import csv, json, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
reps = [json.loads(l) for l in open(sys.argv[2]) if l.startswith('{')]
short = lambda r: r['Kernel_Name'].split('(')[0].replace('void ', '').replace('halo::', '')[:48]
ks = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r)) for r in rows]
ks = [k for k in ks if not k[2].startswith(('k_synth_bases', 'k_shift_windows'))]
# the second repetition: kernels starting after its host start stamp (CLOCK_MONOTONIC, the trace's clock)
r1 = reps[-1]["start_ns"]
rep = [k for k in ks if k[0] >= r1]
t0 = r1
print("rep 1 host times (ms):", reps[-1]["times_ms"])
busy, gaps, end, prev_name = 0, [], t0, '(host start)'
for i, (s, e, n) in enumerate(rep):
    if s > end:
        gaps.append((s - end, end - t0, prev_name, n))
    busy += max(0, e - max(s, end))
    if e > end:
        end, prev_name = e, n
span = end - t0
print(f"kernels {len(rep)}  span {span / 1e6:.2f} ms  busy (union) {busy / 1e6:.2f} ms  idle {(span - busy) / 1e6:.2f} ms")
tot = {}
for g in gaps:
    b = 'lt10us' if g[0] < 1e4 else ('lt50us' if g[0] < 5e4 else 'ge50us')
    tot[b] = tot.get(b, [0, 0])
    tot[b][0] += 1
    tot[b][1] += g[0]
print("gaps by size:", {k: (v[0], round(v[1] / 1e6, 2)) for k, v in tot.items()}, "(count, ms)")
for g in sorted(gaps, reverse=True)[:40]:
    print(f"gap {g[0] / 1e3:8.1f} us at {g[1] / 1e6:8.2f} ms  after {g[2]:<48} before {g[3]}")
# the kernels around the ten largest gaps (start offset, duration)
for g in sorted(gaps, reverse=True)[:10]:
    at = t0 + g[1] + g[0]
    i = next(j for j, k in enumerate(rep) if k[0] >= at)
    print(f"-- gap {g[0] / 1e3:.1f} us at {g[1] / 1e6:.2f} ms")
    for k in rep[max(0, i - 6): i + 4]:
        print(f"   {(k[0] - t0) / 1e6:9.3f} ms {(k[1] - k[0]) / 1e3:8.1f} us  {k[2]}")
PY
rm -rf $O/t
head -50 $O/gaps.txt
