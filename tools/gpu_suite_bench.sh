# Full GPU suite + a headline / NTT bench line that reads the stamped profiles/pmc_summary.json
# (compute_roofline filled), through gpurun from the repo root: bash tools/gpu_suite_bench.sh <tag>
set -o pipefail
O=gpurun_out/suite_${1:-r05}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1; rc=$?
tail -3 $O/gputest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('ms/step', d['ms_per_step']); print('compute', json.dumps(d['compute_roofline'])[:700]); print('traffic', d['roofline']['traffic'])
print('ntt', json.dumps(d['extra']['ntt'])[:900])"
