# Baseline measurements of the current library (gpurun, repo root): full bench line, the headline at
# GPU_MAX_HW_QUEUES 4 vs 8, the pipelined kernel timeline and the per-kernel SQ counters.
#   bash tools/r04_base.sh <tag>
set -o pipefail
tag=${1:-r04a}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$tag
rm -rf $O && mkdir -p $O
HEAD='--no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl ""'
timeout -k 10 400 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -n 1 $O/bench.json | cut -c 1-400
for i in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --steps 20 > $O/hwq$q.$i.json 2> $O/hwq.err || { tail -5 $O/hwq.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/hwq$q.$i.json').read().strip().splitlines()[-1]); e=d['extra']
print('hwq $q', 'ms/step %.3f'%d['ms_per_step'], 'acc %.3f'%d['roofline']['avg_launch_ms'], 'lat %.3f'%e['msm_single_latency_ms'], 'ntt %.3f'%e['ntt']['pair_ms'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv && rm -rf $O/tr
python3 tools/timeline.py $O/kernel_trace.csv 5 > $O/timeline.txt
tail -8 $O/timeline.txt
bash tools/pmc_kernels.sh $tag > /dev/null && cp gpurun_out/pmc_k/$tag/summary.txt $O/pmc_kernels.txt && rm -rf gpurun_out/pmc_k/$tag/[a-e]
cat $O/pmc_kernels.txt | head -30
