# A/B of the number of streams the pipelined MSMs alternate over (bench.py --msm-streams), at the
# headline 2^20 and in the 2^24 sizes leg (gpurun, repo root): bash tools/ab_streams.sh "1 2"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_streams; rm -rf $O; mkdir -p $O
for i in 1 2; do
  for m in ${1:-1 2}; do
    timeout -k 10 300 python bench.py --no-cpu --sizes 24 --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --batch-ntt 0 --pcdl "" --steps 20 --msm-streams $m > $O/s${m}_$i.json 2> $O/s${m}_$i.err || { tail -20 $O/s${m}_$i.err; exit 1; }
    python3 -c "
import json; d = json.loads(open('$O/s${m}_$i.json').read().strip().splitlines()[-1]); s = d['extra']['sizes']['msm_2^24']
print('streams $m run $i: 2^20 ms/step %.4f  k_acc %.3f | 2^24 ms/msm %.2f  k_acc %.2f  single %.2f' % (d['ms_per_step'], d['roofline']['avg_launch_ms'], s['ms_per_msm'], s['k_acc_ms'], s['single_latency_ms']))"
  done
done
