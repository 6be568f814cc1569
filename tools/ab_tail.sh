# A/B of two library builds on the latency-bound paths (run through gpurun from the repo root):
#   bash tools/ab_tail.sh <lib A> <lib B>
# single-call MSM latency, IPA openings and hiding pcdl opens, then the pipelined headline step.
cd $GRAFT_REPO_ROOT
export GPU_MAX_HW_QUEUES=8
for r in 1 2; do
for lib in $1 $2; do
  echo "== $lib (round $r)"
  HALO_LIB=$PWD/$lib timeout -k 10 120 python3 tools/msm_latency.py 2 10 14 16 18 20 || exit 1
  HALO_LIB=$PWD/$lib timeout -k 10 120 python3 tools/pcdl_open_time.py 2 10 16 || exit 1
  HALO_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu --sizes "" --ipa 1 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --steps 20 > gpurun_out/ab_$r.json || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$r.json').read().strip().splitlines()[-1]); e=d['extra']
print('ms/step %.3f'%d['ms_per_step'], 'acc %.3f'%d['roofline']['avg_launch_ms'], 'lat %.3f'%e['msm_single_latency_ms'], 'ntt %.3f'%e['ntt']['pair_ms'], 'ipa2^20 %.2f'%e['ipa_open']['open_ms'])"
done
done
