# Stream-priority A/B at 2^24 (the prio build, tuning msm_front_prio: 0 none, 3 the sort on a
# greatest-priority stream, 4 also the tails on a least-priority stream), gpurun from the repo root.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_prio24; rm -rf $O; mkdir -p $O
for i in 1 2; do
  for m in 0 3 4; do
    HALO_LIB=$PWD/ablib/prio.so timeout -k 10 300 python bench.py --no-cpu --sizes 24 --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --batch-ntt 0 --pcdl "" --steps 20 --tune msm_front_prio=$m > $O/m${m}_$i.json 2> $O/m${m}_$i.err || { tail -20 $O/m${m}_$i.err; exit 1; }
    python3 -c "
import json; d = json.loads(open('$O/m${m}_$i.json').read().strip().splitlines()[-1]); s = d['extra']['sizes']['msm_2^24']
print('mode $m run $i: 2^20 ms/step %.4f | 2^24 ms/msm %.2f  k_acc %.2f  single %.2f' % (d['ms_per_step'], s['ms_per_msm'], s['k_acc_ms'], s['single_latency_ms']))"
  done
done
