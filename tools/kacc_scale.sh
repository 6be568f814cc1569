set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/kacc_scale; rm -rf $O; mkdir -p $O
for lg in 20 21 22 23 24; do
  timeout -k 10 300 python bench.py --no-cpu --logn $lg --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --batch-ntt 0 --pcdl "" --steps 8 --warmup 4 --msm-streams 1 > $O/l$lg.json 2> $O/l$lg.err || { tail -20 $O/l$lg.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/l$lg.json').read().strip().splitlines()[-1]); r = d['roofline']
print('2^$lg: ms/step %.3f  k_acc live %.3f  isolated %.3f  per 2^20 points: isolated %.3f' % (d['ms_per_step'], r['avg_launch_ms'], r['isolated_launch_ms'], r['isolated_launch_ms'] / 2 ** ($lg - 20)))"
done
