# Headline A/B over the values of one tuning key (gpurun, repo root), two interleaved runs each:
#   bash tools/tune_ab.sh <key> <value> [<value> ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tune_ab; rm -rf $O; mkdir -p $O
key=$1; shift
for i in 1 2; do
  for v in "$@"; do
    tag=${key}_${v}_$i
    timeout -k 10 200 python bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --steps 20 --tune $key=$v > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); e=d['extra']
print('$tag', 'ms/step %.3f'%d['ms_per_step'], 'acc %.3f'%d['roofline']['avg_launch_ms'], 'lat %.3f'%e['msm_single_latency_ms'], 'ntt %.3f'%e['ntt']['pair_ms'])"
  done
done
