# Quick A/B (gpurun, repo root): the MSM / NTT GPU tests on the in-tree library, then the headline
# bench alternated over library builds (HALO_LIB), two runs each.   bash tools/ab_quick.sh <lib> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abq; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_northstar.py > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -1 $O/gputest.txt
for i in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)_$i
    HALO_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --steps 20 > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $lib"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); e=d['extra']
print('$tag', 'ms/step %.3f'%d['ms_per_step'], 'acc %.3f'%d['roofline']['avg_launch_ms'], 'lat %.3f'%e['msm_single_latency_ms'], 'ntt %.3f'%e['ntt']['pair_ms'])"
  done
done
