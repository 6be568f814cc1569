# A/B of two library builds on one GPU box (run through gpurun from the repo root):
#   bash tools/ab_lib.sh <lib A> <lib B> [rounds]
# alternates the headline bench (--no-cpu, MSM + NTT legs only) between the two libraries via
# HALO_LIB and prints ms/step, k_acc and single-call latency per run; then a kernel trace of the
# single-call 2^20 latency path for each library (serialised MSMs: isolated kernel durations).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablib
A=$1; B=$2; R=${3:-3}
for i in $(seq 1 $R); do
  for lib in $A $B; do
    tag=$(basename $lib .so)_$i
    HALO_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --steps 20 > gpurun_out/ablib/$tag.json 2> gpurun_out/ablib/$tag.err || { echo "FAIL $lib"; tail -5 gpurun_out/ablib/$tag.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ablib/$tag.json').read().strip().splitlines()[-1]); e=d['extra']
print('$tag', 'ms/step %.3f'%d['ms_per_step'], 'acc %.3f'%d['roofline']['avg_launch_ms'], 'lat %.3f'%e['msm_single_latency_ms'], 'sync_ok', e['pipelined_equals_sync'], 'ntt %.3f'%e['ntt']['pair_ms'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for lib in $A $B; do
  tag=$(basename $lib .so)
  rm -rf gpurun_out/ablib/tr_$tag
  HALO_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ablib/tr_$tag -o run -- python3 tools/msm_latency.py 20 > gpurun_out/ablib/tr_$tag.log 2>&1 || { echo "trace FAIL $lib"; tail -5 gpurun_out/ablib/tr_$tag.log; exit 1; }
  f=$(find gpurun_out/ablib/tr_$tag -name "*kernel_stats.csv" | head -1)
  python3 tools/kstats.py $f > gpurun_out/ablib/kstats_$tag.txt
  echo "== $tag"; grep -E "k_rs_|k_acc|k_merge" gpurun_out/ablib/kstats_$tag.txt
  rm -rf gpurun_out/ablib/tr_$tag
done
