# Env-variable A/B of the pipelined 2^20 MSM bench (gpurun, repo root):
#   bash tools/env_ab.sh <rounds> "<ENV=.. ENV=..>" "<...>" ...
# Each configuration runs <rounds> times, interleaved; gpurun_out/env_ab/sum.txt lists ms/step.
O=gpurun_out/env_ab; rm -rf $O; mkdir -p $O
R=$1; shift
for r in $(seq $R); do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python bench.py --no-cpu --prove 0 --pcdl "" --varbase 0 --commit-batch 0 --ipa 0 --sizes "" --steps 40 ${BENCH_ARGS:-} > $O/c${i}_$r.log 2>&1 || { tail -5 $O/c${i}_$r.log; exit 1; }
    echo "[$cfg] $(grep -o '"ms_per_step": [0-9.]*' $O/c${i}_$r.log)" >> $O/sum.txt
  done
done
cat $O/sum.txt
