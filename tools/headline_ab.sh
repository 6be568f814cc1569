# Interleaved A/B of the headline MSM step over the shifted copies' window width (bench.py --shift-c),
# headline only: bash tools/headline_ab.sh "0 18 19" [rounds]   (through gpurun, from the repo root)
O=gpurun_out/hab; rm -rf $O; mkdir -p $O
for r in $(seq 1 ${2:-2}); do
  for c in $1; do
    timeout -k 10 240 python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" \
      --steps 40 --warmup 5 --shift-c $c > $O/c${c}_$r.json 2> $O/c${c}_$r.err || { tail -5 $O/c${c}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c', sys.argv[2], 'round', sys.argv[3], 'ms/step', round(d['ms_per_step'], 4))" $O/c${c}_$r.json $c $r
  done
done
