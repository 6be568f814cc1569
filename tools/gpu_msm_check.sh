set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_msm.py -x -q > gpurun_out/msm_test.log 2>&1 || { tail -30 gpurun_out/msm_test.log; exit 1; }
tail -2 gpurun_out/msm_test.log
timeout -k 10 300 python bench.py > gpurun_out/bench_cur.json 2> gpurun_out/bench_cur.err || { tail -20 gpurun_out/bench_cur.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_cur.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['roofline']['avg_launch_ms'],d['extra']['msm_single_latency_ms'],d['extra']['pipelined_equals_sync'],d['cpu_baseline']['gpu_matches_cpu'], d['extra']['ntt']['pair_ms'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_cur
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cur -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --sizes "" --ipa 0 > /dev/null 2>&1
python3 tools/kstats.py $(find gpurun_out/prof_cur -name "*kernel_stats.csv" | head -1) | head -24
