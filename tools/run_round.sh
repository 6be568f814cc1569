# GPU test suite + default bench (no CPU leg) + kernel timeline of the pipelined headline bench.
#   bash tools/run_round.sh <tag>       (through gpurun, from the repo root)
set -o pipefail
tag=${1:-r03b}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$tag
rm -rf $O && mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 400 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -n 1 $O/bench.json | cut -c 1-600
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv && rm -rf $O/tr
python3 tools/timeline.py $O/kernel_trace.csv 5 > $O/timeline.txt
tail -8 $O/timeline.txt
