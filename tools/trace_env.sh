# kernel timeline of the pipelined headline bench under env settings: bash tools/trace_env.sh <tag> [ENV=..]...
tag=$1; shift
cd $GRAFT_REPO_ROOT
O=gpurun_out/trace_$tag; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv && rm -rf $O/tr
python3 tools/timeline.py $O/kernel_trace.csv 5 > $O/timeline.txt
tail -7 $O/timeline.txt
