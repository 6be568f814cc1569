# Pipelined kernel timeline (tools/timeline.py) of the headline bench for each value of one tuning key
# (gpurun, repo root):   bash tools/tune_timeline.sh <key> <value> [<value> ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tune_tl; rm -rf $O; mkdir -p $O
key=$1; shift
for v in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --tune $key=$v > $O/trace_$v.log 2>&1 || { tail -20 $O/trace_$v.log; exit 1; }
  cp $(find $O/tr_$v -name "*kernel_trace.csv" | head -1) $O/kernel_trace_$v.csv && rm -rf $O/tr_$v
  python3 tools/timeline.py $O/kernel_trace_$v.csv 5 > $O/timeline_$v.txt
  echo "== $key=$v"; tail -8 $O/timeline_$v.txt
done
