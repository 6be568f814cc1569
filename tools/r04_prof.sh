# GPU suite, small pcdl::open A/B of two libraries, then per-kernel SQ counters and the pipelined
# kernel timeline of the in-tree library (gpurun, repo root).   bash tools/r04_prof.sh <libA> <libB> <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$3; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/ > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -1 $O/gputest.txt
for lib in $1 $2; do
  echo "== pcdl open $(basename $lib)"
  HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/pcdl_open_time.py 2 4 6 8 10 12 16 2>&1 | grep "^2^" | sed 's/begin+eval.*rounds=/rounds=/' || exit 1
done
bash tools/pmc_kernels.sh $3 > /dev/null && cp gpurun_out/pmc_k/$3/summary.txt $O/pmc_kernels.txt && rm -rf gpurun_out/pmc_k/$3/[a-e]
head -20 $O/pmc_kernels.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv && rm -rf $O/tr
python3 tools/timeline.py $O/kernel_trace.csv 5 > $O/timeline.txt
tail -8 $O/timeline.txt
