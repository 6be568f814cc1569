# k_merge lanes per bucket (HALO_MERGE_LANES): isolated kernel times (single-call 2^20 latency path)
# and the pipelined bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/merge_ab; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 120 --timeout-method thread > $O/msmtest.log 2>&1 || { tail -20 $O/msmtest.log; exit 1; }
tail -1 $O/msmtest.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for q in 1 2 4; do
  HALO_MERGE_LANES=$q timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$q -o run -- python3 tools/msm_latency.py 20 > $O/tr$q.log 2>&1 || { tail -5 $O/tr$q.log; exit 1; }
  python3 tools/kstats.py $(find $O/tr$q -name "*kernel_stats.csv" | head -1) > $O/kstats$q.txt
  echo "== lanes=$q"; grep -E "k_merge|k_acc|k_rowcol" $O/kstats$q.txt
  rm -rf $O/tr$q
done
bash tools/env_ab.sh 2 "HALO_MERGE_LANES=1" "HALO_MERGE_LANES=2" "HALO_MERGE_LANES=4"
