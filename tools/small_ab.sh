# Small SRS MSM path A/B (gpurun, repo root): full GPU test suite, then single-call latency at small n
# with the multiples-table path (default) and through the bucket pipeline (HALO_SRS_SMALL=0).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/small
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/small/tests.log 2>&1 || { tail -40 gpurun_out/small/tests.log; exit 1; }
tail -2 gpurun_out/small/tests.log
for i in 1 2; do
  echo "== table path"; timeout -k 10 120 python tools/msm_latency.py 2 4 6 8 10 12 || exit 1
  echo "== bucket path"; HALO_SRS_SMALL=0 timeout -k 10 120 python tools/msm_latency.py 2 4 6 8 10 12 || exit 1
done
