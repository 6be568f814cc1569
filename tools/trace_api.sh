# kernel + HIP API trace of the pipelined headline bench (host enqueue vs GPU timeline)
cd $GRAFT_REPO_ROOT
O=gpurun_out/trace_api; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/tr -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cp $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv
cp $(find $O/tr -name "*hip_api_trace.csv" | head -1) $O/hip_api_trace.csv
rm -rf $O/tr
ls -la $O
