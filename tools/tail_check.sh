# MSM/IPA parity under the current library, then isolated tail-kernel times (single-call 2^20 MSM),
# single-call latencies and the 2^20 opening time
cd $GRAFT_REPO_ROOT
O=gpurun_out/tail_check; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ipa_eval.py tests/test_gpu_transcript.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -1 $O/test.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/msm_latency.py 20 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 tools/kstats.py $(find $O/tr -name "*kernel_stats.csv" | head -1) > $O/kstats.txt
rm -rf $O/tr
grep -E "k_merge|k_acc|k_rowcol|k_bitterms|k_bitcombine" $O/kstats.txt
timeout -k 10 200 python tools/msm_latency.py 2 10 14 16 18 20 2>&1 | tail -8
timeout -k 10 300 python tools/ipa_time.py 2>&1 | tail -6
