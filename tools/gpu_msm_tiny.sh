# MSM tests (the tiny GLV-window path for <= 32 caller points) + prover timing at 2^16 (through gpurun)
set -o pipefail
O=gpurun_out/tiny; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_prover.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
tail -3 $O/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/prove_time.py 16 > $O/prove.txt 2>&1 || { tail -5 $O/prove.txt; exit 1; }
cat $O/prove.txt
