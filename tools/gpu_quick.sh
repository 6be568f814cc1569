set -o pipefail
mkdir -p gpurun_out/r1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_ipa_eval.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r1/test.log 2>&1; rc=$?
tail -5 gpurun_out/r1/test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ntt_time.py 20 22 23 24 > gpurun_out/r1/ntt.txt 2>&1 && cat gpurun_out/r1/ntt.txt && bash tools/pmc_ntt.sh > gpurun_out/r1/pmc_ntt.txt 2>&1; cat gpurun_out/r1/pmc_ntt.txt | head -12
