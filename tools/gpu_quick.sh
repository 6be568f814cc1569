# Quick GPU check of the NTT / IPA changes: their tests, NTT timing (default split and 8-bit passes),
# and the NTT pass counters.  bash tools/gpu_quick.sh (through gpurun, from the repo root)
set -o pipefail
mkdir -p gpurun_out/r1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_ipa_eval.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r1/test.log 2>&1; rc=$?
tail -5 gpurun_out/r1/test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ntt_time.py 20 22 23 24 > gpurun_out/r1/ntt.txt 2>&1 && cat gpurun_out/r1/ntt.txt || exit 1
timeout -k 10 200 python tools/ntt_time.py 20 22 ntt_big_max_log=16 > gpurun_out/r1/ntt8.txt 2>&1 && cat gpurun_out/r1/ntt8.txt || exit 1
bash tools/pmc_ntt.sh > gpurun_out/r1/pmc_ntt.txt 2>&1; cat gpurun_out/r1/pmc_ntt.txt | head -12
