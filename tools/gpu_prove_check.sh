# Prover / IPA GPU tests and prover timings at 2^16 and 2^20 (through gpurun, from the repo root)
set -o pipefail
O=gpurun_out/pc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_prover.py tests/test_gpu_ipa_eval.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
tail -3 $O/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/prove_time.py 16 20 > $O/prove.txt 2>&1 || { tail -5 $O/prove.txt; exit 1; }
cat $O/prove.txt
