# GPU suite for the IPA / pcdl paths (signed tail windows, XYZZ blind / combine) + pcdl open, IPA and
# prover timings.  bash tools/gpu_tail_check.sh (through gpurun, from the repo root)
set -o pipefail
O=gpurun_out/tail; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipa_eval.py tests/test_gpu_transcript.py tests/test_gpu_prover.py tests/test_gpu_northstar.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
tail -3 $O/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/pcdl_open_time.py 2 6 10 12 16 > $O/pcdl.txt 2>&1 || { tail -5 $O/pcdl.txt; exit 1; }
tail -12 $O/pcdl.txt
REPS=3 timeout -k 10 200 python tools/ipa_time.py 16 20 2>&1 | grep "^open"
timeout -k 10 300 python tools/prove_time.py 16 > $O/prove.txt 2>&1 || { tail -5 $O/prove.txt; exit 1; }
cat $O/prove.txt
