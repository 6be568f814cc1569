# GPU suite (MSM / IPA / transcript / prover: the sort changed) + IPA A/B of the paired L/R MSM at 2^19
set -o pipefail
mkdir -p gpurun_out/ipa_ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ipa_ab/gputest.log 2>&1; rc=$?
tail -3 gpurun_out/ipa_ab/gputest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  REPS=3 timeout -k 10 120 python tools/ipa_time.py 16 20 2>&1 | grep "^open" | sed "s/^/default $i /"
  TUNE=ipa_pair_max=524288 REPS=3 timeout -k 10 120 python tools/ipa_time.py 20 2>&1 | grep "^open" | sed "s/^/pair19 $i /"
done
timeout -k 10 120 python tools/pcdl_open_time.py 2 10 16 2>&1 | tail -8
