# IPA / transcript / prover parity on the current library, then the 2^20 opening and prover times
# (A = HALO_LIB library for the timing comparison)
cd $GRAFT_REPO_ROOT
O=gpurun_out/ipa_check; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_ipa_eval.py tests/test_gpu_transcript.py tests/test_gpu_prover.py tests/test_gpu_field_curve.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -1 $O/test.log
A=$PWD/$1
for r in 1 2; do
  echo "-- A"; HALO_LIB=$A timeout -k 10 300 python tools/prove_time.py 20 2>&1 | tail -2
  echo "-- B"; timeout -k 10 300 python tools/prove_time.py 20 2>&1 | tail -2
done
