# IPA / prover A/B of two library builds (gpurun, repo root): the IPA, prover and transcript GPU tests on the
# current library, then tools/ipa_time.py 16 20 and tools/prove_time.py 16 alternating ablib/libhalo_old.so
# (the baseline build) and halo_amd/lib/libhalo_gpu.so.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ipa_ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipa_eval.py tests/test_gpu_prover.py tests/test_gpu_transcript.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ipa_ab/tests.log 2>&1 || { tail -30 gpurun_out/ipa_ab/tests.log; exit 1; }
tail -2 gpurun_out/ipa_ab/tests.log
for i in 1 2; do for lib in ablib/libhalo_old.so halo_amd/lib/libhalo_gpu.so; do
  echo "== $lib ipa"; HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/ipa_time.py 16 20 2>&1 | tail -4 || exit 1
  echo "== $lib prove"; HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/prove_time.py 16 2>&1 | tail -3 || exit 1
done; done
