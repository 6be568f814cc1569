set -o pipefail
cd $GRAFT_REPO_ROOT
#timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r04_gt3.txt 2>&1 || { tail -30 gpurun_out/r04_gt3.txt; exit 1; }
#
for lib in ablib/r04_asm.so ablib/r04_tail3.so; do
  echo "== pcdl open $(basename $lib)"
  HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/pcdl_open_time.py 2 4 6 8 10 12 16 2>&1 | grep "^2^" | sed 's/begin+eval.*rounds=/rounds=/' || exit 1
  HALO_LIB=$PWD/$lib REPS=3 timeout -k 10 200 python tools/ipa_time.py 16 20 2>&1 | grep "^open" || exit 1
done
