# IPA opening A/B (gpurun, repo root): tools/ipa_time.py at the given sizes, alternated over library
# builds (HALO_LIB), two runs each.   SIZES="16 20" bash tools/ipa_ab.sh <lib> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for lib in "$@"; do
    echo "== $(basename $lib) $i"
    HALO_LIB=$PWD/$lib REPS=2 timeout -k 10 300 python tools/ipa_time.py ${SIZES:-16 20} 2>&1 | grep "^open" || exit 1
  done
done
