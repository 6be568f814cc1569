# NTT pair A/B (gpurun, repo root): tools/ntt_time.py alternated over library builds (HALO_LIB).
#   SIZES="22 23 24" bash tools/ntt_ab.sh <lib> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for lib in "$@"; do
    echo "== $(basename $lib) $i"
    HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/ntt_time.py ${SIZES:-22 23 24} 2>&1 | tail -${NL:-3} || exit 1
  done
done
