# pcdl::open sweep A/B (gpurun, repo root): tools/pcdl_open_time.py alternated over library builds.
#   SIZES="2 4 6 8 10" bash tools/pcdl_ab.sh <lib> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for lib in "$@"; do
    echo "== $(basename $lib) $i"
    HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/pcdl_open_time.py ${SIZES:-2 4 6 8 10 12} 2>&1 | grep "^2^" | sed 's/begin+eval.*rounds=/rounds=/' || exit 1
  done
done
