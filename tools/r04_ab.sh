# Round-4 A/B (gpurun, repo root): GPU suite on the in-tree library, then the headline bench and the
# small pcdl::open sweep alternated over library builds given as arguments (HALO_LIB).
#   bash tools/r04_ab.sh <lib> [<lib> ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ab; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/ > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -1 $O/gputest.txt
for i in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)_$i
    HALO_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --pcdl "" --steps 20 > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $lib"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); e=d['extra']
print('$tag', 'ms/step %.3f'%d['ms_per_step'], 'acc %.3f'%d['roofline']['avg_launch_ms'], 'lat %.3f'%e['msm_single_latency_ms'], 'ntt %.3f'%e['ntt']['pair_ms'])"
  done
done
for lib in "$@"; do
  echo "== pcdl open $(basename $lib)"
  HALO_LIB=$PWD/$lib timeout -k 10 200 python tools/pcdl_open_time.py 2 4 6 8 10 12 16 2>&1 | grep "^2^" | sed 's/begin+eval.*rounds=/rounds=/' || exit 1
done
echo "== ipa_mat_n sweep (in-tree library)"
MAT_N=2048,8192,32768,131072 REPS=2 timeout -k 10 300 python tools/ipa_time.py 20 2>&1 | grep "^open" || exit 1
