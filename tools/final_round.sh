# End-of-session evidence on the current library: full GPU suite, prover A/B against HALO_LIB=$1,
# then tools/collect_profiles.sh <tag>
cd $GRAFT_REPO_ROOT
tag=${2:-r03c}
O=gpurun_out/final_$tag; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
if [ -n "$1" ]; then
  A=$PWD/$1
  echo "-- A"; HALO_LIB=$A timeout -k 10 300 python tools/prove_time.py 20 2>&1 | tail -1
  echo "-- B"; timeout -k 10 300 python tools/prove_time.py 20 2>&1 | tail -1
  timeout -k 10 200 python tools/ipa_time.py 2>&1 | tail -2
fi
bash tools/collect_profiles.sh $tag
