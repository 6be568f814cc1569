# Re-stamps profiles/pmc_summary.json for the current library (FETCH_SIZE and WRITE_SIZE in separate
# passes, as tools/collect_profiles.sh), then checks that bench.py picks it up (roofline.traffic)
cd $GRAFT_REPO_ROOT
tag=${1:-r03d}
O=gpurun_out/stamp_$tag; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LEGS='--varbase 0 --commit-batch 0 --batch-ntt 0 --pcdl'
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 $LEGS "" --steps 3 --warmup 1 > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 $LEGS "" --steps 3 --warmup 1 > /dev/null 2>&1 || exit 1
python3 tools/make_pmc_summary.py $O/pmc_f $O/pmc_w $O/pmc_summary.json "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of 'python3 bench.py --no-cpu --sizes \"\" --ipa 0 --prove 0 $LEGS \"\" --steps 3 --warmup 1', ${tag}" > /dev/null || exit 1
rm -rf $O/pmc_f/*/ $O/pmc_w/*/ 2>/dev/null
cp $O/pmc_summary.json profiles/pmc_summary.json
timeout -k 10 300 python bench.py --no-cpu --sizes "" --ipa 0 --prove 0 $LEGS "" > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['traffic'], d['roofline']['traffic_note'])"
