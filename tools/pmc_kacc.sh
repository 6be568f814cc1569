# k_acc counter passes (gpurun, repo root) for one or more library builds:
#   bash tools/pmc_kacc.sh <tag>=<lib.so> ...
# Per build: pass a = SQ issue / wait counters, pass b = GRBM_GUI_ACTIVE, pass c = kernel trace
# (durations), all over the 2^20 MSM bench.  Output: gpurun_out/pmc_kacc/<tag>/ + summary.json.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_kacc; mkdir -p $O
for spec in "$@"; do
  tag=${spec%%=*}; lib=${spec#*=}
  D=$O/$tag; rm -rf $D; mkdir -p $D
  export HALO_LIB=$lib
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $D/a -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --steps 3 --warmup 1 ${BENCH_ARGS:-} > $D/a.log 2>&1 || { tail -5 $D/a.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $D/b -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --steps 3 --warmup 1 ${BENCH_ARGS:-} > $D/b.log 2>&1 || { tail -5 $D/b.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --steps 3 --warmup 1 ${BENCH_ARGS:-} > $D/c.log 2>&1 || { tail -5 $D/c.log; exit 1; }
done
unset HALO_LIB
python3 tools/pmc_kacc_summary.py $O "$@" > $O/summary.json; cat $O/summary.json
