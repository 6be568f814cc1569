# Per-kernel counter passes over the 2^20 MSM bench (gpurun, repo root), for the front's kernels
# by default:  bash tools/pmc_kernels.sh <tag> [bench args...]
# Under --pmc every dispatch is serialised, so the kernel-trace durations of pass a are isolated
# (no concurrent tail).  Summary: tools/pmc_kernels_summary.py -> gpurun_out/pmc_k/<tag>/summary.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
D=gpurun_out/pmc_k/$tag; rm -rf $D; mkdir -p $D
run() {  # run <pass> <rocprofv3 args...>
  local p=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" --output-format csv -d $D/$p -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --batch-ntt 0 --pcdl "" --steps 3 --warmup 1 "${BARGS[@]}" > $D/$p.log 2>&1 || { tail -5 $D/$p.log; return 1; }
}
BARGS=("$@")
run a --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU &&
run b --pmc GRBM_GUI_ACTIVE GRBM_COUNT &&
run c --pmc FETCH_SIZE &&
run d --pmc WRITE_SIZE &&
run e --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES &&
python3 tools/pmc_kernels_summary.py $D > $D/summary.txt && cat $D/summary.txt
