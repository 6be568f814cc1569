# VALU issue evidence for the dominant kernels (k_acc, k_ntt_pass): SQ instruction counters and
# GRBM_GUI_ACTIVE in separate --pmc passes over the 2^20 MSM + 2^22 NTT bench (gpurun, repo root).
# Output: gpurun_out/pmc_valu/valu_summary.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_valu; rm -rf $O; mkdir -p $O
CMD="python3 bench.py --no-cpu --sizes '' --ipa 0 --prove 0 --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/a -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --steps 3 --warmup 1 > $O/a.log 2>&1 || { tail -5 $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/b -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --steps 3 --warmup 1 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
python3 tools/valu_summary.py $O "$CMD" > $O/valu_summary.json
rm -rf $O/a $O/b
cat $O/valu_summary.json
