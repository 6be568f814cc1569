# VALU instruction counts of the roofline kernels (k_acc in the headline bench, k_ntt_pass<2048> in the
# 2^22 NTT pair, k_ntt_pass<1024> in the 2^24 pair), one rocprofv3 --pmc pass each (4 SQ counters), merged into profiles/pmc_summary.json under
# "<key>.valu" together with the kernel's static instruction-class split (tools/valu_mix.py) -- the
# inputs of bench.py's compute roofline.  Run through gpurun from the repo root, after pmc_stamp.sh
# (which rewrites pmc_summary.json for the current library); argument: the summary to merge into
# (default profiles/pmc_summary.json).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_valu; rm -rf $O; mkdir -p $O
C="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/acc -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 --varbase 0 --commit-batch 0 --batch-ntt 0 --pcdl "" --steps 3 --warmup 1 > $O/acc.log 2>&1 || { tail -5 $O/acc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/ntt -o run -- python3 tools/ntt_time.py 22 > $O/ntt.log 2>&1 || { tail -5 $O/ntt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/ntt24 -o run -- python3 tools/ntt_time.py 24 > $O/ntt24.log 2>&1 || { tail -5 $O/ntt24.log; exit 1; }
S=${1:-profiles/pmc_summary.json}
python3 tools/pmc_valu_merge.py $O/acc $O/ntt $S $O/ntt24 || exit 1
rm -rf $O/acc/*/ $O/ntt/*/ $O/ntt24/*/ 2>/dev/null
cp $S $O/
