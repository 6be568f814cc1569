# VALU counters of the 2^${1:-20} naive_prover's kernels (tools/prove_time.py: two proves) and its kernel
# statistics, run through gpurun from the repo root: one rocprofv3 --pmc pass (SQ_INSTS_VALU, _INT32,
# _INT64, SQ_WAVES), merged with the kernels' static instruction classes (tools/valu_mix.py) by
# tools/pmc_prove_merge.py into gpurun_out/pmc_prove/prove_valu.json -- the input of the prover kernels'
# compute rooflines (k_ntt_pass<1024>, the three gate kernels).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_prove; rm -rf $O; mkdir -p $O
lg=${1:-20}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 tools/prove_time.py $lg > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cp $(find $O/t -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && rm -rf $O/t
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES --output-format csv -d $O/v -o run -- python3 tools/prove_time.py $lg > $O/valu.log 2>&1 || { tail -20 $O/valu.log; exit 1; }
python3 tools/pmc_prove_merge.py $O/v $O/kernel_stats.csv $O/prove_valu.json || exit 1
rm -rf $O/v
