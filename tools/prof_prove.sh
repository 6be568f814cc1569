# rocprofv3 kernel statistics of the naive_prover pipeline at 2^${1:-20} (tools/prove_time.py),
# run through gpurun from the repo root.  Output: gpurun_out/prof_prove/kstats.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/prof_prove
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 tools/prove_time.py ${1:-20} > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
cp $(find $O/t -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
python3 tools/kstats.py $O/kernel_stats.csv > $O/kstats.txt
rm -rf $O/t
head -40 $O/kstats.txt
