cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/kmerge; rm -rf $O; mkdir -p $O
for k in 0 4 32 64; do
  if [ $k = 0 ]; then unset HALO_ACC_K; else export HALO_ACC_K=$k; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$k -o run -- python3 tools/msm_latency.py 15 > $O/k$k.log 2>&1 || exit 1
  f=$(find $O/t$k -name "*kernel_stats.csv" | head -1)
  echo "== K=$k $(grep '2^15' $O/k$k.log)" >> $O/sum.txt
  python3 tools/kstats.py $f | grep -E "k_merge|k_acc|k_rowcol|k_bitterms|k_bitcombine|k_final|k_group" >> $O/sum.txt
  rm -rf $O/t$k
done
