# Collects the round's evidence on the GPU box (run through gpurun from the repo root); outputs go to
# gpurun_out/evid_<tag>/ (merged back by gpurun), then copied into profiles/ locally:
#   bench.json           default bench.py line (with the CPU baseline)
#   kernel_stats.csv     rocprofv3 --kernel-trace --stats of the 2^20 MSM + 2^22 NTT bench
#   kstats.txt           its per-kernel table (tools/kstats.py)
#   bench_traced.json    the bench line of that traced run; trace_exit.txt its exit status
#   pmc_summary.json     FETCH_SIZE / WRITE_SIZE per dispatch (separate --pmc passes) and the VALU
#                        counts of k_acc / k_ntt_pass (tools/pmc_valu.sh), stamped with the library's
#                        sha256 (bench.py uses them -- roofline.traffic, compute_roofline -- only if it
#                        matches)
#   pmc_kernels.txt      per-kernel SQ / LDS / HBM counters of the MSM kernels (tools/pmc_kernels.sh)
#   prove_kstats.txt     kernel statistics of the 2^20 naive_prover pipeline (tools/prof_prove.sh)
#   prove_valu.json      the prover kernels' VALU counts and compute fractions (tools/pmc_prove.sh)
#   pmc_ntt22.txt / pmc_ntt24.txt   SQ stall counters of the NTT pass kernels (tools/pmc_ntt.sh)
#   bench_stamped.json   the default bench line again, with pmc_summary.json / prove_valu.json of this
#                        build in place (roofline.traffic and every compute roofline filled)
set -o pipefail
tag=${1:-r02}
cd $GRAFT_REPO_ROOT
O=gpurun_out/evid_${tag}
rm -rf $O && mkdir -p $O
LEGS='--varbase 0 --commit-batch 0 --batch-ntt 0 --pcdl'
timeout -k 10 500 python bench.py > $O/bench_full.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -n 1 $O/bench_full.json > $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 $LEGS "" > $O/trace.log 2>&1
rc=$?; echo "rocprofv3 --kernel-trace exit status: $rc" > $O/trace_exit.txt
grep -n -i "segmentation\|core dumped\|abort" $O/trace.log >> $O/trace_exit.txt || true
[ $rc -eq 0 ] || { tail -20 $O/trace.log; exit 1; }
cp $(find $O/trace -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
grep '^{' $O/trace.log | tail -n 1 > $O/bench_traced.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 $LEGS "" --steps 3 --warmup 1 > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 bench.py --no-cpu --sizes "" --ipa 0 --prove 0 $LEGS "" --steps 3 --warmup 1 > /dev/null 2>&1 || exit 1
python3 tools/make_pmc_summary.py $O/pmc_f $O/pmc_w $O/pmc_summary.json "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of 'python3 bench.py --no-cpu --sizes \"\" --ipa 0 --prove 0 $LEGS \"\" --steps 3 --warmup 1', ${tag}" > /dev/null
rm -rf $O/trace $O/pmc_f/*/ $O/pmc_w/*/ 2>/dev/null
bash tools/pmc_valu.sh $O/pmc_summary.json > $O/pmc_valu.log 2>&1 || { tail -5 $O/pmc_valu.log; exit 1; }
python3 tools/kstats.py $O/kernel_stats.csv > $O/kstats.txt
bash tools/pmc_kernels.sh $tag > /dev/null && cp gpurun_out/pmc_k/$tag/summary.txt $O/pmc_kernels.txt
rm -rf gpurun_out/pmc_k/$tag/[a-e]
bash tools/prof_prove.sh 20 > /dev/null && cp gpurun_out/prof_prove/kstats.txt $O/prove_kstats.txt
bash tools/pmc_prove.sh 20 > $O/pmc_prove.log 2>&1 && cp gpurun_out/pmc_prove/prove_valu.json $O/ || { tail -5 $O/pmc_prove.log; exit 1; }
bash tools/pmc_ntt.sh 22 > $O/pmc_ntt22.txt 2>&1 && bash tools/pmc_ntt.sh 24 > $O/pmc_ntt24.txt 2>&1 || exit 1
cp $O/pmc_summary.json profiles/pmc_summary.json && cp $O/prove_valu.json profiles/prove_valu.json
timeout -k 10 500 python bench.py > $O/bench_stamped_full.json 2> $O/bench_stamped.err || { tail -20 $O/bench_stamped.err; exit 1; }
tail -n 1 $O/bench_stamped_full.json > $O/bench_stamped.json
head -n 30 $O/kstats.txt
