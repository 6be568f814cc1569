mkdir -p gpurun_out/ipa_ab
for m in 1024 4096 16384 65536 262144 1024 16384 65536; do
  HALO_IPA_MAT_N=$m timeout -k 10 120 python3 tools/ipa_time.py 20 > gpurun_out/ipa_ab/m$m.log 2>&1 || exit 1
  echo "MAT_N=$m $(grep 'open 2^20' gpurun_out/ipa_ab/m$m.log | tail -1)" >> gpurun_out/ipa_ab/sum.txt
done
