# NTT pair timing across pass splits (tuning A/B): default, 8-bit passes for 2^22, even radices
set -o pipefail
mkdir -p gpurun_out/sweep
timeout -k 10 120 python tools/ntt_time.py 20 21 22 23 24 > gpurun_out/sweep/default.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ntt_time.py 21 22 ntt_big_max_log=20 > gpurun_out/sweep/big20.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ntt_time.py 21 22 23 24 ntt_big_max_log=20 ntt_even_split=1 > gpurun_out/sweep/even.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ntt_time.py 20 22 ntt_big_max_log=16 ntt_even_split=1 > gpurun_out/sweep/even8.txt 2>&1 || exit 1
grep -h logn gpurun_out/sweep/*.txt
