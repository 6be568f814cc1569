# Two ranks on one GPU over gloo (protocol rehearsal of bench.py --gpus 2, not a scaling number),
# through gpurun from the repo root.  Output: gpurun_out/rehearse/out.txt
set -o pipefail
O=gpurun_out/rehearse; rm -rf $O; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --same-device --steps 5 --warmup 2 ${EXTRA:---prove 0 --ipa 1 --no-cpu} > $O/out.txt 2> $O/err.txt; rc=$?
tail -3 $O/err.txt; grep '^{' $O/out.txt | cut -c1-300
exit $rc
