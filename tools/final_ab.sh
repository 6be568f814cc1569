# quad Horner / quad GLV scalar multiplication: parity, then single-call latencies, A = HALO_LIB
cd $GRAFT_REPO_ROOT
O=gpurun_out/final_ab; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_field_curve.py tests/test_gpu_prover.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -1 $O/test.log
A=$PWD/$1
for r in 1 2; do
  echo "-- A"; HALO_LIB=$A timeout -k 10 120 python tools/varbase_time.py 10 16 20 2>&1 | grep varbase
  HALO_LIB=$A timeout -k 10 120 python tools/curve_op_time.py 2>&1 | grep curve_op
  echo "-- B"; timeout -k 10 120 python tools/varbase_time.py 10 16 20 2>&1 | grep varbase
  timeout -k 10 120 python tools/curve_op_time.py 2>&1 | grep curve_op
done
