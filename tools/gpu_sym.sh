set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sym; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "sym or walk or wave_kernel or shard or synthetic" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
