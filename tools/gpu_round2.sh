# The new multi-rank (shm transport) test first, then the round-end check.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/round
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "shm_transport" \
  > gpurun_out/round/shm.log 2>&1; rc=$?; tail -8 gpurun_out/round/shm.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh
