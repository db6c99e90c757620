mkdir -p gpurun_out/sym1
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "sym or wave_kernel or prefix" > gpurun_out/sym1/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --workload cfg4 --steps 1 --warmup 0 --no-secondary > gpurun_out/sym1/cfg4.json 2> gpurun_out/sym1/cfg4.err
