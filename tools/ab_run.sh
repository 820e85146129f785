# exact-NS conversion kernels A/B (SFHE_CONV_EXACT=0 keeps the guarded NS=16 ones)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab7_parity.log 2>&1
SFHE_CONV_EXACT=0 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab7_mb_base.log 2>&1
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab7_mb_exact.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
SFHE_CONV_EXACT=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab7_base.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab7_exact.log 2>&1
SFHE_CONV_EXACT=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab7_base2.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab7_exact2.log 2>&1
