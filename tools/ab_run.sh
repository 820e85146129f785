# conversion LDS: smod aliased with the FP64 multipliers (always) + NS=13 kernels (SFHE_CONV_NS13=0: NS=16)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab8_parity.log 2>&1
SFHE_CONV_NS13=0 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab8_mb_16.log 2>&1
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab8_mb_13.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
SFHE_CONV_NS13=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab8_16.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab8_13.log 2>&1
SFHE_CONV_NS13=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab8_16b.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab8_13b.log 2>&1
