set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1_parity.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
SFHE_NTT_ROW_PF=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab1_off.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab1_on.log 2>&1
SFHE_NTT_ROW_PF=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab1_off2.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab1_on2.log 2>&1
