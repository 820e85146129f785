# A/B of the PS helper lanes under graph replay (parity first; every step time-limited)
set -e
mkdir -p gpurun_out
SFHE_PS_LANES=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab3_parity.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
timeout -k 10 200 python bench.py $B > gpurun_out/ab3_l0.log 2>&1
SFHE_PS_LANES=1 timeout -k 10 200 python bench.py $B > gpurun_out/ab3_l1.log 2>&1
SFHE_PS_LANES=2 timeout -k 10 200 python bench.py $B > gpurun_out/ab3_l2.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab3_l0b.log 2>&1
SFHE_PS_LANES=2 timeout -k 10 200 python bench.py $B > gpurun_out/ab3_l2b.log 2>&1
