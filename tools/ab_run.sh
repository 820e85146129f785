# NTT write-through stores (SFHE_NTT_WT=1) A/B: parity with the knob on, microbench, bench x2 each
set -e
mkdir -p gpurun_out
SFHE_NTT_WT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab6_parity.log 2>&1
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab6_mb_base.log 2>&1
SFHE_NTT_WT=1 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab6_mb_wt.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
timeout -k 10 200 python bench.py $B > gpurun_out/ab6_base.log 2>&1
SFHE_NTT_WT=1 timeout -k 10 200 python bench.py $B > gpurun_out/ab6_wt.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab6_base2.log 2>&1
SFHE_NTT_WT=1 timeout -k 10 200 python bench.py $B > gpurun_out/ab6_wt2.log 2>&1
