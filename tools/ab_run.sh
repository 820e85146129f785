# NTT COL rounds forming W/q from W (default) vs staging the W/q table (SFHE_NTT_COL_WQ=0)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_ntt_variants.py -x -q --timeout 150 --timeout-method thread > gpurun_out/ab15_parity.log 2>&1
SFHE_NTT_COL_WQ=0 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab15_mb_tab.log 2>&1
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab15_mb_calc.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
SFHE_NTT_COL_WQ=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab15_tab.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab15_calc.log 2>&1
SFHE_NTT_COL_WQ=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab15_tab2.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab15_calc2.log 2>&1
