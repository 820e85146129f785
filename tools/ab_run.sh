# A/B of NTT kernel knobs on one box (parity first; every step time-limited)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2_parity.log 2>&1
SFHE_NTT_ROW_PF=0 SFHE_NTT_COL_UNROLL=0 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab2_mb_base.log 2>&1
SFHE_NTT_COL_UNROLL=0 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab2_mb_pf.log 2>&1
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab2_mb_both.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
SFHE_NTT_COL_UNROLL=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab2_pf.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab2_both.log 2>&1
SFHE_NTT_COL_UNROLL=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab2_pf2.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab2_both2.log 2>&1
