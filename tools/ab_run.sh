# k_ks_inner unrolled over the digits (SFHE_KS_UNROLL=0: runtime loop) A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab9_parity.log 2>&1
SFHE_KS_UNROLL=0 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab9_mb_0.log 2>&1
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab9_mb_1.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
SFHE_KS_UNROLL=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab9_0.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab9_1.log 2>&1
SFHE_KS_UNROLL=0 timeout -k 10 200 python bench.py $B > gpurun_out/ab9_0b.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab9_1b.log 2>&1
