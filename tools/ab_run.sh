# register-round width of the >64-row NTT launches (SFHE_NTT_LE; default 2)
set -e
mkdir -p gpurun_out
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
SFHE_NTT_LE=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab12_parity3.log 2>&1
SFHE_NTT_LE=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab12_parity4.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab12_le2.log 2>&1
SFHE_NTT_LE=3 timeout -k 10 200 python bench.py $B > gpurun_out/ab12_le3.log 2>&1
SFHE_NTT_LE=4 timeout -k 10 200 python bench.py $B > gpurun_out/ab12_le4.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab12_le2b.log 2>&1
SFHE_NTT_LE=3 timeout -k 10 200 python bench.py $B > gpurun_out/ab12_le3b.log 2>&1
SFHE_NTT_LE=3 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab12_mb3.log 2>&1
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/ab12_mb2.log 2>&1
