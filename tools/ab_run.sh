# conversion blocks of 64 coefficients (variants/c64, occupancy 8 at NS=13) against 128 (product)
set -e
mkdir -p gpurun_out
V=$PWD/variants/c64/libsfhe.so
SFHE_PRODUCT_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab10_parity.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
timeout -k 10 200 python bench.py $B > gpurun_out/ab10_128.log 2>&1
SFHE_PRODUCT_LIB=$V timeout -k 10 200 python bench.py $B > gpurun_out/ab10_64.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab10_128b.log 2>&1
SFHE_PRODUCT_LIB=$V timeout -k 10 200 python bench.py $B > gpurun_out/ab10_64b.log 2>&1
