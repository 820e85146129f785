#!/bin/bash
# A/B of the product library against tools/build/libsfhe_prev.so on one box
# (developer script): bit-exact parity of the current build, then the metric
# bench alternating current / previous library.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
O=gpurun_out/${PROBE_TAG:-ab}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_fusion.py tests/test_bootstrap.py tests/test_kway.py ${AB_TESTS} > ${O}_tests.log 2>&1 || exit 1
B="python bench.py --steps 10 --warmup 3 --no-kway --no-cpu-baseline --no-hybrid1 --no-c5 --trials 5"
for r in 1 2; do
    timeout -k 10 200 $B > ${O}_cur$r.log 2>&1 || exit 1
    SFHE_PRODUCT_LIB=$PWD/tools/build/libsfhe_prev.so timeout -k 10 200 $B > ${O}_prev$r.log 2>&1 || exit 1
done
MB_REPS=3 timeout -k 10 120 tools/build/microbench 16 > ${O}_mb_cur.log 2>&1
