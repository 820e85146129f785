#!/bin/bash
# Developer A/B/C of three builds of the product library (tools/build/
# libsfhe_v{a,b,c}.so): parity of variants b and c, then the metric bench
# alternating a / b / c twice on one box.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
O=gpurun_out/${PROBE_TAG:-abc}
for v in b c; do
    SFHE_PRODUCT_LIB=$PWD/tools/build/libsfhe_v$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_parity_metric.py tests/test_fusion.py > ${O}_tests_$v.log 2>&1 || exit $?
done
B="python bench.py --steps 10 --warmup 3 --no-kway --no-cpu-baseline --no-hybrid1 --no-c5 --trials 5"
for r in 1 2; do
    for v in a b c; do
        SFHE_PRODUCT_LIB=$PWD/tools/build/libsfhe_v$v.so timeout -k 10 200 $B > ${O}_${v}$r.log 2>&1 || exit $?
    done
done
exit 0
