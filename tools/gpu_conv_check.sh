#!/bin/bash
# Conversion-kernel change check (developer script): bit-exact parity incl.
# the scale-59 (60-bit prime) bootstrapping / k-way paths, then the k-way
# sort's time and bootstrap attribution.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
O=gpurun_out/${PROBE_TAG:-cv}
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_fusion.py tests/test_bootstrap.py tests/test_kway.py tests/test_gpu_ntt_variants.py \
    > ${O}_tests.log 2>&1 || exit 1
SFHE_BOOT_TRACE=1 timeout -k 10 400 python tools/kway_run.py --sorts 2 > ${O}_kway.log 2> ${O}_kway_boot.log
