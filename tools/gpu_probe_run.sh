#!/bin/bash
# Precision + parity check on the GPU box (developer script): bit-exact HIP vs
# oracle tests, the per-stage precision probe at the BASELINE sizes (lazy
# rescaling on and off), and a short bench.  Output under gpurun_out/.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
P=tools/build/prec_probe_hip
O=gpurun_out/${PROBE_TAG:-probe}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_fusion.py tests/test_gpu_ntt_variants.py -m gpu > ${O}_parity.log 2>&1 || exit 1
timeout -k 10 200 $P h1x 256 17 1 > ${O}_h1x.log 2>&1 || exit 1
SFHE_LAZY=0 timeout -k 10 200 $P h1x 256 17 1 > ${O}_h1x_nolazy.log 2>&1 || exit 1
timeout -k 10 200 $P ds 256 16 0 > ${O}_ds16.log 2>&1 || exit 1
SFHE_LAZY=0 timeout -k 10 200 $P ds 256 16 0 > ${O}_ds16_nolazy.log 2>&1 || exit 1
timeout -k 10 200 $P ds 256 17 1 > ${O}_ds17.log 2>&1 || exit 1
timeout -k 10 200 $P h 256 17 1 > ${O}_h.log 2>&1 || exit 1
timeout -k 10 200 $P h2 256 17 1 > ${O}_h2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-kway --no-c5 --no-cpu-baseline --trials 3 > ${O}_bench.log 2>&1 || exit 1
SFHE_LAZY=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-kway --no-c5 --no-cpu-baseline --no-hybrid1 --trials 3 > ${O}_bench_nolazy.log 2>&1
