#!/bin/bash
# Developer GPU script: the MFMA conversion (SFHE_CONV_MFMA=1) -- lane-map
# probe, bit-exact parity against the oracle, microbench, and an A/B of the
# metric sort against the FP64 conversion on one box.
set -o pipefail
cd "$(dirname "$0")/.."
T=${TAG:-mf}
timeout -k 10 60 tools/build/mfma_i8_probe > gpurun_out/${T}_probe.txt 2>&1 || exit $?
SFHE_CONV_MFMA=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_parity_metric.py tests/test_fusion.py tests/test_gpu_ntt_variants.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
SFHE_CONV_MFMA=1 timeout -k 10 120 tools/build/microbench 16 > gpurun_out/${T}_mb_mf.txt 2>&1 || exit $?
B="python bench.py --steps 10 --warmup 3 --no-kway --no-cpu-baseline --no-hybrid1 --no-c5 --trials 0"
for r in 1 2; do
    SFHE_CONV_MFMA=1 timeout -k 10 300 $B > gpurun_out/${T}_mf$r.json 2> gpurun_out/${T}_mf$r.err || exit $?
    timeout -k 10 300 $B > gpurun_out/${T}_fp$r.json 2> gpurun_out/${T}_fp$r.err || exit $?
done
exit 0
