#!/bin/bash
# Stacked launches / NTT row order: bit-exactness tests, then the metric sort
# A/B/C (leg-free bench), alternated twice on one box.
#   A: defaults (stacked batches, prime-major NTT rows)
#   B: SFHE_STACK_BATCHES=0 (the batches on two streams, round 4)
#   C: SFHE_NTT_ROW_ORDER=0 (poly-major NTT rows)
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r05s}
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_stack.py tests/test_gpu_parity_sort.py::test_metric_sort_bitexact tests/test_gpu_graph.py \
    tests/test_hybrid_variants.py tests/test_gpu_shard.py tests/test_gpu_multigpu.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
fi
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 5 --steps 20 --warmup 3"
for k in 1 2; do
    timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_A_$k.json 2> gpurun_out/${T}_A_$k.err || exit $?
    SFHE_STACK_BATCHES=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_B_$k.json 2> gpurun_out/${T}_B_$k.err || exit $?
    SFHE_NTT_ROW_ORDER=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_C_$k.json 2> gpurun_out/${T}_C_$k.err || exit $?
done
exit 0
