# EvalRotateSum's rotated c0 terms summed by one weighted-sum launch: parity
# tests, then A/B x2 on one box against SFHE_ROTSUM_C0=0 (one add per term).
#   bash tools/gpu_c0sum_ab.sh <tag>
set -o pipefail
T=${1:-r05c0}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_parity_metric.py tests/test_gpu_parity_sort.py tests/test_gpu_graph.py \
    > gpurun_out/$T/gpu_tests.log 2>&1 || exit $?
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 1 --steps 20 --warmup 3"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/onesum_$k.json 2>/dev/null || exit 1
  SFHE_ROTSUM_C0=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/adds_$k.json 2>/dev/null || exit 1
done
