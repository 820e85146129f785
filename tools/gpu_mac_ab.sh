# Multi-output mask sums (sfp_mac_plain2_multi from EvalRotateSum): parity
# tests, then A/B/C x2 on one box: up to 8 sums per launch (the default), 4
# (SFHE_MAC_MULTI_G=4) and single sums (SFHE_MAC_MULTI=0).
#   bash tools/gpu_mac_ab.sh <tag>
set -o pipefail
T=${1:-r05m}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_parity_metric.py tests/test_gpu_parity_sort.py tests/test_gpu_graph.py \
    tests/test_gpu_sort.py > gpurun_out/$T/gpu_tests.log 2>&1 || exit $?
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 1 --steps 20 --warmup 3"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/multi8_$k.json 2>/dev/null || exit 1
  SFHE_MAC_MULTI_G=4 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/multi4_$k.json 2>/dev/null || exit 1
  SFHE_MAC_MULTI=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/single_$k.json 2>/dev/null || exit 1
done
