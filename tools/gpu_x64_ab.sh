# k_mdrsf with 64-coefficient blocks for small ModDowns (<= 16 target rows):
# parity tests of that build (sorting-fhe_amd/build_x64) through the product
# library override, then A/B/C x2 on one box: it, the same build with
# SFHE_MDRS_SMALL_L=0 (128 everywhere), and the default build.
#   bash tools/gpu_x64_ab.sh <tag>
set -o pipefail
T=${1:-r05x64}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
L=$PWD/sorting-fhe_amd/build_x64/libsfhe.so
SFHE_PRODUCT_LIB=$L timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_parity_metric.py tests/test_gpu_parity_sort.py tests/test_gpu_graph.py \
    > gpurun_out/$T/gpu_tests.log 2>&1 || exit $?
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 1 --steps 20 --warmup 3"
for k in 1 2; do
  SFHE_PRODUCT_LIB=$L timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/x64_$k.json 2>/dev/null || exit 1
  SFHE_PRODUCT_LIB=$L SFHE_MDRS_SMALL_L=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/x64off_$k.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/default_$k.json 2>/dev/null || exit 1
done
