# Small-launch latency changes, A/B/C/D x2 on one box: the default build (q_0
# folded into the first FP64 chunk of k_mdrsf / k_convf, the dropped row's
# constants issued early, two-target k_modup_col blocks for small launches,
# k_mac_plain2 four terms per step), the same with SFHE_MODUP_TG_SMALL=0
# (four targets always), the same built with two mac terms per step
# (sorting-fhe_amd/build_mac2), and the previous kernels
# (sorting-fhe_amd/build_base); parity tests of the default build first.
#   bash tools/gpu_fold_ab.sh <tag>
set -o pipefail
T=${1:-r05f}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_parity_metric.py tests/test_gpu_parity_sort.py tests/test_gpu_graph.py \
    tests/test_gpu_ntt_variants.py tests/test_gpu_stack.py > gpurun_out/$T/gpu_tests.log 2>&1 || exit $?
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 1 --steps 20 --warmup 3"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/new_$k.json 2>/dev/null || exit 1
  SFHE_MODUP_TG_SMALL=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/new_tg4_$k.json 2>/dev/null || exit 1
  SFHE_PRODUCT_LIB=$PWD/sorting-fhe_amd/build_mac2/libsfhe.so timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/new_mac2_$k.json 2>/dev/null || exit 1
  SFHE_PRODUCT_LIB=$PWD/sorting-fhe_amd/build_base/libsfhe.so timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/base_$k.json 2>/dev/null || exit 1
done
