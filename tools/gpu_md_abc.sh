# Fused ModDown COL pass A/B/C/D/E on one box, x2: SFHE_MODDOWN_COL=0 (k_mdrsf /
# k_convf + the plain COL pass), the default build (k_moddown_col, 4 targets
# per block) at every level and up to 16 target rows (SFHE_MODDOWN_COL_MAXT),
# and a 2-target build (sorting-fhe_amd/build_md2) likewise; parity tests of
# the default build first.   bash tools/gpu_md_abc.sh <tag>
set -o pipefail
T=${1:-r05md3}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity_metric.py tests/test_gpu_parity_sort.py \
    > gpurun_out/$T/gpu_tests.log 2>&1 || exit $?
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 1 --steps 20 --warmup 3"
L2=$PWD/sorting-fhe_amd/build_md2/libsfhe.so
for k in 1 2; do
  SFHE_MODDOWN_COL=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/unfused_$k.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/tg4_all_$k.json 2>/dev/null || exit 1
  SFHE_MODDOWN_COL_MAXT=16 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/tg4_max16_$k.json 2>/dev/null || exit 1
  SFHE_PRODUCT_LIB=$L2 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/tg2_all_$k.json 2>/dev/null || exit 1
  SFHE_PRODUCT_LIB=$L2 SFHE_MODDOWN_COL_MAXT=16 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/tg2_max16_$k.json 2>/dev/null || exit 1
done
