set -o pipefail
mkdir -p gpurun_out
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 1 --steps 20 --warmup 3"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/tg4_$k.json 2>/dev/null || exit 1
  SFHE_PRODUCT_LIB=$PWD/sorting-fhe_amd/build_tg8/libsfhe.so timeout -k 10 300 python -u bench.py $B > gpurun_out/tg8_$k.json 2>/dev/null || exit 1
  SFHE_PRODUCT_LIB=$PWD/sorting-fhe_amd/build_tg2/libsfhe.so timeout -k 10 300 python -u bench.py $B > gpurun_out/tg2_$k.json 2>/dev/null || exit 1
done
