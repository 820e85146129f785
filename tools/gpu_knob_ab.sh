# Knob / build-variant A/B on one box, x2: the default build against
# conversion blocks of 64 and 256 coefficients (SFHE_CONV_COEFS builds
# sorting-fhe_amd/build_cc64, build_cc256: k_convf / k_mdrsf blocks) and
# SFHE_NTT_T1K_ROWS (1024-word NTT tiles up to this many rows; default 64)
# at 32 and 128.   bash tools/gpu_knob_ab.sh <tag>
set -o pipefail
T=${1:-r05k}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 1 --steps 20 --warmup 3"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/default_$k.json 2>/dev/null || exit 1
  for v in 64 256; do
    SFHE_PRODUCT_LIB=$PWD/sorting-fhe_amd/build_cc$v/libsfhe.so timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/cc${v}_$k.json 2>/dev/null || exit 1
  done
  SFHE_NTT_T1K_ROWS=32 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/t1k32_$k.json 2>/dev/null || exit 1
  SFHE_NTT_T1K_ROWS=128 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/t1k128_$k.json 2>/dev/null || exit 1
done
