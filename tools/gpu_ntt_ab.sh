#!/bin/bash
# NTT prologue / row order A/B/C (unstacked batches), alternated twice:
#   B: defaults (row-arithmetic mask, prime-major rows)
#   D: SFHE_NTT_MASK=0 (both twiddle forms loaded, as round 4)
#   E: SFHE_NTT_MASK=0 SFHE_NTT_ROW_ORDER=0 (round 4's NTT behaviour)
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r05n}
mkdir -p gpurun_out
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 3 --steps 20 --warmup 3"
for k in 1 2; do
    timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_B_$k.json 2> gpurun_out/${T}_B_$k.err || exit $?
    SFHE_NTT_MASK=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_D_$k.json 2> gpurun_out/${T}_D_$k.err || exit $?
    SFHE_NTT_MASK=0 SFHE_NTT_ROW_ORDER=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_E_$k.json 2> gpurun_out/${T}_E_$k.err || exit $?
done
exit 0
