# k_modup_col two-target threshold A/B x2 on one box (no rebuild): launches
# under SFHE_MODUP_TG_SMALL blocks (at four targets per block) take two
# targets per block; default 512 against 1024 and 4096.
#   bash tools/gpu_tgsmall_ab.sh <tag>
set -o pipefail
T=${1:-r05tg}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 1 --steps 20 --warmup 3"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/tg512_$k.json 2>/dev/null || exit 1
  SFHE_MODUP_TG_SMALL=1024 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/tg1024_$k.json 2>/dev/null || exit 1
  SFHE_MODUP_TG_SMALL=4096 timeout -k 10 300 python -u bench.py $B > gpurun_out/$T/tg4096_$k.json 2>/dev/null || exit 1
done
