# One GPU test with its output uncaptured (a crash's own message stays in the log).
#   bash tools/gpu_one.sh <tag> <pytest node id> [env assignments...]
set -o pipefail
T=$1; shift
NODE=$1; shift
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
env "$@" timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread -m gpu "$NODE" \
    > gpurun_out/$T/one.log 2>&1
echo "rc=$?" >> gpurun_out/$T/one.log
