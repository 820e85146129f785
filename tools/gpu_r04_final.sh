#!/bin/bash
# Round-4 closing GPU call (developer script): the whole -m gpu suite as the
# driver runs it, the default bench line, then (PROFILE=1) the round's profile.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r04z}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread --durations=15 tests -m gpu > gpurun_out/${T}_gpu_suite.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
[ -n "$PROFILE" ] && { bash tools/profile_round.sh "$T" || exit $?; }
exit 0
