#!/bin/bash
# Round-end GPU check (developer script): the whole -m gpu suite, as the
# driver runs it, with per-test timings.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
O=gpurun_out/${PROBE_TAG:-fin}
timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread --durations=25 tests -m gpu > ${O}_gpu_suite.log 2>&1
echo "suite rc=$?" >> ${O}_gpu_suite.log
