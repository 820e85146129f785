# Round-end check on one box: full GPU suite, smoke, the default bench line,
# then the rocprof kernel trace + PMC passes (tools/profile_round.sh <tag>).
set -e
tag=${1:-rXX}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_suite.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 360 python bench.py > gpurun_out/${tag}_bench.log 2>&1
tail -1 gpurun_out/${tag}_bench.log > gpurun_out/${tag}_bench.json
bash tools/profile_round.sh ${tag}
