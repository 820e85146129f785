set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcF.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcW.log 2>&1
timeout -k 10 200 python3 tools/hostbound.py > gpurun_out/hostbound.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_full.log 2>&1
find gpurun_out/pmcF gpurun_out/pmcW gpurun_out/prof -name "*.csv" | head -20
