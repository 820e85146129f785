# k_lin_wsum_multi with (w, w/q) staged as doubles: parity, bench x2, kernel trace
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab11_parity.log 2>&1
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
timeout -k 10 200 python bench.py $B > gpurun_out/ab11_a.log 2>&1
timeout -k 10 200 python bench.py $B > gpurun_out/ab11_b.log 2>&1
SFHE_NO_GRAPH_REPLAY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof11 -o run -- python3 bench.py --steps 3 --warmup 1 --trials 0 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5 > gpurun_out/prof11_bench.log 2>&1
python3 tools/trace_segments.py gpurun_out/prof11/run_kernel_trace.csv > gpurun_out/ab11_rocprof_summary.txt 2>&1
