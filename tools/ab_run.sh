# HIP hardware queues per process for the graph-replayed sort (GPU_MAX_HW_QUEUES; box default 4)
set -e
mkdir -p gpurun_out
B="--steps 5 --warmup 2 --trials 6 --no-cpu-baseline --no-hybrid1 --no-kway --no-c5"
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py $B > gpurun_out/ab14_$tag.log 2>&1; }
run base X=1
run q2 GPU_MAX_HW_QUEUES=2
run q1 GPU_MAX_HW_QUEUES=1
run base2 X=1
run q2b GPU_MAX_HW_QUEUES=2
