set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_a.log 2>&1
SIZES="4096 8192 16384" RUNS="DYMU_KERNEL=0" bash tools/sweep.sh
