set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
SIZES="8192" RUNS="DYMU_KERNEL=3;DYMU_KERNEL=4;DYMU_KERNEL=4 DYMU_PRIO_TARGET=8192" bash tools/sweep.sh
