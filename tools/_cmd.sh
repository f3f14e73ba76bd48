set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_solver.py -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_a.log 2>&1 && timeout -k 10 300 python bench.py --cpu-sample 0 --no-profile > gpurun_out/bench_b.log 2>&1
