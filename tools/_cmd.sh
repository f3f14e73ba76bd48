set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_costmap.py -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -30 gpurun_out/gpu_tests.log
exit $rc
