mkdir -p gpurun_out
DYMU_KERNEL=4 DYMU_PRIO_TARGET=1024 DYMU_PRIO_DEBUG=400 timeout -k 10 120 python tools/probe.py 1024 > gpurun_out/dbg.log 2>&1
