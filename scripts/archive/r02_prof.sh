#!/bin/bash
# GPU box: host facts, the default bench line, then the headline profile (trace + PMC passes).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))" > gpurun_out/host.txt
cat /sys/fs/cgroup/cpu.max >> gpurun_out/host.txt 2>&1; nproc >> gpurun_out/host.txt; cat /sys/fs/cgroup/pids.max >> gpurun_out/host.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-r02} ./scripts/profile.sh
