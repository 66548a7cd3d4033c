#!/bin/bash
# quick GPU check: parity probe (short) + stamps
set -o pipefail
timeout -k 10 300 python scripts/gpu_probe.py > gpurun_out/probe.log 2>&1; r1=$?
echo "probe exit $r1"; head -20 gpurun_out/probe.log
[ $r1 -ne 0 ] && exit $r1
timeout -k 10 300 python scripts/gpu_stamps.py > gpurun_out/stamps.log 2>&1; r2=$?
echo "stamps exit $r2"; cat gpurun_out/stamps.log
exit $r2
