#!/bin/bash
# hardware-queue count vs the launch-heavy repair (configs[1] cold start)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
echo "box default GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
for Q in 4 32; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 100 python3 -u scripts/r3_probe.py shapes > gpurun_out/r3q_q$Q.log 2>&1 || { echo "q$Q failed"; exit 1; }
  echo "queues $Q: $(python3 -c 'import json; print([(json.loads(l)["tag"], json.loads(l)["s"]) for l in open("gpurun_out/r3q_q'$Q'.log") if l.startswith("{")])')"
done
