#!/bin/bash
# the run kernel's stay limit (MVC_RUN_LIMIT) in the sparse-mover regime: configs[3] cold start, configs[1] cold, literal
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for L in 64 16 8; do
  MVC_RUN_LIMIT=$L timeout -k 10 150 python3 -u scripts/coldstart.py --config c4 --sweeps 12 --budget-s 100 > gpurun_out/r3n_c4_L$L.log 2>&1 || { echo "c4 L$L failed"; exit 1; }
  echo "c4 L=$L: $(tail -3 gpurun_out/r3n_c4_L$L.log | python3 -c 'import sys,json; print([ (json.loads(l)["s"], json.loads(l)["moves"], json.loads(l)["rounds"]) for l in sys.stdin])')"
  MVC_RUN_LIMIT=$L timeout -k 10 100 python3 -u scripts/r3_probe.py shapes > gpurun_out/r3n_shapes_L$L.log 2>&1 || { echo "shapes L$L failed"; exit 1; }
  echo "shapes L=$L: $(python3 -c 'import sys,json; print([(json.loads(l)["tag"], json.loads(l)["s"]) for l in open("gpurun_out/r3n_shapes_L'$L'.log") if l.startswith("{")])')"
done
