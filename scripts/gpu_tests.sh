cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
rocminfo | grep -m2 -E "gfx950|Marketing" > gpurun_out/rocminfo.txt 2>&1
timeout -k 10 1200 python -m pytest tests -m gpu -q --timeout=300 -rA > gpurun_out/pytest_gpu_r1e.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu_r1e.log
