# Value-prediction loop check: the repair parity tests, then the dense-mover
# legs (the north-star literal, configs[1]'s cold start).
# usage: gpu_vp.sh TAG
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
  -k "value_prediction or repair or config2 or chains or last_customer or parallel_golden or underflow or literal" \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
for L in north_star_literal_gpu cold_start_gpu; do
  timeout -k 10 400 python -u bench.py --leg $L > gpurun_out/${TAG}_$L.json 2> gpurun_out/${TAG}_$L.err || { tail -5 gpurun_out/${TAG}_$L.err; exit 1; }
  tail -c 600 gpurun_out/${TAG}_$L.json; echo
done
