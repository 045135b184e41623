# Round 6 GPU step: a selected test subset (-k), then bench legs.
# usage: gpu_r6.sh TAG "<pytest -k expr>" [legs...]   (legs: bench.py --leg names, or "env:VAR=VAL" before a leg)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; KEXPR=$2; shift 2
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs -k "$KEXPR" \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
fi
ENVV=""
for L in "$@"; do
  case "$L" in
    env:*) ENVV="${L#env:}"; continue;;
  esac
  echo "== leg $L ($ENVV)"
  env $ENVV timeout -k 10 400 python -u bench.py --leg $L > gpurun_out/${TAG}_leg_${L}.json 2> gpurun_out/${TAG}_leg_${L}.err
  rc=$?; tail -c 1500 gpurun_out/${TAG}_leg_${L}.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_leg_${L}.err; exit 1; }
  ENVV=""
done
