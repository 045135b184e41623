# Round 4: the multi-chain diagnosis steps, then the whole GPU suite.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
  local name=$1; local lim=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $lim "$@" > gpurun_out/r4e_$name.log 2>&1
  local rc=$?
  echo "rc=$rc"
  tail -n 5 gpurun_out/r4e_$name.log
  return $rc
}
step conc1 240 python scripts/diag_mc.py chains 4 8 &&
step conc2 240 python scripts/diag_mc.py chains 4 8 &&
step post1 240 python scripts/diag_mc.py post 16 300 &&
step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs
