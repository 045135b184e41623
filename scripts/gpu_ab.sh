# A/B of a build variant against the in-tree library: a test subset on the
# variant, then each bench leg on the variant and on the in-tree library.
# usage: gpu_ab.sh TAG VARIANT "<pytest -k expr>" legs...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; VAR=$PWD/build_variants/$2/libmvc_hip.so; KEXPR=$3; shift 3
if [ -n "$KEXPR" ]; then
  MVC_HIP_LIB=$VAR timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs \
    -k "$KEXPR" > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit 1
fi
for L in "$@"; do
  for side in var head; do
    if [ $side = var ]; then export MVC_HIP_LIB=$VAR; else unset MVC_HIP_LIB; fi
    timeout -k 10 400 python -u bench.py --leg $L > gpurun_out/${TAG}_${L}_${side}.json 2> gpurun_out/${TAG}_${L}_${side}.err \
      || { echo "leg $L $side failed"; tail -5 gpurun_out/${TAG}_${L}_${side}.err; exit 1; }
    echo "== $L $side"; tail -c 700 gpurun_out/${TAG}_${L}_${side}.json; echo
  done
done
