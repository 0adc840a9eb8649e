# GPU pass: parity tests of the in-tree build, then timing of variant builds
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  TASKS=reach,push,pick_and_place timeout -k 10 600 python scripts/time_variants.py "$@" > gpurun_out/variants.log 2>&1
fi
echo "done"
