# GPU pass after a kernel change, run through gpurun from the repo root:
# every -m gpu test without stopping at the first failure (pytest rc 0 or 1
# lets the chain go on; a crash, abort or time limit ends it), then the bench
# line and, with AB=1, the interleaved A/B timing of the library variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest tests -q -m gpu -rf --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "[gpu_check] pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
if [ -n "$AB" ]; then bash scripts/gpu_ab.sh || exit $?; fi
echo "done rc=0"
