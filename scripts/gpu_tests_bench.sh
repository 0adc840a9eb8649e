# GPU pass: the GPU parity tests (a failing test still lets the bench run; a
# crash, abort or time limit ends the call there), then bench lines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -s -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
for t in ${TASKS:-}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --env-id Panda$t-v3 >> gpurun_out/bench_tasks.log 2>&1 || exit $?
done
echo "done rc=$?"
