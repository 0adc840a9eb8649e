# GPU pass: GPU parity tests of the in-tree build, phase split, bench lines.
# A failing test (pytest exit 1) still lets the measurement steps run; a
# crash, abort or time limit (any other status) ends the call there.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -s -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python scripts/phase_profile.py PandaPush-v3 65536 20 > gpurun_out/phase.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 && \
for t in ${TASKS:-Reach Slide PickAndPlace Stack Flip}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --env-id Panda$t-v3 >> gpurun_out/bench_tasks.log 2>&1 || exit $?
done
echo "done rc=$?"
