# GPU pass: every GPU test, then the Push and Stack bench lines and the phase
# splits of both (a failing test still lets the benches run; a crash, abort or
# time limit ends the call there)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -s -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_push.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --env-id PandaStack-v3 > gpurun_out/bench_stack.log 2>&1 && \
timeout -k 10 300 python scripts/phase_profile.py PandaPush-v3 65536 20 > gpurun_out/phase.log 2>&1 && \
timeout -k 10 300 python scripts/phase_profile.py PandaStack-v3 65536 20 >> gpurun_out/phase.log 2>&1
echo "done rc=$?"
