# GPU pass: Stack parity tests, Stack bench and Stack phase split
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -s -rf --timeout 300 --timeout-method thread -k "stack or Stack" > gpurun_out/pytest_stack.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --env-id PandaStack-v3 > gpurun_out/bench_stack.log 2>&1 && \
timeout -k 10 300 python scripts/phase_profile.py PandaStack-v3 65536 20 > gpurun_out/phase_stack.log 2>&1
echo "done rc=$?"
