# GPU pass: Stack parity tests and bench after the Stack LDS change, then the
# Push bench of the default build beside the IEEE-mode-off variant.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -s -rf --timeout 300 --timeout-method thread -k "stack or Stack" > gpurun_out/pytest_stack.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --env-id PandaStack-v3 > gpurun_out/bench_stack.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_push.log 2>&1 && \
PANDASIM_LIB=panda-lang-manip_amd/pandasim/libpandasim_ieee_off.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_push_ieee_off.log 2>&1
echo "done rc=$?"
