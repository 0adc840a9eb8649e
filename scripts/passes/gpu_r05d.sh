# round 5 final pass, part 1: every GPU test, smoke, the bench line, and the
# rocprofv3 kernel trace + PMC passes of the bench command (scripts/gpu_round.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -q -s -m gpu -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
STAGES="smoke bench trace pmc" bash scripts/gpu_round.sh
