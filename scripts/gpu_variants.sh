# GPU pass: time experimental builds of the step kernel (no parity check)
set -o pipefail
mkdir -p gpurun_out
TASKS=reach,push,pick_and_place timeout -k 10 600 python scripts/time_variants.py scripts/bin/variants/*.so > gpurun_out/variants.log 2>&1
echo "done rc=$?"
