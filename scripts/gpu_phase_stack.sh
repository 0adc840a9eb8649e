# GPU pass: phase split of the Stack step kernel (diagnostic build)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/phase_profile.py PandaStack-v3 65536 20 > gpurun_out/phase_stack.log 2>&1 && \
timeout -k 10 300 python scripts/phase_profile.py PandaPush-v3 65536 20 >> gpurun_out/phase_stack.log 2>&1
echo "done rc=$?"
