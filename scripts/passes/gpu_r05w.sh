# round 5 pass w (library of 252bf8b, rebuilt in a fresh container): every
# -m gpu test, smoke, the bench line, its kernel trace and PMC passes
set -o pipefail
mkdir -p gpurun_out
STAGES="tests smoke bench trace pmc" bash scripts/gpu_round.sh
