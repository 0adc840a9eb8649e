# round 5 final pass (library of 37ec464), part 1: every -m gpu test, smoke,
# the bench line, its kernel trace and PMC passes, and the bench at every
# single-GPU config and task (scripts/gpu_configs.sh)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/configs.jsonl
STAGES="tests smoke bench trace pmc" bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_configs.sh
