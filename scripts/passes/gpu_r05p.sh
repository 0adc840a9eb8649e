# round 5 final pass (library of d54809d): smoke, the bench line, its kernel
# trace and PMC passes, every config, and the phase split (Push, Slide, Stack,
# Push 8 192); the per-config PMC passes are scripts/gpu_pmc_configs.sh
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/configs.jsonl gpurun_out/phase.log
STAGES="smoke bench trace pmc" bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_configs.sh || exit $?
STAGES="phase" PHASE_IDS="PandaPush-v3:65536 PandaSlide-v3:65536 PandaStack-v3:65536 PandaPush-v3:8192" bash scripts/gpu_round.sh
