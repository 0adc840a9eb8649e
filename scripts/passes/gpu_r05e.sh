# round 5 final pass, part 2: the bench at every single-GPU config and task
# (scripts/gpu_configs.sh) and the phase split of k_step (Push, Stack)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/configs.jsonl gpurun_out/phase.log
bash scripts/gpu_configs.sh || exit $?
STAGES="phase" PHASE_IDS="PandaPush-v3:65536 PandaStack-v3:65536 PandaPush-v3:8192" bash scripts/gpu_round.sh
