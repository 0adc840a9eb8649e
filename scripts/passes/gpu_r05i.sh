# round 5 final pass, part 3: phase split and per-config PMC passes
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/phase.log
STAGES="phase" PHASE_IDS="PandaPush-v3:65536 PandaStack-v3:65536 PandaPush-v3:8192" bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_pmc_configs.sh
