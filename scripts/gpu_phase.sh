set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/phase.log
STAGES="phase" PHASE_IDS="PandaSlide-v3:65536 PandaPush-v3:65536" bash scripts/gpu_round.sh
