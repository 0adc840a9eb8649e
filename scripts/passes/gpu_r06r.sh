# round 6 final pass (library f03ef581: the group kernels' XCD block order), part 1 (bit-identical to the
# round-5 library on every task, control and lanes-per-env: r06q and earlier
# compare_libs): every -m gpu test, smoke, the bench line with its CPU
# baseline, and the rocprofv3 kernel trace + PMC passes of the bench command
# (FETCH_SIZE, WRITE_SIZE, SQ counters, the FLOPS counters)
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/tf200 gpurun_out/judged
STAGES="tests smoke bench trace pmc" bash scripts/gpu_round.sh
