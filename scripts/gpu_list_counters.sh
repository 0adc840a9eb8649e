# list the PMC counters rocprofv3 offers on the box (gpurun_out/counters.txt)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1
echo "done rc=$?"
