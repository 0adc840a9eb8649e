# GPU pass: parity tests, bench line, rocprof kernel trace and PMC passes of
# the same bench command, FETCH_SIZE calibration, host probes.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="--output-format csv -o run"
BENCH="$R/bench.py --steps 100 --warmup 10 --no-cpu-baseline"
(python -c "import pybullet" > gpurun_out/probe_pybullet.log 2>&1; nproc; lscpu | grep "Model name") \
  > gpurun_out/probe_host.log 2>&1
timeout -k 10 600 python -m pytest tests -x -q -m gpu -s > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $P -d $R/gpurun_out/prof_trace -- python $BENCH > $R/gpurun_out/prof_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d $R/gpurun_out/prof_fetch -- python $BENCH > $R/gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d $R/gpurun_out/prof_write -- python $BENCH > $R/gpurun_out/prof_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES $P -d $R/gpurun_out/prof_valu -- python $BENCH > $R/gpurun_out/prof_valu.log 2>&1 && \
timeout -k 10 120 $R/scripts/bin/calib_fetch > $R/gpurun_out/calib.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d $R/gpurun_out/calib_fetch -- $R/scripts/bin/calib_fetch > $R/gpurun_out/calib_fetch.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d $R/gpurun_out/calib_write -- $R/scripts/bin/calib_fetch > $R/gpurun_out/calib_write.log 2>&1
echo "done rc=$?"
