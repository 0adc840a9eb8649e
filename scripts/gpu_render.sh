# GPU pass for the camera-image row: parity tests, throughput line, montage,
# rocprofv3 kernel stats and PMC (FETCH_SIZE, WRITE_SIZE) of the render bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="--output-format csv -o run"
B="$R/scripts/bench_render.py --reps 5"
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/render_tests.log 2>&1 && \
timeout -k 10 300 python scripts/bench_render.py --png gpurun_out/render_push.png > gpurun_out/render_bench.log 2>&1 && \
timeout -k 10 300 python scripts/bench_render.py --env-id PandaStack-v3 --batch 16 --png gpurun_out/render_stack.png >> gpurun_out/render_bench.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $P -d $R/gpurun_out/prof_render_trace -- python $B > $R/gpurun_out/prof_render.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d $R/gpurun_out/prof_render_fetch -- python $B > $R/gpurun_out/prof_render_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d $R/gpurun_out/prof_render_write -- python $B > $R/gpurun_out/prof_render_write.log 2>&1
echo "done rc=$?"
