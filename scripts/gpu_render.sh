# GPU pass for the camera-image row: parity tests, throughput line, montage,
# rocprofv3 kernel stats of the render bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/render_tests.log 2>&1 && \
timeout -k 10 300 python scripts/bench_render.py --png gpurun_out/render_push.png > gpurun_out/render_bench.log 2>&1 && \
timeout -k 10 300 python scripts/bench_render.py --env-id PandaStack-v3 --batch 16 --png gpurun_out/render_stack.png >> gpurun_out/render_bench.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $R/gpurun_out/prof_render -- python $R/scripts/bench_render.py > $R/gpurun_out/prof_render.log 2>&1
echo "done rc=$?"
