# Round-2 GPU pass: every GPU test, the default bench line (with its CPU
# baseline and FLOP roofline), rocprofv3 kernel trace and separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ instruction counts, FP32 instruction counts) of
# the same bench command, phase profiles, and the bench line at every
# single-GPU BASELINE config.  Each GPU step has its own time limit; after a
# crash or a time limit nothing else runs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="--output-format csv -o run"
BENCH="$R/bench.py --steps 100 --warmup 10 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -s -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $P -d $R/gpurun_out/prof_trace -- python $BENCH > $R/gpurun_out/prof_trace.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d $R/gpurun_out/prof_fetch -- python $BENCH > $R/gpurun_out/prof_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d $R/gpurun_out/prof_write -- python $BENCH > $R/gpurun_out/prof_write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES $P -d $R/gpurun_out/prof_valu -- python $BENCH > $R/gpurun_out/prof_valu.log 2>&1 && \
cd $R && \
timeout -k 10 300 python scripts/phase_profile.py PandaPush-v3 65536 20 > gpurun_out/phase_push65536.log 2>&1 && \
timeout -k 10 300 python scripts/phase_profile.py PandaStack-v3 65536 10 > gpurun_out/phase_stack65536.log 2>&1 && \
timeout -k 10 300 python scripts/phase_profile.py PandaPush-v3 4096 20 16 > gpurun_out/phase_push4096_l16.log 2>&1 && \
timeout -k 10 300 python scripts/phase_profile.py PandaPush-v3 4096 20 1 > gpurun_out/phase_push4096_l1.log 2>&1 && \
for cfg in "PandaReach-v3 4096" "PandaReachJoints-v3 4096" "PandaPush-v3 8192" "PandaPickAndPlace-v3 8192" \
           "PandaPush-v3 65536" "PandaReachDense-v3 65536" "PandaReachJoints-v3 65536" "PandaPickAndPlace-v3 65536" \
           "PandaSlide-v3 65536" "PandaStack-v3 65536" "PandaFlip-v3 65536"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --env-id $1 --batch $2 >> gpurun_out/configs.jsonl 2>/dev/null || exit $?
done
cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 $P -d $R/gpurun_out/prof_flops -- python $BENCH > $R/gpurun_out/prof_flops.log 2>&1
echo "done rc=$?"
