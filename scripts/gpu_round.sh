# GPU pass for a round checkpoint, run through gpurun from the repo root:
#   STAGES="tests smoke bench trace pmc phase" bash scripts/gpu_round.sh
# tests  every -m gpu test (PYTEST_K narrows them)    -> gpurun_out/pytest_gpu.log
# smoke  __graft_entry__.smoke()                      -> gpurun_out/smoke.log
# bench  the default bench line with its CPU baseline -> gpurun_out/bench.json
# trace  rocprofv3 --kernel-trace --stats of the bench command (ENV_ID, BATCH)
# pmc    separate PMC passes of the same command: FETCH_SIZE, WRITE_SIZE, SQ counters
# phase  per-phase cycle split of k_step (libpandasim_prof.so; PHASE_IDS)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
STAGES=${STAGES:-"tests bench trace pmc"}
ENV_ID=${ENV_ID:-PandaPush-v3}
BATCH=${BATCH:-65536}
P="--output-format csv -o run"
BENCH="$R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --env-id $ENV_ID --batch $BATCH"
has() { case " $STAGES " in *" $1 "*) return 0;; esac; return 1; }
run() { echo "[gpu_round] $*" >&2; "$@" || { rc=$?; echo "[gpu_round] failed rc=$rc: $*"; exit $rc; }; }
if has tests; then
  run timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -rf --timeout 120 --timeout-method thread \
      ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
fi
if has smoke; then
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
fi
if has bench; then
  run timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
fi
cd /tmp
if has trace; then
  run timeout -k 10 300 rocprofv3 --kernel-trace --stats $P -d $R/gpurun_out/prof_trace -- python $BENCH > $R/gpurun_out/prof_trace.log 2>&1
fi
if has pmc; then
  run timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d $R/gpurun_out/prof_fetch -- python $BENCH > $R/gpurun_out/prof_fetch.log 2>&1
  run timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d $R/gpurun_out/prof_write -- python $BENCH > $R/gpurun_out/prof_write.log 2>&1
  run timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES $P -d $R/gpurun_out/prof_valu -- python $BENCH > $R/gpurun_out/prof_valu.log 2>&1
  run timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 $P -d $R/gpurun_out/prof_fp32 -- python $BENCH > $R/gpurun_out/prof_fp32.log 2>&1
fi
cd $R
if has phase; then
  DEFAULT_IDS="PandaPush-v3:65536 PandaStack-v3:65536"  # (a quoted default inside ${:-} is one word)
  for id in ${PHASE_IDS:-$DEFAULT_IDS}; do
    run timeout -k 10 300 python scripts/phase_profile.py ${id%%:*} ${id##*:} 20 >> gpurun_out/phase.log 2>&1
  done
fi
echo "done rc=0"
