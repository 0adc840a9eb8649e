# round 6 pass q: the product's XCD remap (tiles at 8 lanes, the whole range at
# 16): bits against round 5 at 1, 8 (ragged) and 16 lanes, C2-C4 timing against
# the same sources without remap (rotating order), FETCH/WRITE against the
# batch, the group-kernel tests
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06q_compare.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1024 10 >> gpurun_out/r06q_compare.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 256 10 >> gpurun_out/r06q_compare.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1000 10 >> gpurun_out/r06q_compare.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1000 10 >> gpurun_out/r06q_compare.log 2>&1 || exit $?
: > gpurun_out/r06q_ab.log
for order in "$V/lib_noremap.so $P" "$P $V/lib_noremap.so" "$V/lib_noremap.so $P" "$P $V/lib_noremap.so"; do
  B=8192 TASKS=push,pick_and_place timeout -k 10 300 python scripts/time_variants.py $order >> gpurun_out/r06q_ab.log 2>&1 || exit $?
  B=4096 TASKS=reach timeout -k 10 300 python scripts/time_variants.py $order >> gpurun_out/r06q_ab.log 2>&1 || exit $?
done
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PP="--output-format csv -o run"
cd /tmp
for cfg in PandaReach-v3:64:16 PandaReach-v3:1024:16 PandaReach-v3:4096:16 PandaPush-v3:128:8 PandaPush-v3:1024:8 PandaPush-v3:8192:8 PandaPickAndPlace-v3:8192:8; do
  IFS=: read id b l <<< "$cfg"
  d=$R/gpurun_out/fvb_${id}_${b}_${l}
  BENCH="$R/bench.py --steps 12 --warmup 2 --no-cpu-baseline --env-id $id --batch $b --lanes $l"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE $PP -d ${d}_fetch -- python $BENCH > ${d}_fetch.log 2>&1 || { echo "failed $cfg fetch"; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE $PP -d ${d}_write -- python $BENCH > ${d}_write.log 2>&1 || { echo "failed $cfg write"; exit 1; }
done
cd $R
python scripts/fetch_vs_batch.py > gpurun_out/r06q_fetch_vs_batch.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_envs.py tests/test_gpu_contacts.py -v -s -k "group or lanes or ragged or config_size or teacher_forced or work_lists" --timeout 300 --timeout-method thread > gpurun_out/r06q_pytest.log 2>&1
echo "done rc=$?"
