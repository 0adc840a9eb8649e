# round 6 pass p: the XCD remap in tiles of G / 2 waves (remaptile) against no
# remap and the whole-range remap: bits, C3/C4 and C2 timing (rotating order),
# FETCH/WRITE at C3 and C2
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06p_compare.log
LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $V/lib_remaptile.so 1000 10 >> gpurun_out/r06p_compare.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $V/lib_remaptile.so 256 10 >> gpurun_out/r06p_compare.log 2>&1 || exit $?
: > gpurun_out/r06p_ab.log
for order in "$V/lib_noremap.so $V/lib_remaptile.so $P" "$P $V/lib_noremap.so $V/lib_remaptile.so" "$V/lib_remaptile.so $P $V/lib_noremap.so"; do
  B=8192 TASKS=push,pick_and_place timeout -k 10 300 python scripts/time_variants.py $order >> gpurun_out/r06p_ab.log 2>&1 || exit $?
  B=4096 TASKS=reach timeout -k 10 300 python scripts/time_variants.py $order >> gpurun_out/r06p_ab.log 2>&1 || exit $?
done
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PP="--output-format csv -o run"
cd /tmp
for cfg in PandaReach-v3:4096:16 PandaPush-v3:8192:8; do
  IFS=: read id b l <<< "$cfg"
  d=$R/gpurun_out/fvbt_${id}_${b}_${l}
  BENCH="$R/bench.py --steps 12 --warmup 2 --no-cpu-baseline --env-id $id --batch $b --lanes $l"
  PANDASIM_LIB=$R/$V/lib_remaptile.so timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE $PP -d ${d}_fetch -- python $BENCH > ${d}_fetch.log 2>&1 || { echo "failed $cfg fetch"; exit 1; }
  PANDASIM_LIB=$R/$V/lib_remaptile.so timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE $PP -d ${d}_write -- python $BENCH > ${d}_write.log 2>&1 || { echo "failed $cfg write"; exit 1; }
done
python scripts/fetch_vs_batch.py fvbt > gpurun_out/r06p_fetch_vs_batch.log 2>&1
echo "done rc=$?"
