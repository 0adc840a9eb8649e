# round 6 pass m: FETCH_SIZE / WRITE_SIZE of the step kernel against the batch
# (Reach on 16 lanes and on 1, Push on 8 and on 1) -- is the small-batch
# configs' traffic above their algorithmic bytes a fixed per-launch part?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="--output-format csv -o run"
cd /tmp
for cfg in PandaReach-v3:64:16 PandaReach-v3:1024:16 PandaReach-v3:4096:16 PandaReach-v3:4096:1 PandaReach-v3:65536:1 PandaPush-v3:128:8 PandaPush-v3:8192:8 PandaPush-v3:8192:1 PandaPush-v3:65536:1; do
  IFS=: read id b l <<< "$cfg"
  d=$R/gpurun_out/fvb_${id}_${b}_${l}
  BENCH="$R/bench.py --steps 12 --warmup 2 --no-cpu-baseline --env-id $id --batch $b --lanes $l"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d ${d}_fetch -- python $BENCH > ${d}_fetch.log 2>&1 || { echo "failed $cfg fetch"; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d ${d}_write -- python $BENCH > ${d}_write.log 2>&1 || { echo "failed $cfg write"; exit 1; }
done
cd $R
python scripts/fetch_vs_batch.py > gpurun_out/r06m_fetch_vs_batch.log 2>&1
echo "done rc=$?"
