set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/hv_budget.py device --ref profiles/r01_hv_oracle_hopper_p5.json --out gpurun_out/hv_dev_hopper_p5.json > gpurun_out/hv_h.log 2>&1 || { tail -30 gpurun_out/hv_h.log; exit 1; }
tail -1 gpurun_out/hv_h.log
timeout -k 10 300 python -u scripts/hv_budget.py device --ref profiles/r01_hv_oracle_walker_p40.json --out gpurun_out/hv_dev_walker_p40.json > gpurun_out/hv_w.log 2>&1 || { tail -30 gpurun_out/hv_w.log; exit 1; }
tail -1 gpurun_out/hv_w.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_hum -o hum --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_hum.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_hum.log; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$GRAFT_REPO_ROOT/gpurun_out/prof_hum/**/*kernel_stats.csv',recursive=True)[0]
for x in csv.DictReader(open(f)):
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1),'us', x['Percentage'])
PY
