set -o pipefail
mkdir -p gpurun_out
for s in 1 2 3 4; do
  timeout -k 10 200 python -u scripts/hv_budget.py device --ref profiles/r01_hv_oracle_hopper_p5_s$s.json --out gpurun_out/hv_dev_hopper_p5_s$s.json > gpurun_out/hv_s$s.log 2>&1 || { tail -20 gpurun_out/hv_s$s.log; exit 1; }
  tail -1 gpurun_out/hv_s$s.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_hum2 -o hum --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --env-name MO-Humanoid-v2 --tasks 20 --num-processes 8 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_hum2.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_hum2.log; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$GRAFT_REPO_ROOT/gpurun_out/prof_hum2/**/*kernel_stats.csv',recursive=True)[0]
for x in list(csv.DictReader(open(f)))[:8]:
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1),'us', x['Percentage'])
PY
