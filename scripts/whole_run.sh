#!/bin/bash
# GPU box: the whole PG-MORL run end to end (python -m pgmorl_amd.run), MO-Walker2d-v2 with pop=40 (40 warm-up
# weights, 40 tasks per generation), prediction-guided selection, update_iter 20, the reference's 5e6 env-step
# budget per task (scripts/walker2d-v2.py:38).  Writes the results tree + timing.json (MOPG vs host split).
set -o pipefail
TAG=${1:-whole}
OUT=$(pwd)/gpurun_out/$TAG
SAVE=${TMPDIR:-/tmp}/pgm_whole_$TAG   # the results tree (EP policies) stays off gpurun_out (64 MiB cap)
mkdir -p $OUT $SAVE
timeout -k 10 ${WHOLE_TIMEOUT:-900} python -u -m pgmorl_amd.run --env-name MO-Walker2d-v2 --obj-num 2 \
  --num-env-steps ${BUDGET:-5000000} --warmup-iter 80 --update-iter 20 --min-weight 0.0 --max-weight 1.0 \
  --delta-weight 0.02564102564102564 --eval-num 1 --pbuffer-num 100 --pbuffer-size 2 \
  --selection-method prediction-guided --num-weight-candidates 7 --num-tasks 40 --sparsity 1.0 \
  --obj-rms --ob-rms --raw --rl-log-interval 40 --seed 0 --save-dir $SAVE > $OUT.log 2>&1 || { echo RUN FAILED; tail -20 $OUT.log; exit 1; }
cp $SAVE/timing.json $SAVE/args.txt $OUT/ && cp -r $SAVE/final/objs.txt $OUT/final_objs.txt && ls $SAVE | head -50 > $OUT/tree.txt
grep -E "timing|Generation" $OUT.log | tail -5
python -c "import json; t=json.load(open('$OUT/timing.json')); print({k: v for k, v in t.items() if k != 'generations'}); print(t['generations'][:2], t['generations'][-2:])"
