#!/bin/bash
# One GPU-box session as a list of steps (replaces the per-call rNNx.sh scripts): each step runs under its own time
# limit, the first failure ends the session (nothing more touches the GPU after it).  libpgm.so / libpgm_test.so are
# prebuilt in-tree.  Outputs under gpurun_out/.
#   bash scripts/gpu_steps.sh TAG STEP [STEP ...]
# STEP:
#   tests[=PYTEST_ARGS]     the -m gpu suite (default: all of it) -> gpu_tests_TAG.log
#   testlib=LIB:PYTEST_ARGS the same against an A/B library (PGM_LIB=LIB) -> gpu_tests_TAG_ab.log
#   smoke                   __graft_entry__.smoke()
#   check                   scripts/round_check.sh TAG --no-tests (bench line + whole run + cpu_baseline + kernel stats)
#   configs                 scripts/configs_check.sh TAG (every BASELINE config's per-GPU line + strong-scaling loads)
#   bench=NAME[@LIB]:ARGS   one bench line (no cpu baseline / whole run) -> bench_TAG_NAME.json; LIB: an A/B library
#   sq=NAME[@KERNEL]:ARGS   SQ counters of the update kernel, or of the kernel whose name contains KERNEL
#                           (scripts/sq_counters.sh)
#   pmc=NAME:ARGS           FETCH/WRITE_SIZE of the update kernel (scripts/pmc.sh)
#   stamps=NAME:VARS        phase stamps (libpgm_stamps.so prebuilt with `python -m pgmorl_amd.build --stamps`,
#                           scripts/stamps.py; VARS = its environment, e.g. ENV=MO-Humanoid-v2,P=20)
#   hv=ENV:ORACLE_JSON      device side of the full-algorithm HV comparison (scripts/hv_full.py)
# ARGS use commas for spaces (e.g. bench=cheetah:--env-name,MO-HalfCheetah-v2,--tasks,20).
set -o pipefail
TAG=$1; shift
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
for step in "$@"; do
  kind=${step%%=*}; val=${step#*=}; [ "$kind" = "$step" ] && val=
  name=${val%%:*}; args=${val#*:}; [ "$args" = "$val" ] && args=; args=${args//,/ }
  echo "== $step"
  case $kind in
    tests)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider ${val//,/ } \
          > $OUT/gpu_tests_$TAG.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR)" $OUT/gpu_tests_$TAG.log | head -20; tail -30 $OUT/gpu_tests_$TAG.log; exit 1; }
      tail -1 $OUT/gpu_tests_$TAG.log ;;
    testlib)
      timeout -k 10 1200 env PGM_LIB=$name python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider $args \
          > $OUT/gpu_tests_${TAG}_ab.log 2>&1 || { echo TESTS FAILED; grep -E "(FAILED|ERROR)" $OUT/gpu_tests_${TAG}_ab.log | head -20; tail -30 $OUT/gpu_tests_${TAG}_ab.log; exit 1; }
      tail -1 $OUT/gpu_tests_${TAG}_ab.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke_$TAG.log; exit 1; }
      tail -1 $OUT/smoke_$TAG.log ;;
    check) bash scripts/round_check.sh $TAG --no-tests || exit 1 ;;
    configs) bash scripts/configs_check.sh $TAG || exit 1 ;;
    bench) lib=; if [ "${name#*@}" != "$name" ]; then lib=${name#*@}; name=${name%@*}; fi
      timeout -k 10 300 env ${lib:+PGM_LIB=$lib} python -u bench.py --no-cpu-baseline --no-whole-run $args > $OUT/bench_${TAG}_$name.json 2> $OUT/bench_${TAG}_$name.err || { echo BENCH $name FAILED; tail -5 $OUT/bench_${TAG}_$name.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/bench_${TAG}_$name.json'));r=d['roofline'];print('$name', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],3),'ms/step', r['kernel'], round(r['avg_launch_ms'],3),'ms frac', round(r['frac'],4))" ;;
    sq) kern=ppo_update; if [ "${name#*@}" != "$name" ]; then kern=${name#*@}; name=${name%@*}; fi
      SQ_KERNEL=$kern bash scripts/sq_counters.sh ${TAG}_$name $args > /dev/null || { echo SQ $name FAILED; exit 1; }
      python -c "import json;d=json.load(open('$OUT/sq_${TAG}_$name.json'));pw=d.get('per_wave',{});sh=d.get('share_of_wave_cycles',{});print('$name', d['kernel'][:60], 'ns', round(d['kernel_ns_profiled']), 'mfma_busy', round(d.get('mfma_busy_share',0),3), 'valu/mfma', round(pw.get('VALU',0)/max(pw.get('MFMA',1),1),2), 'lds_conf', round(d.get('lds_bank_conflict_per_active_lds',0),3), 'wait_any', round(sh.get('SQ_WAIT_ANY',0),3))" ;;
    pmc) bash scripts/pmc.sh ${TAG}_$name $args > /dev/null || { echo PMC $name FAILED; exit 1; }
      python -c "import json;d=json.load(open('$OUT/pmc_${TAG}_$name.json'));print('$name', d['variant'], d['source_hash'], round(d['hbm_bytes_per_launch']/1e9,3),'GB')" ;;
    stamps) timeout -k 10 300 env PGM_LIB=pgmorl_amd/libpgm_stamps.so $args python -u scripts/stamps.py > $OUT/stamps_${TAG}_$name.txt 2>&1 || { echo STAMPS $name FAILED; tail -5 $OUT/stamps_${TAG}_$name.txt; exit 1; }
      tail -4 $OUT/stamps_${TAG}_$name.txt ;;
    hv) timeout -k 10 1100 python -u scripts/hv_full.py device --ref $args --out $OUT/${TAG}_hvfull_$name.json > $OUT/${TAG}_hv_$name.log 2>&1 || { echo HV $name FAILED; tail -20 $OUT/${TAG}_hv_$name.log; exit 1; }
      tail -c 400 $OUT/${TAG}_hv_$name.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo all done
