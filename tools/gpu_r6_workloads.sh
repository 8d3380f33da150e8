#!/bin/bash
# round 6: bench.py --workload lines (1 GPU) with rocprofv3 kernel stats and PMC passes of the same commands
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wl
export TMPDIR=/tmp
declare -A ARGS=( [config2]="--warmup 10 --steps 190" [config4]="--warmup 0 --steps 140" [selfstart]="--warmup 0 --steps 40"
                  [config5]="--warmup 0 --steps 60" )
declare -A WLS=( [config2]="4096:190:10:1:config2" [config4]="16384:140:0:1:config4" [selfstart]="16384:40:0:1:selfstart"
                 [config5]="65536:60:0:1:config5" )
MODE=${MODE:-lines}
for w in ${WORKLOADS:-config2 config4 selfstart config5}; do
  a="--workload $w ${ARGS[$w]} --no-cpu-baseline --no-ring"
  if [ "$MODE" = lines ] || [ "$MODE" = all ]; then
    timeout -k 10 400 python -u bench.py $a > gpurun_out/wl/$w.json 2> gpurun_out/wl/$w.err
    rc=$?; echo "bench $w rc=$rc" >> gpurun_out/wl/$w.err; [ $rc -eq 0 ] || exit $rc
  fi
  if [ "$MODE" = prof ] || [ "$MODE" = all ]; then
    bash tools/gpu_r6_prof.sh $w $a || exit 1
  fi
  if [ "$MODE" = pmc ] || [ "$MODE" = all ]; then
    i=0
    for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"; do
      i=$((i+1))
      timeout -k 10 -s KILL 300 rocprofv3 --pmc $pass --kernel-trace -d /tmp/pmc_${w}_$i -o run \
        --output-format csv -- python3 bench.py $a > gpurun_out/wl/pmc_${w}_$i.log 2>&1
      rc=$?; echo "pmc $w pass $i rc=$rc" >> gpurun_out/wl/pmc_${w}_$i.log; [ $rc -eq 0 ] || exit $rc
    done
    dirs=""
    for k in $(seq 1 $i); do dirs="$dirs $(dirname $(ls /tmp/pmc_${w}_$k/*/run_counter_collection.csv /tmp/pmc_${w}_$k/run_counter_collection.csv 2>/dev/null | head -n 1))"; done
    python3 tools/pmc_summary.py --workload ${WLS[$w]} --window gpurun_out/wl/pmc_summary_$w.json $dirs || exit 1
  fi
done
exit 0
