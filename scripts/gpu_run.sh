#!/bin/bash
# One gpurun call.  STEPS selects what runs (space-separated):
#   tests   GPU test tier (payload on the MI355X), smoke()
#   bench   the driver's bench invocation (20 timed steps), JSON kept
#   configs deployment-shaped rows (etcd latency, TLS, chart defaults at 1000 Crons)
#   rocprof kernel stats of the scheduled payload (rocprofv3 --kernel-trace --stats)
#   soak    200 ticks, 3 shards (SOAK_PARTITIONS fake apiservers, default 3: the headline's layout),
#           20-tick windows: step time, operator and fixture CPU per fire,
#           fixture counters, box calibrations (scripts/soak_windows.py)
#   baseline all five BASELINE.json configs in both reconciler modes (scripts/baseline_configs.py)
#   scale   cron-reconciles/s at 1 / 10 / 100 / 1000 Crons, both modes (scripts/bench_scale.py)
#   scale10k  10000 Crons, this operator only: one process and 3 shards (peak RSS)
#   shards10k  10000 Crons, 3 label-routed shard processes on a first start (peak RSS per shard)
#   routing label vs hash routing on 3 shards, REPS alternating pairs at ROUTING_SIZES Crons (default 3000)
#   mem10k  10000 Crons, the operator in its own process: peak RSS with a shared and with distinct templates
#   split   fixture vs operator CPU, native and Python fake apiserver, 3 shards and one process
#           (scripts/fixture_split.py; REPS alternating repetitions)
#   ranks   the driver's multi-rank line (torch.distributed.run, N=2 and 4 CPU-only ranks): the
#           N=8 scaling run is the driver's; RANKS overrides the list
# Stops at the first failure; every GPU step has its own time limit.
#   TAG=r4a STEPS="tests bench" bash scripts/gpu_run.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
export TMPDIR=/tmp
TAG=${TAG:-r4}
STEPS=${STEPS:-"tests bench"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { echo "== $1 $(date +%T)"; }
check() { local rc=$1; echo "$2 rc=$rc"; [ "$rc" = 0 ] || exit "$rc"; }

for s in $STEPS; do
  case $s in
    tests)
      step "gpu tests"
      timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v -p no:cacheprovider \
        --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
      check $? tests; tail -3 "$OUT/gpu_tests.log"
      step smoke
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      check $? smoke; tail -3 "$OUT/smoke.log" ;;
    bench)
      step bench
      timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 --out "$OUT/bench.json" \
        > "$OUT/bench.log" 2> "$OUT/bench.err"
      check $? bench; cat "$OUT/bench.err"; tail -1 "$OUT/bench.log" | cut -c1-600 ;;
    configs)
      step configs
      timeout -k 10 1100 python -u scripts/bench_configs.py --only "${CONFIGS:-etcd-latency,chart-defaults-1000}" \
        ${CONFIG_MODE:+--mode $CONFIG_MODE} --out "$OUT/configs.json" > "$OUT/configs.log" 2>&1
      check $? configs; tail -8 "$OUT/configs.log" ;;
    rocprof)
      step rocprof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o payload -- \
        python -m cron_operator_amd.models.payloads.train_smoke > "$OUT/rocprof.log" 2>&1
      check $? rocprof; find "$OUT/prof" -name "*kernel_stats.csv" | head -2 ;;
    soak)
      step soak
      timeout -k 10 600 python -u scripts/soak_windows.py --steps 200 --partitions "${SOAK_PARTITIONS:-3}" \
        --out "$OUT/soak200.json" \
        > "$OUT/soak200.log" 2>&1
      check $? soak; tail -1 "$OUT/soak200.log" | cut -c1-400 ;;
    baseline)
      step baseline
      timeout -k 10 900 python -u scripts/baseline_configs.py --out "$OUT/baseline_configs.json" \
        > "$OUT/baseline_configs.log" 2>&1
      check $? baseline; tail -15 "$OUT/baseline_configs.log" ;;
    scale)
      step scale
      timeout -k 10 900 python -u scripts/bench_scale.py --steps 3 --warmup 1 --out "$OUT/scale.json" \
        > "$OUT/scale.log" 2>&1
      check $? scale; tail -12 "$OUT/scale.log" ;;
    scale10k)
      step scale10k
      timeout -k 10 900 python -u scripts/bench_scale.py --sizes 10000 --modes optimized --steps 3 --warmup 1 \
        --out "$OUT/scale10k.json" > "$OUT/scale10k.log" 2>&1
      check $? scale10k; tail -4 "$OUT/scale10k.log"
      timeout -k 10 900 python -u scripts/bench_scale.py --sizes 10000 --modes optimized --steps 3 --warmup 1 \
        --shards 3 --out "$OUT/scale10k_3shards.json" > "$OUT/scale10k_3shards.log" 2>&1
      check $? scale10k_3shards; tail -4 "$OUT/scale10k_3shards.log" ;;
    shards10k)
      step shards10k
      timeout -k 10 900 python -u scripts/bench_scale.py --sizes 10000 --modes optimized --steps 5 --warmup 1 \
        --shards 3 --out "$OUT/shards10k.json" > "$OUT/shards10k.log" 2>&1
      check $? shards10k; tail -4 "$OUT/shards10k.log" ;;
    routing)
      # alternating pairs (REPS of them): the box's run-to-run spread is larger than one pair shows
      for i in $(seq 1 "${REPS:-1}"); do
        for r in labels hash; do
          step "routing $r $i"
          timeout -k 10 900 python -u scripts/bench_scale.py --sizes "${ROUTING_SIZES:-3000}" --modes optimized \
            --steps 5 --warmup 1 --shards 3 --shard-routing $r --out "$OUT/routing_${r}_$i.json" \
            > "$OUT/routing_${r}_$i.log" 2>&1
          check $? "routing $r"; grep "n=" "$OUT/routing_${r}_$i.log"
        done
      done ;;
    mem10k)
      # peak RSS of the operator alone (its own process) at 10,000 Crons / 110,000 jobs over 10
      # ticks: one template shared by every Cron, then a distinct template per Cron
      # (MEM_VARIANTS overrides the list; "--lifecycle realistic": the training-operator's status sequence)
      old_ifs=$IFS; IFS=';'
      for c in ${MEM_VARIANTS:-";--distinct-templates"}; do
        IFS=$old_ifs
        tag=$(echo "$c" | tr -c 'a-z0-9' '_' | sed 's/^_*//; s/_*$//')
        step "mem10k $c"
        timeout -k 10 600 python -u scripts/bench_scale.py --sizes 10000 --modes optimized --steps 10 --warmup 1 \
          --operator-process $c --out "$OUT/mem10k${tag:+_$tag}.json" > "$OUT/mem10k${tag:+_$tag}.log" 2>&1
        check $? "mem10k $c"; head -1 "$OUT/mem10k${tag:+_$tag}.log"
        IFS=';'
      done
      IFS=$old_ifs ;;
    split)
      step split
      timeout -k 10 900 python -u scripts/fixture_split.py --reps "${REPS:-1}" --out "$OUT/split.json" \
        > "$OUT/split.log" 2>&1
      check $? split; cut -c1-400 "$OUT/split.log" ;;
    ranks)
      for n in ${RANKS:-2 4}; do
        step "ranks $n"
        timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
          --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus "$n" --steps 20 --warmup 5 \
          --out "$OUT/ranks$n.json" > "$OUT/ranks$n.log" 2> "$OUT/ranks$n.err"
        check $? "ranks $n"; grep '^{' "$OUT/ranks$n.log" | cut -c1-400
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
