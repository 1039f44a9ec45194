#!/bin/bash
# One gpurun call at a round-3 checkpoint: build, GPU test tier, smoke, rocprofv3 of the smoke
# payload, the driver's bench invocation, the 1/10/100/1000-Cron curve and the
# deployment-shaped configs.  A heartbeat line every 60 s keeps long steps visibly alive.
# Stops at the first timeout/abort/segfault (no further GPU steps after a fault).
#   TAG=r3c bash scripts/gpu_check3.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
export TMPDIR=/tmp
TAG=${TAG:-r3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/prof"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }
( while sleep 60; do echo "heartbeat $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT

echo "== build $(date +%T)"
timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1
rc=$?; echo "build rc=$rc"; fatal $rc build; [ $rc -eq 0 ] || exit $rc

echo "== gpu tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; fatal $rc tests

echo "== smoke $(date +%T)"
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; fatal $rc smoke

echo "== rocprofv3 smoke payload $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof/smoke" -o smoke -- \
    python3 -m cron_operator_amd.models.payloads.train_smoke > "$OUT/prof/rocprof_smoke.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof

echo "== bench, driver invocation $(date +%T)"
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 --out "$OUT/bench_driver.json" > "$OUT/bench_driver.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench_driver.log" | cut -c1-300; fatal $rc bench

if [ -z "$SKIP_SCALE" ]; then
  echo "== scale curve $(date +%T)"
  timeout -k 10 900 python -u scripts/bench_scale.py --steps 3 --warmup 1 --out "$OUT/scale.json" > "$OUT/scale.log" 2>&1
  rc=$?; echo "scale rc=$rc"; tail -12 "$OUT/scale.log"; fatal $rc scale
fi

if [ -z "$SKIP_CONFIGS" ]; then
  echo "== deployment-shaped configs $(date +%T)"
  timeout -k 10 1500 python -u scripts/bench_configs.py ${CONFIGS:+--only $CONFIGS} --out "$OUT/bench_configs.json" \
      > "$OUT/bench_configs.log" 2>&1
  rc=$?; echo "configs rc=$rc"; tail -20 "$OUT/bench_configs.log"; fatal $rc configs
fi
echo "== done $(date +%T)"
