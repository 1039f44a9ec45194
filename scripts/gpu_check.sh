#!/bin/bash
# One gpurun call: build, GPU test tier, headline bench (default + 1 shard), smoke,
# rocprofv3 of the smoke payload.  Stops at the first timeout/abort/segfault.
#   TAG=r1n bash scripts/gpu_check.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
export TMPDIR=/tmp
TAG=${TAG:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/prof"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }

echo "== build $(date)"
timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1
rc=$?; echo "build rc=$rc"; fatal $rc build

echo "== gpu tests $(date)"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; fatal $rc tests

# the driver's invocation (reference baseline measured in the same run), then shard variants
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 --out "$OUT/bench_driver.json" \
    > "$OUT/bench_driver.log" 2>&1
rc=$?; echo "bench driver-shape rc=$rc"; tail -1 "$OUT/bench_driver.log" | cut -c1-400; fatal $rc "bench driver"
for v in "--shards 1" "--shards 4"; do
  name=$(echo "default$v" | tr -d ' -' )
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --baseline none $v --out "$OUT/bench_$name.json" \
      > "$OUT/bench_$name.log" 2>&1
  rc=$?; echo "bench $v rc=$rc"; tail -1 "$OUT/bench_$name.log" | cut -c1-200; fatal $rc "bench $v"
done

echo "== per-process scaling 100 vs 1000 $(date)"
timeout -k 10 600 python scripts/bench_scale.py --sizes 100,1000 --modes optimized --steps 5 --warmup 2 \
    --out "$OUT/scale_1proc.json" > "$OUT/scale_1proc.log" 2>&1
rc=$?; echo "scale rc=$rc"; tail -6 "$OUT/scale_1proc.log"; fatal $rc scale

echo "== smoke $(date)"
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; fatal $rc smoke

echo "== rocprofv3 smoke payload $(date)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof/smoke" -o smoke -- \
    python3 -m cron_operator_amd.models.payloads.train_smoke > "$OUT/prof/rocprof_smoke.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
echo "== done $(date)"
