#!/bin/bash
# One gpurun call: GPU test tier, headline bench, scaling curve, operator profile,
# rocprofv3 of the scheduled MI355X payload, smoke.  Stops at the first
# timeout/abort/segfault (no further GPU steps after a fault).
#   TAG=r1c bash scripts/gpu_round.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/prof"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }

echo "== build $(date)"
timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1
rc=$?; echo "build rc=$rc"; fatal $rc build

echo "== gpu tests $(date)"
timeout -k 10 900 python -m pytest tests/test_gpu.py -m gpu -x -q -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; fatal $rc tests

echo "== bench $(date)"
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log"; fatal $rc bench

echo "== bench variants $(date)"
for v in "--shards 1" "--mode reference --shards 1 --steps 3 --warmup 1" "--mode reference --shards 2 --steps 3 --warmup 1"; do
  name=$(echo "$v" | tr -d ' -' )
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 $v --out "$OUT/bench_$name.json" > "$OUT/bench_$name.log" 2>&1
  rc=$?; echo "bench $v rc=$rc"; tail -1 "$OUT/bench_$name.log" | cut -c1-330; fatal $rc "bench $v"
done

echo "== scale $(date)"
timeout -k 10 900 python scripts/bench_scale.py --steps 3 --warmup 1 --out "$OUT/scale.json" > "$OUT/scale.log" 2>&1
rc=$?; echo "scale rc=$rc"; tail -12 "$OUT/scale.log"; fatal $rc scale

echo "== operator cProfile $(date)"
timeout -k 10 600 python scripts/profile_bench.py --out "$OUT/prof/operator_cprofile.txt" > "$OUT/prof/cprofile.log" 2>&1
rc=$?; echo "cprofile rc=$rc"; fatal $rc cprofile

echo "== rocprofv3 smoke payload $(date)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof/smoke" -o smoke -- \
    python3 -m cron_operator_amd.models.payloads.train_smoke > "$OUT/prof/rocprof_smoke.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof

echo "== smoke $(date)"
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"
