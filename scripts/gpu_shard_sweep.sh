#!/bin/bash
# One gpurun call: bench.py across operator shard counts and routings on the same box
# (box-to-box variance is ~15%, so variants are only compared within one call).
#   TAG=r1h bash scripts/gpu_shard_sweep.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
export TMPDIR=/tmp
TAG=${TAG:-sweep}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/prof"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }

echo "== build $(date)"
timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1
rc=$?; echo "build rc=$rc"; fatal $rc build

for v in "--shards 1" "--shards 2 --shard-routing hash" "--shards 2" "--shards 3" "--shards 4" "--shards 6" \
         "--mode reference --shards 1 --steps 3 --warmup 1"; do
  name=$(echo "$v" | tr -d ' -' )
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 $v --out "$OUT/bench_$name.json" > "$OUT/bench_$name.log" 2>&1
  rc=$?; echo "bench $v rc=$rc"; tail -1 "$OUT/bench_$name.log" | cut -c1-200; fatal $rc "bench $v"
done

echo "== profile 4 shards $(date)"
timeout -k 10 600 python scripts/profile_bench.py --shards 4 --out "$OUT/prof/cprofile_4shards.txt" \
    > "$OUT/prof/cprofile.log" 2>&1
rc=$?; echo "cprofile rc=$rc"; fatal $rc cprofile
echo "== done $(date)"

echo "== deployment-shaped configs $(date)"
timeout -k 10 900 python scripts/bench_configs.py --out "$OUT/configs.json" > "$OUT/configs.log" 2>&1
rc=$?; echo "configs rc=$rc"; tail -11 "$OUT/configs.log"; fatal $rc configs
