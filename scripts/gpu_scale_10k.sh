#!/bin/bash
# One gpurun call: the Cron-count scaling axis past the headline: 1000, 3000
# and 10000 Crons on the default 3 shard processes, both algorithms at 1000.
#   TAG=r2h bash scripts/gpu_scale_10k.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
TAG=${TAG:-scale10k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1 || exit $?
echo "== 3 shards: 1000 / 3000 / 10000 Crons $(date)"
timeout -k 10 1000 python -u scripts/bench_scale.py --sizes 1000,3000,10000 --modes optimized --shards 3 \
    --steps 3 --warmup 1 --out "$OUT/scale_3shards.json" > "$OUT/scale_3shards.log" 2>&1
rc=$?; echo "rc=$rc"; tail -8 "$OUT/scale_3shards.log"; exit $rc
