#!/bin/bash
# One gpurun call at the round-3 final head: the GPU tier, smoke and rocprof checkpoint with the
# driver's bench invocation (scripts/gpu_check3.sh), an 80-tick 3-shard soak (peak RSS per shard)
# and all five BASELINE configs in both reconciler modes.  Stops at the first fault.
#   TAG=r3v bash scripts/gpu_final3.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
TAG=${TAG:-r3final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }
TAG=$TAG SKIP_SCALE=1 SKIP_CONFIGS=1 timeout -k 10 600 bash scripts/gpu_check3.sh
rc=$?; fatal $rc checkpoint; [ $rc -eq 0 ] || exit $rc
( while sleep 60; do echo "heartbeat $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== soak, 3 shards, 80 ticks $(date +%T)"
timeout -k 10 600 python bench.py --steps 80 --warmup 3 --baseline none --single-process none \
    --out "$OUT/soak80.json" > "$OUT/soak80.log" 2>&1
rc=$?; echo "soak rc=$rc"; tail -1 "$OUT/soak80.log" | cut -c1-240; fatal $rc soak
echo "== all five BASELINE configs $(date +%T)"
timeout -k 10 900 python -u scripts/baseline_configs.py --out "$OUT/baseline_configs.json" \
    > "$OUT/baseline_configs.log" 2>&1
rc=$?; echo "baseline configs rc=$rc"; tail -15 "$OUT/baseline_configs.log"; fatal $rc baseline
echo "== done $(date +%T)"
