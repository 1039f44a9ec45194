#!/bin/bash
# One gpurun call: round-3 evidence beyond the checkpoint -- a sampled profile of one operator
# process at 1000 Crons (>= 2000 samples), 80-tick soaks on 3 shards and on one process (native
# connections: flat RSS and CPU per fire), and all five BASELINE.json configs (config 5 trains
# on the MI355X over RCCL).  Heartbeat every 60 s; stops at the first timeout/abort/segfault.
#   TAG=r3d bash scripts/gpu_evidence3.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
export TMPDIR=/tmp
TAG=${TAG:-r3d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }
( while sleep 60; do echo "heartbeat $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT

timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1 || exit $?

echo "== sampled profile, one process, 1000 Crons $(date +%T)"
timeout -k 10 600 python scripts/profile_bench.py --sampler --steps ${PROFILE_STEPS:-40} --warmup 3 --top 60 \
    --out "$OUT/operator_sampled_1000crons.txt" > "$OUT/profile.log" 2>&1
rc=$?; echo "profile rc=$rc"; head -4 "$OUT/operator_sampled_1000crons.txt"; fatal $rc profile

for v in "" "--shards 1"; do
  name=soak80$(echo "$v" | tr -d ' -')
  echo "== soak $v $(date +%T)"
  timeout -k 10 900 python bench.py --steps 80 --warmup 3 --baseline none --single-process none $v \
      --out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
  rc=$?; echo "soak $v rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-240; fatal $rc soak
done

if [ -z "$SKIP_BASELINE_CONFIGS" ]; then
  echo "== all five BASELINE configs $(date +%T)"
  timeout -k 10 1200 python -u scripts/baseline_configs.py --out "$OUT/baseline_configs.json" \
      > "$OUT/baseline_configs.log" 2>&1
  rc=$?; echo "baseline configs rc=$rc"; tail -15 "$OUT/baseline_configs.log"; fatal $rc baseline
fi
echo "== done $(date +%T)"
