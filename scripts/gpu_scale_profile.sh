#!/bin/bash
# One gpurun call: per-process scaling (100/300/1000 Crons, one operator process) with CPU
# and GC per fire, plus operator cProfiles at 100 and 1000 Crons to locate any per-fire cost
# that grows with the fleet.   TAG=r2b bash scripts/gpu_scale_profile.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
TAG=${TAG:-scale}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }

timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1
rc=$?; echo "build rc=$rc"; fatal $rc build
timeout -k 10 600 python scripts/bench_scale.py --sizes 100,300,1000 --modes optimized --steps 10 --warmup 2 \
    --out "$OUT/scale_1proc.json" > "$OUT/scale_1proc.log" 2>&1
rc=$?; echo "scale rc=$rc"; grep "n=" "$OUT/scale_1proc.log"; fatal $rc scale
for n in 100 1000; do
  steps=$(( n == 100 ? 30 : 3 ))
  timeout -k 10 600 python scripts/profile_bench.py --crons $n --steps $steps --warmup 2 --out "$OUT/prof_$n.txt" \
      > "$OUT/prof_$n.log" 2>&1
  rc=$?; echo "profile $n rc=$rc"; sed -n 2,3p "$OUT/prof_$n.txt"; fatal $rc "profile $n"
done
