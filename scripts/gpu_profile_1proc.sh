#!/bin/bash
# One gpurun call: GPU test tier, the shipped-default single-process bench, and a
# statistical profile (>= 2000 SIGPROF samples) of that one operator process at 1000 Crons.
#   TAG=r3a bash scripts/gpu_profile_1proc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
TAG=${TAG:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > "$OUT/gpu_tests.log" 2>&1 && tail -2 "$OUT/gpu_tests.log" &&
timeout -k 10 300 python bench.py --shards 1 --steps 10 --warmup 3 --baseline none > "$OUT/bench_1shard.log" 2>&1 &&
tail -1 "$OUT/bench_1shard.log" | cut -c1-300 &&
timeout -k 10 400 python scripts/profile_bench.py --sampler --steps ${PROF_STEPS:-40} --warmup 3 --top 60 \
    --out "$OUT/sampled_1proc.txt" > "$OUT/prof.log" 2>&1 && head -4 "$OUT/sampled_1proc.txt"
