#!/bin/bash
# One gpurun call: all five BASELINE.json configs in both modes (scripts/baseline_configs.py),
# the 1/10/100/1000-Cron scaling curve (scripts/bench_scale.py) and a sampled operator
# profile at 1000 Crons.  Stops at the first failing step.
#   TAG=r2e bash scripts/gpu_configs_scale.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
TAG=${TAG:-configs}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1 || exit $?
echo "== baseline configs $(date)"
timeout -k 10 900 python -u scripts/baseline_configs.py --out "$OUT/baseline_configs.json" > "$OUT/baseline_configs.log" 2>&1
rc=$?; echo "rc=$rc"; tail -3 "$OUT/baseline_configs.log"; [ $rc -eq 0 ] || exit $rc
echo "== scale $(date)"
timeout -k 10 900 python -u scripts/bench_scale.py --steps 3 --warmup 1 --out "$OUT/scale.json" > "$OUT/scale.log" 2>&1
rc=$?; echo "rc=$rc"; tail -14 "$OUT/scale.log"; [ $rc -eq 0 ] || exit $rc
echo "== sampled operator profile $(date)"
timeout -k 10 600 python scripts/profile_bench.py --sampler --steps 5 --warmup 2 --top 50 \
    --out "$OUT/operator_sampled_1000crons.txt" > "$OUT/profile.log" 2>&1
rc=$?; echo "rc=$rc"; tail -2 "$OUT/profile.log"; exit $rc
