#!/bin/bash
# One gpurun call: all five BASELINE.json configs in both modes (scripts/baseline_configs.py)
# and the 1/10/100/1000-Cron scaling curve (scripts/bench_scale.py).  Stops at the first
# failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/r1s
timeout -k 10 300 python -m cron_operator_amd.ops.build > gpurun_out/r1s/build.log 2>&1 || exit $?
echo "== baseline configs $(date)"
timeout -k 10 900 python -u scripts/baseline_configs.py --out gpurun_out/r1s/baseline_configs.json > gpurun_out/r1s/baseline_configs.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/r1s/baseline_configs.log; [ $rc -eq 0 ] || exit $rc
echo "== scale $(date)"
timeout -k 10 900 python -u scripts/bench_scale.py --steps 3 --warmup 1 --out gpurun_out/r1s/scale.json > gpurun_out/r1s/scale.log 2>&1
rc=$?; echo "rc=$rc"; tail -14 gpurun_out/r1s/scale.log; exit $rc
