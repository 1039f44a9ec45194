#!/bin/bash
# One gpurun call: reference-algorithm baseline + optimized headline bench on the
# box, a host-side cProfile of the operator, and a rocprofv3 kernel trace of the
# MI355X smoke payload.  Stops at the first timeout/abort/segfault.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }
TAG=${TAG:-r1}

echo "== optimized bench $(date)"
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_opt_$TAG.json > gpurun_out/bench_opt_$TAG.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/bench_opt_$TAG.log; fatal $rc bench-opt

echo "== reference-algorithm bench $(date)"
timeout -k 10 900 python bench.py --steps 3 --warmup 1 --mode reference --out gpurun_out/bench_ref_$TAG.json > gpurun_out/bench_ref_$TAG.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/bench_ref_$TAG.log; fatal $rc bench-ref

echo "== operator cProfile $(date)"
timeout -k 10 600 python scripts/profile_bench.py --out gpurun_out/prof/operator_cprofile_$TAG.txt > gpurun_out/prof/cprofile_$TAG.log 2>&1
rc=$?; echo "rc=$rc"; fatal $rc cprofile

echo "== rocprofv3 smoke payload $(date)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/smoke -o smoke -- \
    python3 -m cron_operator_amd.models.payloads.train_smoke > gpurun_out/prof/rocprof_smoke_$TAG.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/prof/rocprof_smoke_$TAG.log; fatal $rc rocprof
find gpurun_out/prof/smoke -name '*stats*' | head -20
