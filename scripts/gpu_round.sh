#!/bin/bash
# One gpurun call: GPU test tier, headline bench, smoke.  Stops at the first
# timeout/abort/segfault (no further GPU steps after a fault).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2; stopping"; exit "$1";; esac; }
echo "== tests $(date)"
timeout -k 10 1500 python -m pytest tests/test_gpu.py -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; fatal $rc tests
echo "== bench $(date)"
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --out gpurun_out/bench_r1.json > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; fatal $rc bench
echo "== smoke $(date)"
timeout -k 10 900 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
