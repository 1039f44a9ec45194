#!/bin/bash
# One gpurun call: bench.py at --gpus 1, 2 and 4 on the 1-GPU box (the ranks are CPU-only
# operator shards, see bench.py), as a rehearsal of the driver's multi-rank scaling run.
# No rank touches the GPU; the N=8 run is the driver's.
#   TAG=r2f bash scripts/gpu_rank_rehearsal.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
TAG=${TAG:-ranks}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "cpus: nproc=$(nproc) affinity=$(python -c 'import os; print(len(os.sched_getaffinity(0)))')"
timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build.log" 2>&1 || exit $?
for n in 1 2 4; do
  echo "== --gpus $n $(date)"
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 --baseline none \
      > "$OUT/bench_gpus$n.log" 2>&1
  rc=$?; echo "rc=$rc"; grep '^{' "$OUT/bench_gpus$n.log" | tail -1 | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
