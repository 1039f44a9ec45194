#!/bin/bash
# One gpurun call: paired A/B of the driver's own bench invocation (bench.py --gpus 1 --steps 20
# --warmup 5: 3-shard headline, one-process run and reference run in one invocation), base tree in
# ab_base/ (git archive <rev> | tar -x -C ab_base) vs this tree, ROUNDS rounds alternating.
#   TAG=r3k_ab ROUNDS=2 bash scripts/gpu_ab_driver.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-abd}
ROUNDS=${ROUNDS:-2}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
for d in ab_base .; do
  (cd "$d" && timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build_$(basename "$(realpath "$d")").log" 2>&1) || exit $?
done
for i in $(seq "$ROUNDS"); do
  for arm in base head; do
    d=.; [ "$arm" = base ] && d=ab_base
    (cd "$d" && PYTHONPATH=$PWD timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/${arm}_$i.log" 2>&1)
    rc=$?; [ $rc -eq 0 ] || { echo "$arm round $i rc=$rc"; exit $rc; }
    python - "$OUT/${arm}_$i.log" "$arm" "$i" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], sys.argv[3], d["value"], d["operator_cpu_ms_per_fire"], d["single_process_value"],
      d["single_process_operator_cpu_ms_per_fire"], d["single_process_p50_ms"], flush=True)
PY
  done
done
