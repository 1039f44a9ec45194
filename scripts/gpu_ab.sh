#!/bin/bash
# One gpurun call: paired A/B of the 1-process 1000-Cron bench on the box.  ab_base/ holds an
# older tree (git archive <rev> | tar -x -C ab_base; git-ignored, shipped with the snapshot).
# ARMS lists the arms run in turn each round: "base", "head", "head:VAR=value" (head with an
# environment override, e.g. head:CRON_OPERATOR_NATIVE_HTTP=python) or "head@--arg=v,--flag" /
# "base@--arg=v" (that tree with extra bench.py arguments, comma-separated).
#   TAG=r3b ROUNDS=4 ARMS="base head:CRON_OPERATOR_NATIVE_HTTP=python head" bash scripts/gpu_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-ab}
ROUNDS=${ROUNDS:-4}
ARMS=${ARMS:-base head}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
for d in ab_base .; do
  [ "$d" = ab_base ] && [[ " $ARMS " != *" base "* && " $ARMS " != *" base@"* ]] && continue
  (cd "$d" && timeout -k 10 300 python -m cron_operator_amd.ops.build > "$OUT/build_$(basename "$(realpath "$d")").log" 2>&1) || exit $?
done
for i in $(seq "$ROUNDS"); do
  for arm in $ARMS; do
    d=.; envs=(); extra=()
    case "$arm" in
      base) d=ab_base ;;
      base@*) d=ab_base; IFS=, read -r -a extra <<< "${arm#base@}" ;;
      head:*) envs=("${arm#head:}") ;;
      head@*) IFS=, read -r -a extra <<< "${arm#head@}" ;;
    esac
    name=$(echo "$arm" | tr ':=@,' '____' | tr -d '-')
    (cd "$d" && env "${envs[@]}" PYTHONPATH=$PWD timeout -k 10 300 python bench.py --shards ${SHARDS:-1} --steps 10 \
        --warmup 3 --baseline none --single-process none $([ "$d" = . ] && echo --deployment none --payload-probe none) "${extra[@]}" \
        > "$OUT/${name}_$i.log" 2>&1)
    rc=$?; [ $rc -eq 0 ] || { echo "$name round $i rc=$rc"; exit $rc; }
    python - "$OUT/${name}_$i.log" "$name" "$i" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], sys.argv[3], d["value"], d["operator_cpu_ms_per_fire"], d["p50_schedule_to_create_ms"], flush=True)
PY
  done
done
