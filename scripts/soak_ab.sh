set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n
(cd ab_base && timeout -k 10 300 python -m cron_operator_amd.ops.build > /dev/null 2>&1) || exit 1
for i in 1 2; do
  for arm in head base; do
    d=.; [ $arm = base ] && d=ab_base
    extra=""; [ $arm = head ] && extra="--deployment none"
    (cd $d && PYTHONPATH=$PWD timeout -k 10 400 python bench.py --steps 80 --warmup 3 --baseline none --single-process none $extra --out "$GRAFT_REPO_ROOT/gpurun_out/r4n/${arm}_$i.json" > /dev/null 2>&1) || exit 1
    python -c "
import json,statistics; d=json.load(open('gpurun_out/r4n/${arm}_$i.json')); s=d['summary']; st=d['rank0']['step_ms']
print('$arm', $i, s['value'], s['operator_cpu_ms_per_fire'], s['apiserver_busy_frac'], [round(statistics.mean(st[j:j+20])) for j in range(0,80,20)], flush=True)"
  done
done
