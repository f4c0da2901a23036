# Round 6 A/B: bench lines of one library under rs_plan_debug overrides.
#   bash tools/r06/ab.sh <tag> <workload> <reps> "<debug A>" "<debug B>" ...   (debug "" = defaults)
# Results: gpurun_out/ab/<tag>_<workload>_<i>_r<rep>.json; a summary line per run on stdout.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
tag=$1; w=$2; reps=$3; shift 3
for r in $(seq 1 $reps); do
  i=0
  for d in "$@"; do
    i=$((i + 1))
    f=gpurun_out/ab/${tag}_${w}_${i}_r$r
    dbg=(); [ -n "$d" ] && dbg=(--plan-debug "$d")
    timeout -k 10 300 python3 bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline "${dbg[@]}" \
        > $f.json 2> $f.err || { echo "FAILED $f rc=$?"; tail -5 $f.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$f.json').read().strip().splitlines()[-1])
k=d.get('kernel_ms_per_step',{}); rf=d.get('roofline',{})
print('$w', 'dbg=[$d]', 'r$r', 'ms', d['ms_per_step'], 'Gk/s', d['value'], 'roof', rf.get('avg_launch_ms'), rf.get('frac'), 'kern', json.dumps(k))"
  done
done
exit 0
