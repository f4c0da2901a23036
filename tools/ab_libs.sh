# A/B bench lines of library variants and / or rs_plan_debug settings, alternated on one box
# (box-to-box spread of one library is ~1 %, so only same-box comparisons count).
#   bash tools/ab_libs.sh <tag> <workload> <reps> <variant> [<variant> ...]
# A variant is `lib` (the in-tree library), `lib:<name>` (webgpu-radix-sort_amd/lib/exp/
# librsort_<name>.so, built by tools/build_variants.sh with OUTD=../lib/exp - list that directory out
# of .gpurunignore for the call), optionally followed by `@<plan-debug fields>` (bench.py
# --plan-debug, e.g. lib@xcd=1 or lib:fused@split=0).  GPU box, from the repo root.
# Results: gpurun_out/ab/<tag>_<workload>_<i>_r<rep>.json; one summary line per run on stdout.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
tag=$1; w=$2; reps=$3; shift 3
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in $(seq 1 "$reps"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    lib=${v%%@*}; dbg=""; [ "$lib" != "$v" ] && dbg=${v#*@}
    L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ "$lib" != lib ] && L=$E/librsort_${lib#lib:}.so
    f=gpurun_out/ab/${tag}_${w}_${i}_r$r
    args=(); [ -n "$dbg" ] && args=(--plan-debug "$dbg")
    RSORT_LIB=$L timeout -k 10 300 python3 bench.py --workload "$w" --steps 20 --warmup 3 --no-cpu-baseline \
        "${args[@]}" > $f.json 2> $f.err || { echo "FAILED $f"; tail -5 $f.err; exit 1; }
    python3 -c "
import json
d = json.loads(open('$f.json').read().strip().splitlines()[-1])
rf = d.get('roofline', {})
print('$w', '$v', 'r$r', 'ms', d['ms_per_step'], 'Gk/s', d['value'], 'roof', rf.get('avg_launch_ms'), rf.get('frac'),
      'kern', json.dumps(d.get('kernel_ms_per_step', {})))"
  done
done
exit 0
