# Round 5: where the workgroups land (XCC_ID vs blockIdx % 8) and the write-pattern probe with both
# groupings; then the lean pass with claims grouped by the hardware XCC_ID vs by blockIdx % 8 vs none.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
N=$PWD/webgpu-radix-sort_amd/lib/librsort.so
soft() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> gpurun_out/soft_failures.txt; if [ $rc -ge 124 ]; then exit $rc; fi; fi; return 0; }
timeout -k 10 150 ./tools/run_probe > gpurun_out/run_probe5.jsonl 2>&1 || exit 10
for r in 1 2; do
  for v in leannx leanhw lean; do
    if [ $v = lean ]; then L=$N; else L=$E/librsort_$v.so; fi
    RSORT_LIB=$L soft timeout -k 10 200 python3 bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/ab5_${v}_config3_r$r.json 2> gpurun_out/ab5_${v}_config3_r$r.err
  done
done
exit 0
