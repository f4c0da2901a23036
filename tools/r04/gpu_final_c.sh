# Round 4 final, part C: SQ counters of the hybrid path's kernels (config3), and the split count
# with two halves in flight (variant library) against the default on config4.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/r04/pmc_onesweep.sh
# the split count with two halves in flight (variant library), A/B on config4
E=$PWD/webgpu-radix-sort_amd/lib/exp
RSORT_LIB=$E/librsort_cnt2.so timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_split_cnt2.log 2>&1 || exit 41
for r in 1 2; do
  for v in base cnt2; do
    if [ $v = base ]; then L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; else L=$E/librsort_$v.so; fi
    RSORT_LIB=$L timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline --steps 10 > gpurun_out/c4_${v}_r$r.json 2> gpurun_out/c4_${v}_r$r.err || exit 42
  done
done
exit 0
