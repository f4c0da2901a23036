# Round 4: split run list with parallel emission, config4 line + trace; scan default (1024 x 32) and
# 40 / 48-element variants.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_split.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline --steps 10 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 --output-format csv -- python3 bench.py --workload config4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prof_c4.log 2>&1 || exit 16
timeout -k 10 400 python -u -m pytest tests/test_robustness_gpu.py tests/test_property_gpu.py tests/test_sort_gpu.py -k "scan or prefix" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_scan.log 2>&1 || exit 12
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in 1 2; do
  for v in base s40 s48; do
    if [ $v = base ]; then L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; else L=$E/librsort_$v.so; fi
    RSORT_LIB=$L timeout -k 10 200 python bench.py --workload prefix_sum --no-cpu-baseline --steps 20 > gpurun_out/ps_${v}_r$r.json 2> gpurun_out/ps_${v}_r$r.err || exit 17
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o ps --output-format csv -- python3 bench.py --workload prefix_sum --no-cpu-baseline --steps 10 > gpurun_out/prof_ps.log 2>&1 || exit 18
exit 0
