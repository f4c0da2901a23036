# Round 4: bucket split v2 (contiguous count ranges, sub-bucket-per-workgroup grid) and the
# 16K-element single-pass scan: parity suites, config4 / prefix_sum / config3 lines, config4 trace.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_split.log 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest tests/test_robustness_gpu.py tests/test_property_gpu.py tests/test_sort_gpu.py -k "scan or prefix" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_scan.log 2>&1 || exit 12
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline --steps 10 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 13
timeout -k 10 300 python bench.py --workload prefix_sum --no-cpu-baseline --steps 20 > gpurun_out/ps.json 2> gpurun_out/ps.err || exit 14
timeout -k 10 200 python bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 15
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 --output-format csv -- python3 bench.py --workload config4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prof_c4.log 2>&1 || exit 16
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in 1 2; do
  RSORT_LIB=$E/librsort_ah.so timeout -k 10 200 python bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/ab_ah_r$r.json 2> gpurun_out/ab_ah_r$r.err || exit 17
  timeout -k 10 200 python bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/ab_base_r$r.json 2> gpurun_out/ab_base_r$r.err || exit 18
done
timeout -k 10 300 python3 -u tools/rank_model.py --reps 5 > gpurun_out/rank_base.json 2> gpurun_out/rank_base.err || exit 19
RSORT_LIB=$E/librsort_wg.so timeout -k 10 300 python3 -u tools/rank_model.py --reps 5 > gpurun_out/rank_wg.json 2> gpurun_out/rank_wg.err || exit 20
exit 0
