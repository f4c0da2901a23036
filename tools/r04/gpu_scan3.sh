#!/bin/bash
# Round 4: the single-pass scan with LB_FIRST (in-tree library) - scan GPU tests, prefix_sum A/B
# against the previous library, then the final part A (full GPU suite, smoke, bench lines).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_robustness_gpu.py tests/test_sort_gpu.py tests/test_property_gpu.py -k "scan or prefix" > gpurun_out/scan_tests.log 2>&1 || exit 10
for r in 1 2; do
  for v in base new; do
    if [ $v = new ]; then L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; else L=$E/librsort_$v.so; fi
    RSORT_LIB=$L timeout -k 10 200 python bench.py --workload prefix_sum --no-cpu-baseline --steps 20 > gpurun_out/ps_${v}_r$r.json 2> gpurun_out/ps_${v}_r$r.err || exit 11
  done
done
bash tools/r04/gpu_final_a.sh
