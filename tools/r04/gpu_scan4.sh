#!/bin/bash
# Round 4: the scan with the next tile's wave scans behind this tile's stores (RS_SCAN_PIPE) and
# without selects on the prefetched values, against the in-tree library: scan GPU tests on the
# variant, then prefix_sum A/B (bench verifies each run).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
RSORT_LIB=$E/librsort_pipe.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_robustness_gpu.py tests/test_sort_gpu.py tests/test_property_gpu.py -k "scan or prefix" > gpurun_out/scan_tests_pipe.log 2>&1 || exit 10
for r in 1 2; do
  for v in base nopipe pipe; do
    if [ $v = base ]; then L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; else L=$E/librsort_$v.so; fi
    RSORT_LIB=$L timeout -k 10 200 python bench.py --workload prefix_sum --no-cpu-baseline --steps 20 > gpurun_out/ps_${v}_r$r.json 2> gpurun_out/ps_${v}_r$r.err || exit 11
  done
done
exit 0
