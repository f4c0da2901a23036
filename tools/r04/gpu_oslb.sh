#!/bin/bash
# Round 4: k_onesweep with its first look-back window read before the next tile's loads (buffer-
# descriptor prefetch, RS_OS_LB_FIRST) against the in-tree library: sort / MSD GPU tests on the
# variant, then config3 / config2 / config4 A/B (bench verifies each run).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
RSORT_LIB=$E/librsort_oslb1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_sort_gpu.py tests/test_msd_gpu.py > gpurun_out/oslb_tests.log 2>&1 || exit 10
for r in 1 2; do
  for v in base oslb1; do
    if [ $v = base ]; then L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; else L=$E/librsort_$v.so; fi
    for wl in config3 config2 config4; do
      RSORT_LIB=$L timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 10 > gpurun_out/${wl}_${v}_r$r.json 2> gpurun_out/${wl}_${v}_r$r.err || exit 11
    done
  done
done
exit 0
