# Round 5: the real pass kernel at digit widths 8/7/6 (run length 64/128/256 records), then the new
# k_hist16_in (no register folds, double-buffered loads) A/B against the round-4 kernels on config3 /
# config2 / config4, then the suites that exercise the histogram on the new library.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
N=$PWD/webgpu-radix-sort_amd/lib/librsort.so
soft() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> gpurun_out/soft_failures.txt; if [ $rc -ge 124 ]; then exit $rc; fi; fi; return 0; }
timeout -k 10 120 ./tools/run_probe > gpurun_out/run_probe_xcd.jsonl 2>&1 || exit 10
timeout -k 10 120 ./tools/pass_probe > gpurun_out/pass_probe.jsonl 2>&1 || exit 11
timeout -k 10 120 ./tools/pass_probe_novm > gpurun_out/pass_probe_novm.jsonl 2>&1 || exit 12
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then L=$E/librsort_base.so; else L=$N; fi
    for w in config3 config2; do
      RSORT_LIB=$L soft timeout -k 10 200 python3 bench.py --workload $w --no-cpu-baseline --steps 20 > gpurun_out/ab2_${v}_${w}_r$r.json 2> gpurun_out/ab2_${v}_${w}_r$r.err
    done
  done
done
RSORT_LIB=$N soft timeout -k 10 200 python3 bench.py --workload config4 --no-cpu-baseline --steps 10 > gpurun_out/ab2_new_config4.json 2> gpurun_out/ab2_new_config4.err
timeout -k 10 900 python -u -m pytest tests/test_sort_gpu.py tests/test_msd_gpu.py tests/test_split_gpu.py tests/test_region_gpu.py tests/test_robustness_gpu.py tests/test_records_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1 || exit 15
exit 0
