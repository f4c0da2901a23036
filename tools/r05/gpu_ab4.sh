# Round 5: the lean MSD pass kernel (k_msd_pass: look-back words read before the next tile's loads,
# branch-free loads, fixed-count scatter) and XCD-grouped tile claims, 2x2 A/B on config3 (+ config2
# for the claims), the ballot ranking's price, then the suites that run the passes.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
N=$PWD/webgpu-radix-sort_amd/lib/librsort.so
soft() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> gpurun_out/soft_failures.txt; if [ $rc -ge 124 ]; then exit $rc; fi; fi; return 0; }
# correctness first (one quick suite on the new default), so a broken kernel stops the call early
timeout -k 10 600 python -u -m pytest tests/test_msd_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t4_msd.log 2>&1 || exit 14
for r in 1 2; do
  for v in osnx os leannx lean; do
    if [ $v = lean ]; then L=$N; else L=$E/librsort_$v.so; fi
    RSORT_LIB=$L soft timeout -k 10 200 python3 bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/ab4_${v}_config3_r$r.json 2> gpurun_out/ab4_${v}_config3_r$r.err
  done
done
for v in osnx lean; do
  if [ $v = lean ]; then L=$N; else L=$E/librsort_$v.so; fi
  RSORT_LIB=$L soft timeout -k 10 200 python3 bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/ab4_${v}_config2.json 2> gpurun_out/ab4_${v}_config2.err
done
for w in config3 config2; do
  RSORT_LIB=$N soft timeout -k 10 200 python3 bench.py --workload $w --rank ballot --no-cpu-baseline --steps 20 > gpurun_out/ab4_ballot_$w.json 2> gpurun_out/ab4_ballot_$w.err
done
RSORT_LIB=$N soft timeout -k 10 200 python3 bench.py --workload config4 --no-cpu-baseline --steps 10 > gpurun_out/ab4_lean_config4.json 2> gpurun_out/ab4_lean_config4.err
timeout -k 10 900 python -u -m pytest tests/test_sort_gpu.py tests/test_split_gpu.py tests/test_region_gpu.py tests/test_robustness_gpu.py tests/test_records_gpu.py tests/test_group_gpu.py tests/test_texture_gpu.py -m "not slow" -x -q --timeout 300 --timeout-method thread > gpurun_out/t4.log 2>&1 || exit 15
exit 0
