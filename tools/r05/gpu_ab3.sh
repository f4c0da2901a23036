# Round 5: XCD-grouped tile claims in k_onesweep (default) vs one ticket counter (noxcd), config3 /
# config2 / config4, the ballot ranking's price (config3 / config2), then the suites that run k_onesweep on the new library.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
N=$PWD/webgpu-radix-sort_amd/lib/librsort.so
soft() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> gpurun_out/soft_failures.txt; if [ $rc -ge 124 ]; then exit $rc; fi; fi; return 0; }
for r in 1 2; do
  for v in noxcd xcd; do
    if [ $v = noxcd ]; then L=$E/librsort_noxcd.so; else L=$N; fi
    for w in config3 config2; do
      RSORT_LIB=$L soft timeout -k 10 200 python3 bench.py --workload $w --no-cpu-baseline --steps 20 > gpurun_out/ab3_${v}_${w}_r$r.json 2> gpurun_out/ab3_${v}_${w}_r$r.err
    done
  done
done
for w in config3 config2; do
  RSORT_LIB=$N soft timeout -k 10 200 python3 bench.py --workload $w --rank ballot --no-cpu-baseline --steps 20 > gpurun_out/ab3_ballot_$w.json 2> gpurun_out/ab3_ballot_$w.err
done
RSORT_LIB=$N soft timeout -k 10 200 python3 bench.py --workload config4 --no-cpu-baseline --steps 10 > gpurun_out/ab3_xcd_config4.json 2> gpurun_out/ab3_xcd_config4.err
timeout -k 10 900 python -u -m pytest tests/test_sort_gpu.py tests/test_msd_gpu.py tests/test_split_gpu.py tests/test_region_gpu.py tests/test_robustness_gpu.py tests/test_records_gpu.py tests/test_group_gpu.py -m "not slow" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_xcd.log 2>&1 || exit 15
exit 0
