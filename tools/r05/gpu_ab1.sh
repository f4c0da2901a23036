# Round 5 A/B: k_onesweep with the explicit vmcnt(0) waits (RS_VMWAIT) and batched staging reads
# (RS_STAGE_BATCH), config3 and config2, two interleaved runs each; then the sort / MSD suites on
# the new default.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
soft() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> gpurun_out/soft_failures.txt; if [ $rc -ge 124 ]; then exit $rc; fi; fi; return 0; }
for r in 1 2; do
  for v in base vm vmnb sb; do
    RSORT_LIB=$E/librsort_$v.so soft timeout -k 10 200 python3 bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/ab_${v}_c3_r$r.json 2> gpurun_out/ab_${v}_c3_r$r.err
  done
done
for v in base vm; do
  RSORT_LIB=$E/librsort_$v.so soft timeout -k 10 200 python3 bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/ab_${v}_c2.json 2> gpurun_out/ab_${v}_c2.err
done
RSORT_LIB=$E/librsort_vm.so timeout -k 10 600 python -u -m pytest tests/test_sort_gpu.py tests/test_msd_gpu.py -m "not slow" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_vm.log 2>&1 || exit 15
exit 0
