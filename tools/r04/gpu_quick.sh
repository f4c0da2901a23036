# Round 4 quick GPU checks: HBM copy ceiling probe, k_onesweep phase stamps on the hybrid path
# (default and RS_AHEAD), A/B of variant libraries on config3, the single-pass prefix sum bench, the
# suites touched this round, the N-rank bench rehearsal (2 gloo ranks on GPU 0).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
# a variant run that fails its own checks is recorded and skipped; a crash / abort / timeout ends the call
soft() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> gpurun_out/soft_failures.txt; if [ $rc -ge 124 ]; then exit $rc; fi; fi; return 0; }
timeout -k 10 120 ./tools/copy_probe > gpurun_out/copy_probe.jsonl 2>&1 || exit 11
RSORT_LIB=$E/librsort_st.so soft timeout -k 10 200 python3 tools/stamp_probe_msd.py > gpurun_out/stamps_msd.jsonl 2> gpurun_out/stamps_msd.err
RSORT_LIB=$E/librsort_ahst.so soft timeout -k 10 200 python3 tools/stamp_probe_msd.py > gpurun_out/stamps_msd_ahead.jsonl 2> gpurun_out/stamps_msd_ahead.err
for r in 1 2; do
  for v in base ah bk3p bk4p; do
    if [ $v = base ]; then L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; else L=$E/librsort_$v.so; fi
    RSORT_LIB=$L soft timeout -k 10 200 python3 bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/ab_${v}_r$r.json 2> gpurun_out/ab_${v}_r$r.err
  done
done
soft timeout -k 10 300 python3 bench.py --workload prefix_sum --steps 10 > gpurun_out/prefix_sum.json 2> gpurun_out/prefix_sum.err
timeout -k 10 600 python -u -m pytest tests/test_robustness_gpu.py tests/test_records_gpu.py tests/test_group_gpu.py -m "not slow" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_quick.log 2>&1 || exit 15
timeout -k 10 400 python3 bench.py --gpus 2 --share-gpu --keys-per-gpu 67108864 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err || exit 16
exit 0
