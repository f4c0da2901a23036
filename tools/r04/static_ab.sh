# Round 4: static-split MSD passes (k_static_pass) - quick parity, then config3 A/B against the
# look-back passes (sweep build, RSORT_STATIC=0/1), then the GPU suites that touch the hybrid path.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_msd_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_msd.log 2>&1 || exit 11
VL=$PWD/webgpu-radix-sort_amd/lib/exp/librsort_sw.so
for r in 1 2; do
  for st in 1 0; do
    RSORT_LIB=$VL RSORT_STATIC=$st timeout -k 10 200 python bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/st${st}_r$r.json 2> gpurun_out/st${st}_r$r.err || exit 12
  done
done
timeout -k 10 200 python bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/prod_c3.json 2> gpurun_out/prod_c3.err || exit 13
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || exit 14
exit 0
