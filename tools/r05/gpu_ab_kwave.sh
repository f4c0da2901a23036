# Round 5: keys wave bucket kernel with the next bucket's count/base prefetched and branch-free
# stores (new) against the committed library (prev): keys tests, then config2 A/B.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abkw
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_msd_gpu.py tests/test_sort_gpu.py \
    > gpurun_out/abkw/tests.log 2>&1 || { tail -30 gpurun_out/abkw/tests.log; exit 1; }
tail -1 gpurun_out/abkw/tests.log
for r in 1 2; do for v in prev new; do
  lib=ab_lib/librsort_$v.so; [ $v = new ] && lib=webgpu-radix-sort_amd/lib/librsort.so
  RSORT_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload config2 --steps 30 --warmup 3 --no-cpu-baseline \
      > gpurun_out/abkw/config2_${v}_r$r.json 2> gpurun_out/abkw/config2_${v}_r$r.err || { tail -5 gpurun_out/abkw/config2_${v}_r$r.err; exit 1; }
done; done
exit 0
