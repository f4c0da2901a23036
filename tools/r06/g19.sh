# Round 6: the plan fused into k_hist16_reduce: the whole GPU suite, then A/B (packed rows vs + fused
# plan vs + fused plan with the 256 x 18 bucket tile, RSORT_BUCKET_SLACK=1.06)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/ab/fused_tests.log 2>&1 || { tail -30 gpurun_out/ab/fused_tests.log; exit 1; }
tail -2 gpurun_out/ab/fused_tests.log
for r in 1 2 3; do for v in packed fused fused18; do
  L=$E/librsort_${v%18}.so; env=(); [ $v = fused18 ] && env=(RSORT_BUCKET_SLACK=1.06)
  env "${env[@]}" RSORT_LIB=$L timeout -k 10 300 python3 bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/fu_${v}_r$r.json 2>gpurun_out/ab/fu_${v}_r$r.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ab/fu_${v}_r$r.json').read().strip().splitlines()[-1]);print('bench $v',$r,d['ms_per_step'],d['kernel_ms_per_step'])"
done; done
