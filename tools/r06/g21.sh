# Round 6: k_msd_pass with the first look-back round issued before the staging (RS_MSD_LBEARLY)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
RSORT_LIB=$E/librsort_early.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_msd_gpu.py > gpurun_out/ab/early_tests.log 2>&1 || { tail -30 gpurun_out/ab/early_tests.log; exit 1; }
tail -1 gpurun_out/ab/early_tests.log
for r in 1 2 3; do for v in base early; do
  RSORT_LIB=$E/librsort_$v.so timeout -k 10 300 python3 bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/ea_${v}_r$r.json 2>gpurun_out/ab/ea_${v}_r$r.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ab/ea_${v}_r$r.json').read().strip().splitlines()[-1]);print('bench $v',$r,d['ms_per_step'],d['roofline']['avg_launch_ms'],d['kernel_ms_per_step']['scatter'])"
done; done
