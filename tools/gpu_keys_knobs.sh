# per-plan keys-path knobs: MSD parity tests incl. the workgroup bucket kernel, config2 full size
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/kk_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u -m pytest tests/test_sort_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config2 or full or baseline" > gpurun_out/kk_tests2.log 2>&1 || exit 12
timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/kk_c2.json 2> gpurun_out/kk.err || exit 13
