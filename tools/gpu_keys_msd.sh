# keys-only hybrid MSD path: parity tests, config2 bench (512x32 and 1024x16 pass tiles, MSD off)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k keys > gpurun_out/km_tests.log 2>&1 || exit 11
timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/km_c2.json 2> gpurun_out/km.err || exit 12
RSORT_MSD_KEYS_CFG=0 timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/km_c2_wide.json 2>> gpurun_out/km.err || exit 13
RSORT_MSD=0 timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/km_c2_lsd.json 2>> gpurun_out/km.err || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o b --output-format csv -- python3 bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/km_c2_prof.json 2>> gpurun_out/km.err || exit 15
