# double-buffered k_hist16_in: MSD parity tests, config3 / texture / config2 bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/hd_tests.log 2>&1 || exit 11
: > gpurun_out/hd_bench.jsonl
for wl in config3 config3_texture config2 config3; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 20 >> gpurun_out/hd_bench.jsonl 2>> gpurun_out/hd.err || exit 12
done
