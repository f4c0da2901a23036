# keys-only MSD pass tiles: 512x32 (default) / 1024x16 / 1024x32, config2 bench + parity
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "keys" > gpurun_out/km4_tests.log 2>&1 || exit 11
: > gpurun_out/km4_sweep.jsonl
for cfg in "RSORT_MSD_KEYS_CFG=1" "RSORT_MSD_KEYS_CFG=2" "RSORT_MSD_KEYS_CFG=0" "RSORT_MSD_KEYS_CFG=2" "RSORT_MSD_KEYS_CFG=1"; do
  echo "{\"cfg\": \"$cfg\"}" >> gpurun_out/km4_sweep.jsonl
  env $cfg timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 >> gpurun_out/km4_sweep.jsonl 2>> gpurun_out/km4.err || exit 12
done
