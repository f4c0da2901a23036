# one-sweep KV tile configurations (RSORT_KV_CFG) on config3 + parity of the one-sweep tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for c in 0 1 4 3 2 0 1; do
  RSORT_KV_CFG=$c timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/kvcfg_$c.json 2> gpurun_out/kvcfg_$c.err || exit 11
  echo "cfg $c $(cut -c1-400 gpurun_out/kvcfg_$c.json)" >> gpurun_out/kvcfg_sweep.txt
done
for c in 1 4; do
RSORT_KV_CFG=$c timeout -k 10 400 python -u -m pytest tests/test_sort_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "onesweep or duplicate_heavy" > gpurun_out/kvcfg_tests_$c.log 2>&1 || exit 12
done
