# Round 4 quick GPU checks: HBM copy ceiling probe, the suites touched this round, the N-rank
# bench rehearsal (2 gloo ranks on GPU 0) with the new multi_gpu breakdown.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 ./tools/copy_probe > gpurun_out/copy_probe.jsonl 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests/test_robustness_gpu.py tests/test_records_gpu.py tests/test_group_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_quick.log 2>&1 || exit 12
timeout -k 10 400 python3 bench.py --gpus 2 --share-gpu --keys-per-gpu 67108864 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err || exit 13
exit 0
