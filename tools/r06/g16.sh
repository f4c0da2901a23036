# Round 6: tests of the one-sweep passes (tail barrier), the rank model, SQ counters (config3, region)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sort_gpu.py tests/test_msd_gpu.py tests/test_split_gpu.py tests/test_texture_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t16.log 2>&1 || { tail -30 gpurun_out/t16.log; exit 1; }
tail -2 gpurun_out/t16.log
timeout -k 10 600 python3 -u tools/rank_model.py > gpurun_out/rank_model.json 2> gpurun_out/rank_model.err || exit 2
cat gpurun_out/rank_model.json
timeout -k 10 700 python3 tools/pmc_sq.py config3 gpurun_out/pmc_sq_config3 || exit 3
timeout -k 10 700 python3 tools/pmc_sq.py region gpurun_out/pmc_sq_region || exit 4
