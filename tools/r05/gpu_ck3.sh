# Round 5: full GPU suite, config4 kernel stats, rank model (after the branch-free load fixes).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ck3
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
    > gpurun_out/ck3/gpu_tests.log 2>&1 || { tail -40 gpurun_out/ck3/gpu_tests.log; exit 1; }
tail -2 gpurun_out/ck3/gpu_tests.log
timeout -k 10 600 python3 -u tools/rank_model.py > gpurun_out/ck3/rank_model.json 2> gpurun_out/ck3/rank_model.err || { tail -20 gpurun_out/ck3/rank_model.err; exit 1; }
tail -c 600 gpurun_out/ck3/rank_model.json
WL=config4 bash tools/r05/gpu_ns_prof.sh > gpurun_out/ck3/nsprof.txt 2>&1 || exit 1
exit 0
