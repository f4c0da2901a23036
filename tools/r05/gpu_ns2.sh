# Round 5: presorted path parity tests + kernel stats of config 4 / config3_check_order.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ns1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_presorted_gpu.py \
    > gpurun_out/ns1/tests.log 2>&1 || { tail -40 gpurun_out/ns1/tests.log; exit 1; }
tail -3 gpurun_out/ns1/tests.log
bash tools/r05/gpu_ns_prof.sh
