# Round 5: the presorted path's parity tests, then config 4 / config3_check_order bench lines.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ns1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_presorted_gpu.py \
    > gpurun_out/ns1/tests.log 2>&1 || { tail -40 gpurun_out/ns1/tests.log; exit 1; }
tail -3 gpurun_out/ns1/tests.log
timeout -k 10 300 python -u bench.py --workload config4 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/ns1/c4.json 2> gpurun_out/ns1/c4.log || { tail -20 gpurun_out/ns1/c4.log; exit 1; }
cat gpurun_out/ns1/c4.json
timeout -k 10 300 python -u bench.py --workload config3_check_order --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/ns1/c3chk.json 2> gpurun_out/ns1/c3chk.log || { tail -20 gpurun_out/ns1/c3chk.log; exit 1; }
cat gpurun_out/ns1/c3chk.json
exit 0
