# Round 6: hist16 probe, side-stream A/B, tests touching the changed paths
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 ./tools/hist_probe > gpurun_out/hist_probe.jsonl 2>&1 || { cat gpurun_out/hist_probe.jsonl; exit 1; }
cat gpurun_out/hist_probe.jsonl
bash tools/r06/ab.sh side config3 2 "xcd=0" "xcd=0,side_stream=0" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_region_gpu.py tests/test_msd_gpu.py tests/test_presorted_gpu.py tests/test_split_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t3.log 2>&1 || { tail -30 gpurun_out/t3.log; exit 1; }
tail -3 gpurun_out/t3.log
