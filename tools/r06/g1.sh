cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_region_gpu.py tests/test_msd_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/t_msd.log 2>&1 || { tail -30 gpurun_out/t_msd.log; exit 1; }
tail -2 gpurun_out/t_msd.log
bash tools/r06/ab.sh xcd1 config3 2 "" "xcd=0"
