cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/r06/ab.sh db config3 2 "" "msd_db=1" || exit 1
AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python3 -u tools/r06/diag_ns.py > gpurun_out/diag_ns.log 2>&1
rc=$?; tail -40 gpurun_out/diag_ns.log; exit $rc
