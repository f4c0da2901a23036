# Round 5 checkpoint on the committed library: full GPU suite, smoke, default bench line, rocprof
# kernel stats of the default line, PMC traffic (config3/2/4), the multi-GPU rank model.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_round.sh 1 3 || exit $?
bash tools/gpu_round.sh 8 10 || exit $?
exit 0
