# Round 4: the host ASan/UBSan/LSan driver over every C-ABI entry point, on the final library's
# sources (tools/gpu_round.sh step 12; the asan build travels only for this call).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_round.sh 12 12
