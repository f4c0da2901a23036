# multi-GPU path at world size 1 on the final build (torch.distributed, RCCL)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --distributed --no-cpu-baseline > gpurun_out/fd_dist1.json 2> gpurun_out/fd.err || exit 12
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/fd_single.json 2>> gpurun_out/fd.err || exit 13
