# bench.py stdout = exactly one JSON line, single-GPU and the RCCL path at world size 1
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --distributed --no-cpu-baseline > gpurun_out/bs_dist1.json 2> gpurun_out/bs.err || exit 12
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bs_single.json 2>> gpurun_out/bs.err || exit 13
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --distributed --no-cpu-baseline > gpurun_out/bs_torchrun.json 2>> gpurun_out/bs.err || exit 14
