"""CPU: how `bench.py --gpus N` is run (bench.launch_plan).  The driver may start it as a plain
`python bench.py --gpus N` or under torch.distributed.run; either way N GPUs are measured, and a
mismatch is an error instead of a 1-GPU line labelled with the wrong count."""
import json
import subprocess
import sys

import pytest

import bench


def test_one_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, 1, []) == ("run", None)
    assert bench.launch_plan(1, {}, 8, ["--steps", "5"]) == ("run", None)


def test_plain_n_gpus_spawns_torchrun_with_same_args():
    what, cmd = bench.launch_plan(8, {}, 8, ["--gpus", "8", "--steps", "5", "--warmup", "2"])
    assert what == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    assert any(a.startswith("--master-port=") and int(a.split("=")[1]) > 0 for a in cmd)
    assert cmd[-7].endswith("bench.py")
    assert cmd[-6:] == ["--gpus", "8", "--steps", "5", "--warmup", "2"]


def test_fewer_gpus_than_asked_is_an_error():
    what, msg = bench.launch_plan(8, {}, 1, ["--gpus", "8"])
    assert what == "error" and "only 1 GPU" in msg
    assert bench.launch_plan(1, {}, 0, [])[0] == "error"
    assert bench.launch_plan(0, {}, 8, [])[0] == "error"


def test_under_a_launcher_world_size_must_match():
    env = {"RANK": "0", "WORLD_SIZE": "4", "LOCAL_RANK": "0"}
    assert bench.launch_plan(4, env, 8, []) == ("run", None)
    what, msg = bench.launch_plan(8, env, 8, [])
    assert what == "error" and "WORLD_SIZE=4" in msg
    assert bench.launch_plan(4, env, 2, [])[0] == "error"


def test_gpus_arg_parsing():
    assert bench._gpus_arg([]) == 1
    assert bench._gpus_arg(["--steps", "3", "--gpus", "4"]) == 4
    assert bench._gpus_arg(["--gpus=2"]) == 2


def test_share_gpu_rehearsal_needs_one_gpu():
    what, cmd = bench.launch_plan(2, {}, 1, ["--gpus", "2", "--share-gpu"])
    assert what == "spawn" and "--nproc-per-node=2" in cmd and cmd[-1] == "--share-gpu"
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}, 1, ["--share-gpu"]) == ("run", None)
    assert bench.launch_plan(2, {}, 0, ["--share-gpu"])[0] == "error"


def test_spawned_command_line_parses_under_torchrun():
    """Every bench option survives torch.distributed.run's own parser (which scans the whole
    command line for abbreviations of its options)."""
    from torch.distributed.run import get_args_parser
    what, cmd = bench.launch_plan(2, {}, 2, ["--gpus", "2", "--steps", "3", "--warmup", "1",
                                             "--workload", "config3", "--keys-per-gpu", "1024",
                                             "--no-cpu-baseline", "--share-gpu", "--radix-bits", "8",
                                             "--rank", "ballot"])
    args = get_args_parser().parse_args(cmd[3:])
    assert args.nproc_per_node == "2" and args.training_script.endswith("bench.py")
    assert "--keys-per-gpu" in args.training_script_args


@pytest.mark.gpu
def test_bench_n_rank_path_rehearsed_on_one_gpu():
    """The driver's N-GPU bench path (plain `bench.py --gpus N` -> torch.distributed.run -> N ranks
    -> distributed_sort + HipLocalOps), rehearsed with 2 ranks on GPU 0 over gloo."""
    out = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--share-gpu",
                          "--keys-per-gpu", str(6 << 20), "--steps", "2", "--warmup", "1",
                          "--no-cpu-baseline"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = out.stdout.strip().splitlines()
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["rccl_ranks"] == 0 and "NOT a measurement" in r["rehearsal"]
    assert r["config"]["global_keys"] == 2 * (6 << 20) and r["value"] > 0
    assert r["recv_keys_rank0"] > 0
