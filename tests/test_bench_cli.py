"""CPU: how `bench.py --gpus N` is run (bench.launch_plan).  The driver may start it as a plain
`python bench.py --gpus N` or under torch.distributed.run; either way N GPUs are measured, and a
mismatch is an error instead of a 1-GPU line labelled with the wrong count."""
import sys

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
