"""The Node host (the reference's own host language) over the N-API addon.

CPU: the addon loads, exports the reference's classes and validates options like the reference.
GPU: the reference's own test flow (example/tests.ts:9-107, seeded) through the JS façade.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE_DIR = os.path.join(ROOT, "webgpu-radix-sort_amd", "node")

pytestmark = pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")


def _run(script, timeout):
    addon = os.path.join(NODE_DIR, "build", "rsort_napi.node")
    if not os.path.exists(addon):
        subprocess.run(["make", "-s", "-C", NODE_DIR], check=True)
    r = subprocess.run(["node", os.path.join(NODE_DIR, "test", script)], capture_output=True,
                       text=True, timeout=timeout, cwd=NODE_DIR)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_node_api_and_validation():
    assert "node api checks ok" in _run("api.js", 60)


@pytest.mark.gpu
def test_node_reference_flow_on_gpu():
    assert "node sort checks ok" in _run("sort.js", 300)


@pytest.mark.gpu
def test_node_group_sort_on_gpu():
    """RadixSortGroup (rs_group_* through the addon): RCCL world 1 and 3 virtual ranks."""
    assert "node group checks ok" in _run("group.js", 300)


def _demo(*args, timeout=300):
    r = subprocess.run(["node", os.path.join(NODE_DIR, "demo.js"), *args], capture_output=True,
                       text=True, timeout=timeout, cwd=NODE_DIR)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_node_demo_rejects_unknown_setting():
    r = subprocess.run(["node", os.path.join(NODE_DIR, "demo.js"), "--noSuchSetting=1"],
                       capture_output=True, text=True, timeout=60, cwd=NODE_DIR)
    assert r.returncode != 0 and "unknown setting" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    (),                                                                  # the demo's defaults
    ("--sortMode=Keys & Values", "--checkOrder", "--consecutiveSorts=3"),
    ("--dataType=texture", "--elementCount=300000", "--bitCount=16", "--workgroupSize=8"),
    ("--initialSort=Sorted", "--localShuffle", "--avoidBankConflicts"),
])
def test_node_demo_cli_report(args):
    """example/index.ts's flow and report; --verify compares the GPU result with the CPU sort."""
    out = _demo(*args, "--verify")
    assert "> CPU Reference:" in out and "GPU Average" in out and "Speedup: x" in out, out
    assert "GPU result matches CPU" in out, out


@pytest.mark.gpu
def test_node_demo_json_line():
    import json
    line = _demo("--elementCount=65536", "--json", "--verify").strip().splitlines()[-1]
    rec = json.loads(line)
    assert rec["verified"] is True and rec["gpu_avg_ms"] > 0 and rec["settings"]["elementCount"] == 65536
