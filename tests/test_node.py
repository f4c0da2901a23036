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
