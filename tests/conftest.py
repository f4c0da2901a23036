"""Shared pytest setup: markers, import paths, golden fixtures."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "webgpu-radix-sort_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) cases")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(GOLDEN_DIR, "golden.npz"))  # allow_pickle=False (default)
    return manifest, arrays


@pytest.fixture
def plan_debug():
    """Path overrides (rs_plan_set_debug) for every plan the test creates through the Python
    wrappers: plan_debug(rank="ballot", tile="small", onesweep=0, ...); reset after the test."""
    from radix_sort_amd import _lib
    saved = dict(_lib._DEBUG)

    def set_(**fields):
        _lib.plan_debug(**fields)          # validates the field names
        _lib._DEBUG.update(fields)

    yield set_
    _lib._DEBUG.clear()
    _lib._DEBUG.update(saved)


def case_arrays(arrays, case):
    keys = arrays[case["name"] + "_keys"]
    exp_k = arrays[case["name"] + "_exp_keys"]
    vals = np.arange(case["n"], dtype=np.uint32) if case["has_values"] else None
    exp_v = arrays[case["name"] + "_exp_values"] if case["has_values"] else None
    return keys, vals, exp_k, exp_v
