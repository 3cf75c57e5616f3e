"""Shared test setup.

Markers: ``gpu`` tests need an MI355X (run by the driver with ``-m gpu`` on a GPU box); every
other test runs on a CPU-only host in a few minutes.
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle_py import fnv1a, length_header, payload_lengths, payloads  # noqa: E402,F401
NATIVE = os.path.join(ROOT, "tests", "native")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def _make(path: str, *targets: str) -> None:
    # one build at a time across pytest-xdist workers (targets share objects)
    import fcntl
    with open(os.path.join(ROOT, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", path, "-j8", *targets], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def oracle_lib():
    """The plain-C oracle (oracle/liboracle.so), built on demand."""
    import ctypes
    _make(os.path.join(ROOT, "oracle"), "liboracle.so")
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    assert L.oracle_self_test() == 0
    return L


@pytest.fixture(scope="session")
def golden_index():
    with open(os.path.join(GOLDEN, "scenarios.json")) as f:
        return json.load(f)


def golden_text(name: str) -> str:
    with gzip.open(os.path.join(GOLDEN, f"{name}.txt.gz"), "rt") as f:
        return f.read()


def sha256(text: str) -> str:
    return hashlib.sha256(text.encode()).hexdigest()


def scenario_params(golden_index, name) -> dict:
    sc = golden_index["scenarios"][name]
    kv = {k: int(v) for k, v in (a.split("=") for a in sc["args"])}
    kv["stream"] = sc["stream"]
    kv["seed_data"] = 1000 + sc["stream"]
    kv["seed_loss"] = 2000 + sc["stream"]
    return kv


def first_diff(a: str, b: str) -> str:
    la, lb = a.splitlines(), b.splitlines()
    for i, (x, y) in enumerate(zip(la, lb)):
        if x != y:
            return f"line {i + 1}: expected {x!r} got {y!r}"
    return f"length differs: expected {len(la)} lines got {len(lb)}"
