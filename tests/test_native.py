"""Runs the native C++ unit-test programs built by parsec_amd._build
(build/tests/*): lock-free containers, mempool, sharded hash map, barrier, futures, rwlock,
the priority-ordered bounded fetch queue of the remote dependency engine."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "tests")


@pytest.mark.parametrize("prog", ["test_containers", "test_futures", "test_fetch_queue"])
def test_native_program(pa, prog):
    exe = os.path.join(BIN, prog)
    if not os.path.exists(exe):
        from parsec_amd import _build

        _build.build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "passed" in r.stdout
