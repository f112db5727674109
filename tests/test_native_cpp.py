"""Runs the C++ unit/integration suite (tests/cpp, incl. the ported sync matrix)."""
import os
import subprocess

from conftest import ROOT


def test_cpp_suite():
    exe = os.path.join(ROOT, "bin", "devspace_tests")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " 0 failed" in r.stdout
