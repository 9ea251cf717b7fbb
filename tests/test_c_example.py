"""The plain-C integration example (examples/c_integration.c): libunsod's side
of the boundary is the header and the link line.  The drop-in symbols over
real mbuf chains from 8 threads (SURVEY.md 8(a) known answers) and a registered
host-memory RX burst verified in place, all from C."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "libunsod_amd", "lib", "c_integration")


def test_c_example_built():
    assert os.path.exists(EXE), "make -C libunsod_amd/csrc builds examples/c_integration.c"


@pytest.mark.gpu
def test_c_integration_runs():
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c_integration ok" in r.stdout
