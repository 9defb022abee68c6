"""The plain-C caller of the BA boundary (tests/c/ba_caller.c) on the device: set_window, optimize, the optimize
tail, the dormant energies and the frame read-back through include/hs_ba.h from a C99 program."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_caller_runs_the_keyframe_sequence():
    exe = os.path.join(ROOT, "h-slam_amd", "lib", "ba_caller")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["iters"] == 15  # a 3-frame window: System::optimize's override
    assert 0 < out["E"] <= out["E0"]
    assert 0 <= out["dropped"] < out["residuals"]
