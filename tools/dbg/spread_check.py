"""Measured GPU-vs-oracle deviations against the oracle's own 1- vs 8-thread spread (for the parity bars in
tests/test_gpu_ba.py): point steps after each solve, the 2-frame window's optimize trajectory."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "h-slam_amd"), os.path.join(ROOT, "oracle")]
from hslam_amd.ba import BAWindow  # noqa: E402
from hslam_amd.scene import make_ba_scene  # noqa: E402
from oracle_ffi import OracleBA  # noqa: E402

scene = make_ba_scene(n_points=2000, seed=20261015)
os.environ["HS_ACC_EXACT"] = "1"
g = BAWindow(scene)
os.environ.pop("HS_ACC_EXACT")
o, o8 = OracleBA(scene), OracleBA(scene, nthreads=8)
g.linearizeAll(reset=True)
for oo in (o, o8):
    oo.linearize_all(reset=True)
    oo.apply_res()
for it in range(3):
    o.backup_state()
    o8.backup_state()
    xo, x8, xg = o.solve_system(it), o8.solve_system(it), g.solveSystem(it)
    po, pg, p8 = o.points()["step"], g.points()["step"], o8.points()["step"]
    sstep = np.abs(p8 - po).max()
    dev = np.abs(pg - po)
    print(f"it {it}: |x| spread {np.linalg.norm(x8 - xo) / np.linalg.norm(xo):.3e} gpu {np.linalg.norm(xg - xo) / np.linalg.norm(xo):.3e};"
          f" step max dev {dev.max():.3e} vs oracle spread {sstep:.3e} (ratio {dev.max() / max(sstep, 1e-30):.2f});"
          f" max rel {np.max(dev / np.maximum(np.abs(po), 1e-30)):.3e}")
    for oo in (o, o8):
        oo.do_step()
    g.doStepFromBackup()
    g.linearizeAll()
    for oo in (o, o8):
        oo.linearize_all()
        oo.apply_res()

s = make_ba_scene(n_points=64, n_frames=2, seed=3)
s.pt_u[:4] = np.float32(3.0)
os.environ["HS_ACC_EXACT"] = "1"
g = BAWindow(s)
os.environ.pop("HS_ACC_EXACT")
o, o8 = OracleBA(s), OracleBA(s, nthreads=8)
g.linearizeAll(reset=True)
o.linearize_all(reset=True)
o8.linearize_all(reset=True)
_, e1 = g.optimize(4)
_, e2 = o.optimize(4)
_, e8 = o8.optimize(4)
print("2-frame: gpu rel dev", np.array2string(np.abs(e1 - e2) / np.abs(e2), precision=2))
print("2-frame: pool rel dev", np.array2string(np.abs(e8 - e2) / np.abs(e2), precision=2))
