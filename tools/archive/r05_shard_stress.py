"""Stress: the full C4 2k window's linearizeAll H, repeated with other contexts created / destroyed in between;
reports any H whose frame rows are all zero (the intermittent test_gpu_shard failure)."""
import sys, os, time
import numpy as np
sys.path.insert(0, "h-slam_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
from hslam_amd.scene import make_ba_scene
from hslam_amd.ba import BAWindow, unpack_system_vector
s = make_ba_scene(n_points=2000)
small = make_ba_scene(n_points=240, seed=7)
bad = 0
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    junk = [BAWindow(small) for _ in range(it % 4)]
    for j in junk:
        j.linearizeAll(reset=True); j.optimize(3)
    if it % 3 == 0:
        for j in junk: j.close()
    w = BAWindow(s)
    e = w.linearizeAll(reset=True)
    n = w.dim
    H, b, E = unpack_system_vector(w.system_vector(), n)
    zr = [i for i in range(n) if not np.any(H[i])]
    if zr:
        bad += 1
        print(f"it {it}: E {e:.6g} zero rows {zr[:3]}..{zr[-3:]} ({len(zr)}) nF {w.nF} n_points {w.n_points} n_res {w.n_res}", flush=True)
        st = w.structure() if hasattr(w, "structure") else None
    w.close()
    if it % 3 != 0:
        for j in junk: j.close()
print("bad", bad, flush=True)
