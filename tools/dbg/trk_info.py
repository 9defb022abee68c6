"""Tracker bench scene facts: reference points per level, LM iterations per level, device ms per track."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "h-slam_amd"))
from hslam_amd.scene import make_track_scene
from hslam_amd.track import CoarseTracker

for nl in (5, 4):
    s = make_track_scene(n_points=2000, n_levels=nl)
    ct = CoarseTracker(s.width, s.height, s.K4, s.n_levels)
    ct.set_scene(s)
    T0 = np.array([0, 0, 0, 1.0, 0, 0, 0])
    minRes = np.full(5, np.nan)
    for _ in range(3):
        ok, T, a = ct.trackNewestCoarse(T0, [0.0, 0.0], s.n_levels - 1, minRes)
    ms = []
    for _ in range(20):
        ct.trackNewestCoarse(T0, [0.0, 0.0], s.n_levels - 1, minRes)
        ms.append(ct.last_ms())
    lv, nr, orr, inc = ct.lm_log(0)
    print("levels", nl, "pc_n", [len(ct.pc(l)["u"]) for l in range(nl)], "ok", ok, "device ms", np.median(ms))
    print("  iterations per level", [int((lv == l).sum()) for l in range(nl)], "total", len(lv))
    ct.close()
