"""Debug: per-block relative error of the GPU systems (get_system 0 / 2) against the oracle."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "h-slam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
from hslam_amd.ba import BAWindow
from hslam_amd.scene import make_ba_scene
from oracle_ffi import OracleBA

for exact in ("1", "0"):
    for nf, npts in ((8, 240), (3, 96)):
        os.environ["HS_ACC_EXACT"] = exact
        s = make_ba_scene(n_points=npts, n_frames=nf, seed=7)
        g = BAWindow(s)
        o = OracleBA(s, nthreads=1)
        g.linearizeAll(reset=True)
        o.linearize_all(reset=True)
        o.apply_res()
        for which in (0, 2):
            Hg, bg = g.system(which)
            Ho, bo = o.accumulate(which)
            n = Ho.shape[0]
            scale = np.abs(np.diag(Ho)).max()
            bad = []
            names = ["c"] + [f"f{i}" for i in range(nf)]
            idx = [range(0, 4)] + [range(4 + 8 * i, 12 + 8 * i) for i in range(nf)]
            for bi, ri in enumerate(idx):
                for bj, cj in enumerate(idx):
                    d = np.abs(Hg[np.ix_(ri, cj)] - Ho[np.ix_(ri, cj)]).max()
                    m = np.abs(Ho[np.ix_(ri, cj)]).max()
                    if d > 1e-6 * (m + 1e-3 * scale):
                        bad.append(f"{names[bi]}{names[bj]}:{d / (m + 1e-30):.2e}(|{m:.2e}|)")
            db = np.abs(bg - bo) / (np.abs(bo) + 1e-3 * np.abs(bo).max())
            print(f"exact={exact} nF={nf} which={which} bad blocks {len(bad)}: {' '.join(bad[:12])}  b worst {db.max():.2e} at {db.argmax()}")
        g.close()
