"""Back-to-back linearize launches of a synthetic window (hs_ba_time_linearize), for library-variant A/B runs:
python tools/lin8_time.py POINTS [REPS]  (HSLAM_AMD_LIB selects the library)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "h-slam_amd"))
from hslam_amd.ba import BAWindow  # noqa: E402
from hslam_amd.scene import make_ba_scene  # noqa: E402

n = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 64
g = BAWindow(make_ba_scene(n_points=n))
g.linearizeAll(reset=True)
ms = [g.time_linearize(reps) for _ in range(3)]
print(json.dumps({"points": n, "kernel": g.partition()["kernel"], "launch_us": [round(m * 1e3, 2) for m in ms]}))
g.close()
