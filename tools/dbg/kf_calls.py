"""Per-call wall time of the keyframe driver's library calls (measurement only): the bench's keyframe sequence,
median ms per (phase, function) over the timed keyframes."""
import collections
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "h-slam_amd"))
import hslam_amd.keyframe as kf  # noqa: E402

calls = collections.defaultdict(list)


class _CallTimer(kf._Timer):
    def run(self, phase, fn, *a, **k):
        t0 = time.perf_counter()
        r = fn(*a, **k)
        dt = time.perf_counter() - t0
        self.t[phase] = self.t.get(phase, 0.0) + dt
        calls[(phase, getattr(fn, "__name__", str(fn)))].append(dt)
        return r


kf._Timer = _CallTimer
from hslam_amd.track import CoarseTracker  # noqa: E402

warm, steps = 2, 10
seq = kf.make_ba_sequence(n_kf=7 + warm + steps, points_per_kf=250)
K4 = np.array([seq.K[0, 0], seq.K[1, 1], seq.K[0, 2], seq.K[1, 2]], np.float32)
drv = kf.KeyframeBA(seq, window=8, tracker=CoarseTracker(seq.width, seq.height, K4, seq.n_levels), image_path="device")
drv.bootstrap()
for k in range(7, 7 + warm):
    drv.add_keyframe(k)
calls.clear()
for k in range(7 + warm, 7 + warm + steps):
    drv.add_keyframe(k)
for (ph, fn), v in sorted(calls.items(), key=lambda kv: -sum(kv[1])):
    print(f"{ph:12s} {fn:28s} calls/KF {len(v) / steps:5.1f}  median {np.median(v) * 1e3:7.3f} ms  total/KF "
          f"{sum(v) / steps * 1e3:7.3f} ms")
