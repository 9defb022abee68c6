#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run from the repo root: python tests/golden/make_golden.py).

The reference ships no tests, fixtures or golden vectors for this path and cannot be built or run here
(SURVEY.md §4, §8c), so these vectors are produced by the CPU restatement (oracle/, -ffp-contract=off
build) from seeded synthetic scenes (hslam_amd.scene).  They pin the oracle against drift and give the GPU
path fixed expected outputs; they are NOT reference outputs ("parity unpinned").
Each fixture stores a SHA-256 digest of its inputs so a change of the scene generator is detected
instead of silently comparing against other inputs.

Fixtures (SURVEY.md §8c list):
  ba_pair64.npz   2 KF x 64 points per host (the two host-target pairs): per-residual state / energy / JpJdF / centre, H/b (A, L, SC),
                  GN step x of iteration 0
  ba_8x200.npz    8 KF x 200 points: the same + the energies of 3 GN iterations
  track_160.npz   CoarseTracker at 160x120: pc arrays per level, calcRes at the truth, trackNewestCoarse
  trace_100.npz   100 traceOn results: ctor outputs, first and second trace
  refine_300.npz  DirectRefinement at 320x240, 300 keypoints: one calcResAndGS (per-point outputs, H/b/Hsc/bsc,
                  res) and the Refine LM log + refined pose
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "h-slam_amd"), os.path.join(ROOT, "oracle")]
OUT = os.path.dirname(os.path.abspath(__file__))


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def ba_scene_digest(s):
    return digest(*[p[0] for p in s.pyramids], s.frames_eval, s.pt_host, s.pt_u, s.pt_v, s.pt_idepth, s.pt_color,
                  s.pt_weights, s.res_point, s.res_target)


def track_scene_digest(s):
    return digest(*s.ref_pyr, *s.new_pyr, s.pt_u, s.pt_v, s.pt_idepth, s.pt_hdi, s.T_true, s.aff_true)


def trace_scene_digest(s):
    return digest(*s.host_imgs, s.new_img, s.KRKi, s.Kt, s.aff, s.pt_host, s.pt_u, s.pt_v)


def refine_scene_digest(s):
    return digest(s.img1, s.img2, s.u, s.v, s.tri, s.z, s.T_init, s.K4)


# ---------------------------------------------------------------- scenes (shared with tests/test_golden.py)
K320 = np.array([[128.0, 0, 159.5], [0, 127.2, 119.5], [0, 0, 1.0]])


def scene_ba_pair64():
    from hslam_amd.scene import make_ba_scene
    return make_ba_scene(n_points=128, n_frames=2, width=320, height=240, K=K320, seed=101)


def scene_ba_8x200():
    from hslam_amd.scene import make_ba_scene
    return make_ba_scene(n_points=200, n_frames=8, width=320, height=240, K=K320, seed=102)


def scene_track160():
    from hslam_amd.scene import make_track_scene
    return make_track_scene(n_points=300, width=160, height=120, n_levels=3, seed=103,
                            K=np.array([[64.0, 0, 79.5], [0, 63.6, 59.5], [0, 0, 1.0]]))


def scene_trace100():
    from hslam_amd.scene import make_trace_scene
    return make_trace_scene(n_points=100, n_hosts=4, width=320, height=240, seed=104)


def scene_refine300():
    from hslam_amd.scene import make_refine_scene
    return make_refine_scene(300, width=320, height=240, K=K320, seed=105)


def refine_outputs(scene):
    from oracle_ffi import OracleRefiner
    o = OracleRefiner(scene)
    H, b, Hsc, bsc, res = o.calc_res(scene.T_init)
    out = dict(calc_H=H, calc_b=b, calc_Hsc=Hsc, calc_bsc=bsc, calc_res=res)
    for k, v in o.points().items():
        out["calc_" + k] = v
    o2 = OracleRefiner(scene)
    T, it, sn = o2.refine(scene.T_init)
    out.update(refine_T=T, refine_iters=np.int64(it), refine_snapped=np.bool_(sn), refine_log=o2.log())
    p = o2.points()
    out.update(refine_idepth=p["idepth"], refine_isGood=p["isGood"])
    return out


def make_refine(scene):
    out = refine_outputs(scene)
    out["digest"] = np.array(refine_scene_digest(scene))
    np.savez_compressed(os.path.join(OUT, "refine_300.npz"), **out)


def ba_outputs(o):
    out = {}
    E0 = o.linearize_all(reset=True)
    o.apply_res()
    r = o.residuals()
    out.update(E0=np.float64(E0), res_state=r["state"], res_energy=r["energy"].astype(np.float32),
               res_energy_wo=r["energy_wo"].astype(np.float32), res_JpJdF=r["JpJdF"], res_center=r["center"],
               energyTH=o.frames()["energyTH"])
    for which, nm in ((0, "A"), (1, "L"), (2, "SC")):
        H, b = o.accumulate(which)
        out["H" + nm], out["b" + nm] = H, b
    o.backup_state()
    out["x0"] = o.solve_system(0)
    return out


def make_ba(name, scene, iters):
    from oracle_ffi import OracleBA
    o = OracleBA(scene)
    out = ba_outputs(o)
    if iters:
        o2 = OracleBA(scene)
        o2.linearize_all(reset=True)
        o2.apply_res()
        out["E_iters"] = o2.iterate(0, iters)
    out["digest"] = np.array(ba_scene_digest(scene))
    np.savez_compressed(os.path.join(OUT, name), **out)


def make_track(scene):
    from oracle_ffi import OracleTracker
    o = OracleTracker(scene.width, scene.height, scene.K4, scene.n_levels)
    o.set_scene(scene)
    out = {}
    for l in range(scene.n_levels):
        pc = o.pc(l)
        for k, v in pc.items():
            out[f"pc{l}_{k}"] = v
    res6, H, b, nw = o.calc_res(0, scene.T_true, scene.aff_true, 20.0)
    out.update(calc_res6=res6, calc_H=H, calc_b=b, calc_nwarped=np.int64(nw))
    t = o.track(np.array([0, 0, 0, 1.0, 0, 0, 0]), [0.0, 0.0], scene.n_levels - 1, np.full(5, np.nan))
    out.update(track_ok=np.bool_(t["ok"]), track_T=t["T"], track_aff=t["aff"], track_lastResiduals=t["lastResiduals"],
               track_flow=t["flow"])
    out["digest"] = np.array(track_scene_digest(scene))
    np.savez_compressed(os.path.join(OUT, "track_160.npz"), **out)


def make_trace(scene):
    from oracle_ffi import OracleTracer
    o = OracleTracer(scene.width, scene.height)
    o.set_scene(scene)
    out = {}
    for k, v in o.points().items():
        out["ctor_" + k] = v
    for rnd in (1, 2):
        out[f"counts{rnd}"] = o.trace(scene.new_img, scene.KRKi, scene.Kt, scene.aff)
        for k, v in o.points().items():
            if k not in ("color", "weights", "gradH", "energyTH"):
                out[f"trace{rnd}_{k}"] = v
    out["digest"] = np.array(trace_scene_digest(scene))
    np.savez_compressed(os.path.join(OUT, "trace_100.npz"), **out)


if __name__ == "__main__":
    make_ba("ba_pair64.npz", scene_ba_pair64(), 0)
    make_ba("ba_8x200.npz", scene_ba_8x200(), 3)
    make_track(scene_track160())
    make_trace(scene_trace100())
    make_refine(scene_refine300())
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)), "bytes")
