"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes bindings of the CPU restatement (oracle/_build/liboracle*.so).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
Parity status: unpinned against the reference (see oracle/oracle_common.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")


class hs_camera(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("n_levels", C.c_int), ("pad", C.c_int),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float)]


class hs_frame(C.Structure):
    _fields_ = [("worldToCam_evalPT", C.c_double * 7), ("state", C.c_double * 10), ("state_zero", C.c_double * 10),
                ("ab_exposure", C.c_float), ("frameEnergyTH", C.c_float), ("id", C.c_int), ("pad", C.c_int)]


class hs_points(C.Structure):
    _fields_ = [("n", C.c_int), ("host", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p), ("idepth", C.c_void_p),
                ("idepth_zero", C.c_void_p), ("color", C.c_void_p), ("weights", C.c_void_p),
                ("has_depth_prior", C.c_void_p)]


class hs_residuals(C.Structure):
    _fields_ = [("n", C.c_int), ("point", C.c_void_p), ("target", C.c_void_p), ("state", C.c_void_p)]


class hs_params(C.Structure):
    _fields_ = [(n, C.c_float) for n in (
        "huberTH", "outlierTHSumComponent", "frameEnergyTHN", "frameEnergyTHFacMedian", "frameEnergyTHConstWeight",
        "overallEnergyTHWeight", "idepthFixPrior", "initialCalibHessian", "affineOptModeA", "affineOptModeB",
        "initialRotPrior", "initialTransPrior", "initialAffAPrior", "initialAffBPrior")] + [
        ("solverModeDelta", C.c_double), ("thOptIterations", C.c_float), ("coarseCutoffTH", C.c_float),
        ("minOptIterations", C.c_int), ("pad", C.c_int)] + [(n, C.c_float) for n in (
        "outlierTH", "maxPixSearch", "trace_slackInterval", "trace_stepsize", "trace_minImprovementFactor",
        "trace_GNThreshold", "trace_extraSlackOnTH")] + [
        ("minTraceTestRadius", C.c_int), ("trace_GNIterations", C.c_int),
        ("idepthFixPriorMargFac", C.c_float), ("margWeightFac", C.c_float),
        ("desiredPointDensity", C.c_float), ("minTraceQuality", C.c_float), ("minIdepthH_act", C.c_float),
        ("GNItsOnPointActivation", C.c_int), ("minGradHistCut", C.c_float), ("minGradHistAdd", C.c_float),
        ("gradDownweightPerLevel", C.c_float), ("selectDirectionDistribution", C.c_int)]


def build(quiet=True):
    r = subprocess.run(["make", "-C", HERE, "-j4"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)


_LIBS = {}


def build_native():
    """-O2 -march=native build for the timed CPU baseline, compiled on the host that times it."""
    r = subprocess.run(["make", "-C", HERE, "-j8", "native"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle native build failed:\n" + r.stdout + r.stderr)


def load(fast=False):
    """fast=False: the parity oracle (-ffp-contract=off); True: portable -march=x86-64-v3; "native": -march=native."""
    name = {False: "liboracle.so", True: "liboracle_fast.so", "native": "liboracle_native.so"}[fast]
    if name in _LIBS:
        return _LIBS[name]
    path = os.path.join(BUILD, name)
    if fast == "native":
        build_native()  # make: a no-op when current
    elif not os.path.exists(path):
        build()
    lib = C.CDLL(path)
    vp = C.c_void_p
    lib.hso_ba_create.restype = vp
    lib.hso_ba_create.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, C.c_int]
    lib.hso_ba_destroy.argtypes = [vp]
    lib.hso_ba_optimize.argtypes = [vp, C.c_int, C.c_int, vp]
    lib.hso_ba_optimize.restype = C.c_int
    lib.hso_ba_iterate.argtypes = [vp, C.c_int, C.c_int, vp]
    lib.hso_ba_linearize_all.argtypes = [vp, C.c_int]
    lib.hso_ba_linearize_all.restype = C.c_double
    lib.hso_ba_apply_res.argtypes = [vp]
    lib.hso_ba_fix_linearization.argtypes = [vp, vp, vp, vp]
    lib.hso_ba_fix_linearization.restype = C.c_double
    lib.hso_ba_calc_energies.argtypes = [vp, vp, vp]
    lib.hso_ba_accumulate.argtypes = [vp, C.c_int, vp, vp]
    lib.hso_ba_solve_system.argtypes = [vp, C.c_int, vp]
    lib.hso_ba_backup_state.argtypes = [vp]
    lib.hso_ba_set_marginal_prior.argtypes = [vp, vp, vp]
    lib.hso_ba_set_calib.argtypes = [vp, vp]
    lib.hso_ba_marginalize_points.argtypes = [vp, C.c_int, vp, C.c_float, C.c_float, vp, vp]
    lib.hso_ba_marginalize_frame.argtypes = [vp, C.c_int, vp, vp]
    lib.hso_ba_do_step.argtypes = [vp]
    lib.hso_ba_do_step.restype = C.c_int
    lib.hso_ba_get_residuals.argtypes = [vp] * 10
    lib.hso_ba_get_points.argtypes = [vp] * 6
    lib.hso_ba_get_frames.argtypes = [vp] * 5
    lib.hso_ba_get_precalc.argtypes = [vp, vp]
    lib.hso_ba_get_nullspaces.argtypes = [vp, vp]
    lib.hso_ba_res_in_A.argtypes = [vp]
    lib.hso_ba_res_in_A.restype = C.c_int
    for n in ("hso_se3_exp", "hso_se3_log", "hso_se3_inverse", "hso_se3_adj", "hso_se3_matrix"):
        getattr(lib, n).argtypes = [vp, vp]
    lib.hso_se3_mul.argtypes = [vp, vp, vp]
    lib.hso_ref_create.restype = vp
    lib.hso_ref_create.argtypes = [C.c_int, C.c_int, vp, vp, vp, C.c_float, C.c_float]
    lib.hso_ref_destroy.argtypes = [vp]
    lib.hso_ref_set_points.argtypes = [vp, C.c_int, vp, vp, vp, vp]
    lib.hso_ref_calc.argtypes = [vp] * 8
    lib.hso_ref_refine.argtypes = [vp, vp, vp, vp]
    lib.hso_ref_refine.restype = C.c_int
    lib.hso_ref_get_log.argtypes = [vp, C.c_int, vp]
    lib.hso_ref_get_log.restype = C.c_int
    lib.hso_ref_get_points.argtypes = [vp, vp, vp, vp]
    lib.hso_trk_create.restype = vp
    lib.hso_trk_create.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp]
    lib.hso_trk_destroy.argtypes = [vp]
    lib.hso_trk_set_ref.argtypes = [vp, vp, C.c_float, vp, C.c_int, vp, vp, vp, vp]
    lib.hso_trk_set_frame.argtypes = [vp, vp, C.c_float]
    lib.hso_trk_get_ref.argtypes = [vp, C.c_int, vp, vp, vp, vp]
    lib.hso_trk_get_ref.restype = C.c_int
    lib.hso_trk_calc_res.argtypes = [vp, C.c_int, vp, vp, C.c_float, vp, vp, vp, vp]
    lib.hso_trk_set_sum_order.argtypes = [vp, C.c_int]
    lib.hso_trk_set_sum_order.restype = None
    lib.hso_trk_track.argtypes = [vp, vp, vp, C.c_int, vp, vp, vp, vp]
    lib.hso_trk_track.restype = C.c_int
    lib.hso_trk_get_log.argtypes = [vp, C.c_int, vp, vp, vp, vp]
    lib.hso_trk_get_log.restype = C.c_int
    lib.hso_trk_track_tries.argtypes = [vp, C.c_int, vp, vp, vp, C.c_float, C.c_int] + [vp] * 6
    lib.hso_dir_pyramid.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, vp]
    lib.hso_trc_create.restype = vp
    lib.hso_trc_create.argtypes = [vp, C.c_int, C.c_int]
    lib.hso_trc_destroy.argtypes = [vp]
    lib.hso_trc_add_points.argtypes = [vp, C.c_int, vp, C.c_int, vp, vp, vp]
    lib.hso_trc_add_points.restype = C.c_int
    lib.hso_trc_set_state.argtypes = [vp] * 6
    lib.hso_trc_set_types.argtypes = [vp, vp]
    lib.hso_trc_activate.argtypes = [vp, vp, C.c_int, vp, vp, vp, C.c_int, vp, vp, vp, vp, C.c_int, vp, C.c_int,
                                     vp, vp, vp, vp, vp, vp]
    lib.hso_trc_activate.restype = C.c_int
    lib.hso_trc_distance_map.argtypes = [vp, vp]
    lib.hso_trc_compact.argtypes = [vp, vp]
    lib.hso_trc_trace.argtypes = [vp] * 4
    lib.hso_trc_get.argtypes = [vp] * 11
    lib.hso_ba_get_frame_eval.argtypes = [vp, vp, vp]
    lib.hso_sel_create.restype = vp
    lib.hso_sel_create.argtypes = [vp, C.c_int, C.c_int]
    lib.hso_sel_destroy.argtypes = [vp]
    lib.hso_sel_make_maps.argtypes = [vp, C.c_int, vp, vp, vp, vp, C.c_float, C.c_int, C.c_float, vp]
    lib.hso_sel_make_maps.restype = C.c_int
    lib.hso_sel_potential.argtypes = [vp]
    lib.hso_sel_potential.restype = C.c_int
    lib.hso_sel_set_potential.argtypes = [vp, C.c_int]
    lib.hso_sel_random_pattern.argtypes = [vp, vp]
    lib.hso_sel_ths.argtypes = [vp, vp, vp]
    _LIBS[name] = lib
    return lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def default_params():
    p = hs_params()
    load().hso_params_default(C.byref(p))
    return p


class OracleBA:
    """The reference's EnergyFunctional/System BA on one window, as a CPU restatement."""

    def __init__(self, scene, nthreads=1, fast=False, params=None):
        self.lib = load(fast)
        self.scene = scene
        nF = scene.n_frames
        self._keep = []
        cam = hs_camera(scene.width, scene.height, scene.n_levels, 0, float(scene.K[0, 0]), float(scene.K[1, 1]),
                        float(scene.K[0, 2]), float(scene.K[1, 2]))
        fr = (hs_frame * nF)()
        for i in range(nF):
            fr[i].worldToCam_evalPT[:] = list(scene.frames_eval[i])
            fr[i].state[:] = list(scene.frames_state[i])
            fr[i].state_zero[:] = list(scene.frames_state_zero[i])
            fr[i].ab_exposure = float(scene.frames_exposure[i])
            fr[i].frameEnergyTH = float(scene.frames_energyTH[i])
            fr[i].id = int(scene.frames_id[i])
        imgs = [np.ascontiguousarray(scene.pyramids[i][0], dtype=np.float32) for i in range(nF)]
        self._keep += imgs
        img_ptrs = (C.c_void_p * nF)(*[im.ctypes.data for im in imgs])
        arrs = dict(host=np.ascontiguousarray(scene.pt_host, np.int32), u=np.ascontiguousarray(scene.pt_u, np.float32),
                    v=np.ascontiguousarray(scene.pt_v, np.float32),
                    idepth=np.ascontiguousarray(scene.pt_idepth, np.float32),
                    idepth_zero=np.ascontiguousarray(scene.pt_idepth_zero, np.float32),
                    color=np.ascontiguousarray(scene.pt_color, np.float32),
                    weights=np.ascontiguousarray(scene.pt_weights, np.float32))
        self._keep += list(arrs.values())
        hp = getattr(scene, "pt_has_prior", None)
        hp = None if hp is None else np.ascontiguousarray(hp, np.uint8)
        self._keep.append(hp)
        pts = hs_points(scene.n_points, *[_p(arrs[k]) for k in ("host", "u", "v", "idepth", "idepth_zero", "color",
                                                                 "weights")], _p(hp))
        rp = np.ascontiguousarray(scene.res_point, np.int32)
        rt = np.ascontiguousarray(scene.res_target, np.int32)
        self._keep += [rp, rt]
        rs = hs_residuals(scene.n_res, _p(rp), _p(rt), None)
        self.params = params if params is not None else default_params()
        self.h = self.lib.hso_ba_create(C.byref(self.params), C.byref(cam), nF, C.cast(fr, C.c_void_p),
                                        C.cast(img_ptrs, C.c_void_p), C.byref(pts),
                                        C.byref(rs), nthreads)
        if not self.h:
            raise RuntimeError("hso_ba_create failed")
        self.nF = nF
        self.dim = 4 + 8 * nF

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.hso_ba_destroy(self.h)
            self.h = None

    def optimize(self, iters=6, allow_break=False):
        e = np.zeros(max(iters, 20) + 2)
        n = self.lib.hso_ba_optimize(self.h, iters, int(allow_break), _p(e))
        return n, e[: n + 1]

    def iterate(self, it0, K):
        e = np.zeros(K)
        self.lib.hso_ba_iterate(self.h, it0, K, _p(e))
        return e

    def linearize_all(self, reset=False):
        return self.lib.hso_ba_linearize_all(self.h, int(reset))

    def apply_res(self):
        self.lib.hso_ba_apply_res(self.h)

    def fix_linearization(self, max_rel_baseline, num_good):
        """System::optimize's tail (newest frame setEvalPT, setAdjointsF, setPrecalcValues, linearizeAll(true)).
        Returns (energy, drop[n_res] uint8, maxRelBaseline, numGoodResiduals)."""
        rb = np.array(max_rel_baseline, np.float32)
        ng = np.array(num_good, np.int32)
        drop = np.zeros(self.scene.n_res, np.uint8)
        e = self.lib.hso_ba_fix_linearization(self.h, _p(rb), _p(ng), _p(drop))
        return e, drop, rb, ng

    def calc_energies(self):
        """EnergyFunctional::calcLEnergyF_MT / calcMEnergyF: (L, M)."""
        el, em = C.c_double(), C.c_double()
        self.lib.hso_ba_calc_energies(self.h, C.byref(el), C.byref(em))
        return el.value, em.value

    def accumulate(self, which):
        H = np.zeros((self.dim, self.dim))
        b = np.zeros(self.dim)
        self.lib.hso_ba_accumulate(self.h, which, _p(H), _p(b))
        return H, b

    def solve_system(self, iteration):
        x = np.zeros(self.dim)
        self.lib.hso_ba_solve_system(self.h, iteration, _p(x))
        return x

    def backup_state(self):
        self.lib.hso_ba_backup_state(self.h)

    def marginalize_points(self, pts):
        """flagPointsForRemoval (per-point part) + marginalizePointsF for window points `pts`; returns (HM, bM)."""
        p = np.ascontiguousarray(pts, np.int32)
        HM, bM = np.zeros((self.dim, self.dim)), np.zeros(self.dim)
        self.lib.hso_ba_marginalize_points(self.h, len(p), _p(p), self.params.idepthFixPriorMargFac,
                                           self.params.margWeightFac, _p(HM), _p(bM))
        return HM, bM

    def marginalize_frame(self, f):
        """EnergyFunctional::marginalizeFrame(f): the (dim-8) HM / bM after removing frame f."""
        n = self.dim - 8
        HM, bM = np.zeros((n, n)), np.zeros(n)
        self.lib.hso_ba_marginalize_frame(self.h, int(f), _p(HM), _p(bM))
        return HM, bM

    def set_calib(self, value4):
        """CalibHessian::setValue of the current (unscaled) camera values; value_zero stays the scene's K."""
        self.lib.hso_ba_set_calib(self.h, _p(np.ascontiguousarray(value4, np.float64)))

    def set_marginal_prior(self, HM, bM):
        self.lib.hso_ba_set_marginal_prior(self.h, _p(np.ascontiguousarray(HM, np.float64)),
                                           _p(np.ascontiguousarray(bM, np.float64)))

    def do_step(self):
        return bool(self.lib.hso_ba_do_step(self.h))

    def residuals(self):
        n = self.scene.n_res
        out = dict(state=np.zeros(n, np.uint8), new_state=np.zeros(n, np.uint8), energy=np.zeros(n),
                   new_energy=np.zeros(n), energy_wo=np.zeros(n), resF=np.zeros((n, 8), np.float32),
                   J=np.zeros((n, 28), np.float32), JpJdF=np.zeros((n, 8), np.float32),
                   center=np.zeros((n, 3), np.float32))
        self.lib.hso_ba_get_residuals(self.h, *[_p(out[k]) for k in ("state", "new_state", "energy", "new_energy",
                                                                      "energy_wo", "resF", "J", "JpJdF", "center")])
        return out

    def points(self):
        n = self.scene.n_points
        out = {k: np.zeros(n, np.float32) for k in ("idepth", "step", "HdiF", "bdSumF", "Hdd_accAF")}
        self.lib.hso_ba_get_points(self.h, *[_p(out[k]) for k in ("idepth", "step", "HdiF", "bdSumF", "Hdd_accAF")])
        return out

    def frames(self):
        st = np.zeros((self.nF, 10))
        th = np.zeros(self.nF, np.float32)
        pose = np.zeros((self.nF, 7))
        cal = np.zeros(4)
        self.lib.hso_ba_get_frames(self.h, _p(st), _p(th), _p(pose), _p(cal))
        return dict(state=st, energyTH=th, pose=pose, calib=cal)

    def frame_eval(self):
        """Each frame's evalPT (data[7]) and state_zero[10]."""
        ev, sz = np.zeros((self.nF, 7)), np.zeros((self.nF, 10))
        self.lib.hso_ba_get_frame_eval(self.h, _p(ev), _p(sz))
        return dict(evalPT=ev, state_zero=sz)

    def precalc(self):
        out = np.zeros((self.nF * self.nF, 39), np.float32)
        self.lib.hso_ba_get_precalc(self.h, _p(out))
        return out

    def nullspaces(self):
        N = np.zeros((7, self.dim))
        self.lib.hso_ba_get_nullspaces(self.h, _p(N))
        return N

    def res_in_A(self):
        return self.lib.hso_ba_res_in_A(self.h)


# ------------------------------------------------------------------ SE3 helpers (Sophus restatement)
def se3_exp(a):
    out = np.zeros(7)
    load().hso_se3_exp(_p(np.ascontiguousarray(a, np.float64)), _p(out))
    return out


def se3_log(d):
    out = np.zeros(6)
    load().hso_se3_log(_p(np.ascontiguousarray(d, np.float64)), _p(out))
    return out


def se3_mul(a, b):
    out = np.zeros(7)
    load().hso_se3_mul(_p(np.ascontiguousarray(a, np.float64)), _p(np.ascontiguousarray(b, np.float64)), _p(out))
    return out


def se3_inverse(a):
    out = np.zeros(7)
    load().hso_se3_inverse(_p(np.ascontiguousarray(a, np.float64)), _p(out))
    return out


def se3_adj(a):
    out = np.zeros(36)
    load().hso_se3_adj(_p(np.ascontiguousarray(a, np.float64)), _p(out))
    return out.reshape(6, 6)


def se3_matrix(a):
    out = np.zeros(9)
    load().hso_se3_matrix(_p(np.ascontiguousarray(a, np.float64)), _p(out))
    return out.reshape(3, 3)


# ------------------------------------------------------------------ CoarseTracker restatement
class OracleTracker:
    """CoarseTracker + System::trackNewCoarse's try loop as a CPU restatement (oracle/track_oracle.cpp)."""

    def __init__(self, width, height, K4, n_levels, params=None, fast=False):
        self.lib = load(fast)
        self.params = params if params is not None else default_params()
        k4 = np.ascontiguousarray(K4, np.float32)
        self.w = [width >> l for l in range(n_levels)]
        self.h_ = [height >> l for l in range(n_levels)]
        self.n_levels = n_levels
        self.h = self.lib.hso_trk_create(C.byref(self.params), width, height, n_levels, _p(k4))
        self._keep = []

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.hso_trk_destroy(self.h)
            self.h = None

    @staticmethod
    def _pyr(pyr):
        arrs = [np.ascontiguousarray(p, np.float32) for p in pyr]
        return arrs, (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])

    def set_ref(self, ref_pyr, ab_exposure, aff, u, v, idepth, hdi):
        arrs, pp = self._pyr(ref_pyr)
        cols = [np.ascontiguousarray(a, np.float32) for a in (u, v, idepth, hdi)]
        self.lib.hso_trk_set_ref(self.h, C.cast(pp, C.c_void_p), float(ab_exposure),
                                 _p(np.ascontiguousarray(aff, np.float64)), len(cols[0]), *[_p(c) for c in cols])

    def set_frame(self, new_pyr, ab_exposure):
        arrs, pp = self._pyr(new_pyr)
        self.lib.hso_trk_set_frame(self.h, C.cast(pp, C.c_void_p), float(ab_exposure))

    def set_scene(self, s):
        self.set_ref(s.ref_pyr, s.ref_exposure, s.ref_aff, s.pt_u, s.pt_v, s.pt_idepth, s.pt_hdi)
        self.set_frame(s.new_pyr, s.new_exposure)

    def pc(self, lvl):
        cap = self.w[lvl] * self.h_[lvl]
        out = {k: np.zeros(cap, np.float32) for k in ("u", "v", "idepth", "color")}
        n = self.lib.hso_trk_get_ref(self.h, lvl, *[_p(out[k]) for k in ("u", "v", "idepth", "color")])
        return {k: a[:n] for k, a in out.items()}

    def calc_res(self, lvl, T7, aff, cutoff):
        res6, H, b = np.zeros(6), np.zeros(64), np.zeros(8)
        nw = C.c_int()
        self.lib.hso_trk_calc_res(self.h, lvl, _p(np.ascontiguousarray(T7, np.float64)),
                                  _p(np.ascontiguousarray(aff, np.float64)), float(cutoff), _p(res6), _p(H), _p(b),
                                  C.byref(nw))
        return res6, H.reshape(8, 8), b, nw.value

    def track(self, T7, aff, coarsest, minRes):
        T = np.array(T7, np.float64)
        a = np.array(aff, np.float64)
        lr, fl = np.zeros(5), np.zeros(3)
        its = C.c_int()
        ok = self.lib.hso_trk_track(self.h, _p(T), _p(a), coarsest, _p(np.ascontiguousarray(minRes, np.float64)),
                                    _p(lr), _p(fl), C.byref(its))
        return dict(ok=bool(ok), T=T, aff=a, lastResiduals=lr, flow=fl, iters=its.value)

    def set_sum_order(self, order):
        """Test hook: 0 = the reference's point order, 1 = reversed (every fp32 sum of calcRes / calcGSSSE formed in
        another order: the spread such a change alone causes bounds the GPU's reduction-order deviation)."""
        self.lib.hso_trk_set_sum_order(self.h, int(order))

    def lm_log(self, cap=512):
        lvl, nr, orr, inc = np.zeros(cap, np.int32), np.zeros(cap), np.zeros(cap), np.zeros(cap)
        n = self.lib.hso_trk_get_log(self.h, cap, _p(lvl), _p(nr), _p(orr), _p(inc))
        n = min(n, cap)
        return lvl[:n], nr[:n], orr[:n], inc[:n]

    def track_tries(self, tries, aff_last, lastCoarseRMSE, reTrackThreshold=1.5, coarsest=None):
        tr = np.ascontiguousarray(np.asarray(tries, np.float64).reshape(-1, 7))
        if coarsest is None:
            coarsest = min(self.n_levels - 1, 4)
        T, a, ach, fl = np.zeros(7), np.zeros(2), np.zeros(5), np.zeros(3)
        good, n = C.c_int(), C.c_int()
        self.lib.hso_trk_track_tries(self.h, len(tr), _p(tr), _p(np.ascontiguousarray(aff_last, np.float64)),
                                     _p(np.ascontiguousarray(lastCoarseRMSE, np.float64)), float(reTrackThreshold),
                                     coarsest, _p(T), _p(a), _p(ach), _p(fl), C.byref(good), C.byref(n))
        return dict(T=T, aff=a, achievedRes=ach, flowVecs=fl, haveOneGood=bool(good.value), tryIterations=n.value)


# ------------------------------------------------------------------ ImmaturePoint::traceOn restatement
TRACE_FIELDS = ("status", "idepth_min", "idepth_max", "quality", "uv", "interval", "energyTH", "color", "weights",
                "gradH")


def trace_hosts_array(KRKi, Kt, aff):
    """[nH] hs_trace_host records (KRKi[9], Kt[3], aff[2] float32) as a contiguous float32 [nH, 14] array."""
    return np.ascontiguousarray(np.concatenate([np.asarray(KRKi, np.float32).reshape(-1, 9),
                                                np.asarray(Kt, np.float32).reshape(-1, 3),
                                                np.asarray(aff, np.float32).reshape(-1, 2)], 1))


class OracleTracer:
    """ImmaturePoint ctor + System::traceNewCoarse / traceOn as a CPU restatement (oracle/trace_oracle.cpp)."""

    def __init__(self, width, height, params=None, fast=False):
        self.lib = load(fast)
        self.params = params if params is not None else default_params()
        self.W, self.H = width, height
        self.h = self.lib.hso_trc_create(C.byref(self.params), width, height)
        self.n = 0

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.hso_trc_destroy(self.h)
            self.h = None

    def add_points(self, host_imgs, host, u, v):
        imgs = [np.ascontiguousarray(a, np.float32) for a in host_imgs]
        pp = (C.c_void_p * len(imgs))(*[a.ctypes.data for a in imgs])
        h, uu, vv = (np.ascontiguousarray(host, np.int32), np.ascontiguousarray(u, np.float32),
                     np.ascontiguousarray(v, np.float32))
        rc = self.lib.hso_trc_add_points(self.h, len(imgs), C.cast(pp, C.c_void_p), len(h), _p(h), _p(uu), _p(vv))
        assert rc == 0
        self.n += len(h)

    def set_state(self, idepth_min=None, idepth_max=None, quality=None, status=None, interval=None):
        arr = [None if a is None else np.ascontiguousarray(a, dt)
               for a, dt in ((idepth_min, np.float32), (idepth_max, np.float32), (quality, np.float32),
                             (status, np.uint8), (interval, np.float32))]
        self.lib.hso_trc_set_state(self.h, *[_p(a) for a in arr])

    def trace(self, new_img, KRKi, Kt, aff):
        img = np.ascontiguousarray(new_img, np.float32)
        hosts = trace_hosts_array(KRKi, Kt, aff)
        counts = np.zeros(6, np.int32)
        self.lib.hso_trc_trace(self.h, _p(img), _p(hosts), _p(counts))
        return counts

    def set_scene(self, s):
        self.add_points(s.host_imgs, s.pt_host, s.pt_u, s.pt_v)

    def points(self):
        n = self.n
        out = dict(status=np.zeros(n, np.uint8), idepth_min=np.zeros(n, np.float32),
                   idepth_max=np.zeros(n, np.float32), quality=np.zeros(n, np.float32), uv=np.zeros((n, 2), np.float32),
                   interval=np.zeros(n, np.float32), energyTH=np.zeros(n, np.float32),
                   color=np.zeros((n, 8), np.float32), weights=np.zeros((n, 8), np.float32),
                   gradH=np.zeros((n, 4), np.float32))
        self.lib.hso_trc_get(self.h, *[_p(out[k]) for k in TRACE_FIELDS])
        return out


    def set_types(self, my_type):
        self.lib.hso_trc_set_types(self.h, _p(np.ascontiguousarray(my_type, np.float32)))

    def activatePointsMT(self, frame_imgs, K4, frames, pairs, act_frame, act_u, act_v, act_idepth, ef_nPoints,
                         currentMinActDist, order=None):
        """System::activatePointsMT restated (oracle/trace_oracle.cpp).  frames / pairs: numpy records laid out as
        hs_act_frame / hs_act_pair; frame_imgs[nF]: DirPyr[0] of the window keyframes."""
        imgs = [np.ascontiguousarray(a, np.float32) for a in frame_imgs]
        pp = (C.c_void_p * len(imgs))(*[a.ctypes.data for a in imgs])
        k4 = np.ascontiguousarray(K4, np.float32)
        fr, pr = np.ascontiguousarray(frames), np.ascontiguousarray(pairs)
        af = np.ascontiguousarray(act_frame, np.int32)
        au, av, ai = (np.ascontiguousarray(x, np.float32) for x in (act_u, act_v, act_idepth))
        od = None if order is None else np.ascontiguousarray(order, np.int32)
        n = self.n
        action, idepth, res_in = np.zeros(n, np.uint8), np.zeros(n, np.float32), np.zeros(n, np.uint8)
        activated = np.zeros(max(n, 1), np.int32)
        cmad = C.c_float(currentMinActDist)
        na = C.c_int()
        rc = self.lib.hso_trc_activate(self.h, _p(k4), len(fr), C.cast(pp, C.c_void_p), _p(fr), _p(pr), len(af),
                                       _p(af), _p(au), _p(av), _p(ai), int(ef_nPoints), C.byref(cmad),
                                       0 if od is None else len(od), _p(od), _p(action), _p(idepth), _p(res_in),
                                       _p(activated), C.byref(na))
        assert rc == 0
        return dict(action=action, idepth=idepth, res_in=res_in, activated=activated[: na.value],
                    currentMinActDist=cmad.value)

    def distance_map(self):
        out = np.zeros((self.H >> 1) * (self.W >> 1), np.float32)
        self.lib.hso_trc_distance_map(self.h, _p(out))
        return out.reshape(self.H >> 1, self.W >> 1)

    def compact(self, keep):
        k = np.ascontiguousarray(keep, np.uint8)
        self.lib.hso_trc_compact(self.h, _p(k))
        self.n = int(k.astype(bool).sum())


# ------------------------------------------------------------------ Frame::CreateDirPyrs restatement
def dir_pyramid(img, n_levels):
    """([(h_l, w_l, 3) float32 DirPyr levels], [(h_l, w_l) absSquaredGrad]) of a W x H fp32 image."""
    img = np.ascontiguousarray(img, np.float32)
    H, W = img.shape
    sizes = [(H >> l, W >> l) for l in range(n_levels)]
    out = np.zeros(sum(h * w * 3 for h, w in sizes), np.float32)
    ag = np.zeros(sum(h * w for h, w in sizes), np.float32)
    load().hso_dir_pyramid(W, H, n_levels, _p(img), _p(out), _p(ag))
    pyr, grads, o3, o1 = [], [], 0, 0
    for h, w in sizes:
        pyr.append(out[o3:o3 + h * w * 3].reshape(h, w, 3))
        grads.append(ag[o1:o1 + h * w].reshape(h, w))
        o3 += h * w * 3
        o1 += h * w
    return pyr, grads


class PixelSelector:
    """PixelSelector (Src/PixelSelector.cpp:14-418) restated (oracle/sel_oracle.cpp)."""

    def __init__(self, width, height, params=None, fast=False):
        self.lib = load(fast)
        self.W, self.H = width, height
        self.h = self.lib.hso_sel_create(C.byref(params) if params is not None else None, width, height)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.hso_sel_destroy(self.h)
            self.h = None

    def makeMaps(self, frame_id, dirpyr0, absg, density, recursionsLeft=1, thFactor=1.0):
        """-> (selection map (H, W) float32, numHaveSub).  dirpyr0: (H, W, 3); absg: levels 0..2."""
        d = np.ascontiguousarray(dirpyr0, np.float32)
        g = [np.ascontiguousarray(x, np.float32) for x in absg[:3]]
        out = np.zeros((self.H, self.W), np.float32)
        n = self.lib.hso_sel_make_maps(self.h, frame_id, _p(d), _p(g[0]), _p(g[1]), _p(g[2]), density,
                                       recursionsLeft, thFactor, _p(out))
        return out, n

    @property
    def currentPotential(self):
        return self.lib.hso_sel_potential(self.h)

    @currentPotential.setter
    def currentPotential(self, p):
        self.lib.hso_sel_set_potential(self.h, int(p))

    def randomPattern(self):
        out = np.zeros(self.W * self.H, np.uint8)
        self.lib.hso_sel_random_pattern(self.h, _p(out))
        return out

    def ths(self):
        n = (self.W // 32) * (self.H // 32)
        a, b = np.zeros(n, np.float32), np.zeros(n, np.float32)
        self.lib.hso_sel_ths(self.h, _p(a), _p(b))
        return a.reshape(self.H // 32, self.W // 32), b.reshape(self.H // 32, self.W // 32)


class OracleRefiner:
    """DirectRefinement (Src/Initializer.cpp:1330-2270) as a CPU restatement (oracle/refine_oracle.cpp)."""

    def __init__(self, scene, fast=False):
        self.lib = load(fast)
        s = scene
        k4 = np.ascontiguousarray(s.K4, np.float64)
        self._img = [np.ascontiguousarray(s.img1, np.float32), np.ascontiguousarray(s.img2, np.float32)]
        self.h = self.lib.hso_ref_create(s.width, s.height, _p(k4), _p(self._img[0]), _p(self._img[1]),
                                         float(s.expo1), float(s.expo2))
        self.n = s.n_points
        cols = [np.ascontiguousarray(s.u, np.float32), np.ascontiguousarray(s.v, np.float32),
                np.ascontiguousarray(s.tri, np.uint8), np.ascontiguousarray(s.z, np.float32)]
        self.lib.hso_ref_set_points(self.h, self.n, *[_p(c) for c in cols])

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.hso_ref_destroy(self.h)
            self.h = None

    def calc_res(self, T7, aff=(0.0, 0.0)):
        H, Hs = np.zeros(64, np.float32), np.zeros(64, np.float32)
        b, bs, res = np.zeros(8, np.float32), np.zeros(8, np.float32), np.zeros(3, np.float32)
        self.lib.hso_ref_calc(self.h, _p(np.ascontiguousarray(T7, np.float64)), _p(np.ascontiguousarray(aff, np.float64)),
                              _p(H), _p(b), _p(Hs), _p(bs), _p(res))
        return H.reshape(8, 8), b, Hs.reshape(8, 8), bs, res

    def refine(self, T7):
        T = np.array(T7, np.float64)
        aff = np.zeros(2)
        sn = C.c_int()
        it = self.lib.hso_ref_refine(self.h, _p(T), _p(aff), C.byref(sn))
        return T, it, bool(sn.value)

    def log(self):
        out = np.zeros((1001, 8), np.float32)
        n = self.lib.hso_ref_get_log(self.h, 1001, _p(out))
        return out[:n]

    def points(self):
        f7 = np.zeros((self.n, 7), np.float32)
        g2 = np.zeros((self.n, 2), np.uint8)
        jb = np.zeros((self.n, 10), np.float32)
        self.lib.hso_ref_get_points(self.h, _p(f7), _p(g2), _p(jb))
        return _ref_points(f7, g2, jb)


def _ref_points(f7, g2, jb):
    return dict(idepth=f7[:, 0], idepth_new=f7[:, 1], iR=f7[:, 2], energy_new0=f7[:, 3], energy_new1=f7[:, 4],
                maxstep=f7[:, 5], lastHessian_new=f7[:, 6], isGood=g2[:, 0], isGood_new=g2[:, 1], jb_new=jb)
