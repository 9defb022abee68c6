"""Loader of the product library ``h-slam_amd/lib/libhslam_amd.so`` (HIP, gfx950).

There is no CPU fallback: if the library is missing, or no HIP device is present
when a context is created, the call raises.  Build with ``make -C h-slam_amd/csrc``
(or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libhslam_amd.so")
# experiment builds only (h-slam_amd/csrc/Makefile `variant`); unset, the in-tree product library is loaded
if os.environ.get("HSLAM_AMD_LIB"):
    LIB_PATH = os.path.abspath(os.environ["HSLAM_AMD_LIB"])

# data-contract structs (include/hs_types.h)


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


# exported symbols of include/hs_ba.h (argument types)
VP, I, D = C.c_void_p, C.c_int, C.c_double
SIGNATURES = {
    "hs_params_default": ([VP], I),
    "hs_last_error": ([], C.c_char_p),
    "hs_create": ([VP, VP, I], I),
    "hs_destroy": ([VP], None),
    "hs_ba_set_window": ([VP, VP, I, VP, VP, VP, VP], I),
    "hs_ba_linearize": ([VP, I, VP], I),
    "hs_ba_solve_system": ([VP, I, VP], I),
    "hs_ba_do_step": ([VP, VP], I),
    "hs_ba_optimize": ([VP, I, I, VP, VP], I),
    "hs_ba_iterate": ([VP, I, I, VP], I),
    "hs_ba_fix_linearization": ([VP, VP, VP, VP, VP, VP], I),
    "hs_ba_calc_energies": ([VP, VP, VP], I),
    "hs_ba_get_system": ([VP, I, VP, VP], I),
    "hs_ba_get_residuals": ([VP] * 7, I),
    "hs_ba_get_points": ([VP] * 5, I),
    "hs_ba_get_frames": ([VP] * 5, I),
    "hs_ba_set_marginal_prior": ([VP, VP, VP], I),
    "hs_ba_marginalize_points": ([VP, I, VP, VP, VP], I),
    "hs_ba_marginalize_frame": ([VP, I, VP, VP], I),
    "hs_ba_get_timings": ([VP, VP], I),
    "hs_ba_time_linearize": ([VP, I, VP], I),
    "hs_ba_get_partition": ([VP, VP], I),
    "hs_ba_reserve": ([VP, VP, I], I),
    "hs_ba_insert_frame": ([VP, VP, VP], I),
    "hs_ba_set_frame_image": ([VP, I, VP], I),
    "hs_ba_set_frame_image_raw": ([VP, I, VP], I),
    "hs_ba_set_frame_image_device": ([VP, I, VP], I),
    "hs_ba_insert_points": ([VP, VP, VP, VP, VP], I),
    "hs_ba_insert_residuals": ([VP, I, VP, VP, VP], I),
    "hs_ba_add_residuals_to_newest": ([VP, VP], I),
    "hs_ba_drop_residuals": ([VP, I, VP, VP], I),
    "hs_ba_drop_inactive_residuals": ([VP, VP], I),
    "hs_ba_remove_points": ([VP, I, VP], I),
    "hs_ba_remove_points_without_residuals": ([VP, VP, VP], I),
    "hs_ba_remove_frame": ([VP, I, I], I),
    "hs_ba_make_idx": ([VP, VP, VP, VP], I),
    "hs_ba_get_structure": ([VP] * 5, I),
    "hs_ba_get_marginal_prior": ([VP, VP, VP], I),
    "hs_ba_synchronize": ([VP], I),
    "hs_ba_get_point_state": ([VP] * 6, I),
    "hs_debug_state_size": ([], I),
    "hs_debug_get_state": ([VP, VP], I),
    "hs_debug_nullspace_error": ([VP, VP], I),
    "hs_debug_set_state": ([VP, VP], I),
    "hs_comm_get_unique_id": ([VP], I),
    "hs_comm_init": ([VP, VP, I, I], I),
    "hs_comm_size": ([VP, VP, VP], I),
    "hs_comm_set_timeout": ([VP, I], I),
    "hs_ba_set_event_timing": ([VP, I], I),
    "hs_ba_get_frame_eval": ([VP, VP, VP], I),
    # test hooks (not in the header): an in-process rank group on one device, the multi-rank exchange by copies
    "hs_ba_debug_group": ([VP, I, I], I),
    "hs_ba_group_linearize": ([VP, I, I, VP], I),
    "hs_ba_group_iterate": ([VP, I, I, I, VP], I),
    # test hooks (not in the header): a stale adjoint upload, a stalled stream
    "hs_debug_stale_adjoints": ([VP, I], I),
    "hs_debug_stall": ([VP, I], I),
    # include/hs_track.h
    "hs_tracker_create": ([VP, VP, I, I, I, I, VP], I),
    "hs_tracker_destroy": ([VP], None),
    "hs_tracker_set_ref": ([VP, VP, C.c_float, VP, I, VP, VP, VP, VP], I),
    "hs_tracker_get_ref": ([VP, I, VP, VP, VP, VP, VP], I),
    "hs_tracker_set_frame": ([VP, VP, C.c_float], I),
    "hs_tracker_calc_res": ([VP, I, VP, VP, C.c_float, VP, VP, VP, VP], I),
    "hs_tracker_track": ([VP, VP, VP, I, VP, VP, VP, VP], I),
    "hs_tracker_track_tries": ([VP, I, VP, VP, VP, C.c_float, VP, VP, VP, VP, VP, VP], I),
    "hs_tracker_get_lm_log": ([VP, I, I, VP, VP, VP, VP, VP], I),
    "hs_tracker_last_ms": ([VP, VP], I),
    "hs_tracker_set_event_timing": ([VP, I], I),
    "hs_tracker_last_stats": ([VP, I, VP, VP, VP], I),
    "hs_tracker_launch_info": ([VP, VP, VP], I),
    "hs_tracker_set_frame_raw": ([VP, VP, C.c_float], I),
    "hs_tracker_set_ref_ba": ([VP, VP, I, C.c_float, VP], I),
    "hs_tracker_frame_texels": ([VP, I, VP], I),
    "hs_tracker_frame_to_ba": ([VP, VP, I], I),
    # include/hs_pyr.h
    "hs_dir_pyramid": ([I, I, I, I, VP, VP, VP], I),
    # include/hs_trace.h
    "hs_tracer_create": ([VP, VP, I, I, I, I], I),
    "hs_tracer_destroy": ([VP], None),
    "hs_tracer_set_host_image": ([VP, I, VP], I),
    "hs_tracer_add_points": ([VP, I, VP, VP, VP], I),
    "hs_tracer_clear": ([VP], I),
    "hs_tracer_set_state": ([VP] * 6, I),
    "hs_tracer_set_types": ([VP, VP], I),
    "hs_tracer_activate": ([VP, VP, I, VP, VP, I, VP, VP, VP, VP, I, VP, I, VP, VP, VP, VP, VP, VP], I),
    "hs_tracer_get_distance_map": ([VP, VP], I),
    "hs_tracer_compact": ([VP, VP], I),
    "hs_tracer_set_frame": ([VP, VP], I),
    "hs_tracer_set_frame_raw": ([VP, VP], I),
    "hs_tracer_trace": ([VP, I, VP, VP], I),
    "hs_tracer_get_points": ([VP] * 12, I),
    "hs_tracer_reinit": ([VP], I),
    "hs_tracer_last_stats": ([VP, VP, VP], I),
    # include/hs_select.h
    "hs_selector_create": ([VP, VP, I, I, I], I),
    "hs_selector_destroy": ([VP], None),
    "hs_selector_make_maps": ([VP, I, VP, VP, VP, VP, C.c_float, I, C.c_float, VP, VP], I),
    "hs_selector_make_maps_raw": ([VP, I, VP, C.c_float, I, C.c_float, VP, VP], I),
    "hs_selector_get_potential": ([VP, VP], I),
    "hs_selector_set_potential": ([VP, I], I),
    "hs_selector_last_stats": ([VP, VP, VP], I),
    # include/hs_refine.h
    "hs_refiner_create": ([VP, I, I, I, VP], I),
    "hs_refiner_destroy": ([VP], None),
    "hs_refiner_set_frames": ([VP, VP, VP, C.c_float, C.c_float], I),
    "hs_refiner_set_points": ([VP, I, VP, VP, VP, VP], I),
    "hs_refiner_refine": ([VP, VP, VP, VP, VP, VP], I),
    "hs_refiner_calc_res": ([VP, VP, VP, VP, VP, VP, VP, VP], I),
    "hs_refiner_get_points": ([VP, VP, VP, VP], I),
    "hs_refiner_get_log": ([VP, I, VP], I),
    "hs_refiner_last_ms": ([VP, VP], I),
}

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C h-slam_amd/csrc` "
                           "(there is no CPU fallback for the hot path)")
    lib = C.CDLL(LIB_PATH)
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


class HsError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise HsError(f"hs call failed ({rc}): {load().hs_last_error().decode(errors='replace')}")


def ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def default_params():
    p = hs_params()
    check(load().hs_params_default(C.byref(p)))
    return p
