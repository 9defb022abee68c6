#!/usr/bin/env python3
"""bench.py — point-residuals/s of H-SLAM's windowed photometric BA on MI355X.

Workload (BASELINE.json configs[3], "C4"): full windowed photometric BA including the
Schur complement, 8 keyframes x 2000 active points, 640x480 synthetic scene
(hslam_amd.scene, seed 20261015), ~13.6k point-residuals.  One *step* = one
Gauss-Newton iteration of System::optimize (solveSystemF + doStepFromBackup +
linearizeAll + applyRes + the accumulations), i.e. hs_ba_iterate(1).  Multi-GPU: one rank
per GPU; by default every rank holds 2000 points of one 8-keyframe window of 2000 N points
("weak" scaling: at N = 1 the metric's own window; SURVEY.md §8e shards points p % N), and
--scaling strong shards the metric's own 2000-point window over the ranks (at
2000 points the step is the single-CU solve plus latency-bound launches, so strong scaling
cannot gain there).  Per step one RCCL exchange: the ranks' system vectors + energies and
their newest-frame candidates, all-gathered in one group call; every rank sums the vectors in
rank order and selects the threshold beside the solve.  --workload ba-kitti runs the same window at KITTI 1232x368 (C5's BA half).

JSON line fields follow the driver contract; `roofline` is for the dominant kernel
(hs_k_linearize, timed with HIP events on the context's own stream), `cpu_baseline` is
the oracle's C++ restatement of the reference SSE/IndexThreadReduce path timed on
this host (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "h-slam_amd"))

METRIC = "point-residuals/sec in windowed photometric BA (8 KF × 2k pts), 1→8 GPU"
BYTES_PER_PRES = 448      # algorithmic bytes per point-residual (fused K1-K5: hs_k_lin accumulates in
                          # registers, no per-residual Jacobian record leaves the kernel)
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
STRONG_LARGE_POINTS = 200000  # N > 1: the window whose strong scaling is reported beside the metric's own
TRACK_BYTES_PER_POINT_PASS = 64  # CoarseTracker bytes per reference point per calcRes+GS pass


def pmc_traffic(points, kernel: str = "hs_k_lin"):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/*_pmc_traffic.json,
    made by tools/archive/r03_pmc.sh + tools/pmc_summary.py: separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this
    bench on the same workload).  points: the workload key -- the C4 window's point count, "kitti<N>" for
    --workload ba-kitti, or the workload name (trace, track).  None when no pass for it has been committed."""
    import glob
    import re

    def version(f):  # r01_v10 after r01_v9: numeric order of the round and version fields
        return [int(x) for x in re.findall(r"\d+", os.path.basename(f))]

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), key=version)
    for f in reversed(files):
        try:
            d = json.load(open(f))
            k = d["points_per_gpu"][str(points)][kernel]
            return k["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
        except (KeyError, ValueError, OSError):
            continue
    return None, None


def pmc_roof(key, kernel: str):
    """Counter evidence for `kernel` on workload `key` from the newest committed profiles/*_pmc_roof.json
    (tools/archive/r04_pmc.sh + tools/pmc_roof.py: separate FETCH_SIZE / WRITE_SIZE / SQ+GRBM rocprofv3 passes with the
    kernel trace beside them): counter DRAM GB/s over the traced launch duration and the SQ issue split.
    {} when no pass for it has been committed."""
    import glob
    import re

    def version(f):
        return [int(x) for x in re.findall(r"\d+", os.path.basename(f))]

    for f in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_roof.json")), key=version)):
        try:
            k = json.load(open(f))["keys"][str(key)][kernel]
        except (KeyError, ValueError, OSError):
            continue
        out = {n: k[n] for n in ("dram_gbs", "dram_frac", "valu_busy_per_simd", "valu_issue_frac", "wait_frac",
                                 "issue_stall_frac", "effective_clock_mhz", "hbm_bytes_per_launch",
                                 "avg_launch_us") if k.get(n) is not None}
        out["source"] = os.path.relpath(f, ROOT)
        return out
    return {}


VALU_LATENCY_FLOOR = 0.3  # below this fraction of both roofs a kernel is latency-bound, not roof-bound


def roof_binding(ctr: dict, hbm_alg_frac: float):
    """What limits a kernel, from its committed counters (pmc_roof), beside the roof its `frac` is priced against.
    `bound` is always "hbm" (the contract's field: achieved is algorithmic bytes per second over the 8 TB/s spec);
    `limiter` says which roof the counters put the kernel closest to: the VALU roof fraction (VALU busy per SIMD
    = 4 SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)) against the HBM fraction (counter DRAM bytes per
    second over the spec, and the algorithmic fraction): "valu" or "hbm" when that roof is the larger one and at least
    VALU_LATENCY_FLOOR, "latency" when neither reaches the floor (the kernel waits on dependent round trips)."""
    valu = ctr.get("valu_busy_per_simd")
    dram = ctr.get("dram_frac")
    out = {"bound": "hbm", "valu_frac": valu, "hbm_counter_frac": dram, "hbm_alg_frac": hbm_alg_frac}
    if valu is None:
        return out
    hbm = max(dram or 0.0, hbm_alg_frac)
    if max(valu, hbm) < VALU_LATENCY_FLOOR:
        out["limiter"] = "latency"
    elif valu >= (dram or 0.0):
        out["limiter"] = "valu"
    else:
        out["limiter"] = "hbm"
    return out


def speedup(res):
    """speedup_vs_cpu, and its range over the CPU baseline's repeats when it has them (the host's noise)."""
    cb = res["cpu_baseline"]
    res["speedup_vs_cpu"] = res["value"] / cb["value"]
    rv = cb.get("repeat_values")
    if rv:
        res["speedup_vs_cpu_range"] = [res["value"] / max(rv), res["value"] / min(rv)]


def host_cpu():
    """Model name of the timing host's CPU (lscpu's 'Model name', read from /proc/cpuinfo) and its logical CPUs."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


def cpu_baseline(points: int, seconds: float, kitti: bool = False):
    """Oracle (C++ restatement of the reference CPU path) on this host, built -O2 -march=native here (the
    reference's flags, CMakeLists.txt:56 + build.sh:4,64; falls back to the portable x86-64-v3 build if the native
    build fails).  Timed twice: with an IndexThreadReduce-style pool of T threads (T = the host threads this job
    may use) and single-threaded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_ffi import OracleBA  # test infrastructure: the CPU baseline leg only
    from hslam_amd.scene import make_ba_scene, make_ba_scene_kitti

    threads = os.cpu_count() or 1
    env_t = os.environ.get("OMP_NUM_THREADS")
    if env_t and env_t.isdigit():
        threads = min(threads, int(env_t))
    flags = "-O2 -march=native"
    try:
        import oracle_ffi
        oracle_ffi.load("native")
        build = "native"
    except Exception:  # no compiler on this host: the portable build
        build, flags = True, "-O2 -march=x86-64-v3"
    scene = make_ba_scene_kitti(points) if kitti else make_ba_scene(n_points=points)

    def timed(nthreads, budget):
        """Per-iteration times of one oracle window over `budget` seconds (after 3 warm-up iterations); the rate
        is taken from the median iteration (host noise on a shared machine shows up as slow outliers)."""
        o = OracleBA(scene, nthreads=nthreads, fast=build)
        o.linearize_all(reset=True)
        o.apply_res()
        o.iterate(0, 3)  # warm-up
        it, t, per = 0, 0.0, []
        while t < budget or it < 3:
            t0 = time.perf_counter()
            o.iterate(3 + it, 1)
            dt = time.perf_counter() - t0
            per.append(dt)
            t += dt
            it += 1
        med = float(np.median(per))
        return {"value": scene.n_res / med, "iterations": it, "median_ms_per_step": med * 1e3,
                "mean_ms_per_step": t / it * 1e3, "spread_ms": [min(per) * 1e3, max(per) * 1e3]}

    # the pool figure is the median of 3 repeats (each its own window and warm-up): one box's host noise varies
    # from run to run, the repeats' spread is reported beside it
    reps = sorted((timed(threads, seconds * 0.5 / 3) for _ in range(3)), key=lambda r: r["value"])
    mt = dict(reps[1])
    mt["repeat_values"] = [r["value"] for r in reps]
    one = timed(1, seconds * 0.25)
    # pool scaling below the job's share, side by side (T = nproc is not run: the GPU pool asks jobs to keep
    # worker pools to their share of a shared host; the curve shows how far the port scales before that)
    scaling = {str(threads): mt["value"], "1": one["value"]}
    for t in (4, 8):
        if t < threads:
            scaling[str(t)] = timed(t, seconds * 0.125)["value"]
    model, ncpu = host_cpu()
    cfg = "C5 BA window (8 KF x %d pts, KITTI 1232x368)" % points if kitti else "C4 window (8 KF x %d pts)" % points
    return {
        "value": mt["value"],
        "unit": "point-residuals/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{mt['iterations']} GN iterations of the {cfg}, {scene.n_res} residuals, after 3 warm-up "
                  f"iterations, IndexThreadReduce-style pool with {threads} threads (chunk 50 / ceil(n/T)); value "
                  f"from the median iteration {mt['median_ms_per_step']:.2f} ms (mean {mt['mean_ms_per_step']:.2f}), "
                  f"the median of 3 repeats; oracle built {flags} on this host",
        "repeat_values": mt["repeat_values"],
        "repeat_spread_rel": (mt["repeat_values"][-1] - mt["repeat_values"][0]) / mt["value"],
        "median_ms_per_step": mt["median_ms_per_step"],
        "mean_ms_per_step": mt["mean_ms_per_step"],
        "spread_ms": mt["spread_ms"],
        "single_thread": one,
        "pool_scaling_value_by_threads": scaling,
        "host_cpu_model": model,
        "host_logical_cpus": ncpu,
        "cores_note": ("the pool uses the host threads this job is allotted (OMP_NUM_THREADS; 16 per GPU on the GPU "
                       "pool, which asks jobs to size worker pools to that share), not every logical CPU of the "
                       "shared machine (host_logical_cpus); the reference sizes its pool by ProcessorCount "
                       "(CMakeLists.txt:52-54), i.e. it would take the whole host"),
        "build_flags": flags,
    }


TRACE_BYTES_PER_STEP = 8 * 4 * 12   # SURVEY.md §8(d) traceOn unit: 8 pattern taps x 4 texels x 12 B per search step


def bench_trace(args):
    """C5 (BASELINE.json configs[4]): ImmaturePoint::traceOn of 20k immature points (8 hosts x 2.5k, KITTI
    1232x368, first trace: idepth_max = NaN, full maxPixSearch).  One step = the ImmaturePoint ctor of every
    point on the device (a fresh first-trace state) + traceNewCoarse over all of them.  Single GPU
    (traceOn shards by point with no collective)."""
    from hslam_amd.scene import make_trace_scene
    from hslam_amd.trace import ImmatureTracer

    s = make_trace_scene(n_points=args.points if args.points != 2000 else 20000)
    t = ImmatureTracer(s.width, s.height, s.n_points)
    t.set_scene(s)
    for _ in range(max(1, args.warmup)):
        t.reinit()
        t.traceNewCoarse(s.KRKi, s.Kt, s.aff, counts=False)
    t.last_stats()
    kern, steps = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t.reinit()
        t.traceNewCoarse(s.KRKi, s.Kt, s.aff, counts=False)
        ms, st = t.last_stats()  # waits for the step: per-step device time of the traceOn kernel
        kern += ms
        steps += st
    dt = time.perf_counter() - t0
    counts = t.traceNewCoarse(s.KRKi, s.Kt, s.aff)  # one more (second-trace state) only for the tallies
    kern_ms = kern / args.steps
    algo_bytes = steps / args.steps * TRACE_BYTES_PER_STEP
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    res = {
        "metric": "immature points traced/sec (ImmaturePoint::traceOn, C5 KITTI 1232x368, 20k points)",
        "value": s.n_points * args.steps / dt, "unit": "points/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "C5 (BASELINE.json configs[4]) traceOn part: ctor + first traceOn of 20k immature "
                               "points, 8 host KFs, 1232x368", "points": s.n_points, "hosts": s.n_hosts,
                   "search_steps_per_trace": steps // args.steps, "parallelism": "single GPU"},
        "roofline": dict({"bound": "hbm", "kernel": "hs_k_trace_on", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_roof("trace", "hs_k_trace_on").get("hbm_bytes_per_launch", pmc_traffic("trace", "hs_k_trace_on")[0]),
                     "bytes_per_unit": TRACE_BYTES_PER_STEP, "unit_of_bytes": "discrete-search step (GN taps excluded)",
                     "avg_launch_ms": kern_ms, "counters": pmc_roof("trace", "hs_k_trace_on")},
                     **roof_binding(pmc_roof("trace", "hs_k_trace_on"), achieved / HBM_PEAK_GBS)),
        "second_trace_counts": dict(zip(("good", "oob", "outlier", "skipped", "badcondition", "uninitialized"),
                                        map(int, counts))),
        "cpu_baseline": None,
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle_ffi import OracleTracer  # test infrastructure: the CPU baseline leg only
        o = OracleTracer(s.width, s.height, fast=True)
        o.set_scene(s)
        n, tt = 0, 0.0
        while tt < args.cpu_seconds / 2 and n < 200:
            o2 = OracleTracer(s.width, s.height, fast=True)
            o2.set_scene(s)
            t1 = time.perf_counter()
            o2.trace(s.new_img, s.KRKi, s.Kt, s.aff)
            tt += time.perf_counter() - t1
            n += 1
        res["cpu_baseline"] = {"value": s.n_points * n / tt, "unit": "points/s", "cores": 1, "kind": "port",
                               "sample": f"{n} first traces of the same 20k points (System::traceNewCoarse is serial "
                                         "in the reference, Src/Mapping.cpp:494-538), ctor excluded"}
        speedup(res)
    t.close()
    return res


def bench_track(args):
    """C2 (BASELINE.json configs[1]): CoarseTracker::trackNewestCoarse, 5-level pyramid, 640x480, one
    hypothesis from identity.  One step = one trackNewestCoarse on the device."""
    from hslam_amd.scene import make_track_scene
    from hslam_amd.track import CoarseTracker

    s = make_track_scene(n_points=2000, n_levels=5)
    ct = CoarseTracker(s.width, s.height, s.K4, s.n_levels)
    ct.set_scene(s)
    T0 = np.array([0, 0, 0, 1.0, 0, 0, 0])
    minRes = np.full(5, np.nan)
    for _ in range(max(1, args.warmup)):
        ct.trackNewestCoarse(T0, [0.0, 0.0], s.n_levels - 1, minRes)
    # the timed loop in the library's default mode (no per-call event pair: the host takes the results from the
    # hypotheses' done words); the device time per track from an untimed loop with event timing on afterwards
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ok, T, a = ct.trackNewestCoarse(T0, [0.0, 0.0], s.n_levels - 1, minRes)
    dt = time.perf_counter() - t0
    ct.set_event_timing(True)
    dev = 0.0
    for _ in range(args.steps):
        ct.trackNewestCoarse(T0, [0.0, 0.0], s.n_levels - 1, minRes)
        dev += ct.last_ms()
    # roofline: 64 B of algorithmic traffic and ~230 FLOP per point-pass (reference point
    # x calcRes(+calcGSSSE) pass); the units come from the kernel's own pass counters
    _, passes, point_passes = ct.last_stats(0)
    dev_ms = dev / args.steps
    if dev_ms <= 0:  # no device timing (HS_TRK_NOEVT=1): the host clock per call
        dev_ms = dt * 1e3 / args.steps
    achieved = point_passes * TRACK_BYTES_PER_POINT_PASS / (dev_ms * 1e-3) / 1e9
    res = {
        "metric": "frames tracked/sec (CoarseTracker::trackNewestCoarse, C2 640x480, 5 levels)",
        "value": args.steps / dt, "unit": "frames/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps, "higher_is_better": True, "scaling": "replicas only",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "C2 (BASELINE.json configs[1]): trackNewestCoarse from identity, 2000 reference "
                               "points, 640x480, 5 levels", "ok": bool(ok), "device_ms_per_track": dev_ms,
                   "passes": passes, "point_passes": point_passes,
                   "timing": "value / ms_per_step: host clock over the timed loop in the library's default mode "
                             "(no per-call event pair, done-word results); device_ms_per_track: the event pair "
                             "(hs_tracker_set_event_timing), in an untimed loop after it"},
        "roofline": {"bound": "hbm", "kernel": "hs_k_track", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": pmc_roof("track", "hs_k_track").get("hbm_bytes_per_launch",
                                                                    pmc_traffic("track", "hs_k_track")[0]),
                     "counters": pmc_roof("track", "hs_k_track"),
                     "bytes_per_unit": TRACK_BYTES_PER_POINT_PASS,
                     "unit_of_bytes": "reference point x calcRes+calcGSSSE pass", "units_per_launch": point_passes,
                     "avg_launch_ms": dev_ms, "flop_per_unit": 230,
                     "achieved_tflops": point_passes * 230 / (dev_ms * 1e-3) / 1e12,
                     "timing": "HIP events around the single hs_k_track launch of each trackNewestCoarse"},
        "cpu_baseline": None,
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle_ffi import OracleTracker  # test infrastructure: the CPU baseline leg only
        o = OracleTracker(s.width, s.height, s.K4, s.n_levels, fast=True)
        o.set_scene(s)
        n, tt = 0, 0.0
        while tt < args.cpu_seconds / 2 and n < 500:
            t1 = time.perf_counter()
            o.track(T0, [0.0, 0.0], s.n_levels - 1, minRes)
            tt += time.perf_counter() - t1
            n += 1
        res["cpu_baseline"] = {"value": n / tt, "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{n} trackNewestCoarse calls (the reference's SSE path is single-threaded)"}
        speedup(res)
    ct.close()
    return res


def bench_act(args):
    """System::activatePointsMT on a KITTI window (1232x368, 8 KFs, 2000 MapPoints, 14k traced
    immature points over the 8 hosts).  One step = one activation: makeDistanceMap + growDistBFS, the greedy
    selection with addIntoDistFinal, optimizeImmaturePoint of every selected point, read-back of the outputs.
    The call leaves the immature points unchanged, so steps repeat the same activation."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from hslam_amd.scene import make_activation_scene
    from hslam_amd.trace import ImmatureTracer, act_frames_array, act_pairs_array

    s = make_activation_scene(2000, 14000, width=1232, height=368, kitti=True, seed=3)
    g = ImmatureTracer(s.width, s.height, len(s.imm_u))
    for f in range(s.n_frames):
        g.set_host_image(int(s.slots[f]), s.imgs[f])
    g.add_points(s.slots[s.imm_frame], s.imm_u, s.imm_v)
    g.set_state(s.imm_idepth_min, s.imm_idepth_max, s.imm_quality, s.imm_status, s.imm_interval)
    g.set_types(s.imm_type)
    fr = act_frames_array(s.slots, s.flagged, s.KRKi1, s.Kt1)
    pr = act_pairs_array(s.RTll, s.tTll, s.aff)
    call = (s.K4, fr, pr, s.act_frame, s.act_u, s.act_v, s.act_idepth, s.ef_nPoints, s.currentMinActDist, s.order)
    for _ in range(max(1, args.warmup)):
        r = g.activatePointsMT(*call)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = g.activatePointsMT(*call)
    dt = time.perf_counter() - t0
    n_opt = int((r["action"] == 2).sum() + 0)
    res = {
        "metric": "point activations/sec (System::activatePointsMT, KITTI 1232x368 window, 14k immature points)",
        "value": args.steps / dt, "unit": "activations/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps, "higher_is_better": True, "scaling": "replicas only",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "activatePointsMT: 8 KFs 1232x368, 2000 MapPoints, 14000 immature points",
                   "activated": len(r["activated"]), "deleted": int((r["action"] == 1).sum()),
                   "immature_points": len(s.imm_u)},
        "cpu_baseline": None,
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from test_act import oracle_tracer  # test infrastructure: the CPU baseline leg only
        o = oracle_tracer(s)
        n, tt = 0, 0.0
        while tt < args.cpu_seconds / 2 and n < 500:
            t1 = time.perf_counter()
            o.activatePointsMT(s.imgs, *call)
            tt += time.perf_counter() - t1
            n += 1
        res["cpu_baseline"] = {"value": n / tt, "unit": "activations/s", "cores": 1, "kind": "port",
                               "sample": f"{n} activations of the same window (the reference's selection loop and "
                                         "BFS are serial; optimizeImmaturePoint runs on its thread pool)"}
        speedup(res)
    g.close()
    return res


def bench_refine(args):
    """the initializer's DirectRefinement::Refine (level-0 LM over calcResAndGS, doStep,
    applyStep, calcEC, optReg) on a 640x480 two-frame pair with 2000 ORB-like keypoints (85% triangulated).
    One step = one Refine from the initializer's pose: the point set-up upload (the ctor) is outside the timed
    call, the kernel, its read-back of the pose and the _videpth write-back are inside."""
    from hslam_amd.refine import DirectRefinement
    from hslam_amd.scene import make_refine_scene

    s = make_refine_scene(2000)
    g = DirectRefinement(s)
    for _ in range(max(1, args.warmup)):
        g.set_points(s.u, s.v, s.tri, s.z)
        T, vid, good, it, sn = g.Refine(s.T_init)
    dt, dev = 0.0, 0.0
    for _ in range(args.steps):
        g.set_points(s.u, s.v, s.tri, s.z)
        t0 = time.perf_counter()
        T, vid, good, it, sn = g.Refine(s.T_init)
        dt += time.perf_counter() - t0
        dev += g.last_ms()
    passes = it + 1  # calcResAndGS evaluations per Refine
    res = {
        "metric": "refinements/sec (DirectRefinement::Refine, 640x480 pair, 2000 keypoints)",
        "value": args.steps / dt, "unit": "refinements/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps, "higher_is_better": True, "scaling": "replicas only",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "DirectRefinement::Refine: 640x480, 2000 keypoints, 85% triangulated",
                   "lm_iterations": it, "snapped": sn, "good_points": int(good.sum()),
                   "device_ms_per_refine": dev / args.steps, "calcResAndGS_passes": passes,
                   "device_us_per_pass": dev / args.steps * 1e3 / passes},
        "cpu_baseline": None,
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle_ffi import OracleRefiner  # test infrastructure: the CPU baseline leg only
        n, tt = 0, 0.0
        while tt < args.cpu_seconds / 2 and n < 2000:
            o = OracleRefiner(s, fast=True)
            t1 = time.perf_counter()
            o.refine(s.T_init)
            tt += time.perf_counter() - t1
            n += 1
        res["cpu_baseline"] = {"value": n / tt, "unit": "refinements/s", "cores": 1, "kind": "port",
                               "sample": f"{n} Refine calls on the same pair (the reference's Refine is serial)"}
        speedup(res)
    g.close()
    return res


def bench_select(args):
    """PixelSelector::makeMaps (makeHists + select + the random sub-sampling) of a new
    640x480 frame at setting_desiredPointDensity = 2000, from its raw image (the pyramid is built on the device).
    One step = one makeMaps of a new frame id (makeHists runs every step, as for every new keyframe)."""
    from hslam_amd.scene import make_select_frames
    from hslam_amd.select import PixelSelector

    frames = make_select_frames(3, quantize=True)
    H, W = frames[0].shape
    sel = PixelSelector(W, H)
    fid = 0
    for _ in range(max(1, args.warmup)):
        sel.makeMapsRaw(frames[fid % 3], fid, 2000.0, want_map=False)
        fid += 1
    dev, n_sel = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, n_sel = sel.makeMapsRaw(frames[fid % 3], fid, 2000.0, want_map=False)
        dev += sel.last_stats()[0]
        fid += 1
    dt = time.perf_counter() - t0
    res = {
        "metric": "frames selected/sec (PixelSelector::makeMaps, 640x480, density 2000)",
        "value": args.steps / dt, "unit": "frames/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps, "higher_is_better": True, "scaling": "replicas only",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "PixelSelector::makeMaps from the raw 640x480 frame (device pyramid), 8-bit texture",
                   "selected": n_sel, "device_ms_per_frame": dev / args.steps},
        "cpu_baseline": None,
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle_ffi import PixelSelector as OracleSelector, dir_pyramid  # the CPU baseline leg only
        pyrs = [dir_pyramid(f, 3) for f in frames]
        o = OracleSelector(W, H, fast=True)
        n, tt = 0, 0.0
        while tt < args.cpu_seconds / 2 and n < 500:
            p, g = pyrs[n % 3]
            t1 = time.perf_counter()
            o.makeMaps(10000 + n, p[0], g, 2000.0)
            tt += time.perf_counter() - t1
            n += 1
        res["cpu_baseline"] = {"value": n / tt, "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{n} makeMaps calls from the host pyramid (the reference's selector is serial)"}
        speedup(res)
    return res


def bench_keyframe(args):
    """System::AddKeyframe's BA part per keyframe (Src/Mapping.cpp:12-140) through the incremental C-ABI, the C4
    window in steady state: 8 KFs x 250 points per host KF during optimize, a new KF's frame image taken from the
    tracker's device pyramid, residuals of the old points into it, 250 activated points (+ their residuals), makeIDX,
    optimize(6) + the tail, toRemove / removeOutliers, the tracker's new reference from the BA on the device,
    flagPointsForRemoval's marginalization (hs_ba_marginalize_points) and drops, marginalizeFrame of the oldest KF.
    One step = one keyframe.  Phases are the wall time spent in library calls (each call that reads back waits for
    its work; setup ends with a stream sync); the driver's own System-level decisions (numpy) are excluded."""
    from hslam_amd.keyframe import KeyframeBA, make_ba_sequence
    from hslam_amd.track import CoarseTracker

    n_kf = 7 + args.warmup + args.steps
    seq = make_ba_sequence(n_kf=n_kf, points_per_kf=max(1, args.points // 8))
    K4 = np.array([seq.K[0, 0], seq.K[1, 1], seq.K[0, 2], seq.K[1, 2]], np.float32)
    tr = CoarseTracker(seq.width, seq.height, K4, seq.n_levels)
    drv = KeyframeBA(seq, window=8, tracker=tr, image_path="device", allow_break=True)
    drv.bootstrap()
    for k in range(7, 7 + args.warmup):
        drv.add_keyframe(k)
    rows = []
    t0 = time.perf_counter()
    for k in range(7 + args.warmup, n_kf):
        rows.append(drv.add_keyframe(k))
    dt = time.perf_counter() - t0
    lib = np.array([r["lib_s"] for r in rows]) * 1e3
    ph = {p: np.array([r["phase_s"].get(p, 0.0) for r in rows]) * 1e3
          for p in ("setup", "optimize", "tail", "post", "track_frame")}
    pres = np.array([r["n_res"] for r in rows])
    iters = np.array([r["iters"] for r in rows])
    res = {
        "metric": "keyframes/sec (System::AddKeyframe BA part: window update + optimize(6) + tail + tracker "
                  "reference + marginalization, C4 8 KF x 2k pts)",
        "value": 1e3 / float(np.mean(lib)), "unit": "keyframes/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": float(np.mean(lib)), "higher_is_better": True,
        "scaling": "replicas only", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "C4 keyframe sequence (BASELINE.json configs[3] window in steady state): 8 KF x "
                               f"{max(1, args.points // 8)} pts per host KF, 640x480, incremental window "
                               "(hs_ba_insert_* / remove_* / make_idx), frame image from the tracker's device "
                               "pyramid, tracker reference handed over on the device",
                   "points_mean": float(np.mean([r["n_points"] for r in rows])),
                   "point_residuals_mean": float(np.mean(pres)), "gn_iterations": int(iters.max()),
                   "gn_iterations_mean": float(np.mean(iters)), "allow_break": True,
                   "marginalized_points_mean": float(np.mean([r.get("marginalized_points", 0) for r in rows])),
                   "parallelism": "single GPU"},
        "phase_ms_per_keyframe": {p: float(np.median(v)) for p, v in ph.items()},
        "phase_ms_per_keyframe_mean": {p: float(np.mean(v)) for p, v in ph.items()},
        "call_ms_per_keyframe": {c: float(np.median([r.get("call_s", {}).get(c, 0.0) for r in rows])) * 1e3
                                 for c in sorted({c for r in rows for c in r.get("call_s", {})})},
        "setup_over_gn": float(np.median(ph["setup"]) / np.median(ph["optimize"])),
        "driver_wall_ms_per_keyframe": dt * 1e3 / args.steps,
        "roofline": None,
        "cpu_baseline": None,
    }
    if not args.no_cpu:
        cb = cpu_baseline(args.points, args.cpu_seconds)
        # a keyframe's BA on the CPU path: optimize(6) = the GN iterations run (the same break test) after the initial
        # linearization, plus the tail's linearizeAll(true): (iterations + 1) GN-iteration equivalents of the same
        # window (the initial linearization and the window edits not counted)
        n_eq = float(np.mean(iters)) + 1
        kf_ms = n_eq * cb["median_ms_per_step"]
        res["cpu_baseline"] = {"value": 1e3 / kf_ms, "unit": "keyframes/s", "cores": cb["cores"], "kind": "port",
                               "sample": f"{n_eq:.2f} x the median GN iteration of the oracle on the C4 window (" +
                                         cb["sample"] + "); the reference's window edits are not timed",
                               "single_thread_keyframes_per_s": 1e3 / (n_eq * cb["single_thread"]["median_ms_per_step"])}
        speedup(res)
    tr.close()
    drv.ba.close()
    return res


def count_gpus(root: str = "/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this process may use, without loading any HIP / ROCm library: the KFD topology nodes with SIMDs
    (/sys/class/kfd/kfd/topology/nodes/*/properties 'simd_count' > 0; CPU nodes have none), narrowed by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set.  0 without a KFD (no amdgpu
    driver: no GPU); None when a topology file is unreadable (the ranks then fail loudly on their own)."""
    import glob
    if not os.path.isdir(root):
        return 0
    n = 0
    try:
        for f in glob.glob(os.path.join(root, "*", "properties")):
            with open(f) as fh:
                for line in fh:
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
    except (OSError, ValueError):
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(n: int, argv, plumbing: bool = False) -> int:
    """`--gpus N` without a launcher (WORLD_SIZE unset): N child rank processes, one per GPU, with the
    torch.distributed.run environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT).  This
    process never touches the GPU (children are started, nothing is exec'd); it counts devices without initialising
    HIP and fails loudly when there are fewer than N.  Returns the first failing child's exit code (the others are
    then stopped by PID), else 0.  Rank 0 prints the JSON line."""
    import socket
    import subprocess

    if not plumbing:
        ndev = count_gpus()  # from the KFD topology in sysfs: no HIP library is loaded in this process
        if ndev is not None and ndev < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, this node has {ndev}", file=sys.stderr)
            return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def plumbing_rank(args, world, rank, local):
    """--plumbing-check (CPU test of the launcher): every rank joins a gloo group with the launcher's environment,
    all-reduces (rank + 1) and reports what it saw; no GPU, no library."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    n = dist.get_world_size()
    pts = [len(range(r, args.points, world)) for r in range(world)]  # the strong shard sizes (p % N == rank)
    if rank == 0:
        print(json.dumps({"plumbing": True, "world": world, "group_size": n, "allreduce": float(t.item()),
                          "gpus_flag": args.gpus, "strong_shard_points": pts}))
    dist.barrier()
    dist.destroy_process_group()


def run_window(args, n_window, kitti, world, rank, local, dist):
    """Builds the 8-KF window of n_window points, loads this rank's shard (points p % world == rank), runs W warm-up
    and then K timed GN iterations between barriers; returns the timing (max over ranks) and the live BAWindow."""
    from hslam_amd.ba import BAWindow
    from hslam_amd.scene import make_ba_scene, make_ba_scene_kitti

    scene = make_ba_scene_kitti(n_window) if kitti else make_ba_scene(n_points=n_window)
    shard = scene.shard(rank, world) if world > 1 else scene
    comm = None
    if world > 1:
        uid = [BAWindow.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = (uid[0], rank, world)
    ba = BAWindow(shard, device=local if world > 1 else 0, comm=comm)
    ranks, my_rank = ba.comm_size()
    if ranks != world or my_rank != rank:
        raise SystemExit(f"bench.py: the RCCL communicator holds {ranks} ranks (this one {my_rank}), "
                         f"the launcher started {world} (this one {rank})")
    ba.linearizeAll(reset=True)
    if args.warmup > 0:
        ba.iterate(0, args.warmup)

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    ba.iterate(args.warmup, args.steps)  # K device-resident GN iterations, one host sync at the end
    t1 = time.perf_counter()
    barrier()
    dt = t1 - t0
    n_res_total = shard.n_res
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        nr = torch.tensor([shard.n_res], dtype=torch.int64, device="cuda")
        dist.all_reduce(nr)
        n_res_total = int(nr.item())
    return dict(ba=ba, shard=shard, dt=dt, n_res_total=n_res_total, n_window=n_window, ranks=ranks,
                value=n_res_total * args.steps / dt, ms_per_step=dt * 1e3 / args.steps)


def phase_split(ba, first, steps):
    """Per-phase device time of the GN step, from HIP event pairs around each launch group of an extra, untimed loop
    of `steps` iterations (after the timed loop: the event records add ~1-2 us per pair, so the timed loop carries
    none).  solve = hs_k_solve (solve + step + precalc); linearize = the linearize kernel; accumulate_stitch =
    hs_k_reduce + hs_k_stitch (+ the RCCL exchange on N > 1)."""
    ba.set_event_timing(2)
    ba.iterate(first, steps)
    ba.set_event_timing(0)
    t = ba.timings()
    n = max(1, t["timed_iters"])
    return {"solve_step_kernel": t["solve_ms"] / n, "linearize_kernel": t["linearize_ms"] / n,
            "accumulate_stitch": t["acc_stitch_ms"] / n, "event_timed_steps": t["timed_iters"],
            "timing": "HIP event pairs per launch group in an untimed loop after the timed one"}


def optimize_calls(scene, reps=15):
    """Wall time of whole library calls on the window (median of reps, host clock around the ctypes call):
    hs_ba_optimize(6) as System::optimize calls it (initial linearizeAll + 6 GN iterations + the energy read-back),
    once with the break test off and once with it on (allow_break: Src/FullSystemOptimize.cpp:493, tested on the
    device) under thOptIterations = 0, so canbreak never holds and both run all 6 iterations; and the optimize tail
    hs_ba_fix_linearization (setEvalPT + setAdjointsF + setPrecalcValues on the device, linearizeAll(true),
    read-backs)."""
    from hslam_amd._lib import default_params
    from hslam_amd.ba import BAWindow
    p = default_params()
    p.thOptIterations = 0.0
    ba = BAWindow(scene, params=p)
    out = {}
    for name, brk in (("optimize6_ms", False), ("optimize6_break_ms", True)):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            n, _ = ba.optimize(6, allow_break=brk)
            ts.append(time.perf_counter() - t0)
            assert n == 6
        out[name] = float(np.median(ts)) * 1e3
    z = np.zeros(scene.n_points, np.float32)
    zi = np.zeros(scene.n_points, np.int32)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ba.fixLinearization(z, zi)
        ts.append(time.perf_counter() - t0)
    out["tail_ms"] = float(np.median(ts)) * 1e3
    ba.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("ba", "ba-kitti", "keyframe", "trace", "track", "act", "refine", "select"),
                    default="ba",
                    help="ba = the headline metric (C4, 640x480); ba-kitti = C5's BA half (KITTI 1232x368, 5 levels); "
                         "trace = C5 traceOn; track = C2 CoarseTracker; act = point activation; refine = initializer "
                         "DirectRefinement; select = PixelSelector; keyframe = AddKeyframe's BA part per keyframe")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU): without a launcher's WORLD_SIZE, bench.py starts the N rank processes "
                         "itself; under torch.distributed.run WORLD_SIZE must equal N")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--points", type=int, default=2000,
                    help="active points of the window (strong scaling) or per GPU (--scaling weak)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong (default): `value` is the metric's own 8 KF x --points window sharded over the N "
                         "GPUs; weak: --points per GPU (a window of --points x N).  The other one is measured too "
                         "(N > 1) and reported beside it")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--phase-events", type=int, default=None, choices=(0, 1, 2),
                    help="HIP event pairs inside the timed GN loop (sets HS_EVENT_TIMING; default: the environment's "
                         "value, else 0 = none; each pair adds ~2 us per step), 1 linearize only, 2 every phase")
    ap.add_argument("--no-phase-split", action="store_true", help="skip the untimed event-timed phase-split loop")
    ap.add_argument("--no-large-strong", action="store_true",
                    help="N > 1: skip the strong-scaling run of the 200k-point window reported beside `value`")
    ap.add_argument("--plumbing-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.workload not in ("ba", "ba-kitti"):
        if args.gpus != 1:
            raise SystemExit(f"bench.py: --workload {args.workload} is single-GPU (replicas only); --gpus {args.gpus}")
        res = {"trace": bench_trace, "track": bench_track, "act": bench_act, "refine": bench_refine,
               "select": bench_select, "keyframe": bench_keyframe}[args.workload](args)
        print(json.dumps(res))
        return

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], plumbing=args.plumbing_check))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} from the launcher but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plumbing_check:
        plumbing_rank(args, world, rank, local)
        return
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    # the timed loop carries no instrumentation unless asked: the roofline's launch duration comes from
    # hs_ba_time_linearize's back-to-back launches, the phase split from an untimed event-timed loop afterwards
    if args.phase_events is not None:
        os.environ["HS_EVENT_TIMING"] = str(args.phase_events)
    args.phase_events = int(os.environ.get("HS_EVENT_TIMING", "0") or 0)

    kitti = args.workload == "ba-kitti"
    n_window = args.points * world if args.scaling == "weak" else args.points
    run = run_window(args, n_window, kitti, world, rank, local, dist)
    ba, shard = run["ba"], run["shard"]
    tim = ba.timings()
    nt = max(1, tim["timed_iters"])
    # per-launch event pairs inside the GN loop (+~3 us event overhead); None without --phase-events
    lin_loop_ms = tim["linearize_ms"] / nt if tim["timed_iters"] > 0 else None
    # continues the timed loop's GN iterations (collective on N > 1: every rank runs it)
    split = None if args.no_phase_split else phase_split(ba, args.warmup + args.steps, min(max(args.steps, 20), 100))
    # the same kernel, same inputs, launched back to back between one event pair: the launch duration
    # rocprofv3 reports (the in-loop pairs add the event-record overhead to a ~9 us kernel)
    lin_ms = ba.time_linearize(max(64, args.steps))
    achieved = BYTES_PER_PRES * shard.n_res / (lin_ms * 1e-3) / 1e9
    lin_kernel = ba.partition()["kernel"]  # hs_k_lin (one point per wave) or hs_k_lin8 (8 points per wave)
    roof_ctr = pmc_roof(f"kitti{args.points}" if kitti else args.points, lin_kernel) if world == 1 else {}
    traffic, traffic_src = ((roof_ctr["hbm_bytes_per_launch"], roof_ctr["source"]) if "hbm_bytes_per_launch" in roof_ctr
                            else pmc_traffic(f"kitti{args.points}" if kitti else args.points, lin_kernel) if world == 1
                            else (None, None))
    ba.close()
    other = large = None
    if world > 1:  # the other scaling mode, same ranks and communicator set-up, reported beside `value`
        mode = "weak" if args.scaling == "strong" else "strong"
        o = run_window(args, args.points * world if mode == "weak" else args.points, kitti, world, rank, local, dist)
        other = {"scaling": mode, "value": o["value"], "ms_per_step": o["ms_per_step"], "points": o["n_window"],
                 "points_per_gpu_rank0": o["shard"].n_points, "point_residuals": o["n_res_total"]}
        o["ba"].close()
        if not kitti and args.points < STRONG_LARGE_POINTS:
            # strong scaling where the linearization outweighs the replicated solve: the 200k window over the N
            # ranks (DESIGN.md §7's projection); --no-large-strong skips it
            if not args.no_large_strong:
                a2 = argparse.Namespace(**vars(args))
                a2.steps, a2.warmup = min(args.steps, 20), min(args.warmup, 3)
                o = run_window(a2, STRONG_LARGE_POINTS, kitti, world, rank, local, dist)
                large = {"scaling": "strong", "value": o["value"], "ms_per_step": o["ms_per_step"],
                         "points": o["n_window"], "points_per_gpu_rank0": o["shard"].n_points,
                         "point_residuals": o["n_res_total"], "steps": a2.steps, "warmup": a2.warmup,
                         "note": "compare with `python bench.py --points 200000` at N = 1 (same window)"}
                o["ba"].close()
    if kitti:
        wl = ("C5 BA half (BASELINE.json configs[4]): full windowed photometric BA incl. Schur complement, 8 KF x "
              f"{n_window} pts, KITTI 1232x368, 5 pyramid levels")
    else:
        wl = ("C4 (BASELINE.json configs[3]): full windowed photometric BA incl. Schur complement, 8 KF x "
              f"{n_window} pts, 640x480, 4 pyramid levels")
    wl += (f", {args.scaling} scaling over {world} GPU(s) ({shard.n_points} pts on rank {rank}); GN step = "
           "solve+step+linearize+accumulate (fp32 residuals, fp64 stitch/solve)")
    result = {
        "metric": METRIC,
        "value": run["value"],
        "unit": "point-residuals/s",
        "n_gpus": run["ranks"],
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": run["ms_per_step"],
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": wl,
            "frames": shard.n_frames,
            "points": n_window,
            "points_per_gpu": shard.n_points,
            "point_residuals": run["n_res_total"],
            "parallelism": f"point-shard x{world}" + (" (one RCCL all-gather group call per GN step)" if world > 1
                                                     else ""),
            "launcher": "bench.py child ranks" if env_world is None and world > 1 else (
                "torch.distributed.run" if world > 1 else "single process"),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": lin_kernel,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "bytes_per_unit": BYTES_PER_PRES,
            "units_per_launch": shard.n_res,
            "avg_launch_ms": lin_ms,
            "avg_launch_ms_in_loop_events": lin_loop_ms,
            "timing": f"HIP events on the context stream around back-to-back {lin_kernel} launches (fused "
                      "linearize + applyRes + top / Schur accumulation into block partials)",
            # the GN loop's launch also applies the previous solve's point step (resubstituteFPt, fused): it reads the
            # last linearization's JpJdF (32 B per residual) and the step's chain heads every point group
            "avg_launch_ms_gn_loop": (split or {}).get("linearize_kernel"),
            "frac_gn_loop": (BYTES_PER_PRES * shard.n_res / ((split or {})["linearize_kernel"] * 1e-3) / 1e9
                             / HBM_PEAK_GBS) if (split or {}).get("linearize_kernel") else None,
            "gn_loop_timing": "the same kernel inside the fused GN loop (with the point step of the previous solve), "
                              "HIP event pairs per launch in an untimed loop after the timed one (+~3 us event "
                              "overhead per launch)",
            "counters": roof_ctr,
            "limiter_note": "one point per wave at 2k: dependent memory round trips (the step is a chain of 4 "
                            "dependent launches, the single-workgroup fp64 solve the longest)" if shard.n_points < 60000
                            else "VALU issue + gather latency at occupancy 2 (DESIGN.md §9)",
        },
        "phase_ms_per_step": split,
        "cpu_baseline": None,
    }
    result["roofline"].update(roof_binding(roof_ctr, achieved / HBM_PEAK_GBS))
    if other is not None:
        result[f"{other['scaling']}_scaling"] = other
    if large is not None:
        result["strong_scaling_200k"] = large
    if world == 1 and not args.no_phase_split:
        calls = optimize_calls(shard)
        calls["six_steps_ms"] = 6 * run["ms_per_step"]
        result["calls_ms"] = calls
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(n_window, args.cpu_seconds, kitti)
        speedup(result)
    if rank == 0:
        print(json.dumps(result))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
