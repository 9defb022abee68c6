/*
 * hs_trace.h — C-ABI of the epipolar-search path on MI355X.
 *
 * Replaces, in AUBVRL/H-SLAM:
 *   hs_tracer_add_points   ImmaturePoint::ImmaturePoint (Src/ImmaturePoint.cpp:7-32; Include/ImmaturePoint.h:34-71):
 *                          colour / weights / gradH / energyTH sampled from the host keyframe's DirPyr[0]
 *                          (getInterpolatedElement33BiLin), idepth_min 0, idepth_max NaN, quality 10000,
 *                          lastTraceStatus IPS_UNINITIALIZED.
 *   hs_tracer_trace        System::traceNewCoarse (Src/Mapping.cpp:494-538): ImmaturePoint::traceOn
 *                          (Src/ImmaturePoint.cpp:40-350) of every immature point of every host keyframe
 *                          against the new frame, with that host's (KRKi, Kt, aff) — the exact arguments
 *                          traceNewCoarse passes (Mapping.cpp:505-511).
 *   hs_tracer_get_points   read-back of ImmaturePoint's public members (lastTraceStatus, idepth_min/max,
 *                          quality, lastTraceUV, lastTracePixelInterval, energyTH, color, weights, gradH).
 *   hs_tracer_activate     System::activatePointsMT (Src/Mapping.cpp:330-480): the currentMinActDist update,
 *                          CoarseDistanceMap::makeDistanceMap / growDistBFS / addIntoDistFinal
 *                          (Src/CoarseTracker.cpp:726-868), the immature-point selection loop and
 *                          System::optimizeImmaturePoint (Src/FullSystemOptPoint.cpp:24-175) with
 *                          ImmaturePoint::linearizeResidual (Src/ImmaturePoint.cpp:389-451) for every selected
 *                          point.  The MapPoint / PointFrameResidual objects themselves are built by the caller
 *                          from the outputs (activated flag, idepth, IN-residual mask).
 *
 * Conventions as include/hs_ba.h: status codes (hs_types.h), caller-owned host buffers copied in/out,
 * the context owns device memory and its own HIP stream, single caller.  Images are Frame::DirPyr[0]:
 * W*H (I, dI/dx, dI/dy) float triplets.  Points are held in the order they are added.
 */
#ifndef HS_TRACE_H
#define HS_TRACE_H

#include "hs_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ImmaturePointStatus, Include/ImmaturePoint.h:25-31 */
enum { HS_IPS_GOOD = 0, HS_IPS_OOB = 1, HS_IPS_OUTLIER = 2, HS_IPS_SKIPPED = 3, HS_IPS_BADCONDITION = 4,
       HS_IPS_UNINITIALIZED = 5 };

/* per host keyframe: the traceOn arguments of Src/Mapping.cpp:505-511 */
typedef struct hs_trace_host {
  float KRKi[9];  /* K * R(hostToNew) * K^-1, row-major (Mat33f) */
  float Kt[3];    /* K * t(hostToNew) */
  float aff[2];   /* AffLight::fromToVecExposure(host, new).cast<float>() */
} hs_trace_host;

typedef struct hs_tracer hs_tracer;

/* width/height: CalibData::Width/Height (level 0); capacity: maximum number of immature points */
int hs_tracer_create(hs_tracer** out, const hs_params* params, int device_id, int width, int height, int capacity);
void hs_tracer_destroy(hs_tracer* t);

/* host keyframe images (level 0) used by hs_tracer_add_points; slot = host index */
int hs_tracer_set_host_image(hs_tracer* t, int slot, const float* img_lvl0);
/* ImmaturePoint ctor for n new points on host slots host[i] at (u[i], v[i]); appended after existing points */
int hs_tracer_add_points(hs_tracer* t, int n, const int* host, const float* u, const float* v);
/* drop all points (a new window) */
int hs_tracer_clear(hs_tracer* t);
/* overwrite the search state of all points (nullable arrays of length n_points): a point traced before;
   interval = lastTracePixelInterval */
int hs_tracer_set_state(hs_tracer* t, const float* idepth_min, const float* idepth_max, const float* quality,
                        const uint8_t* status, const float* interval);

/* the frame to trace on (level 0 image); stays resident until the next call */
int hs_tracer_set_frame(hs_tracer* t, const float* img_lvl0);
/* the same from the raw level-0 image (W*H floats): DirPyr[0] built on the device (include/hs_pyr.h) */
int hs_tracer_set_frame_raw(hs_tracer* t, const float* img);
/* traceOn of every point; hosts[n_hosts] indexed by the points' host slot.  counts6 (nullable): number of
   points per ImmaturePointStatus after the call (the trace_good/oob/... tallies of Mapping.cpp:513-520);
   with counts6 == NULL the call returns without waiting for the device. */
int hs_tracer_trace(hs_tracer* t, int n_hosts, const hs_trace_host* hosts, int counts6[6]);

/* read-back, all nullable: status[n], idepth_min[n], idepth_max[n], quality[n], uv[n][2] (lastTraceUV),
   interval[n] (lastTracePixelInterval), energyTH[n], color[n][8], weights[n][8], gradH[n][4] */
int hs_tracer_get_points(hs_tracer* t, int* n, uint8_t* status, float* idepth_min, float* idepth_max,
                         float* quality, float* uv, float* interval, float* energyTH, float* color, float* weights,
                         float* gradH);
/* ImmaturePoint::my_type of every stored point (n_points floats; PixelSelector's 1 / 2 / 4).  Points are
   added with my_type 1. */
int hs_tracer_set_types(hs_tracer* t, const float* my_type);

/* ---- point activation (activatePointsMT) ----------------------------------------------------------------- */

/* one window keyframe, in frameHessians order (the newest keyframe last) */
typedef struct hs_act_frame {
  int slot;              /* tracer image slot holding this keyframe's DirPyr[0] (hs_tracer_set_host_image) */
  int flagged_for_marg;  /* Frame::FlaggedForMarginalization (Mapping.cpp:397) */
  float KRKi[9];         /* CoarseDistanceMap::K[1] * R(frame -> newest) * Ki[0], row-major (Mapping.cpp:368,
                            CoarseTracker.cpp:745); unused for the newest keyframe */
  float Kt[3];           /* K[1] * t(frame -> newest) */
} hs_act_frame;

/* Frame::targetPrecalc[target] of a host keyframe (FrameFramePrecalc::set, Src/OptimizationClasses.cpp:13-39) */
typedef struct hs_act_pair {
  float RTll[9];         /* PRE_RTll, row-major */
  float tTll[3];         /* PRE_tTll */
  float aff[2];          /* PRE_aff_mode */
} hs_act_pair;

/* what activatePointsMT did to an immature point */
enum { HS_ACT_KEEP = 0, HS_ACT_DELETED = 1, HS_ACT_ACTIVATED = 2 };

/* One activatePointsMT call.
     K4            level-0 fx, fy, cx, cy (CalibData fxl .. cyl); fxli = 1/fx and fyli = 1/fy in float
     frames[nF]    the window (nF <= 8), pairs[nF*nF] at [host*nF + target]
     active points (for makeDistanceMap): window frame index act_frame[i], u, v, idepth of every MapPoint
     ef_nPoints, *currentMinActDist: EnergyFunctional::nPoints and System::currentMinActDist (updated in place)
     order[n_order]: the tracer points in the reference's loop order (for host in frameHessians, for i in
                   host->ImmaturePoints); NULL = storage order.  Points whose slot is no window frame's, and
                   points of the newest keyframe, are left untouched (HS_ACT_KEEP).
   Outputs (nullable, indexed by tracer point): action[n] (HS_ACT_*), idepth[n] (the new MapPoint's idepth
   and idepth_zero, activated points only), res_in[n] (bit f set: a PointFrameResidual into window frame f in
   state IN); activated[n] = the activated points in the reference's toOptimize order, *n_activated their
   number.  The tracer's points are not removed: hs_tracer_compact does that. */
int hs_tracer_activate(hs_tracer* t, const float K4[4], int nF, const hs_act_frame* frames, const hs_act_pair* pairs,
                       int n_active, const int* act_frame, const float* act_u, const float* act_v,
                       const float* act_idepth, int ef_nPoints, float* currentMinActDist, int n_order,
                       const int* order, uint8_t* action, float* idepth, uint8_t* res_in, int* activated,
                       int* n_activated);
/* the distance map of the last hs_tracer_activate after its selection loop (fwdWarpedIDDistFinal,
   (W/2)*(H/2) floats) */
int hs_tracer_get_distance_map(hs_tracer* t, float* dist);
/* drop the points with keep[i] == 0; the survivors keep their relative order */
int hs_tracer_compact(hs_tracer* t, const uint8_t* keep);

/* re-run the ImmaturePoint ctor on every point already added (same host / u / v, no upload): a fresh
   first-trace state (idepth_min 0, idepth_max NaN, quality 10000, IPS_UNINITIALIZED) */
int hs_tracer_reinit(hs_tracer* t);
/* last hs_tracer_trace: device time (ms) of the traceOn kernel (HIP events on the tracer stream) and the
   number of discrete-search steps it evaluated (sum of numSteps over the points that reached the search).
   No reference counterpart (its tallies are commented-out printf, Src/Mapping.cpp:521-528). */
int hs_tracer_last_stats(hs_tracer* t, double* ms, long long* search_steps);

#ifdef __cplusplus
}
#endif
#endif /* HS_TRACE_H */
