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
/* overwrite the search state of all points (nullable arrays of length n_points): a point traced before */
int hs_tracer_set_state(hs_tracer* t, const float* idepth_min, const float* idepth_max, const float* quality,
                        const uint8_t* status);

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
