/*
 * hs_track.h — C-ABI drop-in boundary of H-SLAM's CoarseTracker (direct image alignment of a new frame
 * against the newest keyframe) on MI355X (gfx950).  Same conventions as hs_ba.h: plain C, caller-owned
 * host buffers copied in/out, the tracker owns its device memory and HIP stream, status codes from
 * hs_types.h, no exception crosses the ABI, one tracker per calling thread.
 *
 * Reference interface each entry point replaces (AUBVRL/H-SLAM):
 *   hs_tracker_create / destroy   CoarseTracker(w, h) + makeK(HCalib)           Src/CoarseTracker.cpp:29-101
 *   hs_tracker_set_ref            setCoarseTrackingRef + makeCoarseDepthL0        Src/CoarseTracker.cpp:492-504,105-263
 *   hs_tracker_get_ref            read-back of pc_u / pc_v / pc_idepth / pc_color / pc_n  Include/CoarseTracker.h:73-77
 *   hs_tracker_set_frame          newFrame->frame->DirPyr (the frame being tracked)  Include/Frame.h:39
 *   hs_tracker_calc_res           calcRes (+ calcGSSSE on its warped buffer)      Src/CoarseTracker.cpp:329-485,267-324
 *   hs_tracker_track              trackNewestCoarse                                Src/CoarseTracker.cpp:506-683
 *   hs_tracker_track_tries        the try loop of System::trackNewCoarse          Src/System.cpp:413-481
 *                                 (the caller builds the motion / rotation hypotheses, System.cpp:346-411)
 *
 * Images: per pyramid level l (0 = finest, w_l = w >> l, h_l = h >> l) a host pointer to w_l*h_l*3 floats
 * (I, dI/dx, dI/dy) — Frame::DirPyr[l].  Poses: Sophus SE3d::data() order (qx qy qz qw tx ty tz),
 * refToNew.  Affine: AffLight (a, b).
 */
#ifndef HS_TRACK_H
#define HS_TRACK_H
#include "hs_types.h"
#include "hs_ba.h" /* hs_ctx (the BA context of hs_tracker_set_ref_ba) */
#ifdef __cplusplus
extern "C" {
#endif

#define HS_TRK_MAXLEV 6

typedef struct hs_tracker hs_tracker;

/* K4 = (fx, fy, cx, cy) of level 0 as CalibData::fxl()/fyl()/cxl()/cyl() (scaled, float);
   n_levels = DirPyrLevels (<= HS_TRK_MAXLEV; trackNewestCoarse requires coarsest level < 5). */
int hs_tracker_create(hs_tracker** out, const hs_params* params, int device_id, int width, int height,
                      int n_levels, const float K4[4]);
void hs_tracker_destroy(hs_tracker* t);

/* lastRef = the newest keyframe: its pyramid, ab_exposure and aff_g2l; the points whose residual into
   it is IN (ph->lastResiduals[0]), in the reference's frame / point order: centerProjectedTo (u, v,
   new idepth) and the point's HdiF.  Runs makeCoarseDepthL0 on the device. */
int hs_tracker_set_ref(hs_tracker* t, const float* const* ref_pyr, float ab_exposure, const double aff_g2l[2],
                       int n_pts, const float* center_u, const float* center_v, const float* center_idepth,
                       const float* HdiF);
/* setCoarseTrackingRef(frameHessians) as System::AddKeyframe calls it after optimize (Src/Mapping.cpp:93-100;
   Src/CoarseTracker.cpp:492-504,105-263), fed from a BA context on the same device: the reference points are the BA
   window's points whose residual into its newest frame is IN (ph->lastResiduals[0], Src/CoarseTracker.cpp:117),
   in window order, with their centerProjectedTo and the last solve's HdiF -- gathered and scattered on the device,
   no host round trip and no host synchronisation (the tracker's stream waits on the BA's).
   promote_frame = 1: the frame last given to hs_tracker_set_frame* is the newest keyframe and becomes the reference
   pyramid as it is (no copy; set the next frame to track afterwards); 0: the reference pyramid is rebuilt on the
   device from the BA's newest frame image.  ab_exposure / aff_g2l: the newest keyframe's.
   The new reference replaces the tracker's in place (the reference builds it in coarseTracker_forNewKF and swaps
   the two under a lock): the tracker must not be tracking on another thread during this call.  A caller that tracks
   while the next reference is built keeps two trackers and swaps them itself, as the reference does. */
int hs_tracker_set_ref_ba(hs_tracker* t, hs_ctx* ba, int promote_frame, float ab_exposure, const double aff_g2l[2]);
/* device pointer of level lvl of the frame last given to hs_tracker_set_frame* (w_l*h_l float4 texels
   (I, dI/dx, dI/dy, 0)), valid until the next set_frame / set_ref_ba(promote) call: a keyframe's image goes to the
   BA context with hs_ba_set_frame_image_device, without crossing PCIe again. */
int hs_tracker_frame_texels(hs_tracker* t, int lvl, const void** d_texels);
/* System::AddKeyframe's image hand-off (Src/Mapping.cpp:22: the keyframe's Frame::DirPyr[0] becomes the new window
   frame's image, EnergyFunctional::insertFrame): level 0 of the frame last given to hs_tracker_set_frame* becomes
   window frame `frame`'s image in the BA context on the same device.  Ordered on the device both ways, no host
   synchronisation: the copy follows the tracker's queued work and the tracker's next work follows the copy (unlike
   hs_ba_set_frame_image_device, which must wait on the host for a producer it cannot order against). */
int hs_tracker_frame_to_ba(hs_tracker* t, hs_ctx* ba, int frame);
/* pc arrays of one level (nullable outputs, capacity w_l*h_l); *n = pc_n[lvl] */
int hs_tracker_get_ref(hs_tracker* t, int lvl, int* n, float* u, float* v, float* idepth, float* color);
/* the frame to track: its pyramid and ab_exposure */
int hs_tracker_set_frame(hs_tracker* t, const float* const* new_pyr, float ab_exposure);
/* the frame to track as its raw level-0 image (W*H floats, ImageData::fImgL): Frame::CreateDirPyrs runs on the
   device (include/hs_pyr.h, Src/Frame.cpp:104-181) into the tracker's pyramid */
int hs_tracker_set_frame_raw(hs_tracker* t, const float* img, float ab_exposure);
/* one calcRes at (refToNew, aff) with cutoffTH; res6 = {E, numTermsInE, flowT, 0, flowRT, saturated ratio};
   H64 / b8 (nullable) = calcGSSSE on the warped buffer; n_warped = buf_warped_n (padded to 4) */
int hs_tracker_calc_res(hs_tracker* t, int lvl, const double T7[7], const double aff[2], float cutoffTH,
                        double res6[6], double H64[64], double b8[8], int* n_warped);
/* trackNewestCoarse: T_inout / aff_inout updated only on success (like the reference);
   lastResiduals[5], flow[3] = lastFlowIndicators; *ok = return value */
int hs_tracker_track(hs_tracker* t, double T_inout[7], double aff_inout[2], int coarsest_lvl,
                     const double minResForAbort[5], double lastResiduals[5], double flow[3], int* ok);
/* System::trackNewCoarse try loop over n_tries refToNew candidates (tries7[n][7]), all starting from
   aff_last_2_l; the tries run concurrently on the device (one workgroup each) and the reference's
   sequential take-over / early-abort logic is replayed exactly on their per-level residual logs.
   Outputs: the chosen pose / aff, achievedRes[5], flowVecs[3], have_one_good, n_tried (tries the
   reference would have run before its early break). */
int hs_tracker_track_tries(hs_tracker* t, int n_tries, const double* tries7, const double aff_last_2_l[2],
                           const double lastCoarseRMSE[5], float reTrackThreshold, double T_out[7],
                           double aff_out[2], double achievedRes[5], double flowVecs[3], int* have_one_good,
                           int* n_tried);
/* trace: the LM accept / break test operands of hypothesis try_idx of the last track / track_tries call, one
   entry per iteration: level, resNew[0]/resNew[1], resOld[0]/resOld[1] (Src/CoarseTracker.cpp:611) and the
   step norm |inc| (:642);
   *n = iterations run, at most min(cap, 256) entries written.  No reference counterpart (its logs are
   commented-out printf, Src/CoarseTracker.cpp:613-625). */
int hs_tracker_get_lm_log(hs_tracker* t, int try_idx, int cap, int* n, int* lvl, double* new_ratio,
                          double* old_ratio, double* inc_norm);
/* device time (ms) of the last track / track_tries call (HIP events on the tracker stream); 0 unless event timing
   is on */
int hs_tracker_last_ms(hs_tracker* t, double* ms);
/* per-call event timing (off by default): on, every track / track_tries call records an event pair around its launch
   and waits for the stream's end (hs_tracker_last_ms reports the device time); off, the host takes each hypothesis'
   results from its done word as soon as the device wrote it (~3-4 us less host time per call) */
int hs_tracker_set_event_timing(hs_tracker* t, int on);

/* Work of hypothesis try_idx in the last trackNewestCoarse / try-loop call: the device time of the call (ms), the
   calcRes(+calcGSSSE) passes it ran and the sum of their levels' reference-point counts (the point-pass units
   of the tracker's roofline).  Outputs nullable. */
int hs_tracker_last_stats(hs_tracker* t, int try_idx, double* ms, int* passes, long long* point_passes);
/* workgroups per hypothesis of the last track launch (G members meeting once per pass, sized from the device's
   compute units) and the number of launches so far rerun with G = 1 after a member meeting timed out (members not
   co-resident: a smaller partition, kernels of other streams). */
int hs_tracker_launch_info(hs_tracker* t, int* G, int* fallbacks);

#ifdef __cplusplus
}
#endif
#endif /* HS_TRACK_H */
