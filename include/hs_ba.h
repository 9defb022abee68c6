/*
 * hs_ba.h — C-ABI drop-in boundary of H-SLAM's windowed photometric BA hot path
 * on MI355X (gfx950).  Plain C: pointers + sizes, caller-owned host buffers
 * copied in/out, the context owns all device memory and its HIP stream.
 * Every entry point returns an hs status code (hs_types.h); no exception
 * crosses the ABI.  A context is single-caller (not thread-safe); use one
 * context per thread (tracking vs mapping, Src/System.cpp:182-212).
 *
 * Reference interface each entry point replaces (AUBVRL/H-SLAM):
 *   hs_create / hs_destroy      new/delete EnergyFunctional + its IndexThreadReduce pool
 *                               (Src/System.cpp:51; Include/EnergyFunctional.h:37-38)
 *   hs_ba_set_window            EnergyFunctional::insertFrame/insertPoint/insertResidual + makeIDX +
 *                               setAdjointsF + System::setPrecalcValues
 *                               (Src/EnergyFunctional.cpp:371-425,819-840,22-82; Src/System.cpp:321-331)
 *   hs_ba_linearize             System::linearizeAll(false) + applyRes_Reductor + setNewFrameEnergyTH
 *                               (Src/FullSystemOptimize.cpp:102-124,55-59,60-101); on the GPU the
 *                               accumulateAF/SCF_MT point loops (Src/EnergyFunctional.cpp:155-220)
 *                               are fused into the same pass.
 *   hs_ba_solve_system          System::solveSystem -> EnergyFunctional::solveSystemF
 *                               (Src/FullSystemOptimize.cpp:552-561; Src/EnergyFunctional.cpp:705-817):
 *                               stitch, prior, Schur, scaled LDLT, orthogonalize, resubstituteF_MT.
 *   hs_ba_do_step               System::backupState + doStepFromBackup(1,1,1,1,1) + setPrecalcValues
 *                               (Src/FullSystemOptimize.cpp:269-314,171-264)
 *   hs_ba_optimize              System::optimize GN loop (Src/FullSystemOptimize.cpp:362-494),
 *                               setting_forceAceptStep = true.
 *   hs_ba_iterate               the loop body of System::optimize (Src/FullSystemOptimize.cpp:420-494)
 *   hs_ba_calc_energies         calcLEnergyF_MT / calcMEnergyF (dormant under setting_forceAceptStep)
 *                               (Src/EnergyFunctional.cpp:277-368)
 *   hs_ba_fix_linearization     System::optimize's tail: newest frame setEvalPT, setAdjointsF,
 *                               setPrecalcValues, linearizeAll(true) (Src/FullSystemOptimize.cpp:498-516,
 *                               19-52, 102-160)
 *   hs_ba_get_system            HA/bA (accumulateAF_MT), HL/bL (accumulateLF_MT), H_sc/b_sc (accumulateSCF_MT)
 *   hs_ba_get_* / hs_ba_set_marginal_prior   read-back of PointFrameResidual / MapPoint / FrameOptimizationData
 *                               state; EnergyFunctional::HM/bM.
 *   hs_ba_marginalize_points    System::flagPointsForRemoval (per-point part) + EnergyFunctional::marginalizePointsF
 *                               (Src/Mapping.cpp:280-293; Src/EnergyFunctional.cpp:545-609).
 *   hs_ba_marginalize_frame     EnergyFunctional::marginalizeFrame (Src/EnergyFunctional.cpp:456-543).
 *   hs_comm_*                   (new) RCCL communicator for point-sharded windows; one rank per GPU.
 */
#ifndef HS_BA_H
#define HS_BA_H

#include "hs_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hs_ctx hs_ctx;

int hs_params_default(hs_params* out);
const char* hs_last_error(void);

int hs_create(hs_ctx** out, const hs_params* params, int device_id);
void hs_destroy(hs_ctx* ctx);

/* images: nF host pointers to level-0 (I, dI/dx, dI/dy) float triplets, W*H*3 floats each
   (Frame::DirPyr[0] layout).  points MUST be sorted by host, residuals grouped by point. */
int hs_ba_set_window(hs_ctx* ctx, const hs_camera* cam, int nF, const hs_frame* frames,
                     const float* const* images, const hs_points* points, const hs_residuals* residuals);

/* one linearizeAll(false) + applyRes over all residuals; reset=1 applies resetOOB first (optimize() entry).
   energy_out: sum of the linearize() energies (nullable; forces a sync). */
int hs_ba_linearize(hs_ctx* ctx, int reset, double* energy_out);

/* solveSystemF on the systems accumulated by the last hs_ba_linearize. x_out: dim = 4 + 8*nF (nullable). */
int hs_ba_solve_system(hs_ctx* ctx, int iteration, double* x_out);

/* doStepFromBackup with all step factors 1; canbreak_out nullable. */
int hs_ba_do_step(hs_ctx* ctx, int* canbreak_out);

/* System::optimize loop.  Windows of fewer than 4 frames run 15 iterations whatever max_iters says (the
   reference's override, Src/FullSystemOptimize.cpp:366-367); energies_out (nullable) receives at most
   max_iters + 1 energies, iters_done (nullable) the number of iterations actually run. */
int hs_ba_optimize(hs_ctx* ctx, int max_iters, int allow_break, double* energies_out, int* iters_done);

/* n_iters GN iterations (solve + step + linearize) continuing from the current linearization,
   iteration numbers first_iteration.. (orthogonalize from iteration 2); no early break.
   energies_out[n_iters] nullable.  This is the benchmark's "step". */
int hs_ba_iterate(hs_ctx* ctx, int first_iteration, int n_iters, double* energies_out);

/* System::optimize's tail after the GN loop (Src/FullSystemOptimize.cpp:498-516): the newest frame's
   setEvalPT(PRE_worldToCam, state = state_zero = (0,..,0, a, b, 0, 0)) (Include/Frame.h:213-218), setAdjointsF and
   setPrecalcValues, then linearizeAll(true) (:19-52, :102-160): every active residual is linearized and applied
   (applyRes(true)); for each residual still active its point's maxRelBaseline = max(relBS) and
   numGoodResiduals++ (the reference never clears PointFrameResidual::isNew, so every active residual counts);
   setNewFrameEnergyTH.
     energy_out        linearizeAll(true)'s energy; non-finite -> HS_ERR_NONFINITE (the reference's isLost).
     drop_out[nR]      1 = not active after the pass: the toRemove list (the caller resets the point's
                       lastResiduals[i].first and calls ef->dropResidual).  The new residual states
                       (lastResiduals[i].second) and centerProjectedTo come from hs_ba_get_residuals.
     maxRelBaseline[nP], numGoodResiduals[nP]   the points' values, updated in place (both or neither).
     HdiF_out[nP]      HdiF of the linearization the last solve consumed (the last accumulateSCF_MT's
                       AccumulatedSCHessianSSE::addPoint, Src/AccumulatedSCHessian.cpp:28): makeCoarseDepthL0's
                       weights (Src/CoarseTracker.cpp:124).
   All outputs nullable.  The context's window afterwards is the fixed one (evalPT moved, system re-stitched). */
int hs_ba_fix_linearization(hs_ctx* ctx, double* energy_out, uint8_t* drop_out, float* maxRelBaseline,
                            int* numGoodResiduals, float* HdiF_out);

/* EnergyFunctional::calcLEnergyF_MT and calcMEnergyF (Src/EnergyFunctional.cpp:277-368) on the current state: the
   energies System::optimize evaluates only when setting_forceAceptStep is off (System::calcLEnergy /
   calcMEnergy return 0 otherwise, Src/FullSystemOptimize.cpp:337-345,565-572) -- the caller keeps that flag.
   energyL: frame priors + calib prior + the points' depth priors (the window holds no linearized residuals);
   energyM: delta . (2 bM + HM delta).  On a multi-rank window energyL's point term is this rank's share. */
int hs_ba_calc_energies(hs_ctx* ctx, double* energyL, double* energyM);

/* which: 0 = HA/bA, 1 = HL/bL (priors), 2 = H_sc/b_sc. H: dim*dim row-major, b: dim. */
int hs_ba_get_system(hs_ctx* ctx, int which, double* H, double* b);

/* per-residual read-back (all nullable): ResState, isActive, energy, energy-with-outlier (-1 = none),
   JpJdF [n][8], centerProjectedTo [n][3] */
int hs_ba_get_residuals(hs_ctx* ctx, uint8_t* state, uint8_t* active, float* energy, float* energy_wo,
                        float* JpJdF, float* center);
/* per-point read-back (all nullable) */
int hs_ba_get_points(hs_ctx* ctx, float* idepth, float* step, float* HdiF, float* bdSumF);
/* per-frame: state[nF][10], frameEnergyTH[nF], PRE_worldToCam[nF][7]; calib value[4] (all nullable) */
int hs_ba_get_frames(hs_ctx* ctx, double* state, float* energyTH, double* pose7, double* calib4);
/* per-frame linearization point: worldToCam_evalPT[nF][7] (Sophus data order, as hs_frame) and state_zero[nF][10]
   (FrameHessian::get_worldToCam_evalPT / get_state_zero, Include/Frame.h:157-176; the optimize tail's setEvalPT
   moves the newest frame's).  Both nullable. */
int hs_ba_get_frame_eval(hs_ctx* ctx, double* evalPT7, double* state_zero);
/* EnergyFunctional::HM / bM (marginalization prior); dim*dim and dim */
int hs_ba_set_marginal_prior(hs_ctx* ctx, const double* HM, const double* bM);

/* Marginalization of n window points (indices into the hs_points of hs_ba_set_window), replacing
   System::flagPointsForRemoval's per-point part (Src/Mapping.cpp:280-293: resetOOB, linearize, applyRes,
   fixLinearizationF of the active residuals) and EnergyFunctional::marginalizePointsF
   (Src/EnergyFunctional.cpp:545-609: priorF *= idepthFixPriorMargFac, AccumulatedTopHessianSSE::addPoint<2>,
   AccumulatedSCHessianSSE::addPoint(p, false), HM += margWeightFac (M - Msc), bM likewise).
   HM_out / bM_out (nullable, dim*dim / dim): the updated prior, also kept by the context.  The call consumes the
   window's current linearization: the caller drops the points (removePoint: hs_ba_set_window without them),
   passes HM / bM to hs_ba_set_marginal_prior and linearizes again. */
int hs_ba_marginalize_points(hs_ctx* ctx, int n, const int* points, double* HM_out, double* bM_out);

/* EnergyFunctional::marginalizeFrame (Src/EnergyFunctional.cpp:456-543) of window frame `frame` on the
   context's HM / bM: the frame's prior is added, its 8 rows are Schur-complemented out of the scaled prior.
   HM_out / bM_out: (dim-8)^2 / dim-8, the prior of the window without that frame (pass it to
   hs_ba_set_marginal_prior after the next hs_ba_set_window).  The context's own window is unchanged. */
int hs_ba_marginalize_frame(hs_ctx* ctx, int frame, double* HM_out, double* bM_out);

/* device-event timing of the last hs_ba_optimize / hs_ba_iterate (ms, summed over the timed iterations):
   [0] linearize kernel, [1] accumulate + stitch (+ RCCL exchange), [2] solve + step kernel,
   [3] number of event-timed iterations, [4] total GN loop wall (host clock), [5] iterations.
   Env HS_EVENT_TIMING: 0 (default) none, 1 times the linearize kernel only, 2 every phase. */
int hs_ba_get_timings(hs_ctx* ctx, double* out6);
/* Sets the HS_EVENT_TIMING mode (0 / 1 / 2 as above) of this context's later GN loops (the bench times its loop
   without events, then runs an untimed event-timed loop for the per-phase split).  Measurement only. */
int hs_ba_set_event_timing(hs_ctx* ctx, int mode);

/* Roofline timing: reps back-to-back launches of the linearize kernel (no fused point step) on the
   context's stream between one HIP event pair; avg_ms = elapsed / reps.  Leaves the residual states of a
   re-linearization at the current point depths.  Measurement only (no reference counterpart). */
int hs_ba_time_linearize(hs_ctx* ctx, int reps, double* avg_ms);

/* The linearize partitioning of the current window: out4 = [kernel (0 hs_k_lin: one point per wave, 1 hs_k_lin8:
   8 points per wave, the production choice from 60k points; env HS_LIN8 forces it), blocks, waves per block that
   take points, HS_ACC_EXACT].  Introspection only (no reference counterpart). */
int hs_ba_get_partition(hs_ctx* ctx, int* out4);

/* ---------------------------------------------------------------------------------------------------------------
 * Incremental window: the keyframe path.  System::AddKeyframe (Src/Mapping.cpp:12-140) edits the window one object
 * at a time through EnergyFunctional::insertFrame / insertPoint / insertResidual / dropResidual / removePoint /
 * marginalizeFrame / makeIDX (Src/EnergyFunctional.cpp:371-454,456-543,632-646,819-840) and System::marginalizeFrame
 * (Src/FullSystemMarginalize.cpp:108-176).  These calls do the same on a context whose device memory hs_ba_reserve
 * allocated once: an edit changes the host mirror of the window's structure (frames in frameHessians order, each
 * frame's points in pointHessians order, each point's residual list in PointHessian::residuals order, with the
 * reference's swap-with-last removals); the next call that needs the device window commits the edits (makeIDX: one
 * pinned upload of the changed index tables plus new points, one gather kernel that moves the device-resident point
 * state -- idepth, idepth_zero, priors, colours, maxRelBaseline / numGoodResiduals, the last solve's HdiF, residual
 * states and centre projections -- into the new order).  Points are named by the handles hs_ba_insert_points
 * returns, frames by their window index.  After a commit the window equals the one hs_ba_set_window builds from the
 * same frames, points (window order) and residuals (point order, list order), and every read-back (residuals in
 * that order) refers to it.  hs_ba_set_window leaves a context these calls can continue from.
 * --------------------------------------------------------------------------------------------------------------- */

/* Capacity for windows of up to HS_MAX_FRAMES frames of cam's size and max_points points (device memory allocated
   once; no allocation on the keyframe path).  Starts an empty incremental window. */
int hs_ba_reserve(hs_ctx* ctx, const hs_camera* cam, int max_points);

/* EnergyFunctional::insertFrame: `frame` becomes the newest window frame (index nF), with takeData's priors; the
   marginal prior HM / bM grows by 8 zero rows / columns.  image (nullable): level-0 (I, dI/dx, dI/dy) triplets,
   W*H*3 floats (Frame::DirPyr[0]); else set it with one of the hs_ba_set_frame_image* calls before the next commit. */
int hs_ba_insert_frame(hs_ctx* ctx, const hs_frame* frame, const float* image);
/* the frame's level-0 image: host (I, dI/dx, dI/dy) triplets | host raw W*H image (ImageData::fImgL: level 0 of
   Frame::CreateDirPyrs runs on the device, Src/Frame.cpp:104-181) | device texels (W*H float4 (I, dI/dx, dI/dy, any)
   on the context's device, e.g. hs_tracker_frame_texels: the keyframe's image never crosses PCIe again; the producer
   must have completed, as it has when its call returned; the device copy has read the texels when this call returns,
   so the producer may overwrite them next).  Copies, ordered on the context's stream. */
int hs_ba_set_frame_image(hs_ctx* ctx, int frame, const float* image);
int hs_ba_set_frame_image_raw(hs_ctx* ctx, int frame, const float* raw);
int hs_ba_set_frame_image_device(hs_ctx* ctx, int frame, const void* d_texels);

/* EnergyFunctional::insertPoint for pts->n points (pts->host: window frame index; each appended to its host's point
   list, Src/Mapping.cpp:449).  maxRelBaseline / numGoodResiduals (nullable => 0) seed the linearizeAll(true)
   bookkeeping the context keeps per point.  handles_out[n]: the points' handles. */
int hs_ba_insert_points(hs_ctx* ctx, const hs_points* pts, const float* maxRelBaseline, const int* numGoodResiduals,
                        int* handles_out);
/* EnergyFunctional::insertResidual: n residuals (point handle, target window frame), each appended to its point's
   residual list; states (nullable => IN). */
int hs_ba_insert_residuals(hs_ctx* ctx, int n, const int* point_handles, const int* targets, const uint8_t* states);
/* AddKeyframe's loop (Src/Mapping.cpp:40-56): a residual in state IN from every point not hosted by the newest frame
   into it, frames and points in window order.  n_added (nullable). */
int hs_ba_add_residuals_to_newest(hs_ctx* ctx, int* n_added);
/* EnergyFunctional::dropResidual (swap with the last of the point's list) for n (point handle, target) pairs, in
   the given order. */
int hs_ba_drop_residuals(hs_ctx* ctx, int n, const int* point_handles, const int* targets);
/* linearizeAll(true)'s toRemove loop (Src/FullSystemOptimize.cpp:137-159): every residual not active after the last
   hs_ba_fix_linearization is dropped, in activeResiduals order.  n_dropped (nullable). */
int hs_ba_drop_inactive_residuals(hs_ctx* ctx, int* n_dropped);
/* EnergyFunctional::removePoint for n handles; each host's point list is compacted the way
   System::flagPointsForRemoval does it (Src/Mapping.cpp:318-326: a removed entry takes the list's last one). */
int hs_ba_remove_points(hs_ctx* ctx, int n, const int* handles);
/* System::removeOutliers (Src/FullSystemOptimize.cpp:575-598): every point without residuals is removed.
   handles_out (nullable, capacity nP): the removed handles in removal order; n_out (nullable). */
int hs_ba_remove_points_without_residuals(hs_ctx* ctx, int* handles_out, int* n_out);
/* System::marginalizeFrame (Src/FullSystemMarginalize.cpp:108-176) of window frame `frame`, which must host no point:
   marginalize = 1 runs EnergyFunctional::marginalizeFrame on the context's HM / bM (as hs_ba_marginalize_frame) and
   keeps the result; 0 drops the frame's rows / columns instead.  Every residual into the frame is dropped (window
   order), the frame leaves the window (order-preserving, deleteOutOrder) and its image slot is freed. */
int hs_ba_remove_frame(hs_ctx* ctx, int frame, int marginalize);
/* EnergyFunctional::makeIDX: commit the pending edits now (otherwise the next call that needs the device window
   does).  Returns the committed sizes (nullable). */
int hs_ba_make_idx(hs_ctx* ctx, int* nF, int* nP, int* nR);
/* waits for the context's queued device work (keyframe timing; no reference counterpart) */
int hs_ba_synchronize(hs_ctx* ctx);
/* EnergyFunctional::HM / bM as the context keeps them (dim*dim, dim; nullable).  Commits first. */
int hs_ba_get_marginal_prior(hs_ctx* ctx, double* HM, double* bM);
/* the device-resident per-point state a caller mirrors into its MapPoints (window order; commits first; nullable):
   idepth, idepth_zero, maxRelBaseline, numGoodResiduals, and HdiF of the last solve (efPoint->HdiF as
   makeCoarseDepthL0 reads it; idepth_hessian = 1 / HdiF for points with an active residual). */
int hs_ba_get_point_state(hs_ctx* ctx, float* idepth, float* idepth_zero, float* maxRelBaseline, int* numGoodResiduals,
                          float* HdiF);
/* the committed window's structure (commits first): handles[nP], pt_host[nP], nres[nP] (residual-list lengths),
   res_target[nR] (targets in activeResiduals order: points in window order, each point's list in order).
   All nullable. */
int hs_ba_get_structure(hs_ctx* ctx, int* handles, int* pt_host, int* nres, int* res_target);

/* multi-GPU (point sharding): 128-byte RCCL unique id from rank 0, broadcast by the caller.
   hs_comm_init must be called before hs_ba_set_window.  Each rank loads its own point shard (same frames);
   per linearization ONE exchange (two all-gathers in one RCCL group call): every rank's stitched system vector +
   energies and its newest-frame energies.  Every rank sums the vectors in rank order (the same system on every
   rank, replacing the reduction of Src/EnergyFunctional.cpp:155-220 over the reference's threads) and selects
   setNewFrameEnergyTH over the gathered energies beside the solve. */
int hs_comm_get_unique_id(char* id128);
int hs_comm_init(hs_ctx* ctx, const char* id128, int rank, int nranks);
/* the communicator's own rank count and this context's rank (ncclCommCount / ncclCommUserRank); 1 / 0 without a
   communicator.  The bench reports n_gpus from it, not from the launcher's environment. */
int hs_comm_size(hs_ctx* ctx, int* nranks, int* rank);
/* failure handling of a multi-rank context ("RCCL errors are mapped to status codes"; the reference's
   isLost, Src/FullSystemOptimize.cpp:512-516): every wait of a context with a communicator polls the stream and
   ncclCommGetAsyncError under a wall-clock bound (default 60000 ms).  A collective that reports an error, or does not
   finish within the bound (a peer rank died or stalled), aborts the communicator (ncclCommAbort) and the call returns
   HS_ERR_RCCL; every later call on the context returns HS_ERR_RCCL as well (destroy it and rebuild the ranks). */
int hs_comm_set_timeout(hs_ctx* ctx, int timeout_ms);

#ifdef __cplusplus
}
#endif
#endif /* HS_BA_H */
