/*
 * hs_refine.h — C-ABI drop-in boundary of H-SLAM's initializer refinement (DirectRefinement, SURVEY.md §8f
 * rank 4) on MI355X (gfx950).  Same conventions as hs_ba.h: plain C, caller-owned host buffers copied in/out,
 * the refiner owns its device memory and HIP stream, status codes from hs_types.h, one refiner per calling
 * thread.
 *
 * Reference interface each entry point replaces (AUBVRL/H-SLAM):
 *   hs_refiner_create / destroy   DirectRefinement ctor buffers (JbBuffer, points)  Src/Initializer.cpp:1330-1360,1404-1410
 *   hs_refiner_set_frames         FirstFrame / SecondFrame ->frame->DirPyr[0] and ab_exposure
 *                                 (Include/Initializer.h:123-124, Include/Frame.h:39)
 *   hs_refiner_set_points         the ctor's Pnt set-up from mvKeys / Pts3D / Triangulated  Src/Initializer.cpp:1362-1382
 *   hs_refiner_refine             Refine (Src/Initializer.cpp:1412-1564) + the ctor's write-back of
 *                                 _Pose and _videpth (:1387-1396)
 *   hs_refiner_calc_res           resetPoints + one calcResAndGS (Src/Initializer.cpp:1897-2153)
 *   hs_refiner_get_points / get_log   read-back of the Pnt state / the LM trajectory (parity and debugging)
 *
 * Images: W*H*3 floats (I, dI/dx, dI/dy) = Frame::DirPyr[0].  Poses: Sophus SE3d::data() order
 * (qx qy qz qw tx ty tz), refToNew (first -> second frame).  Affine: AffLight (a, b).
 */
#ifndef HS_REFINE_H
#define HS_REFINE_H
#include <stdint.h>

#include "hs_types.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct hs_refiner hs_refiner;

/* K4 = (fx, fy, cx, cy) of CalibData::pyrK[0] (double, as the reference's Mat33) */
int hs_refiner_create(hs_refiner** out, int device_id, int width, int height, const double K4[4]);
void hs_refiner_destroy(hs_refiner* r);
/* exposures: FrameShell::ab_exposure of the two frames (<= 0: Refine keeps thisToNext_aff = (0, 0)) */
int hs_refiner_set_frames(hs_refiner* r, const float* first_dirpyr0, const float* second_dirpyr0,
                          float first_exposure, float second_exposure);
/* the first frame's keypoints (mvKeys[i].pt), Triangulated[i] and Pts3D[i].z (read when triangulated) */
int hs_refiner_set_points(hs_refiner* r, int n, const float* u, const float* v, const uint8_t* triangulated,
                          const float* z);
/* Refine: pose_inout = thisToNext (in: the initializer's pose, out: the refined pose, like _Pose);
   idepth_out[n] (nullable) = the refined idepth where the point is good and triangulated, unchanged
   elsewhere (the reference's _videpth write-back); good_out[n] (nullable) = isGood;
   *iterations = LM iterations run; *snapped = the alpha regularizer switched off. */
int hs_refiner_refine(hs_refiner* r, double pose_inout[7], float* idepth_out, uint8_t* good_out, int* iterations,
                      int* snapped);
/* resetPoints + calcResAndGS(lvl 0) at (T7, aff) on the current point state (no step applied):
   H64/b8 = H_out/b_out, Hsc64/bsc8 = H_out_sc/b_out_sc, res3 = (E, alphaEnergy, E.num) */
int hs_refiner_calc_res(hs_refiner* r, const double T7[7], const double aff[2], float* H64, float* b8, float* Hsc64,
                        float* bsc8, float res3[3]);
/* per point: f7[n*7] = idepth, idepth_new, iR, energy_new[0], energy_new[1], maxstep, lastHessian_new;
   g2[n*2] = isGood, isGood_new; jb_new[n*10] (nullable) = JbBuffer_new */
int hs_refiner_get_points(hs_refiner* r, float* f7, uint8_t* g2, float* jb_new);
/* LM log of the last refine: 8 floats per iteration (eTotalOld, eTotalNew, accept, lambda, |inc|, resNew[0],
   resNew[1], calcEC new); returns the number of iterations logged (<= cap written) */
int hs_refiner_get_log(hs_refiner* r, int cap, float* out);
/* device time of the last refine / calc_res kernel (HIP events on the refiner's stream), ms */
int hs_refiner_last_ms(hs_refiner* r, double* ms);

#ifdef __cplusplus
}
#endif
#endif /* HS_REFINE_H */
