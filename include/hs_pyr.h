/*
 * hs_pyr.h — the direct-image pyramid on MI355X.
 *
 * Replaces Frame::CreateDirPyrs (Src/Frame.cpp:104-181): from a frame's photometrically undistorted level-0
 * image (ImageData::fImgL, Include/DatasetLoader.h:436-506; W*H floats) it builds DirPyr[lvl] (w_l*h_l (I, dI/dx,
 * dI/dy) float triplets, w_l = W >> lvl) and absSquaredGrad[lvl] (w_l*h_l floats) for DirPyrLevels levels.
 * The contexts take raw frames directly (hs_tracker_set_frame_raw, hs_tracer_set_frame_raw): the pyramid is
 * built on the device and never crosses PCIe.  Border rows of dI are 0 (the reference leaves them
 * uninitialised); absSquaredGrad skips the gamma weighting (Calib->PhotoUnDistL is null).
 */
#ifndef HS_PYR_H
#define HS_PYR_H

#include "hs_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Standalone: builds the pyramid on device `device_id` and copies it back.  dirpyr_out (nullable): levels
   concatenated, sum_l w_l*h_l*3 floats; abs_squared_grad_out (nullable): sum_l w_l*h_l floats. */
int hs_dir_pyramid(int device_id, int width, int height, int n_levels, const float* img, float* dirpyr_out,
                   float* abs_squared_grad_out);

#ifdef __cplusplus
}
#endif
#endif /* HS_PYR_H */
