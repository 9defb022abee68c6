/*
 * hs_select.h — C-ABI of the pixel selection step on MI355X.
 *
 * Replaces, in AUBVRL/H-SLAM:
 *   hs_selector_create     PixelSelector::PixelSelector (Src/PixelSelector.cpp:14-33): the randomPattern of
 *                          std::srand(3141592) / rand() & 0xFF (the C library generator, restated on the host),
 *                          currentPotential 3.
 *   hs_selector_make_maps  PixelSelector::makeMaps (Src/PixelSelector.cpp:118-262) with makeHists (:57-117) and
 *                          select (:265-415): the 32x32 gradient histograms and their smoothed thresholds, the
 *                          pot / 2pot / 4pot block selection with the reference's direction sequence, the
 *                          re-selection recursion and the random sub-sampling.  map_out is selectionMap
 *                          (FeatureDetector::ExtractFeatures, Src/Detector.cpp:58): 0, 1, 2 or 4 per pixel.
 *
 * Conventions as include/hs_ba.h: status codes (hs_types.h), caller-owned host buffers, the context owns device
 * memory and its own HIP stream, single caller.
 */
#ifndef HS_SELECT_H
#define HS_SELECT_H

#include "hs_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hs_selector hs_selector;

/* width/height: CalibData::Width/Height (level 0) */
int hs_selector_create(hs_selector** out, const hs_params* params, int device_id, int width, int height);
void hs_selector_destroy(hs_selector* s);

/* makeMaps on a frame given as its DirPyr[0] ((I, dx, dy) float triplets, W*H) and absSquaredGrad of levels 0, 1, 2
   (W*H, (W/2)*(H/2), (W/4)*(H/4) floats).  frame_id: makeHists runs only when it differs from the last call's
   (gradHistFrame).  density: numWant; recursions_left / th_factor: makeMaps' recursionsLeft (reference default 1)
   and thFactor (default 1).  map_out[W*H] (nullable) receives the selection map, *n_selected the returned count. */
int hs_selector_make_maps(hs_selector* s, int frame_id, const float* dirpyr0, const float* absg0, const float* absg1,
                          const float* absg2, float density, int recursions_left, float th_factor, float* map_out,
                          int* n_selected);
/* the same from the raw level-0 image (W*H floats): Frame::CreateDirPyrs runs on the device (include/hs_pyr.h) */
int hs_selector_make_maps_raw(hs_selector* s, int frame_id, const float* img, float density, int recursions_left,
                              float th_factor, float* map_out, int* n_selected);
/* PixelSelector::currentPotential (read / overwrite) */
int hs_selector_get_potential(hs_selector* s, int* potential);
int hs_selector_set_potential(hs_selector* s, int potential);
/* last make_maps: device time (ms, HIP events on the selector stream) and the select passes it ran (1 or 2) */
int hs_selector_last_stats(hs_selector* s, double* ms, int* passes);

#ifdef __cplusplus
}
#endif
#endif /* HS_SELECT_H */
