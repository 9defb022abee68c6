// hs_sel_kernels.h — PixelSelector (Src/PixelSelector.cpp:54-418) kernels and their argument blocks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// makeHists (:57-117): 32x32 gradient histograms -> ths, then (last block) the 3x3 smoothing -> thsSmoothed
struct HsSelHistArgs {
  int W, H, w32, h32;
  const float* absg0;  // absSquaredGrad[0], W*H
  float minGradHistCut, minGradHistAdd;
  float* ths;          // w32*h32
  float* thsSmoothed;  // w32*h32 (+ zeroed slack, see hs_select.cpp)
  unsigned int* ticket;
};

// select (:265-415) at one potential.  Work unit = one pot-block ("slot"), slots numbered in the reference's
// traversal order with a padded index: slot = (b4 * 4 + sub3) * 4 + sub2, b4 the raster index of the 4pot-block,
// sub3 the raster position of the 2pot-block inside it, sub2 that of the pot-block inside the 2pot-block.
struct HsSelArgs {
  int W, H, pot, n4x, n4y, nslots;
  const float* dI;  // Frame::DirPyr[0]: dx at dI[dstride*idx+1], dy at dI[dstride*idx+2]
  int dstride;
  const float* g0;  // absSquaredGrad[0..2]
  const float* g1;
  const float* g2;
  int w1, w2;
  const float* thsSmoothed;
  int thsStep;
  float dw1, dw2, thFactor;
  int dirDist;               // setting_selectDirectionDistribution
  const uint8_t* pattern;    // randomPattern, W*H
  uint16_t* mask;            // [nslots] level-2 existence per direction (bit d: a pixel with |g . dir_d| > 0)
  int* n2b;                  // [nslots] n2 before the slot (the count select's dir2/dir3/dir4 index with)
  uint8_t* has2;             // [nslots] the slot selects a level-2 pixel
  float* map;                // W*H selection map (zeroed before hs_k_sel_pick)
  int* counts;               // n2, n3, n4 (zeroed before hs_k_sel_pick)
};

// makeMaps' random sub-sampling (:226-243): rank of every selected pixel in raster order
struct HsSelSubArgs {
  int n;               // W*H
  float* map;
  const uint8_t* pattern;
  int* tile_cnt;       // [ntiles] selected pixels per tile of kSelSubTile pixels, then their exclusive prefix
  int ntiles;
  uint8_t charTH;
  int* removed;
};

constexpr int kSelSubTile = 2048;  // 256 threads x 8 pixels

__global__ void hs_k_sel_hist(HsSelHistArgs a);
__global__ void hs_k_sel_mask(HsSelArgs a);
__global__ void hs_k_sel_scan(HsSelArgs a);
__global__ void hs_k_sel_pick(HsSelArgs a);
__global__ void hs_k_sel_subcount(HsSelSubArgs a);
__global__ void hs_k_sel_subscan(HsSelSubArgs a);
__global__ void hs_k_sel_subapply(HsSelSubArgs a);
