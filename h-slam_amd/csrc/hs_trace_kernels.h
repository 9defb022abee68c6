// hs_trace_kernels.h — argument blocks of the ImmaturePoint kernels (hs_trace_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hs_trace.h"

#define HS_TRC_MAXHOST 64

// ImmaturePoint ctor for points [first, first + n)
struct HsImmCtorArgs {
  int n, first, W, H;
  const float4* const* host_img;  // device array of [HS_TRC_MAXHOST] level-0 images
  const int* host;
  const float* u;
  const float* v;
  float outlierTHSumComponent, outlierTH, overallEnergyTHWeight;
  float* color;     // [n][8]
  float* weights;   // [n][8]
  float* gradH;     // [n][4]
  float* energyTH;
  float* quality;
  float* idepth_min;
  float* idepth_max;
  uint8_t* status;
  float* uv;        // [n][2]
  float* interval;
};

struct HsTraceArgs {
  int n, W, H;
  const float4* img;            // the new frame, level 0
  const hs_trace_host* hosts;   // per host slot
  const int* host;
  const float* u;
  const float* v;
  const float* color;
  const float* weights;
  const float* gradH;
  const float* energyTH;
  float* quality;
  float* idepth_min;
  float* idepth_max;
  uint8_t* status;
  float* uv;
  float* interval;
  int* steps;                   // [n] discrete-search steps evaluated (0 = no search)
  float huberTH, maxPixSearch, slackInterval, stepsize, minImprovementFactor, GNThreshold, extraSlackOnTH;
  int minTraceTestRadius, GNIterations;
};

__global__ void hs_k_imm_ctor(HsImmCtorArgs a);
__global__ void hs_k_trace_on(HsTraceArgs a);
__global__ void hs_k_trace_count(int n, const uint8_t* status, const int* steps, int* out);

// ---- point activation (System::activatePointsMT), hs_act_kernels.hip ----------------------------------------
#define HS_ACT_BFS_STEPS 40    // growDistBFS: k = 1 .. 39

// candidate states of the selection loop (per entry of the loop order)
enum { HS_CAND_SKIP = 0, HS_CAND_DELETE = 1, HS_CAND_PENDING = 2 };

// makeDistanceMap seeds: every active point's level-1 projection into the newest keyframe
struct HsActSeedArgs {
  int n, newest, w1, h1;
  const hs_act_frame* frames;
  const int* frame;
  const float* u;
  const float* v;
  const float* idepth;
  uint8_t* dist;   // [w1*h1] distance bytes (255 = 1000, untouched)
  int* list;       // [w1*h1] seed cells x | y << 16 (deduplicated)
  int* count;
};

// per loop-order entry: the state-only part of the selection loop (Mapping.cpp:378-426 up to the distance test)
struct HsActCandArgs {
  int m, newest, w1, h1;
  float minTraceQuality, currentMinActDist;
  const int* order;          // nullable: identity
  const int* frame_of_slot;  // [HS_TRC_MAXHOST] window frame index of a tracer slot, -1 = none
  const hs_act_frame* frames;
  const int* host;
  const float* u;
  const float* v;
  const float* idepth_min;
  const float* idepth_max;
  const float* quality;
  const float* interval;
  const float* my_type;
  const uint8_t* status;
  uint8_t* cand;     // [m] HS_CAND_*
  int* cell;         // [m] projected cell u | v << 16 of a pending entry
  float* frac;       // [m] ptp[0] - floorf(ptp[0])
  float* thr;        // [m] currentMinActDist * my_type
  uint8_t* action;   // [n points] HS_ACT_*
};

// a distance map from seeds in closed form (hs_act_kernels.hip bfs_dist): mode 0, makeDistanceMap's multi-seed
// growDistBFS (Src/CoarseTracker.cpp:726-756); mode 1, the map the greedy loop leaves (makeDistanceMap's map + every
// addIntoDistFinal, in call order).  Interior cells in 16 x 16 tiles, then the border cells, one thread each.
struct HsActDistArgs {
  int w1, h1, mode, n_tiles_x, n_tiles;
  int dbg;                   // experiments (env HS_ACT_DBG): 1 border blocks return, 2 tile blocks return, 4 no seeds
  const int* seeds;          // cells x | y << 16
  const int* n_seeds;
  const uint8_t* init;       // [w1*h1] mode 0: 0 at the seeds, 255 elsewhere; mode 1: makeDistanceMap's map
  uint8_t* out;              // [w1*h1]
};

// the sequential part: the greedy distance test + addIntoDistFinal in loop order
struct HsActSelectArgs {
  int m, w1, h1, lds_map;
  const int* order;
  const uint8_t* cand;
  const int* cell;
  const float* frac;
  const float* thr;
  uint8_t* dist;             // global working map when the map does not fit LDS (then hs_k_act_dist mode 1 overwrites it)
  const uint8_t* map0;       // [w1*h1] makeDistanceMap's map (hs_k_act_dist mode 0)
  int* seeds;                // [m] out: the cells addIntoDistFinal was called on, in call order
  int* plist;                // [m] scratch: the pending entries' indices in loop order
  int* toopt;                // [m] points to optimize, in order (+ 64 scratch slots after m)
  int* n_toopt;
  long long* prof;           // nullable: wall_clock64 at entry, after the seed BFS, at exit (HS_ACT_PROF=1)
};

// optimizeImmaturePoint, one wave per point to optimize
struct HsActOptArgs {
  int n, nF, W, H;
  float fxl, fyl, cxl, cyl, fxli, fyli;
  float huberTH, minIdepthH_act;
  int GNIts;
  const int* toopt;
  const int* frame_of_slot;
  const hs_act_frame* frames;
  const hs_act_pair* pairs;
  const float4* const* img;  // per tracer slot
  const int* host;
  const float* u;
  const float* v;
  const float* idepth_min;
  const float* idepth_max;
  const float* color;
  const float* weights;
  const float* energyTH;
  uint8_t* action;
  float* idepth_out;
  uint8_t* res_in;
};

__global__ void hs_k_act_seed(HsActSeedArgs a);
__global__ void hs_k_act_cand(HsActCandArgs a);
__global__ void hs_k_act_dist(HsActDistArgs a);
__global__ void hs_k_act_select(HsActSelectArgs a);
__global__ void hs_k_act_optimize(HsActOptArgs a);
