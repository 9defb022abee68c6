// hs_win_kernels.hip — device side of the incremental keyframe window (hs_ba_window.cpp).
//
//   hs_k_win_gather   the structural commit (EnergyFunctional::makeIDX after insertFrame / insertPoint /
//                     insertResidual / dropResidual / removePoint / marginalizeFrame): every point of the new layout
//                     takes its device-resident state from its old position (or from the staged upload of a point
//                     inserted since the last commit), its residual slots from the old frame column of the same
//                     target (frames keep their order; removed frames' columns vanish, new ones start empty); the
//                     frames' setNewFrameEnergyTH thresholds follow their frames.  One lane per (point, slot): the
//                     [n][8] arrays move as coalesced rows.  Pure copies: a commit changes no value, only places.
//   hs_k_win_newest   the BA -> tracker hand-off (CoarseTracker::makeCoarseDepthL0's point loop,
//                     Src/CoarseTracker.cpp:110-129): the points whose residual into the newest frame is IN, in point
//                     order, as (centerProjectedTo u, v, idepth, HdiF); one workgroup, ballot prefix sums per chunk.
#include <hip/hip_runtime.h>

#include "hs_win_kernels.h"

__global__ __launch_bounds__(256) void hs_k_win_gather(HsWinGatherArgs a) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the thresholds follow their frames (in place: one thread)
    float old[HS_MAXF];
    for (int f = 0; f < HS_MAXF; f++) old[f] = a.frameTH[f];
    for (int f = 0; f < a.nF; f++) a.frameTH[f] = a.col_src[f] >= 0 ? old[a.col_src[f]] : a.th_init[f];
  }
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int p = gid >> 3, t = gid & 7;
  if (p >= a.n) return;
  const int src = a.src[p];
  const size_t o = (size_t)p * 8 + t;
  if (src >= 0) {
    const size_t i = (size_t)src * 8 + t;
    a.to.color[o] = a.from.color[i];
    a.to.weight[o] = a.from.weight[i];
    if (t == 0) {
      a.to.u[p] = a.from.u[src];
      a.to.v[p] = a.from.v[src];
      a.to.idepth[p] = a.from.idepth[src];
      a.to.idepth_zero[p] = a.from.idepth_zero[src];
      a.to.priorF[p] = a.from.priorF[src];
      a.to.relBL[p] = a.from.relBL[src];
      a.to.nGood[p] = a.from.nGood[src];
      a.hdif_to[p] = a.hdif_from[src];
    }
  } else {
    const HsStagedPoint& s = a.staged[-src - 1];
    a.to.color[o] = s.color[t];
    a.to.weight[o] = s.weight[t];
    if (t == 0) {
      a.to.u[p] = s.u;
      a.to.v[p] = s.v;
      a.to.idepth[p] = s.idepth;
      a.to.idepth_zero[p] = s.idepth_zero;
      a.to.priorF[p] = s.priorF;
      a.to.relBL[p] = s.relBL;
      a.to.nGood[p] = s.nGood;
      a.hdif_to[p] = 0.f;
    }
  }
  // residual slot t: a committed residual keeps its state and centre projection (old column of the same frame), a new
  // one starts in the given state, a slot without a residual is OOB
  const unsigned code = a.newres[o];
  uint8_t st = HS_RES_OOB;
  float c0 = 0.f, c1 = 0.f, c2 = 0.f;
  if (code == HS_WIN_KEEP) {
    const size_t i = (size_t)src * 8 + a.col_src[t];
    st = a.from.r_state[i];
    c0 = a.from.r_center[3 * i]; c1 = a.from.r_center[3 * i + 1]; c2 = a.from.r_center[3 * i + 2];
  } else if (code != HS_WIN_NONE) {
    st = (uint8_t)code;
  }
  a.to.r_state[o] = st;
  a.to.r_center[3 * o] = c0;
  a.to.r_center[3 * o + 1] = c1;
  a.to.r_center[3 * o + 2] = c2;
}

// points p (in order) with res_of_slot[p][newest] >= 0 and state IN -> out[cap * {0,1,2,3}] = cu, cv, cid, HdiF
__global__ __launch_bounds__(1024) void hs_k_win_newest(int n, int newest, const int* __restrict__ res_of_slot,
                                                        const uint8_t* __restrict__ r_state,
                                                        const float* __restrict__ r_center,
                                                        const float* __restrict__ hdif, float* __restrict__ out,
                                                        int cap, int* __restrict__ n_out) {
  __shared__ int wsum[16];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int p = c0 + tid;
    bool take = false;
    if (p < n) {
      const size_t sl = (size_t)p * 8 + newest;
      take = res_of_slot[sl] >= 0 && r_state[sl] == HS_RES_IN;
    }
    const unsigned long long m = __ballot(take);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wv] = __popcll(m);
    __syncthreads();
    int off = base_s;
    for (int w = 0; w < wv; w++) off += wsum[w];
    if (take) {
      const int q = off + before;
      const size_t sl = (size_t)p * 8 + newest;
      out[q] = r_center[3 * sl];
      out[cap + q] = r_center[3 * sl + 1];
      out[2 * cap + q] = r_center[3 * sl + 2];
      out[3 * cap + q] = hdif[p];
    }
    __syncthreads();
    if (tid == 0) {
      int s = 0;
      for (int w = 0; w < 16; w++) s += wsum[w];
      base_s += s;
    }
    __syncthreads();
  }
  if (tid == 0) *n_out = base_s;
}
