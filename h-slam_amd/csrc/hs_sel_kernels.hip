// hs_sel_kernels.hip — PixelSelector (Src/PixelSelector.cpp:54-418) on CDNA4.
//
// The reference's select() walks 4pot -> 2pot -> pot blocks in one serial loop, and the only state that crosses
// block boundaries is n2: the count of level-2 selections so far, which picks the direction every block scores
// against (randomPattern[n2] & 0xF, :318,325,332).  Whether a pot-block selects at level 2 depends on that
// direction only through "|g . dir| > 0" of a passing pixel, so the device splits select into
//   hs_k_sel_mask  thread per pot-block ("slot", in traversal order): a 16-bit mask, bit d = some pixel passing
//                  the level-0 threshold has |g . dir_d| > 0 under direction d
//   hs_k_sel_scan  one workgroup: the exclusive count n2 before every slot.  A slot whose mask is 0 or 0xFFFF
//                  selects independently of its direction (a block scan of those); the rest ("ambiguous", e.g.
//                  axis-aligned gradients of 8-bit images under the axis directions) are resolved in traversal
//                  order by one lane from the prefix it has so far, then the chunk is re-scanned
//   hs_k_sel_pick  thread per slot again, now with dir2 / dir3 / dir4 known: the per-block argmax of the
//                  reference (strict '>', first in traversal order wins) for the three levels, combined across the
//                  4 (2pot) and 16 (4pot) slots of a block with lane shuffles; writes the map and n2 / n3 / n4.
// makeHists is hs_k_sel_hist (block per 32x32 cell, LDS histogram, last block smooths) and makeMaps' random
// sub-sampling is hs_k_sel_sub{count,scan,apply} (raster rank of every selected pixel).
// Bandwidth: one pass over absSquaredGrad[0] + (dx, dy) of DirPyr[0] per select pass (+ levels 1, 2 at 1/4,
// 1/16), i.e. ~ W*H*(4 + 8) B read twice (mask + pick) and W*H*4 B of map written.
#include <hip/hip_runtime.h>

#include "hs_sel_kernels.h"

#pragma clang fp contract(off)

namespace {

// the directions table of select (:283-299)
__constant__ float kDir[16][2] = {
    {0.f, 1.0000f},     {0.3827f, 0.9239f},  {0.1951f, 0.9808f},  {0.9239f, 0.3827f},
    {0.7071f, 0.7071f}, {0.3827f, -0.9239f}, {0.8315f, 0.5556f},  {0.8315f, -0.5556f},
    {0.5556f, -0.8315f}, {0.9808f, 0.1951f}, {0.9239f, -0.3827f}, {0.7071f, -0.7071f},
    {0.5556f, 0.8315f}, {0.9808f, -0.1951f}, {1.0000f, 0.0000f},  {0.1951f, -0.9808f}};

// computeHistQuantil (:45-54)
__device__ int hist_quantil(const int* hist, float below) {
  int th = hist[0] * below + 0.5f;
  for (int i = 0; i < 90; i++) {
    th -= hist[i + 1];
    if (th < 0) return i;
  }
  return 90;
}

// exclusive scan of one int per thread over the workgroup (blockDim.x = 64 * nw); *total = the sum
template <int NW>
__device__ int block_excl_scan(int v, int* s_w, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  if (w == 0) {
    int t = lane < NW ? s_w[lane] : 0;
#pragma unroll
    for (int o = 1; o < NW; o <<= 1) {
      const int y = __shfl_up(t, o);
      if (lane >= o) t += y;
    }
    if (lane < NW) s_w[NW + lane] = t;
  }
  __syncthreads();
  const int wexcl = w ? s_w[NW + w - 1] : 0;
  *total = s_w[2 * NW - 1];
  __syncthreads();  // s_w is reused by the next call
  return wexcl + x - v;
}

struct SlotGeo {
  bool valid;
  int x0, y0, mx1, my1;
};

__device__ __forceinline__ SlotGeo slot_geo(const HsSelArgs& a, int s) {
  SlotGeo g;
  const int b4 = s >> 4, sub3 = (s >> 2) & 3, sub2 = s & 3;
  const int b4y = b4 / a.n4x, b4x = b4 - b4y * a.n4x;
  const int x34 = b4x * 4 * a.pot + (sub3 & 1) * 2 * a.pot, y34 = b4y * 4 * a.pot + (sub3 >> 1) * 2 * a.pot;
  g.x0 = x34 + (sub2 & 1) * a.pot;
  g.y0 = y34 + (sub2 >> 1) * a.pot;
  // x3 < mx3 <=> x34 < W; x2 < mx2 <=> x234 < W (and the same in y)
  g.valid = s < a.nslots && b4y < a.n4y && x34 < a.W && y34 < a.H && g.x0 < a.W && g.y0 < a.H;
  g.mx1 = min(a.pot, a.W - g.x0);
  g.my1 = min(a.pot, a.H - g.y0);
  return g;
}

__device__ __forceinline__ bool border_out(const HsSelArgs& a, int xf, int yf) {
  return xf < 4 || xf >= a.W - 5 || yf < 4 || yf > a.H - 4;  // (:342; yf == H-4 is inside)
}

__device__ __forceinline__ float th0_of(const HsSelArgs& a, int xf, int yf) {
  return a.thsSmoothed[(xf >> 5) + (yf >> 5) * a.thsStep];
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// makeHists: block per 32x32 cell (256 threads x 4 pixels); the last block to finish smooths
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void hs_k_sel_hist(HsSelHistArgs a) {
  __shared__ int hist[100];
  __shared__ int s_last;
  const int t = threadIdx.x;
  const int bx = blockIdx.x % a.w32, by = blockIdx.x / a.w32;
  if (t < 100) hist[t] = 0;
  __syncthreads();
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int p = t + 256 * k;
    const int it = (p & 31) + 32 * bx, jt = (p >> 5) + 32 * by;
    if (it > a.W - 2 || jt > a.H - 2 || it < 1 || jt < 1) continue;
    int g = sqrtf(a.absg0[it + jt * a.W]);
    if (g > 48) g = 48;
    atomicAdd(&hist[g + 1], 1);
    cnt++;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((t & 63) == 0) atomicAdd(&hist[0], cnt);
  __syncthreads();
  if (t == 0) {
    const float th = hist_quantil(hist, a.minGradHistCut) + a.minGradHistAdd;
    __hip_atomic_store(&a.ths[blockIdx.x], th, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every thread of the last block sees the other blocks' ths
  const int w32 = a.w32, h32 = a.h32;
  auto T = [&](int x, int y) { return __hip_atomic_load(&a.ths[x + y * w32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int c = t; c < w32 * h32; c += 256) {
    const int x = c % w32, y = c / w32;
    float sum = 0, num = 0;  // the reference's neighbour order (:89-110)
    if (x > 0) {
      if (y > 0) { num++; sum += T(x - 1, y - 1); }
      if (y < h32 - 1) { num++; sum += T(x - 1, y + 1); }
      num++;
      sum += T(x - 1, y);
    }
    if (x < w32 - 1) {
      if (y > 0) { num++; sum += T(x + 1, y - 1); }
      if (y < h32 - 1) { num++; sum += T(x + 1, y + 1); }
      num++;
      sum += T(x + 1, y);
    }
    if (y > 0) { num++; sum += T(x, y - 1); }
    if (y < h32 - 1) { num++; sum += T(x, y + 1); }
    num++;
    sum += T(x, y);
    a.thsSmoothed[c] = (sum / num) * (sum / num);
  }
  if (t == 0) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
// select, pass 1: level-2 existence mask per slot and direction
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void hs_k_sel_mask(HsSelArgs a) {
  // 16 lanes per slot: lane `sub` takes the slot's rows y1 = sub, sub + 16, ...; the masks are OR-combined
  // (order-free, so the result is the sequential loop's)
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = t >> 4, sub = t & 15;
  const SlotGeo g = slot_geo(a, min(s, a.nslots - 1));
  uint32_t m = 0;
  if (s < a.nslots && g.valid) {
    // every load of a pixel is unconditional (clamped index) and the tests are selects, so the loads of
    // several pixels are in flight together instead of one dependent round trip per pixel
    const int last = a.W * a.H - 1;
    for (int y1 = sub; y1 < g.my1; y1 += 16) {
#pragma unroll 4
      for (int x1 = 0; x1 < g.mx1; x1++) {
        const int xf = g.x0 + x1, yf = g.y0 + y1;
        const int idx = min(xf + a.W * yf, last);
        const float ag0 = a.g0[idx];
        const float th = th0_of(a, xf, yf);
        const float dx = a.dI[a.dstride * idx + 1], dy = a.dI[a.dstride * idx + 2];
        const bool pass = !border_out(a, xf, yf) && (ag0 > th * a.thFactor);
        uint32_t mm;
        if (!a.dirDist) {
          mm = 0xFFFFu;  // dirNorm = ag0 > 0
        } else {
          mm = 0;
#pragma unroll
          for (int d = 0; d < 16; d++) mm |= (fabsf(dx * kDir[d][0] + dy * kDir[d][1]) > 0.f) ? (1u << d) : 0u;
        }
        m |= pass ? mm : 0u;
      }
    }
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) m |= (uint32_t)__shfl_xor((int)m, o);
  if (sub == 0 && s < a.nslots) a.mask[s] = (uint16_t)m;
}

// ------------------------------------------------------------------------------------------------
// select, pass 2: n2 before every slot (one workgroup of 1024, chunks of 4096 slots in traversal order)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void hs_k_sel_scan(HsSelArgs a) {
  constexpr int kChunk = 4096;
  __shared__ uint16_t s_mask[kChunk];
  __shared__ uint8_t s_fix[kChunk];
  __shared__ uint8_t s_pat[kChunk];
  __shared__ int s_amb[kChunk];
  __shared__ int s_texcl[1024];
  __shared__ int s_w[32];
  const int t = threadIdx.x;
  const int area = a.W * a.H;
  int carry = 0;
  for (int base = 0; base < a.nslots; base += kChunk) {
    uint32_t m[4];
    int f = 0, am = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int s = base + 4 * t + k;
      m[k] = s < a.nslots ? a.mask[s] : 0u;
      s_mask[4 * t + k] = (uint16_t)m[k];
      f += m[k] == 0xFFFFu;
      am += m[k] != 0u && m[k] != 0xFFFFu;
    }
    int total;
    const int excl = block_excl_scan<16>((am << 16) | f, s_w, &total);
    uint32_t fin = 0;  // final level-2 flags of this thread's 4 slots
#pragma unroll
    for (int k = 0; k < 4; k++) fin |= (uint32_t)(m[k] == 0xFFFFu) << k;
    if (total >> 16) {
      // ambiguous slots: list them in order, one lane resolves them with the running n2
      int pos = excl >> 16;
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (m[k] != 0u && m[k] != 0xFFFFu) s_amb[pos++] = 4 * t + k;
      s_texcl[t] = excl & 0xFFFF;
      for (int i = t; i < kChunk; i += 1024) s_pat[i] = carry + i < area ? a.pattern[carry + i] : 0;
      __syncthreads();
      if (t == 0) {
        const int namb = total >> 16;
        int delta = 0;
        for (int k = 0; k < namb; k++) {
          const int p = s_amb[k], th = p >> 2;
          int pre = s_texcl[th];
          for (int q = th * 4; q < p; q++) pre += s_mask[q] == 0xFFFFu;
          const int n2 = pre + delta;  // relative to carry (< kChunk)
          const int bit = (s_mask[p] >> (s_pat[n2] & 0xF)) & 1;
          s_fix[p] = (uint8_t)bit;
          delta += bit;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (m[k] != 0u && m[k] != 0xFFFFu && s_fix[4 * t + k]) fin |= 1u << k;
    }
    int tot2;
    int run = carry + block_excl_scan<16>(__builtin_popcount(fin), s_w, &tot2);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int s = base + 4 * t + k;
      if (s < a.nslots) {
        a.n2b[s] = run;
        a.has2[s] = (fin >> k) & 1;
      }
      run += (fin >> k) & 1;
    }
    carry += tot2;
  }
}

// ------------------------------------------------------------------------------------------------
// select, pass 3: per-level argmax with the resolved directions, map + counts
// ------------------------------------------------------------------------------------------------
// 4 lanes per slot, so a wave is one 4pot-block (16 slots): lane `sub` scans the slot's rows y1 = sub, sub + 4, ...
// in traversal order; the 4 per-lane argmaxes are combined by (value, first traversal position) — the strict '>'
// of the reference's row-major loop keeps the first maximum
__device__ __forceinline__ void argmax4(float& v, int& i, int pos) {
  uint64_t key = v > 0.f ? ((uint64_t)__float_as_uint(v) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)pos) : 0ull;
#pragma unroll
  for (int o = 1; o < 4; o <<= 1) {
    const uint64_t ky = __shfl_xor(key, o);
    const int iy = __shfl_xor(i, o);
    const bool take = ky > key;
    key = take ? ky : key;
    i = take ? iy : i;
  }
  v = key ? __uint_as_float((uint32_t)(key >> 32)) : 0.f;
  if (!key) i = -1;
}

__global__ __launch_bounds__(256) void hs_k_sel_pick(HsSelArgs a) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;  // nslots is a multiple of 16; a wave = one 4pot-block
  const int s = t >> 2, sub = t & 3;
  const SlotGeo g = slot_geo(a, min(s, a.nslots - 1));
  const int sc = min(s, a.nslots - 1);
  const int n2 = a.n2b[sc], n3 = a.n2b[sc & ~3], n4 = a.n2b[sc & ~15];
  const int d2 = a.pattern[n2] & 0xF, d3 = a.pattern[n3] & 0xF, d4 = a.pattern[n4] & 0xF;
  const float d2x = kDir[d2][0], d2y = kDir[d2][1], d3x = kDir[d3][0], d3y = kDir[d3][1];
  const float d4x = kDir[d4][0], d4y = kDir[d4][1];
  const bool valid = s < a.nslots && g.valid;
  const bool h2 = valid && a.has2[sc];
  float b2v = 0.f, b3v = 0.f, b4v = 0.f;
  int b2i = -1, b3i = -1, b4i = -1, b2p = 0, b3p = 0, b4p = 0;
  if (valid) {
    // unconditional (clamped) loads and select-form updates, in traversal order (strict '>': the first maximum)
    const int last = a.W * a.H - 1;
    for (int y1 = sub; y1 < g.my1; y1 += 4) {
#pragma unroll 4
      for (int x1 = 0; x1 < g.mx1; x1++) {
        const int xf = g.x0 + x1, yf = g.y0 + y1;
        const int pos = y1 * g.mx1 + x1;
        const bool in = !border_out(a, xf, yf);
        const int idx = min(xf + a.W * yf, last);
        const float pixelTH0 = th0_of(a, xf, yf);
        const float pixelTH1 = pixelTH0 * a.dw1;
        const float pixelTH2 = pixelTH1 * a.dw2;
        const float dx = a.dI[a.dstride * idx + 1], dy = a.dI[a.dstride * idx + 2];
        const float ag0 = a.g0[idx];
        const int i1 = min((int)(xf * 0.5f + 0.25f) + (int)(yf * 0.5f + 0.25f) * a.w1, a.w1 * (a.H >> 1) - 1);
        const int i2 = min((int)(xf * 0.25f + 0.125) + (int)(yf * 0.25f + 0.125) * a.w2, a.w2 * (a.H >> 2) - 1);
        const float ag1 = a.g1[i1];
        const float ag2 = a.g2[i2];
        {
          const float dn = a.dirDist ? fabsf(dx * d2x + dy * d2y) : ag0;
          const bool up = in && (ag0 > pixelTH0 * a.thFactor) && (dn > b2v);
          b2v = up ? dn : b2v;
          b2i = up ? idx : b2i;
          b2p = up ? pos : b2p;
        }
        {
          const float dn = a.dirDist ? fabsf(dx * d3x + dy * d3y) : ag1;
          const bool up = in && (ag1 > pixelTH1 * a.thFactor) && (dn > b3v);
          b3v = up ? dn : b3v;
          b3i = up ? idx : b3i;
          b3p = up ? pos : b3p;
        }
        {
          const float dn = a.dirDist ? fabsf(dx * d4x + dy * d4y) : ag2;
          const bool up = in && (ag2 > pixelTH2 * a.thFactor) && (dn > b4v);
          b4v = up ? dn : b4v;
          b4i = up ? idx : b4i;
          b4p = up ? pos : b4p;
        }
      }
    }
  }
  argmax4(b2v, b2i, b2p);
  argmax4(b3v, b3i, b3p);
  argmax4(b4v, b4i, b4p);
  const bool lead = sub == 0;
  // level 2: the slot's own argmax (h2 <=> b2v > 0, the same expression as hs_k_sel_mask)
  if (h2 && lead) a.map[b2i] = 1.f;
  // level 3 per 2pot-block: only when none of its 4 slots selected at level 2; max value, first slot on ties
  const uint64_t key = 0xFFFFFFFFull - (uint32_t)s;
  const uint64_t p3 = (valid && b3v > 0.f) ? ((uint64_t)__float_as_uint(b3v) << 32) | key : 0ull;
  uint64_t m3 = p3;
  int any2 = h2;
#pragma unroll
  for (int o = 4; o < 16; o <<= 1) {  // the 4 slots of the 2pot-block (4 lanes each)
    const uint64_t y = __shfl_xor(m3, o);
    m3 = y > m3 ? y : m3;
    any2 |= __shfl_xor(any2, o);
  }
  const bool sel3 = !any2 && p3 != 0ull && p3 == m3;
  if (sel3 && lead) a.map[b3i] = 2.f;
  // level 4 per 4pot-block: only when no slot selected at level 2 and no level-3 candidate appeared
  const uint64_t p4 = (valid && b4v > 0.f) ? ((uint64_t)__float_as_uint(b4v) << 32) | key : 0ull;
  uint64_t m4 = p4;
  int any23 = h2 || p3 != 0ull;
#pragma unroll
  for (int o = 4; o < 64; o <<= 1) {  // the 16 slots of the 4pot-block: the whole wave
    const uint64_t y = __shfl_xor(m4, o);
    m4 = y > m4 ? y : m4;
    any23 |= __shfl_xor(any23, o);
  }
  const bool sel4 = !any23 && p4 != 0ull && p4 == m4;
  if (sel4 && lead) a.map[b4i] = 4.f;
  const uint64_t c2 = __ballot(h2 && lead), c3 = __ballot(sel3 && lead), c4 = __ballot(sel4 && lead);
  if ((threadIdx.x & 63) == 0) {
    if (c2) atomicAdd(&a.counts[0], __popcll(c2));
    if (c3) atomicAdd(&a.counts[1], __popcll(c3));
    if (c4) atomicAdd(&a.counts[2], __popcll(c4));
  }
}

// ------------------------------------------------------------------------------------------------
// makeMaps' sub-sampling: rn = raster rank of the selected pixel; drop it when randomPattern[rn] > charTH
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void hs_k_sel_subcount(HsSelSubArgs a) {
  __shared__ int s_w[32];
  const int i0 = blockIdx.x * kSelSubTile + threadIdx.x * 8;
  int c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) c += (i0 + k < a.n) && a.map[i0 + k] != 0.f;
  int total;
  (void)block_excl_scan<4>(c, s_w, &total);
  if (threadIdx.x == 0) a.tile_cnt[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void hs_k_sel_subscan(HsSelSubArgs a) {
  __shared__ int s_w[32];
  int carry = 0;
  for (int base = 0; base < a.ntiles; base += 1024) {
    const int i = base + threadIdx.x;
    const int v = i < a.ntiles ? a.tile_cnt[i] : 0;
    int total;
    const int e = block_excl_scan<16>(v, s_w, &total);
    if (i < a.ntiles) a.tile_cnt[i] = carry + e;
    carry += total;
  }
}

__global__ __launch_bounds__(256) void hs_k_sel_subapply(HsSelSubArgs a) {
  __shared__ int s_w[32];
  const int i0 = blockIdx.x * kSelSubTile + threadIdx.x * 8;
  float v[8];
  int c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    v[k] = i0 + k < a.n ? a.map[i0 + k] : 0.f;
    c += v[k] != 0.f;
  }
  int total;
  int rn = a.tile_cnt[blockIdx.x] + block_excl_scan<4>(c, s_w, &total);
  int rem = 0;
#pragma unroll
  for (int k = 0; k < 8; k++)
    if (v[k] != 0.f) {
      if (a.pattern[rn] > a.charTH) {
        a.map[i0 + k] = 0.f;
        rem++;
      }
      rn++;
    }
  for (int o = 32; o > 0; o >>= 1) rem += __shfl_xor(rem, o);
  if ((threadIdx.x & 63) == 0 && rem) atomicAdd(a.removed, rem);
}
