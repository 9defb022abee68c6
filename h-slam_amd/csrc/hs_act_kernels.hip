// hs_act_kernels.hip — point activation (System::activatePointsMT, Src/Mapping.cpp:330-480) on CDNA4.
//
// hs_k_act_seed      makeDistanceMap (Src/CoarseTracker.cpp:726-756): one thread per active point, level-1
//                    projection into the newest keyframe, seed byte set to 0 with a word CAS (duplicates dropped).
// hs_k_act_cand      the per-point part of the selection loop (Mapping.cpp:378-426): delete / skip / the
//                    projected cell, the sub-pixel fraction and the threshold of every entry of the loop order.
// hs_k_act_dist      mode 0: makeDistanceMap's growDistBFS over the seeds in closed form (bfs_dist), per cell.
// hs_k_act_select    one workgroup, the greedy loop: per batch of 64 entries wave 0 takes, in loop order,
//                    each entry whose distance passes and applies its addIntoDistFinal to the rest of the batch
//                    in closed form (bfs_dist); the workgroup then folds the batch's seeds into the map.
//                    The map lives in LDS as bytes (0..39, 255 = the reference's 1000) when it fits.
//                    mode 1: the exact distance map after the loop (+ every addIntoDistFinal), per cell.
// hs_k_act_optimize  optimizeImmaturePoint (Src/FullSystemOptPoint.cpp:24-175) with
//                    ImmaturePoint::linearizeResidual (Src/ImmaturePoint.cpp:389-451): one wave per point,
//                    lane = residual (target frame) x pattern pixel; energy, Hdd and bd are summed in the
//                    reference's sequential order from readlane, including the partial sums a mid-pattern OOB
//                    leaves behind.
#include <hip/hip_runtime.h>

#include "hs_trace_kernels.h"

#pragma clang fp contract(off)
#include "hs_interp.h"

namespace {

constexpr int kPat[8][2] = {{0, -2}, {-1, -1}, {1, -1}, {-2, 0}, {0, 0}, {2, 0}, {-1, 1}, {0, 2}};
constexpr uint8_t kIpsGood = 0, kIpsOob = 1, kIpsOutlier = 2, kIpsSkipped = 3, kIpsBadCondition = 4;
constexpr int kResIn = 0, kResOob = 1, kResOut = 2;

// Eigen `KRKi * Vec3f(x, y, 1) + Kt * s`
__device__ __forceinline__ void proj3(const float* K, const float* t, float x, float y, float s, float p[3]) {
#pragma unroll
  for (int i = 0; i < 3; i++) p[i] = (K[3 * i] * x + K[3 * i + 1] * y + K[3 * i + 2] * 1.0f) + t[i] * s;
}

// lower the distance byte of cell q to k when it is larger; true when this call lowered it
__device__ __forceinline__ bool lower_cell(uint8_t* map, int q, uint32_t k) {
  uint32_t* w = reinterpret_cast<uint32_t*>(map + (q & ~3));
  const int sh = (q & 3) * 8;
  uint32_t old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (((old >> sh) & 0xffu) > k) {
    const uint32_t nw = (old & ~(0xffu << sh)) | (k << sh);
    const uint32_t prev = atomicCAS(w, old, nw);
    if (prev == old) return true;
    old = prev;
  }
  return false;
}

__device__ __forceinline__ float decode(uint8_t b) { return b == 255 ? 1000.f : (float)b; }

}  // namespace

__global__ void __launch_bounds__(256) hs_k_act_seed(HsActSeedArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int f = a.frame[i];
  if (f == a.newest) return;
  const hs_act_frame& fr = a.frames[f];
  float ptp[3];
  proj3(fr.KRKi, fr.Kt, a.u[i], a.v[i], a.idepth[i], ptp);
  const int u = ptp[0] / ptp[2] + 0.5f;
  const int v = ptp[1] / ptp[2] + 0.5f;
  if (!(u > 0 && v > 0 && u < a.w1 && v < a.h1)) return;
  if (lower_cell(a.dist, u + a.w1 * v, 0)) a.list[atomicAdd(a.count, 1)] = u | (v << 16);
}

__global__ void __launch_bounds__(256) hs_k_act_cand(HsActCandArgs a) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.m) return;
  const int i = a.order ? a.order[j] : j;
  const int f = a.frame_of_slot[a.host[i]];
  uint8_t c = HS_CAND_SKIP;
  if (f >= 0 && f != a.newest) {
    const float idmax = a.idepth_max[i], idmin = a.idepth_min[i];
    const uint8_t st = a.status[i];
    if (!isfinite(idmax) || st == kIpsOutlier) {
      c = HS_CAND_DELETE;
    } else {
      const bool canActivate =
          (st == kIpsGood || st == kIpsSkipped || st == kIpsBadCondition || st == kIpsOob) && a.interval[i] < 8 &&
          a.quality[i] > a.minTraceQuality && (idmax + idmin) > 0;
      if (!canActivate) {
        c = (a.frames[f].flagged_for_marg || st == kIpsOob) ? HS_CAND_DELETE : HS_CAND_SKIP;
      } else {
        float ptp[3];
        proj3(a.frames[f].KRKi, a.frames[f].Kt, a.u[i], a.v[i], 0.5f * (idmax + idmin), ptp);
        const int u = ptp[0] / ptp[2] + 0.5f;
        const int v = ptp[1] / ptp[2] + 0.5f;
        if (u > 0 && v > 0 && u < a.w1 && v < a.h1) {
          c = HS_CAND_PENDING;
          a.cell[j] = u | (v << 16);
          a.frac[j] = ptp[0] - floorf((float)(ptp[0]));
          a.thr[j] = a.currentMinActDist * a.my_type[i];
        } else {
          c = HS_CAND_DELETE;
        }
      }
    }
  }
  a.cand[j] = c;
  a.action[i] = (c == HS_CAND_DELETE) ? HS_ACT_DELETED : HS_ACT_KEEP;
}

// addIntoDistFinal without a BFS.  growDistBFS from one seed takes 8-neighbour steps at odd k and 4-neighbour steps
// at even k, so an unobstructed cell at (dx, dy) is first reached at the smallest k with max(|dx|, |dy|) <= k and
// |dx| + |dy| <= k + ceil(k / 2): k = max(M, (2 L + 1) / 3).  With the map before the call being a union of such
// waves, the pruned BFS leaves every interior cell at min(map, k) (k <= 39), and a border cell (never expanded)
// at min(map, k_n + 1) over its interior neighbours n whose value the wave lowered (k_n < map(n), or n the seed),
// a diagonal move only on an odd step k_n + 1; a seed on the border only sets itself.  Checked against the
// reference's growDistBFS on random maps and seed sequences, every cell of every map
// (tests/test_act.py::test_closed_form_bfs_matches_grow_dist_bfs).
__device__ __forceinline__ int bfs_dist(int dx, int dy) {
  dx = abs(dx);
  dy = abs(dy);
  return max(max(dx, dy), (2 * (dx + dy) + 1) / 3);
}

// the interior neighbours of a border cell (x == w1 - 1 or y == h1 - 1; x, y > 0) as packed cells, -1 = none
__device__ __forceinline__ void border_nbrs(int x, int y, int w1, int h1, int nb[3]) {
  int cx[3], cy[3];
  if (x == w1 - 1) {
    cx[0] = cx[1] = cx[2] = x - 1;
    cy[0] = y - 1; cy[1] = y; cy[2] = y + 1;
  } else {
    cy[0] = cy[1] = cy[2] = y - 1;
    cx[0] = x - 1; cx[1] = x; cx[2] = x + 1;
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const bool in = cx[i] >= 1 && cx[i] <= w1 - 2 && cy[i] >= 1 && cy[i] <= h1 - 2;
    nb[i] = in ? (cx[i] | (cy[i] << 16)) : -1;
  }
}

// one addIntoDistFinal from seed s applied to a border cell (value v) with interior neighbour values nv, limit r
__device__ __forceinline__ void border_step(int x, int y, int s, int r, const int nb[3], int& v, int nv[3]) {
  const int sx = s & 0xffff, sy = s >> 16;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    if (nb[i] < 0) continue;
    const int nx = nb[i] & 0xffff, ny = nb[i] >> 16;
    const int dn = bfs_dist(nx - sx, ny - sy);
    const int t = dn + 1;
    const bool diag = (nx != x) & (ny != y);
    if ((dn < nv[i] || nb[i] == s) && t <= r && (!diag || (t & 1))) v = min(v, t);
    if (dn <= r) nv[i] = min(nv[i], dn);
  }
}

__device__ __forceinline__ uint32_t ld_word(const uint8_t* map, int w) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(map) + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_cell(const uint8_t* map, int q) {
  const uint32_t b = (ld_word(map, q >> 2) >> ((q & 3) * 8)) & 0xffu;
  return b == 255u ? 1000 : (int)b;
}

// workgroup barrier that orders LDS only: a global-memory operation in flight (wave 0's prefetch of the next batch,
// its toopt / seeds stores) is not waited for, as __syncthreads' release fence would
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// makeDistanceMap's map (hs_k_act_map0) in the working map, then the selection loop in batches of 64 entries: wave 0 takes, in loop
// order, every entry whose distance passes, updating the rest of the batch from each new seed in registers; then
// the whole workgroup folds the batch's seeds into the working map.  The working map only has to decide the test
// dist + frac >= thr (thr <= T = the largest threshold of the call): it is kept exact up to r = ceil(T) - 1 (seed
// patches of radius r; cells farther away keep a larger value, which passes every test anyway), and the exact
// map is formed afterwards by hs_k_act_dist (mode 1).
constexpr int kBorderWords = 128;  // border-candidate bitmap of select_body: maps with w1 + h1 <= 4096

__device__ __forceinline__ int select_body(const HsActSelectArgs& a, uint8_t* map, int* s_n, int* s_seeds,
                                           float* s_red, uint32_t* s_bcand, int* s_wc) {
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int w1 = a.w1, h1 = a.h1;
  float tmax = 0.f;
  bool tnan = false;
  for (int j = tid; j < a.m; j += nthr)
    if (a.cand[j] == HS_CAND_PENDING) {
      const float t = a.thr[j];
      tnan |= !(t == t);
      tmax = fmaxf(tmax, t);
    }
  for (int o = 32; o > 0; o >>= 1) {
    tmax = fmaxf(tmax, __shfl_xor(tmax, o));
    tnan |= __shfl_xor((int)tnan, o) != 0;
  }
  // the right column / bottom row cells some pending entry sits on (bit x: bottom row; bit w1 + y: right column);
  // the border pass of a batch only forms those
  const bool bfilter = w1 + h1 <= 32 * kBorderWords;
  for (int j = tid; j < a.m; j += nthr)
    if (bfilter && a.cand[j] == HS_CAND_PENDING) {
      const int c = a.cell[j], cx = c & 0xffff, cy = c >> 16;
      if (cy == h1 - 1) atomicOr(&s_bcand[cx >> 5], 1u << (cx & 31));
      if (cx == w1 - 1) atomicOr(&s_bcand[(w1 + cy) >> 5], 1u << ((w1 + cy) & 31));
    }
  if ((tid & 63) == 0) s_red[tid >> 6] = tnan ? 1e30f : tmax;
  __syncthreads();  // (also: the map is in place)
  float T = 0.f;
  for (int i = 0; i < nthr / 64; i++) T = fmaxf(T, s_red[i]);
  const int r = T >= 40.f ? HS_ACT_BFS_STEPS - 1 : max(0, (int)ceilf(T) - 1);
  if (a.prof && tid == 0) {
    a.prof[1] = wall_clock64();
    a.prof[6] = clock64();
  }
  const int lane = tid & 63;
  const bool w0 = tid < 64;
  // the pending entries (the only ones a batch can take; the others stay as they are) in loop order, compacted into
  // a.plist, so the batches run over them alone (ballot prefix sums per chunk of the workgroup)
  for (int c0 = 0; c0 < a.m; c0 += nthr) {
    const int j = c0 + tid;
    const bool p = j < a.m && a.cand[j] == HS_CAND_PENDING;
    const unsigned long long bm = __ballot(p);
    if (lane == 0) s_wc[tid >> 6] = __popcll(bm);
    __syncthreads();
    int off = s_n[2];
    for (int w = 0; w < (tid >> 6); w++) off += s_wc[w];
    if (p) a.plist[off + __popcll(bm & ((1ull << lane) - 1ull))] = j;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int w = 0; w < nthr / 64; w++) tot += s_wc[w];
      s_n[2] += tot;
    }
    __syncthreads();
  }
  const int np = s_n[2];
  int nt = 0;
  long long npatch = 0;
  // wave 0's candidate batches of 64, the next batch's loads in flight while the current one is processed
  unsigned int ncand = 0u;
  int ncell = 0, npt = 0;
  float nfrac = 0.f, nthr_ = 0.f;
  auto fetch = [&](int jj) {
    const int jc = a.plist[max(0, min(jj, np - 1))];
    ncand = a.cand[jc];
    ncell = a.cell[jc];
    npt = a.order ? a.order[jc] : jc;
    nfrac = a.frac[jc];
    nthr_ = a.thr[jc];
  };
  if (w0 && np > 0) fetch(lane);
  const int rows = 2 * r + 1, wpr = (2 * r + 1 + 3) / 4 + 1;
  int wb_shift = 0, rb_shift = 0;
  while ((1 << wb_shift) < wpr) wb_shift++;
  while ((1 << rb_shift) < rows) rb_shift++;
  const int ps_shift = wb_shift + rb_shift;
  long long t_dec = 0, t_fold = 0, t_p1 = 0;
  for (int base = 0; base < np; base += 64) {
    const long long c0 = a.prof ? wall_clock64() : 0;
    if (w0) {
      bool pend = (base + lane < np) && ncand == HS_CAND_PENDING;
      const int cell = pend ? ncell : (1 | (1 << 16));
      const float frac = nfrac, thr = nthr_;
      const int pt = npt;
      fetch(base + 64 + lane);
      const int x = cell & 0xffff, y = cell >> 16;
      const bool border = (x == w1 - 1) | (y == h1 - 1);
      int v = ld_cell(map, x + w1 * y);
      int nb[3], nv[3] = {1000, 1000, 1000};
      border_nbrs(x, y, w1, h1, nb);
      if (border) {
#pragma unroll
        for (int i = 0; i < 3; i++)
          if (nb[i] >= 0) nv[i] = ld_cell(map, (nb[i] & 0xffff) + w1 * (nb[i] >> 16));
      }
      int myslot = -1, ns = 0, myseed = 0;  // lane k: the batch's k-th seed
      int bxm = 0, bym = 0;  // the batch seeds' largest x / y (the border pass is skipped when no seed is near)
      for (;;) {
        // dist = fwdWarpedIDDistFinal[u + w1 * v] + (ptp[0] - floorf(ptp[0])) >= currentMinActDist * my_type
        const bool acc = pend && ((float)v + frac >= thr);
        const unsigned long long bm = __ballot(acc);
        if (bm == 0) break;  // every remaining entry of the batch fails: they stay immature
        const int first = (int)__builtin_ctzll(bm);
        const int sc = __builtin_amdgcn_readlane(cell, first);
        if (lane == first) myslot = nt;
        if (lane == ns) myseed = sc;
        ns++;
        nt++;
        bxm = max(bxm, sc & 0xffff);
        bym = max(bym, sc >> 16);
        if (lane <= first) pend = false;
        // addIntoDistFinal(sc) on the batch's later entries
        const int sx = sc & 0xffff, sy = sc >> 16;
        if ((sx == w1 - 1) | (sy == h1 - 1)) {  // a border seed only sets its own cell
          if (cell == sc) v = 0;
        } else if (!border) {
          const int d = bfs_dist(x - sx, y - sy);
          if (d <= HS_ACT_BFS_STEPS - 1) v = min(v, d);
        } else if (pend && max(abs(x - sx), abs(y - sy)) <= HS_ACT_BFS_STEPS) {
          // (a seed farther than limit + 1 reaches no neighbour: border_step would change nothing)
          border_step(x, y, sc, HS_ACT_BFS_STEPS - 1, nb, v, nv);
        }
      }
      // one unconditional store per batch (the lanes not taken write their scratch slot toopt[m + lane]); the
      // batch's seeds from LDS (no global store inside the loop: its completion would be waited for with the
      // next batch's prefetch)
      a.toopt[myslot >= 0 ? myslot : a.m + lane] = pt;
      if (lane < ns) {
        a.seeds[nt - ns + lane] = myseed;
        s_seeds[lane] = myseed;  // the fold's copy (read after the barrier)
      }
      if (lane == 0) {
        s_n[0] = ns;
        s_n[1] = (bxm + r + 1 >= w1 - 1) | (bym + r + 1 >= h1 - 1);
      }
    }
    lds_barrier();  // wave 0's prefetch loads and its toopt / seeds stores stay in flight across it
    const long long c1 = a.prof ? wall_clock64() : 0;
    const int ns = s_n[0];
    if (ns > 0) {
      npatch += ns;
      // the right column / bottom row cells near a seed (the only border cells an entry can sit on), seeds in order:
      // one item per (seed near the edge, cell within r + 1 of it along the edge); a cell near two seeds is formed
      // twice, the same value
      const int span = 2 * r + 3;
      for (int it = s_n[1] ? tid : 2 * ns * span; it < 2 * ns * span; it += nthr) {
        const int jj = it / (2 * span), rem = it - jj * 2 * span, side = rem >= span, o = rem - side * span;
        const int s0 = s_seeds[jj], s0x = s0 & 0xffff, s0y = s0 >> 16;
        int x, y;
        if (side == 0) {  // the right column
          if (s0x + r + 1 < w1 - 1) continue;
          x = w1 - 1;
          y = s0y - r - 1 + o;
        } else {  // the bottom row
          if (s0y + r + 1 < h1 - 1) continue;
          y = h1 - 1;
          x = s0x - r - 1 + o;
        }
        if (x < 1 || y < 1 || x > w1 - 1 || y > h1 - 1) continue;
        if (bfilter) {  // no entry sits on this cell: its value decides nothing
          const int bi = side == 0 ? w1 + y : x;
          if (!((s_bcand[bi >> 5] >> (bi & 31)) & 1u)) continue;
        }
        int nb[3], nv[3] = {1000, 1000, 1000};
        border_nbrs(x, y, w1, h1, nb);
        for (int k = 0; k < 3; k++)
          if (nb[k] >= 0) nv[k] = ld_cell(map, (nb[k] & 0xffff) + w1 * (nb[k] >> 16));
        const int q = x + w1 * y;
        const int v0 = ld_cell(map, q);
        int v = v0;
        for (int j = 0; j < ns; j++) {
          const int sc = s_seeds[j];
          if (((sc & 0xffff) == w1 - 1) | ((sc >> 16) == h1 - 1)) {
            if (sc == (x | (y << 16))) v = 0;
          } else if (max(abs(x - (sc & 0xffff)), abs(y - (sc >> 16))) <= r + 1) {  // else: no neighbour reached
            border_step(x, y, sc, r, nb, v, nv);
          }
        }
        if (v < v0) {  // the interior pass below runs after the barrier; two items of one cell store the same byte
          uint32_t* wp = reinterpret_cast<uint32_t*>(map) + (q >> 2);
          const int sh = (q & 3) * 8;
          uint32_t old = ld_word(map, q >> 2);
          for (;;) {
            const uint32_t nw = (old & ~(0xffu << sh)) | ((uint32_t)v << sh);
            const uint32_t pv = atomicCAS(wp, old, nw);
            if (pv == old) break;
            old = pv;
          }
        }
      }
      lds_barrier();
      if (a.prof) t_p1 += wall_clock64() - c1;
      // interior cells: min(map, k) over each seed's patch of radius r, one 4-cell word per (seed, row, word) item
      // (items laid out in powers of two: shifts, no divisions)
      for (int it = tid; it < (ns << ps_shift); it += nthr) {
        const int j = it >> ps_shift, rem = it & ((1 << ps_shift) - 1);
        const int row = rem >> wb_shift, wi = rem & ((1 << wb_shift) - 1);
        if (row >= rows || wi >= wpr) continue;
        const int sc = s_seeds[j], sx = sc & 0xffff, sy = sc >> 16;
        if ((sx == w1 - 1) | (sy == h1 - 1)) continue;
        const int y = sy - r + row;
        const int x0 = max(1, sx - r), x1 = min(w1 - 2, sx + r);
        if (y < 1 || y > h1 - 2 || x0 > x1) continue;
        const int rb = y * w1;
        const int w = ((rb + x0) >> 2) + wi;
        if (w > ((rb + x1) >> 2)) continue;
        uint32_t* wp = reinterpret_cast<uint32_t*>(map) + w;
        uint32_t old = ld_word(map, w);
        for (;;) {
          uint32_t nw = old;
#pragma unroll
          for (int b = 0; b < 4; b++) {
            const int xx = w * 4 + b - rb;
            if (xx < x0 || xx > x1) continue;
            const int d = bfs_dist(xx - sx, y - sy);
            const uint32_t cur = (nw >> (8 * b)) & 0xffu;
            if (d <= r && (uint32_t)d < cur) nw = (nw & ~(0xffu << (8 * b))) | ((uint32_t)d << (8 * b));
          }
          if (nw == old) break;
          const uint32_t pv = atomicCAS(wp, old, nw);
          if (pv == old) break;
          old = pv;
        }
      }
    }
    lds_barrier();
    if (a.prof) {
      t_dec += c1 - c0;
      t_fold += wall_clock64() - c1;
    }
  }
  if (a.prof && tid == 0) {
    a.prof[3] = (np + 63) / 64;
    a.prof[4] = npatch;
    a.prof[5] = r;
    a.prof[8] = t_dec;
    a.prof[9] = t_fold;
    a.prof[10] = t_p1;
  }
  return nt;
}

__global__ void __launch_bounds__(1024) hs_k_act_select(HsActSelectArgs a) {
  extern __shared__ uint32_t s_map32[];
  __shared__ int s_n[3];  // batch seeds, near-border flag, pending entries
  __shared__ int s_seeds[64];
  __shared__ float s_red[16];
  __shared__ int s_wc[16];
  __shared__ uint32_t s_bcand[kBorderWords];
  for (int w = threadIdx.x; w < kBorderWords; w += blockDim.x) s_bcand[w] = 0u;
  if (threadIdx.x == 0) s_n[2] = 0;
  __syncthreads();
  const int words = (a.w1 * a.h1 + 3) / 4;
  if (a.prof && threadIdx.x == 0) a.prof[0] = wall_clock64();
  const uint32_t* g = reinterpret_cast<const uint32_t*>(a.map0);
  // one inlined instance per map location, so the LDS one compiles to ds_* instructions (a pointer that may be
  // either would make every map access a flat one); select_body's first barrier orders the copies before any use
  int nt;
  if (a.lds_map) {
    for (int w = threadIdx.x; w < words; w += blockDim.x) s_map32[w] = g[w];
    nt = select_body(a, reinterpret_cast<uint8_t*>(s_map32), s_n, s_seeds, s_red, s_bcand, s_wc);
  } else {
    uint32_t* m32 = reinterpret_cast<uint32_t*>(a.dist);
    for (int w = threadIdx.x; w < words; w += blockDim.x) m32[w] = g[w];
    nt = select_body(a, a.dist, s_n, s_seeds, s_red, s_bcand, s_wc);
  }
  if (threadIdx.x == 0) *a.n_toopt = nt;
  if (a.prof && threadIdx.x == 0) {
    a.prof[2] = wall_clock64();
    a.prof[7] = clock64();
  }
}

// Distance maps from seeds in closed form.  Mode 0, makeDistanceMap (Src/CoarseTracker.cpp:726-756): growDistBFS
// from every seed at once is, per interior cell, the minimum of the seeds' single-seed distances (bfs_dist, <= 39);
// a border cell (never expanded) takes k_n + 1 from its interior neighbours n (a diagonal move only on an odd
// step); a seed on the border only sets itself.  Mode 1, the map the greedy loop leaves: makeDistanceMap's map and
// every addIntoDistFinal in call order -- interior cells the same minimum, border cells the sequential rule of
// border_step (their neighbours' values before each seed).  Both checked against growDistBFS (tests/test_act.py).
// Blocks [0, n_tiles): one 16 x 16 tile of interior cells; blocks after: 4 waves of border cells each, every wave
// within one row or column.  Each wave takes only the seeds within reach of its cells (Chebyshev 39, 40 for border
// cells): per chunk of 1024 seeds it compacts them, in seed order, into its own LDS list and reads them four at a
// time as uniform values.
__global__ void __launch_bounds__(256) hs_k_act_dist(HsActDistArgs a) {
  __shared__ int4 wtile[4][256];  // per wave: the seeds of the current chunk within reach of its cells, in order
  constexpr int R = HS_ACT_BFS_STEPS - 1;
  const int w1 = a.w1, h1 = a.h1, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const bool itile = (int)blockIdx.x < a.n_tiles;
  if (((a.dbg & 1) && !itile) || ((a.dbg & 2) && itile)) return;
  int x, y;
  bool live;
  if (itile) {  // 16 x 16 interior cells; wave wv: rows 4 wv .. 4 wv + 3
    const int tx = blockIdx.x % a.n_tiles_x, ty = blockIdx.x / a.n_tiles_x;
    x = 1 + 16 * tx + (tid & 15);
    y = 1 + 16 * ty + (tid >> 4);
    live = x <= w1 - 2 && y <= h1 - 2;
  } else {  // border cells: each segment (top row, bottom row, left column, right column) padded to whole waves,
            // so a wave's cells are at most 64 consecutive cells of one row or column
    const int gw = ((int)blockIdx.x - a.n_tiles) * 4 + wv;  // global border wave
    const int sw0 = (w1 + 63) / 64, sw1 = (h1 - 2 + 63) / 64;
    int seg, off;
    if (gw < sw0) { seg = 0; off = gw * 64; }
    else if (gw < 2 * sw0) { seg = 1; off = (gw - sw0) * 64; }
    else if (gw < 2 * sw0 + sw1) { seg = 2; off = (gw - 2 * sw0) * 64; }
    else { seg = 3; off = (gw - 2 * sw0 - sw1) * 64; }
    const int k = off + lane;
    if (seg < 2) { x = k; y = seg == 0 ? 0 : h1 - 1; live = k < w1 && gw < 2 * sw0 + 2 * sw1; }
    else { x = seg == 2 ? 0 : w1 - 1; y = 1 + k; live = k < h1 - 2 && gw < 2 * sw0 + 2 * sw1; }
  }
  // the wave's bounding box (uniform)
  int bx0 = live ? x : 1 << 20, bx1 = live ? x : -(1 << 20), by0 = live ? y : 1 << 20, by1 = live ? y : -(1 << 20);
  for (int o = 32; o > 0; o >>= 1) {
    bx0 = min(bx0, __shfl_xor(bx0, o));
    bx1 = max(bx1, __shfl_xor(bx1, o));
    by0 = min(by0, __shfl_xor(by0, o));
    by1 = max(by1, __shfl_xor(by1, o));
  }
  if (__builtin_amdgcn_readfirstlane(bx1) < 0) return;  // no live cell in this wave
  const int q = live ? x + w1 * y : 0;
  auto val = [&](int c) { const uint8_t b = a.init[c]; return b == 255 ? 1000 : (int)b; };
  int v = live ? val(q) : 1000;
  const int self = x | (y << 16);
  int nb[3] = {-1, -1, -1}, nv[3] = {1000, 1000, 1000};
  if (!itile && live) {
    int kk = 0;
    for (int dy = -1; dy <= 1; dy++)
      for (int dx = -1; dx <= 1; dx++) {
        const int nx = x + dx, ny = y + dy;
        if ((dx | dy) == 0 || nx < 1 || nx > w1 - 2 || ny < 1 || ny > h1 - 2 || kk >= 3) continue;
        nb[kk] = nx | (ny << 16);
        nv[kk] = a.mode ? val(nx + w1 * ny) : 1000;  // mode 1: the neighbours' values before the first seed
        kk++;
      }
  }
  const int reach = itile ? R : R + 1;
  const int rx0 = bx0 - reach, rx1 = bx1 + reach, ry0 = by0 - reach, ry1 = by1 + reach;
  const int ns = (a.dbg & 4) ? 0 : *a.n_seeds;
  int* wt = reinterpret_cast<int*>(wtile[wv]);
  for (int t0 = 0; t0 < ns; t0 += 1024) {
    const int tn = min(1024, ns - t0);
    // this wave's seeds of the chunk within reach, compacted in seed order (16 per lane, a wave prefix sum); the
    // list is the wave's own LDS, whose operations complete in order: no barrier
    unsigned int msk = 0u;
    int sv[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int i = j * 64 + lane;  // coalesced
      sv[j] = i < tn ? a.seeds[t0 + i] : 0;
      const int sx = sv[j] & 0xffff, sy = sv[j] >> 16;
      const bool r = i < tn && sx >= rx0 && sx <= rx1 && sy >= ry0 && sy <= ry1;
      msk |= (unsigned int)r << j;
    }
    // seed order is i = j 64 + lane: compact chunk by chunk of 64 (j), each by a ballot prefix
    int base = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const bool r = (msk >> j) & 1u;
      const unsigned long long bm = __ballot(r);
      if (r) wt[base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u))] = sv[j];
      base += (int)__popcll(bm);
    }
    // pad to a multiple of 4 with a seed out of reach of every cell
    if (lane < ((4 - (base & 3)) & 3)) wt[base + lane] = 0x7000 | (0x7000 << 16);
    const int n4 = (base + 3) >> 2;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int i4 = 0; i4 < n4; i4++) {
      const int4 s4 = wtile[wv][i4];
      const int sc4[4] = {__builtin_amdgcn_readfirstlane(s4.x), __builtin_amdgcn_readfirstlane(s4.y),
                          __builtin_amdgcn_readfirstlane(s4.z), __builtin_amdgcn_readfirstlane(s4.w)};
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int sc = sc4[u];
        const int sx = sc & 0xffff, sy = sc >> 16;
        if ((sx == w1 - 1) | (sy == h1 - 1)) {  // a border seed only sets itself (mode 0: already 0 in init)
          if (sc == self) v = 0;
          continue;
        }
        if (itile) {
          const int d = bfs_dist(x - sx, y - sy);
          v = min(v, d <= R ? d : 1000);
        } else if (a.mode) {
          if (sc == self) v = 0;
          border_step(x, y, sc, R, nb, v, nv);
        } else {
#pragma unroll
          for (int k = 0; k < 3; k++) {
            const int d = bfs_dist((nb[k] & 0xffff) - sx, (nb[k] >> 16) - sy);
            if (d <= R) nv[k] = min(nv[k], d);
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (!live) return;
  if (!itile && !a.mode) {  // makeDistanceMap: every reached interior neighbour was expanded
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (nb[k] < 0 || nv[k] >= 1000) continue;
      const int t = nv[k] + 1;
      const bool diag = ((nb[k] & 0xffff) != x) & ((nb[k] >> 16) != y);
      if (t <= R && (!diag || (t & 1))) v = min(v, t);
    }
  }
  a.out[q] = v >= 255 ? 255 : (uint8_t)v;
}

__global__ void __launch_bounds__(256) hs_k_act_optimize(HsActOptArgs a) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= a.n) return;  // wave-uniform
  const int p = a.toopt[wave];
  const int hostF = a.frame_of_slot[a.host[p]];
  const int nres = a.nF - 1;
  const int r = lane >> 3, idx = lane & 7;
  const bool live = r < nres;
  const int tf = r < hostF ? r : r + 1;  // the r-th window frame other than the host
  const int tfc = live ? tf : 0;
  const hs_act_pair& pc = a.pairs[hostF * a.nF + tfc];
  const float4* img = a.img[a.frames[tfc].slot];
  const float pu = a.u[p], pv = a.v[p];
  const float color = a.color[8 * p + idx], wgt = a.weights[8 * p + idx];
  const float energyTH = a.energyTH[p];
  float R[9], t[3], aff0, aff1;
#pragma unroll
  for (int k = 0; k < 9; k++) R[k] = pc.RTll[k];
#pragma unroll
  for (int k = 0; k < 3; k++) t[k] = pc.tTll[k];
  aff0 = pc.aff[0];
  aff1 = pc.aff[1];
  const float KliP0 = (pu + kPat[idx][0] - a.cxl) * a.fxli;
  const float KliP1 = (pv + kPat[idx][1] - a.cyl) * a.fyli;

  // ImmaturePointTemporaryResidual of this lane's residual (replicated over its 8 lanes)
  int st_state = kResIn, st_new = kResOut;
  float st_energy = 0.f, st_newE = 0.f;

  // one pass of linearizeResidual over all residuals at idepth; returns the summed energy (float +=)
  auto evaluate = [&](float idepth, float slack, float& Hdd, float& bd) -> float {
    float ptp[3];
#pragma unroll
    for (int i = 0; i < 3; i++) ptp[i] = (R[3 * i] * KliP0 + R[3 * i + 1] * KliP1 + R[3 * i + 2] * 1.0f) + t[i] * idepth;
    const float drescale = 1.0f / ptp[2];
    const float u = ptp[0] * drescale, v = ptp[1] * drescale;
    const float Ku = u * a.fxl + a.cxl, Kv = v * a.fyl + a.cyl;
    bool ok = (drescale > 0) & (Ku > 1.1f) & (Kv > 1.1f) & (Ku < (float)(a.W - 3)) & (Kv < (float)(a.H - 3));
    const float Kuc = ok ? Ku : 2.f, Kvc = ok ? Kv : 2.f;
    const float3 hit = hs_img::interp33(img, Kuc, Kvc, a.W, a.H);
    ok = ok & isfinite(hit.x);
    const float residual = hit.x - (aff0 * color + aff1);
    float hw = fabsf(residual) < a.huberTH ? 1 : a.huberTH / fabsf(residual);
    const float eterm = wgt * wgt * hw * residual * residual * (2 - hw);
    const float dxInterp = hit.y * a.fxl;
    const float dyInterp = hit.z * a.fyl;
    const float d_idepth = (dxInterp * drescale * (t[0] - t[2] * u) + dyInterp * drescale * (t[1] - t[2] * v)) * 1.0f;
    hw *= wgt * wgt;
    const float hterm = (hw * d_idepth) * d_idepth;
    const float bterm = (hw * residual) * d_idepth;
    const unsigned long long bad = __ballot(live && !ok);
    float E = 0.f;
    for (int rr = 0; rr < nres; rr++) {
      const int l0 = rr * 8;
      const int sst = __builtin_amdgcn_readlane(st_state, l0);
      const float sE = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(st_energy), l0));
      float contrib;
      int ns;
      float nE = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(st_newE), l0));
      if (sst == kResOob) {
        ns = kResOob;
        contrib = sE;
      } else {
        const unsigned badr = (unsigned)(bad >> l0) & 0xffu;
        const int nvalid = badr ? __builtin_ctz(badr) : 8;
        for (int q = 0; q < nvalid; q++) {
          Hdd += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hterm), l0 + q));
          bd += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bterm), l0 + q));
        }
        if (badr) {
          ns = kResOob;
          contrib = sE;
        } else {
          float el = 0.f;
          for (int q = 0; q < 8; q++) el += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eterm), l0 + q));
          const float cap = energyTH * slack;
          if (el > cap) {
            el = cap;
            ns = kResOut;
          } else {
            ns = kResIn;
          }
          nE = el;
          contrib = el;
        }
      }
      if (r == rr) {
        st_new = ns;
        st_newE = nE;
      }
      E = (float)((double)E + (double)contrib);
    }
    return E;
  };
  auto take = [&]() {
    st_state = st_new;
    st_energy = st_newE;
  };

  float lastHdd = 0.f, lastbd = 0.f;
  float currentIdepth = (a.idepth_max[p] + a.idepth_min[p]) * 0.5f;
  float lastEnergy = evaluate(currentIdepth, 1000.f, lastHdd, lastbd);
  take();
  bool good = isfinite(lastEnergy) && !(lastHdd < a.minIdepthH_act);
  if (good) {
    float lambda = 0.1f;
    for (int it = 0; it < a.GNIts; it++) {
      float H = lastHdd;
      H *= 1 + lambda;
      const float step = (float)((1.0 / (double)H) * (double)lastbd);
      const float newIdepth = currentIdepth - step;
      float newHdd = 0.f, newbd = 0.f;
      const float newEnergy = evaluate(newIdepth, 1.f, newHdd, newbd);
      if (!isfinite(lastEnergy) || newHdd < a.minIdepthH_act) {
        good = false;
        break;
      }
      if (newEnergy < lastEnergy) {
        currentIdepth = newIdepth;
        lastHdd = newHdd;
        lastbd = newbd;
        lastEnergy = newEnergy;
        take();
        lambda = (float)((double)lambda * 0.5);
      } else {
        lambda = (float)((double)lambda * 5.0);
      }
      if ((double)fabsf(step) < 0.0001 * (double)currentIdepth) break;
    }
  }
  good = good && isfinite(currentIdepth);
  const unsigned long long inb = __ballot(live && idx == 0 && st_state == kResIn);
  unsigned mask = 0;
  for (int rr = 0; rr < nres; rr++)
    if ((inb >> (rr * 8)) & 1ull) mask |= 1u << (rr < hostF ? rr : rr + 1);
  good = good && mask != 0 && isfinite(energyTH);
  if (lane == 0) {
    a.action[p] = good ? HS_ACT_ACTIVATED : HS_ACT_DELETED;
    a.idepth_out[p] = currentIdepth;
    a.res_in[p] = good ? (uint8_t)mask : 0;
  }
}
