// hs_act_kernels.hip — point activation (System::activatePointsMT, Src/Mapping.cpp:330-480) on CDNA4.
//
// hs_k_act_seed      makeDistanceMap (Src/CoarseTracker.cpp:726-756): one thread per active point, level-1
//                    projection into the newest keyframe, seed byte set to 0 with a word CAS (duplicates dropped).
// hs_k_act_cand      the per-point part of the selection loop (Mapping.cpp:378-426): delete / skip / the
//                    projected cell, the sub-pixel fraction and the threshold of every entry of the loop order.
// hs_k_act_select    one workgroup: growDistBFS of the seeds over the whole workgroup, then the greedy loop on
//                    wave 0 alone — per batch of 64 entries the first one (in loop order) whose distance passes
//                    is taken, addIntoDistFinal grows the map from it, the rest of the batch is re-tested.
//                    BFS steps are frontier-parallel; a cell joins the next frontier only through the CAS that
//                    lowered it, so the map after each step is the reference's (its per-step result does not
//                    depend on the order the frontier is walked in).
//                    The map lives in LDS as bytes (0..39, 255 = the reference's 1000) when it fits.
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

// Frontier entries are packed cells x | y << 16 (no division to find a cell's neighbours).
__device__ __forceinline__ int xy_index(int xy, int w1) { return (xy & 0xffff) + w1 * (xy >> 16); }

// One growDistBFS step's work for one frontier entry: probe the 4 / 8 neighbour words, CAS the bytes that are
// larger than k (the probe's word is the CAS's expected value), report which neighbours this lane lowered.
__device__ __forceinline__ unsigned expand_cell(uint8_t* map, int w1, int h1, int xy, bool valid, uint32_t k,
                                                bool diag, int nbxy[8]) {
  const int x = xy & 0xffff, y = xy >> 16;
  const bool live = valid & (x != 0) & (y != 0) & (x != w1 - 1) & (y != h1 - 1);
  const int idx = live ? x + w1 * y : w1 + 1;
  const int nbi[8] = {idx + 1, idx - 1, idx + w1, idx - w1, idx + 1 + w1, idx - 1 + w1, idx - 1 - w1, idx + 1 - w1};
  const int dxy[8] = {1, -1, 1 << 16, -(1 << 16), 1 + (1 << 16), -1 + (1 << 16), -1 - (1 << 16), 1 - (1 << 16)};
  const int cnt = diag ? 8 : 4;
  uint32_t word[8];
#pragma unroll
  for (int d = 0; d < 8; d++) {
    nbxy[d] = xy + dxy[d];
    word[d] = d < cnt ? *reinterpret_cast<const uint32_t*>(map + (nbi[d] & ~3)) : 0u;
  }
  // every wanted CAS is issued before any result is waited for; a CAS that lost to another lane's update of
  // the same word is retried
  unsigned want = 0;
  uint32_t prev[8];
#pragma unroll
  for (int d = 0; d < 8; d++) {
    const int sh = (nbi[d] & 3) * 8;
    const bool w = live & (d < cnt) & (((word[d] >> sh) & 0xffu) > k);
    want |= (unsigned)w << d;
    if (w)
      prev[d] = atomicCAS(reinterpret_cast<uint32_t*>(map + (nbi[d] & ~3)), word[d],
                          (word[d] & ~(0xffu << sh)) | (k << sh));
  }
  unsigned got = 0;
#pragma unroll
  for (int d = 0; d < 8; d++) {
    if (!((want >> d) & 1u)) continue;
    const int sh = (nbi[d] & 3) * 8;
    uint32_t old = word[d];
    uint32_t pv = prev[d];
    while (pv != old) {  // lost a race on this word: retry while the byte still needs lowering
      old = pv;
      if (((old >> sh) & 0xffu) <= k) break;
      pv = atomicCAS(reinterpret_cast<uint32_t*>(map + (nbi[d] & ~3)), old, (old & ~(0xffu << sh)) | (k << sh));
    }
    got |= (unsigned)(pv == old && ((old >> sh) & 0xffu) > k) << d;
  }
  return got;
}

// growDistBFS from the n cells in *in (Src/CoarseTracker.cpp:759-857), frontier-parallel over the workgroup
// (makeDistanceMap's multi-seed BFS; its frontiers can span the map).  s_n[0] holds the frontier size on entry.
__device__ __forceinline__ void bfs_grow_wg(uint8_t* map, int w1, int h1, int*& in, int*& out, int* s_n) {
  const int lane = threadIdx.x & 63;
  for (int k = 1; k < HS_ACT_BFS_STEPS; k++) {
    const int n = s_n[0];
    if (n == 0) break;  // the reference keeps looping over empty lists: nothing changes
    if (threadIdx.x == 0) s_n[1] = 0;
    __syncthreads();
    const bool diag = (k & 1) != 0;
    for (int e0 = threadIdx.x & ~63; e0 < n; e0 += blockDim.x) {  // wave-uniform trip count
      const int e = e0 + lane;
      const int xy = e < n ? in[e] : 0;
      int nbxy[8];
      const unsigned got = expand_cell(map, w1, h1, xy, e < n, (uint32_t)k, diag, nbxy);
#pragma unroll
      for (int d = 0; d < 8; d++) {
        const unsigned long long bm = __ballot((got >> d) & 1u);
        if (bm == 0) continue;
        int base = 0;
        if (lane == (int)__builtin_ctzll(bm)) base = atomicAdd(&s_n[1], (int)__popcll(bm));
        base = __shfl(base, (int)__builtin_ctzll(bm));
        if ((got >> d) & 1u)
          out[base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u))] =
              nbxy[d];
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_n[0] = s_n[1];
    int* t = in;
    in = out;
    out = t;
    __syncthreads();
  }
}

// addIntoDistFinal's growDistBFS from one cell, run by a single wave: the frontier of a one-seed BFS is at most
// the ring of its step (<= 8k cells), so one wave walks it with no workgroup barrier.  Lane = frontier entry
// (8 or 16 per pass) x neighbour direction, so a pass is one straight-line sequence: read entry, probe word, lower,
// append (ballot + mbcnt, no atomics).  The lists are LDS.  This form (the map in global memory) lowers by CAS;
// the LDS map uses bfs_grow_wave_claim below.
__device__ __forceinline__ void bfs_grow_wave(uint8_t* map, int w1, int h1, int* in, int* out, int n,
                                              long long* cnt) {
  const int lane = threadIdx.x & 63;
  // growDistBFS's neighbour order: +x, -x, +y, -y, then the diagonals (+1+w1, -1+w1, -1-w1, +1-w1)
  const int sub8 = lane & 7, sub4 = lane & 3;
  const int dx8 = (sub8 == 0 || sub8 == 4 || sub8 == 7) ? 1 : ((sub8 == 1 || sub8 == 5 || sub8 == 6) ? -1 : 0);
  const int dy8 = (sub8 == 2 || sub8 == 4 || sub8 == 5) ? 1 : ((sub8 == 3 || sub8 == 6 || sub8 == 7) ? -1 : 0);
  const int dx4 = sub4 == 0 ? 1 : (sub4 == 1 ? -1 : 0);
  const int dy4 = sub4 == 2 ? 1 : (sub4 == 3 ? -1 : 0);
  n = __builtin_amdgcn_readfirstlane(n);  // uniform: the pass loop is a scalar loop
  for (int k = 1; k < HS_ACT_BFS_STEPS && n > 0; k++) {
    // odd steps: 8 entries x 8 directions per pass; even steps: 16 entries x 4 directions
    const bool diag = (k & 1) != 0;
    const int slot = diag ? lane >> 3 : lane >> 2;
    const int per = diag ? 8 : 16;
    const int dx = diag ? dx8 : dx4, dy = diag ? dy8 : dy4;
    const int dxy = dx + dy * 65536;
    int m = 0;
    cnt[0]++;
    int xyn = in[min(slot, n - 1)];  // the entries of the next pass are read one pass ahead
    for (int e0 = 0; e0 < n; e0 += per) {
      cnt[1]++;
      const int e = e0 + slot;
      const bool valid = e < n;
      const int xy = xyn;
      xyn = in[min(e + per, n - 1)];
      const int x = xy & 0xffff, y = xy >> 16;
      const bool live = valid & (x != 0) & (y != 0) & (x != w1 - 1) & (y != h1 - 1);
      const int q = live ? (x + dx) + (y + dy) * w1 : 0;
      const int sh = (q & 3) * 8;
      uint32_t* wp = reinterpret_cast<uint32_t*>(map + (q & ~3));
      uint32_t old = *wp;
      bool want = live & (((old >> sh) & 0xffu) > (uint32_t)k);
      bool got = false;
      while (want) {
        const uint32_t pv = atomicCAS(wp, old, (old & ~(0xffu << sh)) | ((uint32_t)k << sh));
        got = pv == old;
        old = pv;
        want = !got & (((old >> sh) & 0xffu) > (uint32_t)k);
      }
      const unsigned long long bm = __ballot(got);
      if (got)
        out[m + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u))] =
            xy + dxy;
      m += (int)__popcll(bm);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    n = __builtin_amdgcn_readfirstlane(m < HS_ACT_WAVE_LIST ? m : HS_ACT_WAVE_LIST);
    int* t = in;
    in = out;
    out = t;
  }
}

// bfs_grow_wave for the LDS map with claim bits: every writer of step k stores the same byte k, so the lowering is a
// plain byte store (no compare-and-swap retries when lanes hit the same word) and the one lane that appends the
// cell to the next frontier is the one whose ds_or sets its claim bit; a cell's bit is cleared when its entry is
// expanded (the last frontier's at the end), so every bit is zero between calls.  The pass is branch-free: the
// lanes that do not lower / clear / append address a dummy word (claim[cwords]) or or / and a no-op mask.
__device__ __forceinline__ void bfs_grow_wave_claim(uint8_t* map, int w1, int h1, int* in, int* out, int n,
                                                    long long* cnt, uint32_t* claim, uint32_t* dummy) {
  const int lane = threadIdx.x & 63;
  const int sub8 = lane & 7, sub4 = lane & 3;
  const int dx8 = (sub8 == 0 || sub8 == 4 || sub8 == 7) ? 1 : ((sub8 == 1 || sub8 == 5 || sub8 == 6) ? -1 : 0);
  const int dy8 = (sub8 == 2 || sub8 == 4 || sub8 == 5) ? 1 : ((sub8 == 3 || sub8 == 6 || sub8 == 7) ? -1 : 0);
  const int dx4 = sub4 == 0 ? 1 : (sub4 == 1 ? -1 : 0);
  const int dy4 = sub4 == 2 ? 1 : (sub4 == 3 ? -1 : 0);
  uint8_t* dummy_byte = reinterpret_cast<uint8_t*>(dummy);
  int* dummy_int = reinterpret_cast<int*>(dummy);
  n = __builtin_amdgcn_readfirstlane(n);
  for (int k = 1; k < HS_ACT_BFS_STEPS && n > 0; k++) {
    const bool diag = (k & 1) != 0;
    const int slot = diag ? lane >> 3 : lane >> 2;
    const int per = diag ? 8 : 16;
    const int dx = diag ? dx8 : dx4, dy = diag ? dy8 : dy4;
    const int dxy = dx + dy * 65536;
    const int doff = dx + dy * w1;
    const bool lead = (diag ? sub8 : sub4) == 0;  // the lane that releases its entry's claim
    int m = 0;
    cnt[0]++;
    int xyn = in[min(slot, n - 1)];  // the entries of the next pass are read one pass ahead
    for (int e0 = 0; e0 < n; e0 += per) {
      cnt[1]++;
      const int e = e0 + slot;
      const bool valid = e < n;
      const int xy = xyn;
      xyn = in[min(e + per, n - 1)];
      const int x = xy & 0xffff, y = xy >> 16;
      const bool live = valid & (x != 0) & (y != 0) & (x != w1 - 1) & (y != h1 - 1);
      const int base = (int)__umul24((unsigned)y, (unsigned)w1) + x;
      const int q = live ? base + doff : 0;
      const uint32_t old = *reinterpret_cast<const uint32_t*>(map + (q & ~3));
      const bool want = live & (((old >> ((q & 3) * 8)) & 0xffu) > (uint32_t)k);
      atomicAnd(&claim[base >> 5], (valid & lead) ? ~(1u << (base & 31)) : ~0u);
      *(want ? map + q : dummy_byte) = (uint8_t)k;
      const uint32_t bit = want ? 1u << (q & 31) : 0u;
      const bool got = want & ((atomicOr(&claim[q >> 5], bit) & bit) == 0u);
      const unsigned long long bm = __ballot(got);
      *(got ? out + m + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u))
            : dummy_int) = xy + dxy;
      m += (int)__popcll(bm);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    n = __builtin_amdgcn_readfirstlane(m < HS_ACT_WAVE_LIST ? m : HS_ACT_WAVE_LIST);
    int* t = in;
    in = out;
    out = t;
  }
  // the last frontier is never expanded: release its claims
  for (int e = lane; e < n; e += 64) {
    const int xy = in[e];
    const int qe = (xy & 0xffff) + w1 * (xy >> 16);
    atomicAnd(&claim[qe >> 5], ~(1u << (qe & 31)));
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// seeds taken in one round of the greedy loop: at most kMaxSeeds (their BFS frontiers share the wave list:
// 6 x a step-39 ring of 312 cells < HS_ACT_WAVE_LIST), pairwise at Chebyshev distance >= kSeedSep (2 x 39 + 2)
constexpr int kMaxSeeds = 6;
constexpr int kSeedSep = 2 * (HS_ACT_BFS_STEPS - 1) + 2;

// makeDistanceMap's BFS (whole workgroup), then the selection loop (wave 0).  Inlined once per map location so
// the LDS instance compiles to ds_* instructions.
__device__ __forceinline__ int select_body(const HsActSelectArgs& a, uint8_t* map, int* s_n, int* wl0, int* wl1,
                                           uint32_t* claim = nullptr, uint32_t* dummy = nullptr) {
  int* in = a.list_a;
  int* out = a.list_b;
  bfs_grow_wg(map, a.w1, a.h1, in, out, s_n);
  if (threadIdx.x >= 64) return 0;  // the greedy loop is sequential: wave 0 alone
  if (a.prof && threadIdx.x == 0) {
    a.prof[1] = wall_clock64();
    a.prof[6] = clock64();
  }
  const int lane = threadIdx.x;
  int nt = 0;
  long long cnt[3] = {0, 0, 0};
  // candidate batches of 64, the next batch's loads in flight while the current one is processed: every load is
  // unconditional (clamped index) and nothing tests a loaded value before the next batch, so no wait sits at the
  // prefetch (a per-entry "pending ? load : 0" made the compiler branch around each load and drain the queue)
  int j = lane;
  unsigned int ncand = 0u;
  int ncell = 0, npt = 0;
  float nfrac = 0.f, nthr = 0.f;
  auto fetch = [&](int jj) {
    const int jc = max(0, min(jj, a.m - 1));
    ncand = a.cand[jc];
    ncell = a.cell[jc];
    npt = a.order ? a.order[jc] : jc;
    nfrac = a.frac[jc];
    nthr = a.thr[jc];
  };
  if (a.m > 0) fetch(j);
  for (int base = 0; base < a.m; base += 64) {
    bool pend = (base + lane < a.m) && ncand == HS_CAND_PENDING;
    const int cell = pend ? ncell : 0;
    const int cidx = xy_index(cell, a.w1);
    const float frac = nfrac, thr = nthr;
    const int pt = npt;
    j = base + 64 + lane;
    fetch(j);
    int myslot = -1;  // this lane's place in toopt when it is taken (stored once after the batch: no global store
                      // inside the round loop, whose completion a later wait would have to drain)
    for (;;) {
      // dist = fwdWarpedIDDistFinal[u + w1 * v] + (ptp[0] - floorf(ptp[0])) >= currentMinActDist * my_type
      const bool acc = pend && (decode(map[cidx]) + frac >= thr);
      const unsigned long long bm = __ballot(acc);
      if (bm == 0) break;  // every remaining entry of the batch fails: they stay immature
      const int first = (int)__builtin_ctzll(bm);
      // The first passing entry is taken, as in the reference.  Later passing entries of the batch are taken in
      // the same round while each is provably unaffected by the round's earlier seeds: at Chebyshev distance
      // >= kSeedSep from all of them (their addIntoDistFinal BFS regions, radius <= 39, are disjoint, so one
      // multi-seed BFS leaves the map the sequential BFS passes leave) and with cheb + frac >= thr (a BFS
      // distance is >= the Chebyshev distance, so its own test still passes after those seeds).  Entries that
      // fail now stay failing (the map only decreases); the first passing entry that is not provably
      // unaffected ends the round.
      unsigned long long take = 1ull << first;
      {
        int sc[kMaxSeeds];
        sc[0] = __shfl(cell, first);
        int ns = 1;
        unsigned long long rest = bm & ~((2ull << first) - 1ull);
        while (rest && ns < kMaxSeeds) {
          const int c = (int)__builtin_ctzll(rest);
          const int cc = __shfl(cell, c);
          const float cf = __shfl(frac, c), ct = __shfl(thr, c);
          bool ok = true;
          for (int q = 0; q < ns; q++) {
            const int ddx = abs((cc & 0xffff) - (sc[q] & 0xffff)), ddy = abs((cc >> 16) - (sc[q] >> 16));
            const int ch = ddx > ddy ? ddx : ddy;
            ok = ok && ch >= kSeedSep && ((float)ch + cf >= ct);
          }
          if (!ok) break;
          sc[ns++] = cc;
          take |= 1ull << c;
          rest &= rest - 1ull;
        }
      }
      if (lane <= first) pend = false;
      const bool mine = (take >> lane) & 1ull;
      if (mine) {
        pend = false;
        const int rank = (int)__popcll(take & ((1ull << lane) - 1ull));
        myslot = nt + rank;
        lower_cell(map, cidx, 0);  // addIntoDistFinal: the cell becomes 0 even when it already was
        wl0[rank] = cell;
      }
      const int ntake = (int)__popcll(take);
      nt += ntake;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const long long c0 = a.prof ? wall_clock64() : 0;
      if (claim) bfs_grow_wave_claim(map, a.w1, a.h1, wl0, wl1, ntake, cnt, claim, dummy);
      else bfs_grow_wave(map, a.w1, a.h1, wl0, wl1, ntake, cnt);
      if (a.prof) cnt[2] += wall_clock64() - c0;
    }
    // one unconditional store per batch (the lanes not taken write their scratch slot toopt[m + lane]), so the
    // compiler counts it and the next batch waits for its loads only
    a.toopt[myslot >= 0 ? myslot : a.m + lane] = pt;
  }
  if (a.prof && lane == 0) {
    a.prof[3] = cnt[0];
    a.prof[4] = cnt[1];
    a.prof[5] = cnt[2];
  }
  return nt;
}

__global__ void __launch_bounds__(1024) hs_k_act_select(HsActSelectArgs a) {
  extern __shared__ uint32_t s_map32[];
  __shared__ int s_n[2];
  __shared__ int s_wl[2][HS_ACT_WAVE_LIST];
  const int words = (a.w1 * a.h1 + 3) / 4;
  if (a.prof && threadIdx.x == 0) a.prof[0] = wall_clock64();
  if (threadIdx.x == 0) s_n[0] = *a.seed_count;
  int nt;
  if (a.lds_map) {
    const uint32_t* g = reinterpret_cast<const uint32_t*>(a.dist);
    for (int w = threadIdx.x; w < words; w += blockDim.x) s_map32[w] = g[w];
    uint32_t* claim = s_map32 + words;  // one bit per cell, zero between the BFS calls; then one dummy word
    const int cwords = (a.w1 * a.h1 + 31) / 32;
    for (int w = threadIdx.x; w <= cwords; w += blockDim.x) claim[w] = 0u;
    __syncthreads();
    nt = select_body(a, reinterpret_cast<uint8_t*>(s_map32), s_n, s_wl[0], s_wl[1], claim, claim + cwords);
    if (threadIdx.x >= 64) return;
    uint32_t* go = reinterpret_cast<uint32_t*>(a.dist);
    for (int w = threadIdx.x; w < words; w += 64) go[w] = s_map32[w];
  } else {
    __syncthreads();
    nt = select_body(a, a.dist, s_n, s_wl[0], s_wl[1]);
    if (threadIdx.x >= 64) return;
  }
  if (threadIdx.x == 0) *a.n_toopt = nt;
  if (a.prof && threadIdx.x == 0) {
    a.prof[2] = wall_clock64();
    a.prof[7] = clock64();
  }
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
