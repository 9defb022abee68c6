// hs_lin8_kernels.hip — the production linearize + accumulate kernel of the BA hot path (gfx950).
//
// Same work and outputs as hs_k_lin (hs_ba_kernels.hip) for the production partitioning of the GN loop:
//   resubstituteFPt + point step of the previous solve (Src/EnergyFunctional.cpp:249-274),
//   PointFrameResidual::linearize + applyRes / takeData (Src/OptimizationClasses.cpp:43-256),
//   the per-point Schur prelude of AccumulatedSCHessianSSE::addPoint (Src/AccumulatedSCHessian.cpp:10-33),
//   and the AccumulatorApprox / accD / accE / accEB / accHcc / accbc updates
//   (Src/AccumulatedTopHessian.cpp:21-141, Src/AccumulatedSCHessian.cpp:32-51, Include/MatrixAccumulators.h)
//   into block partials in hs_k_lin's production layout (hs_kernels.h, HS_E_TOP), which hs_k_reduce / hs_k_stitch
//   consume unchanged.
// Lane layout: lane = (point pl, target slot t); a wave takes 8 consecutive points at a time and every lane loops
// over the 8 pattern pixels of its residual.  So the per-residual work (centre projection, Jacobians, state
// decision, takeData) and the per-point work (fused step, residual-list sums, Schur prelude) are done once per
// lane instead of once per pixel lane, and the pattern-order sums are plain in-lane running sums: one wave
// instruction now serves 8 points where hs_k_lin's serves one.  Per-residual arithmetic keeps the reference's
// operation order (fp contraction off): states, energies, JpJdF, centre projections, HdiF / bdSumF / Hcd and the
// point steps are bit-identical to hs_k_lin's (and the oracle's).  The accumulators are production sums (fp32 per
// lane, the block partial in fixed wave / lane order, FMA-contracted), checked against the reference's order by
// tolerance like hs_k_lin's production partitioning.  Not used for the marginalization pass, linearizeAll(true)'s
// bookkeeping or HS_ACC_EXACT (hs_k_lin serves those).
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "hs_kernels.h"

namespace {

typedef float l8f2 __attribute__((ext_vector_type(2)));  // a packed-fp32 pair (v_pk_fma_f32)
// accD's 28 (o1 <= o2) entries as 9 register pairs (o2, o2 + 1) with o2 even -- so the operand pair is an aligned
// half of the loaded JpJdF quads -- and 10 singles; kind 0: pair p (.x / .y by o2 parity), kind 1: single
struct DSlot {
  int kind, idx;
};
__host__ __device__ constexpr DSlot d_slot(int o1, int o2) {
  int np = 0, ns = 0;
  for (int a = 0; a < 7; a++)
    for (int b = a; b < 7; b++) {
      const bool paired = (b & 1) == 0 ? b + 1 < 7 : b - 1 >= a;  // (b, b + 1) or (b - 1, b) inside row a
      if (a == o1 && b == o2) return paired ? DSlot{0, np} : DSlot{1, ns};
      if (paired) np += (b & 1);  // a pair is counted at its odd member
      else ns++;
    }
  return DSlot{-1, -1};
}
constexpr float SCALE_F8 = 50.0f, SCALE_C8 = 50.0f, SCALE_IDEPTH8 = 1.0f;
constexpr int L8_NW = HS_LIN8_NT / 64;  // waves per block
constexpr int NTOP = 91;  // AccumulatorApprox entries of one (host, target) block: Data 55 | TopRight 30 | BotRight 6
constexpr int Q8_N = 17;  // per-pixel quantities summed over the pattern
#ifndef L8_TAP_GROUP
#define L8_TAP_GROUP 8  // pixels whose taps may be in flight together (8: no scheduling barrier)
#endif
// Production: occupancy 2 (two waves per SIMD hide each other's tap latency), which the accumulators in LDS and no
// cross-group prefetch make fit in 256 registers without spills (244).  Measured (r03_b1): 2M points 1929 -> 1512 us
// per launch (HBM frac 0.39 -> 0.50), 200k 243 -> 200 us, per-residual outputs bit-identical.
#ifndef L8_MIN_WAVES
#define L8_MIN_WAVES 2  // waves per SIMD the register budget must allow (launch bounds)
#endif
#ifndef L8_PREFETCH
#define L8_PREFETCH 0   // 1: the next point group's inputs are loaded while the current group computes (occupancy 1)
#endif
#ifndef L8_FAST_OPS
#define L8_FAST_OPS 7   // div_nr / sqrt_nr for: 1 the projection quotients, 2 the gradient weight, 4 the Huber weight
#endif
// Issue priority.  The two waves sharing a SIMD are VALU-bound together; with equal priority the arbiter's
// oldest-first rule runs the older one ahead and leaves the younger alone on the SIMD at the end.  4 (production):
// the pair takes turns, priority 1 on alternate groups.  Measured (r05_l6 / r05_l8, per launch, HBM roofline
// fraction): 2M points 0.516 (4-wave blocks, no priority) -> 0.560 (8-wave blocks + turns); 200k 0.387 -> 0.378 ..
// 0.388 (VALU-bound either way: the turns equalise the waves' end times, not the SIMD's work).
// 0: none; 1: alternate per group (all waves in phase); 2: a wave ahead of the block's slowest yields.
#ifndef L8_PRIO
#define L8_PRIO 4
#endif
#ifndef L8_BOUNDS_BITS
#define L8_BOUNDS_BITS 1  // the pixel bounds test on float bits (one unsigned range compare per coordinate)
#endif
#ifndef L8_TEXEL_BYTES
#define L8_TEXEL_BYTES 12  // the taps' texel stride: 12 = the packed (I, dx, dy) copy, 16 = the float4 texels
#endif
#ifndef L8_BUFFER_TAPS
#define L8_BUFFER_TAPS 1  // the pixel taps as buffer loads with 32-bit offsets (interp33_8b)
#endif
#ifndef L8_LDS_ACC
#define L8_LDS_ACC 1    // the per-lane accumulators (T slice, accD / accE / accEB / accHcc) live in LDS between groups
#endif
#ifndef L8_PK_SC
// the Schur accumulators' accD / accE updates as packed-fp32 pairs (v_pk_fma_f32) on operand pairs that are aligned
// halves of the loaded JpJdF quads (no moves to form them); the same fmas, bit for bit.  Measured (per launch,
// profiles/r06_mfma/valu_mfma_pk_ab.txt): 200k 151 -> 144 us, 2M 1324 -> 1254 us, 25k 38.2 -> 37.0 us.  (As one
// product on v_mfma_f32_16x16x4_f32 they measured 137 / 1167 / 36.9 us; the path's specification keeps these small
// accumulations off the matrix cores, so that form is kept out: tools/archive/r06_lin8_mfma_schur.diff)
#define L8_PK_SC 1
#endif

// Data (r, c), r <= c < 10, in the natural per-lane layout
__host__ __device__ constexpr int didx(int r, int c) { return r * 10 - (r * (r - 1)) / 2 + (c - r); }
constexpr int TR0 = 55, BR0 = 85;

// getInterpolatedElement33 (Include/GlobalTypes.h:377-388) on float4 texels, through one buffer resource over every
// frame's image: 32-bit texel offsets (one 24-bit multiply-add and one shift-add per pixel instead of 64-bit address
// arithmetic), the next row by the scalar offset, the x + 1 texel by the instruction offset; dx = fract(x), which is
// x - (int)x exactly for the non-negative coordinates the caller passes
__device__ __forceinline__ float3 ld_texel3(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, vo, so, 0);
  return make_float3(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]));
}
__device__ __forceinline__ float3 interp33_8b(__amdgpu_buffer_rsrc_t img, int slot_b, float x, float y, int w) {
  constexpr int TB = L8_TEXEL_BYTES;
  const int ix = (int)x, iy = (int)y;
  const float dx = __builtin_amdgcn_fractf(x), dy = __builtin_amdgcn_fractf(y), dxdy = dx * dy;
  const int vo = __mul24(__mul24(iy, w) + ix, TB) + slot_b;
  const int row = __builtin_amdgcn_readfirstlane(w * TB);
  const float3 p00 = ld_texel3(img, vo, 0), p10 = ld_texel3(img, vo + TB, 0), p01 = ld_texel3(img, vo, row),
               p11 = ld_texel3(img, vo + TB, row);
  const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
  float3 r;
  r.x = w11 * p11.x + w01 * p01.x + w10 * p10.x + w00 * p00.x;
  r.y = w11 * p11.y + w01 * p01.y + w10 * p10.y + w00 * p00.y;
  r.z = w11 * p11.z + w01 * p01.z + w10 * p10.z + w00 * p00.z;
  return r;
}
__device__ __forceinline__ float3 interp33_8(const float4* __restrict__ img, float x, float y, int w) {
  int ix = (int)x, iy = (int)y;
  float dx = x - ix, dy = y - iy, dxdy = dx * dy;
  const float4* bp = img + ix + iy * w;
  const float4 p00 = bp[0], p10 = bp[1], p01 = bp[w], p11 = bp[w + 1];
  const float w11 = dxdy, w01 = dy - dxdy, w10 = dx - dxdy, w00 = 1 - dx - dy + dxdy;
  float3 r;
  r.x = w11 * p11.x + w01 * p01.x + w10 * p10.x + w00 * p00.x;
  r.y = w11 * p11.y + w01 * p01.y + w10 * p10.y + w00 * p00.y;
  r.z = w11 * p11.z + w01 * p01.z + w10 * p10.z + w00 * p00.z;
  return r;
}

// the block's constants (host h's precalc by target slot, thresholds, xAd[h][t][.], calib step)
struct __align__(16) L8Const {
  HsPrecalc pre[HS_MAXF];
  float th[HS_MAXF];
  float xad[HS_MAXF * 8];
  float cs[4];
};
// per-wave LDS scratch of a point group
struct __align__(16) L8Scratch {
  float ps[8][8][8];  // [point][slot][tbd, tHdd, tc0..3, econ, -]: the residuals' terms of the per-point sums
  float jb[8][8][8];  // [point][pattern row i][non-host slot o]: JpJdF (0 unless active), accD / accE operand
  float pp[8][8];     // [point][HdiF, bdSumF, Hcd0..3, -, -]
};
// the epilogue's per-wave partials: T (natural layout, summed over the wave's point lanes) and the D / E / C lanes
struct __align__(16) L8Part {
  float T[L8_NW][8][NTOP + 1];
  float DEC[L8_NW][HS_ND_PROD + 6][64];
};
#if L8_LDS_ACC
union __align__(16) L8Lds {
  L8Scratch s[L8_NW];
};
// the per-lane accumulators in LDS, [wave][entry][lane] (lane-consecutive: conflict-free b32 accesses): T slice
// entries 0..11 (lane (pl, t) holds entries 12 pl + i of slot t's natural layout), accD 12..39, accE / accEB 40..44,
// accHcc / accbc 45
constexpr int L8_NACC = 12 + HS_ND_PROD + 6;
#else
union __align__(16) L8Lds {
  L8Scratch s[L8_NW];
  L8Part part;
};
#endif

// the owner of entry e of lane (t, k) in hs_k_lin's production layout, as an index of the natural T layout
// (-1: the entry is never read by hs_k_reduce / hs_k_stitch)
__device__ __forceinline__ int owner_map(int e, int k) {
  if (e < 8) return e <= k ? didx(e, k) : -1;           // Data (e, k), e <= k
  if (e == 8) return didx(k, 8);                         // Data (k, 8)
  if (e == 9) return didx(k, 9);                         // Data (k, 9)
  if (e == 10) return k == 0 ? didx(8, 8) : k == 1 ? didx(8, 9) : k == 2 ? didx(9, 9) : -1;
  if (e < 14) return TR0 + k * 3 + (e - 11);             // TopRight (k, a | b | r)
  if (e == 14) return k < 6 ? TR0 + (8 + k / 3) * 3 + k % 3 : -1;  // TopRight (8 + k/3, k%3)
  return k < 6 ? BR0 + k : -1;                           // BotRight[k]
}

// fp32 quotient and square root as the compiler's correctly rounded expansions WITHOUT their range steps
// (v_div_scale's operand scaling, v_div_fmas's rescale, v_div_fixup; sqrt's 2^32 pre-scale, its 2^-16 unscale and
// class fix-up).  Where those steps are identities the results are bit-identical to a / b and sqrtf(x)
// (tests/test_gpu_lin8.py::test_fast_div_sqrt_match_ieee sweeps the ranges):
//   div_nr(a, b, rcp_nr(b)) == a / b   for |b| in [2^-60, 2^60], |a| >= 2^-60 and |a / b| in [2^-90, 2^90];
//   sqrt_nr(x) == sqrtf(x)             for x >= 2^-96 (and 0).
// The pixel loop (9 + 8 VALU per quotient pair / further quotient and 9 per root instead of 22 / 11 / 16) flags a
// lane whose operands may leave those ranges; its wave then redoes the group with a / b and sqrtf.
__device__ __forceinline__ float rcp_nr(float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  return __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
}
__device__ __forceinline__ float div_nr(float a, float b, float r) {
  float q = a * r;
  q = __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
  return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
}
__device__ __forceinline__ float sqrt_nr(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __int_as_float(__float_as_int(s) - 1), sp = __int_as_float(__float_as_int(s) + 1);
  const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
  const float o = rm <= 0.f ? sm : s;
  return rp > 0.f ? sp : o;
}

__device__ __forceinline__ float dpp_ror8(float v) {  // lane l <- lane l ^ 8 (rotate a row of 16 by 8)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
}

constexpr int NTP = 96;  // NTOP padded to 8 x 12: entries NTOP .. NTP-1 of the reduce-scatter are zero
static_assert(NTP == 8 * 12 && NTP >= NTOP, "12 entries per point lane");

// entry e of the natural layout -> (kind, r, c): Data (r, c) r <= c < 10 | TopRight (r, c) r < 10, c < 3 | BotRight c
struct TopEntry {
  int kind, r, c;
};
__host__ __device__ constexpr TopEntry top_entry(int e) {
  if (e < TR0) {
    int r = 0;
    while (didx(r, 9) < e) r++;
    return TopEntry{0, r, r + (e - didx(r, r))};
  }
  if (e < BR0) return TopEntry{1, (e - TR0) / 3, (e - TR0) % 3};
  if (e < NTOP) return TopEntry{2, 0, e - BR0};
  return TopEntry{3, 0, 0};
}

// the lane's contribution to entry e (0 for an inactive residual: its operands are zeroed by the caller)
struct TopOps {
  float uu[10], ww[10], jx[10], jy[10], tr0[3], tr1[3], br[6];
};
template <int E>
__device__ __forceinline__ float top_value(const TopOps& o) {
#pragma clang fp contract(fast)
  constexpr TopEntry te = top_entry(E);
  if constexpr (te.kind == 0) return o.uu[te.r] * o.jx[te.c] + o.ww[te.r] * o.jy[te.c];
  else if constexpr (te.kind == 1) return o.jx[te.r] * o.tr0[te.c] + o.jy[te.r] * o.tr1[te.c];
  else if constexpr (te.kind == 2) return o.br[te.c];
  else return 0.f;
}

__device__ __forceinline__ float swap32_add(float x, float y) {  // lanes < 32: x + x(lane + 32); else y(lane - 32) + y
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16_add(float x, float y) {  // rows 0, 2: x + x(row + 1); rows 1, 3: y(row - 1) + y
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Reduce-scatter of the NTP entries over the 8 point lanes of every target slot (lane = 8 pl + t): afterwards lane
// (pl, t) holds, for entries e = 12 pl + j (j < 12), the sum over the slot's 8 lanes.  v_permlane32_swap (pl bit 2)
// and v_permlane16_swap (pl bit 1) exchange half of the remaining entries between partner lanes in one instruction
// per pair, DPP row_ror:8 (pl bit 0) the last quarter: 84 exchanges + 84 adds for 96 entries, no LDS.  The entries
// are formed pairwise as the first exchange consumes them, so at most 48 partial sums are live.
template <int I>
__device__ __forceinline__ void rs_step_a(const TopOps& o, float (&a)[48]) {
  if constexpr (I < 48) {
    a[I] = swap32_add(top_value<I>(o), top_value<48 + I>(o));
    rs_step_a<I + 1>(o, a);
  }
}
__device__ __forceinline__ void slot_reduce_scatter(const TopOps& o, float (&out)[12], int pl) {
  float a[48];
  rs_step_a<0>(o, a);
  float b[24];
#pragma unroll
  for (int i = 0; i < 24; i++) b[i] = swap16_add(a[i], a[24 + i]);
  const bool odd = (pl & 1) != 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const float keep = odd ? b[12 + i] : b[i];
    const float send = odd ? b[i] : b[12 + i];
    out[i] = keep + dpp_ror8(send);
  }
}

// a point group's inputs of one lane (point pl, target slot t), loaded one group ahead (software pipelining: the
// next group's loads are in flight while the current group computes)
struct L8In {
  float idep, idep0, pu, pv;
  int res, st_raw;
  float oldE, oldNewE;
  uint2 ro2;
  unsigned fm;
  float4 jp0, jp1;
  float bds, hdi;
  float4 hcd, co0, co1, we0, we1;
  float priorF;
};
__device__ __forceinline__ void l8_load(const HsLinArgs& a, int pc, int t, L8In& in) {
  const int sl = pc * 8 + t;
  in.idep = a.idepth[pc];
  in.idep0 = a.idepth_zero[pc];
  in.pu = a.u[pc];
  in.pv = a.v[pc];
  in.res = a.res_of_slot[sl];
  in.st_raw = (int)a.r_state[sl];
  in.oldE = a.r_energy[sl];
  in.oldNewE = a.r_newEnergy[sl];
  in.ro2 = reinterpret_cast<const uint2*>(a.res_order)[pc];
  in.fm = a.p_actmask[pc];
  in.jp0 = reinterpret_cast<const float4*>(a.p_JpJdF)[sl * 2];
  in.jp1 = reinterpret_cast<const float4*>(a.p_JpJdF)[sl * 2 + 1];
  in.bds = a.p_bdSumF[pc];
  in.hdi = a.p_HdiF_prev[pc];
  in.hcd = reinterpret_cast<const float4*>(a.p_Hcd)[pc];
  in.co0 = reinterpret_cast<const float4*>(a.color)[pc * 2];
  in.co1 = reinterpret_cast<const float4*>(a.color)[pc * 2 + 1];
  in.we0 = reinterpret_cast<const float4*>(a.weight)[pc * 2];
  in.we1 = reinterpret_cast<const float4*>(a.weight)[pc * 2 + 1];
  in.priorF = a.priorF[pc];
}

}  // namespace

__global__ __launch_bounds__(HS_LIN8_NT, L8_MIN_WAVES) void hs_k_lin8(HsLinArgs a) {
  __shared__ L8Const K;
  __shared__ L8Lds U;
  __shared__ unsigned int H1[HS_TH_BINS];  // the block's pass-1 histogram of its candidates (a.th_hist)
#if L8_LDS_ACC
  __shared__ float ACC[L8_NW][L8_NACC][64];
#endif
  if (a.brk && a.st->stop) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pl = lane >> 3, t = lane & 7;  // point of the group, target slot
  const int b = blockIdx.x;
  const int nF = a.nF;
  int h = 0;  // the block's host
#pragma unroll
  for (int i = 1; i < HS_MAXF; i++) h += (i < nF && b >= a.blk_begin[i]) ? 1 : 0;
  const int nb = a.blk_begin[h + 1] - a.blk_begin[h], q = b - a.blk_begin[h];
  const int hb = a.host_begin[h], nh = a.host_begin[h + 1] - hb;
  const int pb = hb + (int)((long long)nh * q / nb), pe = hb + (int)((long long)nh * (q + 1) / nb);
  if (a.trace && tid == 0) a.trace[(size_t)b * 16] = wall_clock64();
  {  // block constants: as hs_k_lin
    constexpr int PW = (int)(sizeof(HsPrecalc) / 4);
    const int* src = reinterpret_cast<const int*>(a.pre + h * nF);
    int* dst = reinterpret_cast<int*>(K.pre);
    for (int i = tid; i < nF * PW; i += HS_LIN8_NT) dst[i] = src[i];
    if (tid < nF) K.th[tid] = a.frameTH[tid];
    if (a.fuse_step && tid < nF * 8) {
      // xAd[h][t][c] of the last solve (resubstituteF_MT, Src/EnergyFunctional.cpp:222-247), the solve's order
      const int tt = tid >> 3, c = tid & 7;
      const float* aH = a.adHostF + (h + nF * tt) * 64;
      const float* aT = a.adTargetF + (h + nF * tt) * 64;
      const double* lx = a.st->lastX;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int rr = 0; rr < 8; rr++) s1 += (float)lx[4 + 8 * h + rr] * aH[rr * 8 + c];
#pragma unroll
      for (int rr = 0; rr < 8; rr++) s2 += (float)lx[4 + 8 * tt + rr] * aT[rr * 8 + c];
      K.xad[tid] = s1 + s2;
    }
    if (tid < 4) K.cs[tid] = a.st->cstep[tid];
    if (a.th_hist)
      for (int i = tid; i < HS_TH_BINS; i += HS_LIN8_NT) H1[i] = 0u;
  }
  __syncthreads();
  if (a.trace && tid == 0) a.trace[(size_t)b * 16 + 11] = wall_clock64();  // the block constants are in

  const HsCalib cal = a.st->dcal;
  const HsLinParams lp = a.lp;
  // div_nr / sqrt_nr in the pixel loop: the two thresholds bound its quotients' and roots' ranges (uniform)
#if L8_BOUNDS_BITS
  // the pixel bounds 1.1 < PKu < W - 3, 1.1 < PKv < H - 3 (Src/OptimizationClasses.cpp:152) as unsigned spans of
  // float bits above 1.1f (an empty interval: span 0)
  constexpr unsigned kLo1 = 0x3f8ccccdu + 1u;  // __float_as_uint(1.1f) + 1
  const float wmax = (float)(cal.W - 3), hmax = (float)(cal.H - 3);
  const unsigned spanU = __builtin_amdgcn_readfirstlane(wmax > 1.1f ? __float_as_uint(wmax) - kLo1 : 0u);
  const unsigned spanV = __builtin_amdgcn_readfirstlane(hmax > 1.1f ? __float_as_uint(hmax) - kLo1 : 0u);
#endif
  const bool fast_ok = lp.outlierTHSumComponent >= 0x1p-30f && lp.outlierTHSumComponent <= 0x1p30f &&
                       lp.huberTH >= 0x1p-30f && lp.huberTH <= 0x1p30f;
  const int tc = t < nF ? t : 0;
#if L8_BUFFER_TAPS
  // every image slot through one resource (num_records: the whole 32-bit range; taps stay inside the slot's image):
  // the packed 12-byte (I, dx, dy) copy (L8_TEXEL_BYTES 12) or the float4 texels (16)
  const void* ibase = L8_TEXEL_BYTES == 12 ? (const void*)a.img3 : (const void*)a.img;
  const __amdgpu_buffer_rsrc_t timg = __builtin_amdgcn_make_buffer_rsrc((void*)ibase, 0, 0x7fffffff, 0x00020000);
  const int slot16 = hs_img_slot(a.img_slot, tc) * (int)a.img_stride * L8_TEXEL_BYTES;  // past the window: frame 0
#else
  const float4* timg = a.img + (long long)hs_img_slot(a.img_slot, tc) * a.img_stride;  // past the window: frame 0
#endif
  L8Scratch& W = U.s[wv];
  const int oslot = t - (t > h ? 1 : 0);           // non-host slot index of t (t != h)

  // accumulators: T, the (host h, target t) block in natural layout, spread over the slot's 8 point lanes (lane (pl,
  // t) keeps entries 12 pl .. 12 pl + 11, summed per point group); D lane (row, col) = (pl, t), E lane (t, k) =
  // (pl, t) read as (slot pl, row t); C lanes 0..19
#if L8_LDS_ACC
#pragma unroll
  for (int i = 0; i < L8_NACC; i++) ACC[wv][i][lane] = 0.f;
#else
  float Td[12];
#pragma unroll
  for (int i = 0; i < 12; i++) Td[i] = 0.f;
  float D[HS_ND_PROD];
#pragma unroll
  for (int i = 0; i < HS_ND_PROD; i++) D[i] = 0.f;
  float E[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float C = 0.f;
#endif
  double eA = 0.0, sidA = 0.0, npA = 0.0;

  const int ngroups = (pe - pb + 7) >> 3;
  auto clamp_p = [&](int g) {
    const int pp = pb + g * 8 + pl;
    return pp < pe ? pp : (pe > pb ? pe - 1 : pb);
  };
  L8In nx;  // the next group's inputs (loaded ahead; clamped addresses, so always valid)
#if L8_PREFETCH
  if (wv < ngroups) l8_load(a, clamp_p(wv), t, nx);
#endif
#if L8_PRIO == 2
  __shared__ int l8_prog[L8_NW];
  if (lane == 0) l8_prog[wv] = 0;
  __syncthreads();
#endif
  for (int gi = wv; gi < ngroups; gi += a.W) {  // wave-uniform
#if L8_PRIO == 1
    if (((gi - wv) / a.W) & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#elif L8_PRIO == 4
    // the two waves sharing a SIMD (wv, wv + 4: workgroup waves go round-robin over the 4 SIMDs) take turns
    if ((((gi - wv) / a.W) + (wv >> 2)) & 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#elif L8_PRIO == 2
    {  // the block's waves progress together: a wave ahead of the slowest one yields its issue priority
      const int k = (gi - wv) / a.W;
      if (lane == 0) l8_prog[wv] = k;
      int mn = k;
#pragma unroll
      for (int w = 0; w < L8_NW; w++) mn = min(mn, l8_prog[w]);
      if (__builtin_amdgcn_readfirstlane(mn) < k) __builtin_amdgcn_s_setprio(0);
      else __builtin_amdgcn_s_setprio(2);
    }
#endif
#if L8_PREFETCH
    const L8In in = nx;
    if (gi + a.W < ngroups) l8_load(a, clamp_p(gi + a.W), t, nx);  // in flight during this group's work
#else
    l8_load(a, clamp_p(gi), t, nx);
    const L8In in = nx;
#endif
    const int p = pb + gi * 8 + pl;
    const bool valid = p < pe;
    const int pc = valid ? p : pe - 1;
    const int sl = pc * 8 + t;
    float idep = in.idep, idep0 = in.idep0;
    const float pu = in.pu, pv = in.pv;
    const int res = in.res;
    const int st_raw = in.st_raw;
    const float oldE = in.oldE, oldNewE = in.oldNewE;
    const uint2 ro2 = in.ro2;
    const unsigned fm = in.fm;
    const float4 jp0 = in.jp0, jp1 = in.jp1;
    const float bds = in.bds, hdi = in.hdi;
    const float4 hcd = in.hcd;
    const float4 co0 = in.co0, co1 = in.co1, we0 = in.we0, we1 = in.we1;
    const float priorF = in.priorF;
    const float colK[8] = {co0.x, co0.y, co0.z, co0.w, co1.x, co1.y, co1.z, co1.w};
    const float wgtK[8] = {we0.x, we0.y, we0.z, we0.w, we1.x, we1.y, we1.z, we1.w};
    auto res_slot = [&](int qq) -> int { return (int)(int8_t)(((qq < 4 ? ro2.x : ro2.y) >> (8 * (qq & 3))) & 0xffu); };
    const HsPrecalc pcr = K.pre[tc];
    const float thr = fmaxf(K.th[h], K.th[tc]);  // std::max<float>(host TH, target TH)

    if (a.fuse_step) {
      // resubstituteFPt + the point part of doStepFromBackup (stepfacD = 1): the slot's 8-term dot in order, the
      // listed residuals' dots subtracted in list order (each lane of the point's octet does the same)
      const unsigned m = fm;
      const bool on = (m >> t) & 1u;
      const float4 x0 = *reinterpret_cast<const float4*>(&K.xad[tc * 8]);
      const float4 x1 = *reinterpret_cast<const float4*>(&K.xad[tc * 8 + 4]);
      const float xa[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      const float jpj[8] = {jp0.x, jp0.y, jp0.z, jp0.w, jp1.x, jp1.y, jp1.z, jp1.w};
      float dsum = 0.f;
#pragma unroll
      for (int k = 0; k < 8; k++) dsum = dsum + (on ? xa[k] * jpj[k] : 0.f);
      float bq = bds;
      float dot = 0.f;
      dot += K.cs[0] * hcd.x;
      dot += K.cs[1] * hcd.y;
      dot += K.cs[2] * hcd.z;
      dot += K.cs[3] * hcd.w;
      bq -= dot;
      float dl[8];
#pragma unroll
      for (int qq = 0; qq < 8; qq++) {
        const int tt = res_slot(qq);
        dl[qq] = __shfl(dsum, pl * 8 + (tt < 0 ? 0 : tt));
      }
      bool live = true;
#pragma unroll
      for (int qq = 0; qq < 8; qq++) {
        const int tt = res_slot(qq);
        live = live && tt >= 0;
        const int ts = tt < 0 ? 0 : tt;
        const float bn = bq - dl[qq];
        bq = (live && ((m >> ts) & 1u)) ? bn : bq;
      }
      const float step = m != 0u ? -bq * hdi : 0.f;
      idep = idep + 1.0f * step;
      idep0 = idep;
      if (valid && t == 0) {
        a.idepth[p] = idep;
        a.idepth_zero[p] = idep;
        a.p_step[p] = step;
      }
    }

    const bool has = valid && res >= 0;
    const int st = has ? st_raw : HS_RES_OOB;
    const bool live0 = has && st != HS_RES_OOB;
    // ---- centre projection + geometric Jacobian: projectPoint(u, v, idepth_zero, 0, 0, R_0, t_0)
    //      (Include/DirectProjection.h:20-38, Src/OptimizationClasses.cpp:62-118)
    float Jx[10], Jy[10], Jd0, Jd1, centre[3];
    bool okC;
    {
      const float Kl0 = (pu + 0 - cal.cxl) * cal.fxli;
      const float Kl1 = (pv + 0 - cal.cyl) * cal.fyli;
      float pt0 = pcr.R0[0] * Kl0 + pcr.R0[1] * Kl1 + pcr.R0[2] * 1.f;
      float pt1 = pcr.R0[3] * Kl0 + pcr.R0[4] * Kl1 + pcr.R0[5] * 1.f;
      float pt2 = pcr.R0[6] * Kl0 + pcr.R0[7] * Kl1 + pcr.R0[8] * 1.f;
      pt0 = pt0 + pcr.t0[0] * idep0;
      pt1 = pt1 + pcr.t0[1] * idep0;
      pt2 = pt2 + pcr.t0[2] * idep0;
      const float drescale = 1.0f / pt2;
      const float new_idepth = idep0 * drescale;
      const float u = pt0 * drescale, v = pt1 * drescale;
      const float Ku = u * cal.fxl + cal.cxl, Kv = v * cal.fyl + cal.cyl;
      okC = (drescale > 0) && (Ku > 1.1f && Kv > 1.1f && Ku < (cal.W - 3) && Kv < (cal.H - 3));
      centre[0] = Ku; centre[1] = Kv; centre[2] = new_idepth;
      const float* R0 = pcr.R0;
      const float* t0 = pcr.t0;
      Jd0 = drescale * (t0[0] - t0[2] * u) * SCALE_IDEPTH8 * cal.fxl;
      Jd1 = drescale * (t0[1] - t0[2] * v) * SCALE_IDEPTH8 * cal.fyl;
      float cx[4], cy[4];
      cx[2] = drescale * (R0[6] * u - R0[0]);
      cx[3] = cal.fxl * drescale * (R0[7] * u - R0[1]) * cal.fyli;
      cx[0] = Kl0 * cx[2];
      cx[1] = Kl1 * cx[3];
      cy[2] = cal.fyl * drescale * (R0[6] * v - R0[3]) * cal.fxli;
      cy[3] = drescale * (R0[7] * v - R0[4]);
      cy[0] = Kl0 * cy[2];
      cy[1] = Kl1 * cy[3];
      cx[0] = (cx[0] + u) * SCALE_F8;
      cx[1] *= SCALE_F8;
      cx[2] = (cx[2] + 1) * SCALE_C8;
      cx[3] *= SCALE_C8;
      cy[0] *= SCALE_F8;
      cy[1] = (cy[1] + v) * SCALE_F8;
      cy[2] *= SCALE_C8;
      cy[3] = (cy[3] + 1) * SCALE_C8;
      const float fx = cal.fxl, fy = cal.fyl;
      Jx[0] = cx[0]; Jx[1] = cx[1]; Jx[2] = cx[2]; Jx[3] = cx[3];
      Jy[0] = cy[0]; Jy[1] = cy[1]; Jy[2] = cy[2]; Jy[3] = cy[3];
      Jx[4] = new_idepth * fx;
      Jx[5] = 0;
      Jx[6] = -new_idepth * u * fx;
      Jx[7] = -u * v * fx;
      Jx[8] = (1 + u * u) * fx;
      Jx[9] = -v * fx;
      Jy[4] = 0;
      Jy[5] = new_idepth * fy;
      Jy[6] = -new_idepth * v * fy;
      Jy[7] = -(1 + v * v) * fy;
      Jy[8] = u * v * fy;
      Jy[9] = u * fy;
    }
    // ---- the 8 pattern pixels (staticPattern[8], Include/GlobalTypes.h:181-184) in order: in-lane running sums
    //      are the reference's pattern-order sums; a failing pixel (the reference's early exit) marks the slot OOB
    //      and its (redirected, finite) values are never read
    float S[Q8_N];
    bool slotOob = false;
    // FAST: quotients / square roots by div_nr / sqrt_nr, `bad` set where an operand may leave their exact range
    // range guards of the FAST forms as integer max / min over the pattern of the operands' magnitude bits (NaN
    // sorts above +inf): |q2| | the gradient-weight divisor | |residual|
    unsigned gq2max = 0u, gq2min = 0xffffffffu, gwmax = 0u, grmax = 0u;
    auto pixels = [&](auto fast_tag) {
    constexpr bool FAST = decltype(fast_tag)::value;
#pragma unroll
    for (int i = 0; i < Q8_N; i++) S[i] = 0.f;
    slotOob = false;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      constexpr int PDX[8] = {0, -1, 1, -2, 0, 2, -1, 0};
      constexpr int PDY[8] = {-2, -1, -1, 0, 0, 0, 1, 2};
      const float px = pu + PDX[k], py = pv + PDY[k];
      float q0 = pcr.KRKi[0] * px + pcr.KRKi[1] * py + pcr.KRKi[2] * 1.f;
      float q1 = pcr.KRKi[3] * px + pcr.KRKi[4] * py + pcr.KRKi[5] * 1.f;
      float q2 = pcr.KRKi[6] * px + pcr.KRKi[7] * py + pcr.KRKi[8] * 1.f;
      q0 = q0 + pcr.Kt[0] * idep;
      q1 = q1 + pcr.Kt[1] * idep;
      q2 = q2 + pcr.Kt[2] * idep;
      float PKu, PKv;
      if constexpr (FAST && (L8_FAST_OPS & 1)) {
        // |q2| in range: every in-bounds quotient is exact (out of bounds it stays out of bounds, or NaN)
        const unsigned aq2 = __float_as_uint(fabsf(q2));
        gq2max = max(gq2max, aq2);
        gq2min = min(gq2min, aq2);
        const float r2 = rcp_nr(q2);
        PKu = div_nr(q0, q2, r2);
        PKv = div_nr(q1, q2, r2);
      } else {
        PKu = q0 / q2;
        PKv = q1 / q2;
      }
      // (the short-circuit form is a branch region per pixel, which keeps the scheduler from hoisting every pixel's
      // taps at once: the bitwise form spills)
#if L8_BOUNDS_BITS
      // 1.1 < PK < W - 3 as one unsigned range test on the float bits (ordered like the values for positive floats;
      // negatives, -0 and NaN land above the range): the four compares' short-circuit form became 16-bit flag packing
      const bool okP = okC && (__float_as_uint(PKu) - kLo1 < spanU) && (__float_as_uint(PKv) - kLo1 < spanV);
#else
      const bool okP = okC && (PKu > 1.1f && PKv > 1.1f && PKu < (cal.W - 3) && PKv < (cal.H - 3));
#endif
#if L8_BUFFER_TAPS
      const float3 hit = interp33_8b(timg, slot16, okP ? PKu : 2.f, okP ? PKv : 2.f, cal.W);
#else
      const float3 hit = interp33_8(timg, okP ? PKu : 2.f, okP ? PKv : 2.f, cal.W);
#endif
      const float color = colK[k];
      const float residual = hit.x - (float)(pcr.aff[0] * color + pcr.aff[1]);
      const float drdA = (color - pcr.b0);
      const bool okI = okP && isfinite(hit.x);
      slotOob = slotOob || (live0 && !okI);
      const float wden = lp.outlierTHSumComponent + (hit.y * hit.y + hit.z * hit.z);
      float w, hw;
      // the uniform thresholds are in [2^-30, 2^30] (checked by the caller): wden <= 2^60 and |residual| <= 2^60
      // keep both quotients and both square-root arguments in range (NaN operands fail the tests)
      if constexpr (FAST && (L8_FAST_OPS & 2)) {
        gwmax = max(gwmax, __float_as_uint(wden));  // wden >= 0 (or NaN)
        w = sqrt_nr(div_nr(lp.outlierTHSumComponent, wden, rcp_nr(wden)));
      } else {
        w = sqrtf(lp.outlierTHSumComponent / wden);
      }
      if constexpr (FAST && (L8_FAST_OPS & 4)) {
        grmax = max(grmax, __float_as_uint(fabsf(residual)));
        // == (|residual| < huberTH ? 1 : huberTH / |residual|): below the threshold the quotient rounds to >= 1 (or
        // is NaN for a zero / denormal divisor), and min returns 1 then; a NaN residual is flagged.  No select, so
        // the compiler keeps the quotient unconditional instead of branching around it
        hw = fminf(1.0f, div_nr(lp.huberTH, fabsf(residual), rcp_nr(fabsf(residual))));
      } else {
        hw = fabsf(residual) < lp.huberTH ? 1 : lp.huberTH / fabsf(residual);
      }
      w = 0.5f * (w + wgtK[k]);
      float qv[Q8_N];
      qv[0] = w * w * hw * residual * residual * (2 - hw);
      if constexpr (FAST && (L8_FAST_OPS & 4)) hw = sqrt_nr(hw);  // hw <= 1 and sqrt(1) == 1: == (hw < 1 ? sqrt(hw) : hw)
      else hw = hw < 1 ? sqrtf(hw) : hw;
      hw = hw * w;
      const float hy = hit.y * hw, hz = hit.z * hw;
      const float resF = residual * hw;
      float jab0 = drdA * hw;
      float jab1 = hw;
      qv[1] = hy * hy;
      qv[2] = hz * hz;
      qv[3] = hy * hz;
      qv[4] = drdA * hw * hy;
      qv[5] = drdA * hw * hz;
      qv[6] = hw * hy;
      qv[7] = hw * hz;
      qv[8] = drdA * drdA * hw * hw;
      qv[9] = drdA * hw * hw;
      qv[10] = hw * hw;
      qv[11] = hw * hw * (hy * hy + hz * hz);
      if (lp.affineOptModeA < 0) jab0 = 0;
      if (lp.affineOptModeB < 0) jab1 = 0;
      const float rz = resF;  // addPoint<0>: resApprox = resF
      qv[12] = rz * hy;
      qv[13] = rz * hz;
      qv[14] = rz * jab0;
      qv[15] = rz * jab1;
      qv[16] = rz * rz;
#pragma unroll
      for (int i = 0; i < Q8_N; i++) S[i] = S[i] + qv[i];
      // the taps of at most L8_TAP_GROUP pixels in flight per wave (register budget of two waves per SIMD: the
      // other wave hides the gather latency the compiler's full hoisting hid at one wave per SIMD)
      if (L8_TAP_GROUP < 8 && (k + 1) % L8_TAP_GROUP == 0) __builtin_amdgcn_sched_barrier(0);
    }
    };
    {
      if (fast_ok) pixels(std::true_type{});
      constexpr unsigned LOb = 0x21800000u, HIb = 0x5d800000u;  // 2^-60, 2^60
      const bool bad = !fast_ok || gq2max > HIb || gq2min < LOb || gwmax > HIb || grmax > HIb;
      if (__builtin_expect(__ballot(bad) != 0ull, 0)) pixels(std::false_type{});  // rare: the wave redoes the group
    }

    // ---- state decision + applyRes (Src/OptimizationClasses.cpp:128-133,235-256)
    const bool eval = live0 && !slotOob;
    const bool isOut = S[0] > thr || S[11] < 2;
    const float energyLeft = isOut ? thr : S[0];
    const bool active = eval && !isOut;
    const float econ = eval ? energyLeft : oldE;
    if (has) {
      a.r_ewo[sl] = eval ? S[0] : -1.f;
      if (live0) {
        a.r_state[sl] = (uint8_t)(slotOob ? HS_RES_OOB : (isOut ? HS_RES_OUT : HS_RES_IN));
        a.r_active[sl] = active ? 1 : 0;
        a.r_energy[sl] = slotOob ? oldNewE : energyLeft;
        if (!slotOob) a.r_newEnergy[sl] = energyLeft;
      }
      if (a.write_center && live0 && okC) {
        a.r_center[sl * 3 + 0] = centre[0];
        a.r_center[sl * 3 + 1] = centre[1];
        a.r_center[sl * 3 + 2] = centre[2];
      }
    }
    if (valid && t == nF - 1) {
      const float cv = eval ? S[0] : -1.f;
      a.newest_cand[p] = cv;
      const unsigned cb = __float_as_uint(cv);
      if (a.th_hist && cb <= 0x7f800000u) atomicAdd(&H1[cb >> 19], 1u);  // >= 0 and not NaN, as red_th_hist_block
    }
    // ---- takeData (Include/OptimizationClasses.h:155-161): JpJdF and the slot's terms of the per-point sums
    float jj[8], tbd, tHdd, tcd[4];
    {
      const float J00 = S[1], J11 = S[2], J10 = S[3];
      const float aa = J00 * Jd0 + J10 * Jd1;
      const float bb = J10 * Jd0 + J11 * Jd1;
      tbd = S[12] * Jd0 + S[13] * Jd1;
      tHdd = aa * Jd0 + bb * Jd1;
#pragma unroll
      for (int c = 0; c < 4; c++) tcd[c] = Jx[c] * aa + Jy[c] * bb;
#pragma unroll
      for (int k = 0; k < 6; k++) jj[k] = Jx[4 + k] * aa + Jy[4 + k] * bb;
      jj[6] = S[4] * Jd0 + S[5] * Jd1;
      jj[7] = S[6] * Jd0 + S[7] * Jd1;
      if (active) {
        float4* jo = reinterpret_cast<float4*>(a.p_JpJdF) + sl * 2;
        jo[0] = make_float4(jj[0], jj[1], jj[2], jj[3]);
        jo[1] = make_float4(jj[4], jj[5], jj[6], jj[7]);
      }
    }
    // ---- per-point sums in the point's residual-list order (every lane of the octet forms them)
    const unsigned long long actBits = __ballot(active);
    const unsigned amask8 = (unsigned)(actBits >> (pl * 8)) & 0xffu;  // the point's active slots
    *reinterpret_cast<float4*>(&W.ps[pl][t][0]) = make_float4(tbd, tHdd, tcd[0], tcd[1]);
    *reinterpret_cast<float4*>(&W.ps[pl][t][4]) = make_float4(tcd[2], tcd[3], econ, 0.f);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float qs[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    double eSum = 0.0;
    unsigned mask = 0u;
    {
      float g[8][8];
#pragma unroll
      for (int qq = 0; qq < 8; qq++) {
        const int tt = res_slot(qq) & 7;
        const float4 g0 = *reinterpret_cast<const float4*>(&W.ps[pl][tt][0]);
        const float4 g1 = *reinterpret_cast<const float4*>(&W.ps[pl][tt][4]);
        g[qq][0] = g0.x; g[qq][1] = g0.y; g[qq][2] = g0.z; g[qq][3] = g0.w;
        g[qq][4] = g1.x; g[qq][5] = g1.y; g[qq][6] = g1.z;
      }
      bool listed = true;
#pragma unroll
      for (int qq = 0; qq < 8; qq++) {
        const int tr = res_slot(qq);
        listed = listed && tr >= 0;
        const int tt = tr & 7;
        const double e1 = eSum + (double)g[qq][6];
        eSum = listed ? e1 : eSum;
        const bool act = listed && ((amask8 >> tt) & 1u);
        mask |= act ? 1u << tt : 0u;
#pragma unroll
        for (int i = 0; i < 6; i++) {
          const float s1 = qs[i] + g[qq][i];
          qs[i] = act ? s1 : qs[i];
        }
      }
    }
    const float bd = qs[0], Hdd = qs[1];
    float HdiF = 0.f, bdSumF = 0.f;
    if (mask != 0u) {
      float Hh = Hdd + 0.f + priorF;  // Hdd_accAF + Hdd_accLF + priorF
      if ((double)Hh < 1e-10) Hh = (float)1e-10;
      HdiF = (float)(1.0 / (double)Hh);
      bdSumF = bd + 0.f;
      bdSumF += priorF * (idep - idep0);
    }
    const float4 hc4 = make_float4(qs[2] + 0.f, qs[3] + 0.f, qs[4] + 0.f, qs[5] + 0.f);
    if (valid && t == 0) {
      a.p_actmask[p] = (uint8_t)mask;
      a.p_HdiF[p] = HdiF;
      a.p_bdSumF[p] = bdSumF;
      reinterpret_cast<float4*>(a.p_Hcd)[p] = hc4;
      eA += eSum;
      sidA += (double)fabsf(idep);
      npA += 1.0;
    }
    if (!a.accumulate) continue;

    // ---- AccumulatedTopHessianSSE::addPoint<0> of this lane's residual (AccumulatorApprox update / updateTopRight
    //      / updateBotRight, Include/MatrixAccumulators.h:754-915): the 13x13 block of (host, t) in natural layout,
    //      this group's 8 residuals of every slot summed by the reduce-scatter (an inactive residual contributes 0)
    {
#pragma clang fp contract(fast)
      TopOps o;
#pragma unroll
      for (int r = 0; r < 10; r++) {
        o.jx[r] = active ? Jx[r] : 0.f;
        o.jy[r] = active ? Jy[r] : 0.f;
      }
      const float a_ = active ? S[1] : 0.f, b_ = active ? S[3] : 0.f, c_ = active ? S[2] : 0.f;  // JIdx2 00, 01, 11
#pragma unroll
      for (int r = 0; r < 10; r++) {
        o.uu[r] = a_ * o.jx[r] + b_ * o.jy[r];
        o.ww[r] = b_ * o.jx[r] + c_ * o.jy[r];
      }
      const float tr0[3] = {S[4], S[6], S[12]}, tr1[3] = {S[5], S[7], S[13]};
#pragma unroll
      for (int c = 0; c < 3; c++) {
        o.tr0[c] = active ? tr0[c] : 0.f;
        o.tr1[c] = active ? tr1[c] : 0.f;
      }
      const float br[6] = {S[8], S[9], S[14], S[10], S[15], S[16]};
#pragma unroll
      for (int i = 0; i < 6; i++) o.br[i] = active ? br[i] : 0.f;
      float red[12];
      slot_reduce_scatter(o, red, pl);
#if L8_LDS_ACC
#pragma unroll
      for (int i = 0; i < 12; i++) ACC[wv][i][lane] += red[i];
#else
#pragma unroll
      for (int i = 0; i < 12; i++) Td[i] += red[i];
#endif
    }
    // ---- Schur accumulators (Src/AccumulatedSCHessian.cpp:32-51) through the wave's scratch: accD (lane = (row,
    //      col) of every (o1 <= o2) block), accE / accEB (lane = (slot, row)), accHcc / accbc (lanes 0..19)
    if (t != h) {
#pragma unroll
      for (int i = 0; i < 8; i++) W.jb[pl][i][oslot] = active ? jj[i] : 0.f;
    }
    if (t == 0) {
      *reinterpret_cast<float4*>(&W.pp[pl][0]) = make_float4(HdiF, bdSumF, hc4.x, hc4.y);
      *reinterpret_cast<float4*>(&W.pp[pl][4]) = make_float4(hc4.z, hc4.w, 0.f, 0.f);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {
#pragma clang fp contract(fast)
      const int dr = pl, dc = t;         // accD lane (row, col)
      const int es = pl, ek = t;         // accE lane (slot es, row ek)
      const int eo = es - (es > h ? 1 : 0);
      const int cr = (lane >> 2) & 3, ccol = lane & 3;
      const unsigned long long wbits = actBits;
#if L8_PK_SC
      l8f2 DP[9];
      float DS[10];
#pragma unroll
      for (int o1 = 0; o1 < 7; o1++)
#pragma unroll
        for (int o2 = o1; o2 < 7; o2++) {
          const float v = ACC[wv][12 + o1 * 7 - (o1 * (o1 - 1)) / 2 + (o2 - o1)][lane];
          const DSlot ds = d_slot(o1, o2);
          if (ds.kind == 1) DS[ds.idx] = v;
          else if (o2 & 1) DP[ds.idx].y = v;
          else DP[ds.idx].x = v;
        }
      float E[5], C;
#pragma unroll
      for (int i = 0; i < 5; i++) E[i] = ACC[wv][12 + HS_ND_PROD + i][lane];
      C = ACC[wv][12 + HS_ND_PROD + 5][lane];
#elif L8_LDS_ACC
      float D[HS_ND_PROD], E[5], C;
#pragma unroll
      for (int i = 0; i < HS_ND_PROD; i++) D[i] = ACC[wv][12 + i][lane];
#pragma unroll
      for (int i = 0; i < 5; i++) E[i] = ACC[wv][12 + HS_ND_PROD + i][lane];
      C = ACC[wv][12 + HS_ND_PROD + 5][lane];
#endif
#pragma unroll
      for (int qp = 0; qp < 8; qp++) {
        const unsigned mq = (unsigned)(wbits >> (qp * 8)) & 0xffu;  // uniform
        if (mq == 0u) continue;
        const float4 pp0 = *reinterpret_cast<const float4*>(&W.pp[qp][0]);
        const float4 pp1 = *reinterpret_cast<const float4*>(&W.pp[qp][4]);
        const float hdf = pp0.x, bsf = pp0.y;
        const float hcv[4] = {pp0.z, pp0.w, pp1.x, pp1.y};
        const float4 r0 = *reinterpret_cast<const float4*>(&W.jb[qp][dr][0]);
        const float4 r1 = *reinterpret_cast<const float4*>(&W.jb[qp][dr][4]);
        const float4 c0 = *reinterpret_cast<const float4*>(&W.jb[qp][dc][0]);
        const float4 c1 = *reinterpret_cast<const float4*>(&W.jb[qp][dc][4]);
        const float j1[7] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z};
        const float j2[7] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z};
#if L8_PK_SC
        const l8f2 j2p[3] = {l8f2{c0.x, c0.y}, l8f2{c0.z, c0.w}, l8f2{c1.x, c1.y}};
#pragma unroll
        for (int o1 = 0; o1 < 7; o1++) {
          const float wl = hdf * j1[o1];
#pragma unroll
          for (int o2 = o1; o2 < 7; o2++) {
            const DSlot ds = d_slot(o1, o2);
            if (ds.kind == 1) DS[ds.idx] = __builtin_fmaf(wl, j2[o2], DS[ds.idx]);
            else if ((o2 & 1) == 0) DP[ds.idx] = __builtin_elementwise_fma(l8f2{wl, wl}, j2p[o2 >> 1], DP[ds.idx]);
          }
        }
        {  // predicated, not branched: jb holds 0 for an inactive residual, and the host slot reads 0
          const float jv = es != h ? W.jb[qp][ek][min(eo, 6)] : 0.f;
          const float wl = hdf * jv;
          const l8f2 e01 = __builtin_elementwise_fma(l8f2{wl, wl}, l8f2{pp0.z, pp0.w}, l8f2{E[0], E[1]});
          const l8f2 e23 = __builtin_elementwise_fma(l8f2{wl, wl}, l8f2{pp1.x, pp1.y}, l8f2{E[2], E[3]});
          E[0] = e01.x; E[1] = e01.y; E[2] = e23.x; E[3] = e23.y;
          E[4] += (hdf * bsf) * jv;
        }
#else
#pragma unroll
        for (int o1 = 0; o1 < 7; o1++) {
          const float wl = hdf * j1[o1];
#pragma unroll
          for (int o2 = o1; o2 < 7; o2++) D[o1 * 7 - (o1 * (o1 - 1)) / 2 + (o2 - o1)] += wl * j2[o2];
        }
        {  // predicated, not branched: jb holds 0 for an inactive residual, and the host slot reads 0
          const float jv = es != h ? W.jb[qp][ek][min(eo, 6)] : 0.f;
          const float wl = hdf * jv;
#pragma unroll
          for (int c = 0; c < 4; c++) E[c] += wl * hcv[c];
          E[4] += (hdf * bsf) * jv;
        }
#endif
        const float hr = W.pp[qp][2 + cr], hc = W.pp[qp][2 + ccol];  // per-lane LDS addresses, no select chains
        C += lane < 16 ? (hdf * hr) * hc : (bsf * hdf) * hc;
      }
#if L8_LDS_ACC
#if L8_PK_SC
#pragma unroll
      for (int o1 = 0; o1 < 7; o1++)
#pragma unroll
        for (int o2 = o1; o2 < 7; o2++) {
          const DSlot ds = d_slot(o1, o2);
          ACC[wv][12 + o1 * 7 - (o1 * (o1 - 1)) / 2 + (o2 - o1)][lane] =
              ds.kind == 1 ? DS[ds.idx] : ((o2 & 1) ? DP[ds.idx].y : DP[ds.idx].x);
        }
#else
#pragma unroll
      for (int i = 0; i < HS_ND_PROD; i++) ACC[wv][12 + i][lane] = D[i];
#endif
#pragma unroll
      for (int i = 0; i < 5; i++) ACC[wv][12 + HS_ND_PROD + i][lane] = E[i];
      ACC[wv][12 + HS_ND_PROD + 5][lane] = C;
#endif
    }
    __builtin_amdgcn_wave_barrier();  // the scratch is rewritten by the next group
    if (a.trace && tid == 0 && gi == wv) a.trace[(size_t)b * 16 + 12] = wall_clock64();  // wave 0's first group
  }
  if (a.trace && tid == 0) a.trace[(size_t)b * 16 + 1] = wall_clock64();
  if (a.trace && lane == 0 && wv < 8) a.trace[(size_t)b * 16 + 3 + wv] = wall_clock64();  // each wave's loop end
#if L8_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
  if (!a.accumulate) return;

  // ---- epilogue: the block partial in hs_k_lin's production layout (T entries from their owner lanes), waves in
  //      order
  // the energies of the wave (lanes t == 0 of the 8 point slots, in point-slot order)
  double eW = 0.0, sW = 0.0, nW = 0.0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    eW += __shfl(eA, j * 8);
    sW += __shfl(sidA, j * 8);
    nW += __shfl(npA, j * 8);
  }
  __syncthreads();  // every wave is done with its scratch (the partials area aliases it)
#if !L8_LDS_ACC
  L8Part& P = U.part;
#pragma unroll
  for (int i = 0; i < 12; i++)
    if (12 * pl + i < NTOP) P.T[wv][t][12 * pl + i] = Td[i];
#pragma unroll
  for (int i = 0; i < HS_ND_PROD; i++) P.DEC[wv][i][lane] = D[i];
#pragma unroll
  for (int i = 0; i < 5; i++) P.DEC[wv][HS_ND_PROD + i][lane] = E[i];
  P.DEC[wv][HS_ND_PROD + 5][lane] = C;
#endif
  __shared__ double se[L8_NW][3];
  if (lane == 0) {
    se[wv][0] = eW;
    se[wv][1] = sW;
    se[wv][2] = nW;
  }
  __syncthreads();
  constexpr int NE = hs_ne(false);
  static_assert(NE == HS_E_TOP + HS_ND_PROD + 6, "production partial layout");
  float* out = a.part + (size_t)b * NE * 64;
  for (int i = tid; i < NE * 64; i += HS_LIN8_NT) {
    const int e = i >> 6, l = i & 63;
    float s = 0.f;
    if (e < HS_E_TOP) {
      const int tt = l >> 3, kk = l & 7;
      const int m = owner_map(e, kk);
      if (m >= 0) {
#if L8_LDS_ACC
        const int sl8 = (m / 12) * 8 + tt, si = m % 12;  // entry m of slot tt: lane (m / 12, tt), slice entry m % 12
        s = ACC[0][si][sl8];
#pragma unroll
        for (int w = 1; w < L8_NW; w++) s += ACC[w][si][sl8];
#else
        s = P.T[0][tt][m];
#pragma unroll
        for (int w = 1; w < L8_NW; w++) s += P.T[w][tt][m];
#endif
      }
    } else {
      const int d = e - HS_E_TOP;
#if L8_LDS_ACC
      s = ACC[0][12 + d][l];
#pragma unroll
      for (int w = 1; w < L8_NW; w++) s += ACC[w][12 + d][l];
#else
      s = P.DEC[0][d][l];
#pragma unroll
      for (int w = 1; w < L8_NW; w++) s += P.DEC[w][d][l];
#endif
    }
    out[i] = s;
  }
  if (tid < 3) {
    double s = se[0][tid];
#pragma unroll
    for (int w = 1; w < L8_NW; w++) s += se[w][tid];
    a.part_e[(size_t)b * 4 + tid] = s;
  }
  if (a.th_hist)  // (every wave's candidates are in: the barriers above)
    for (int i = tid; i < HS_TH_BINS; i += HS_LIN8_NT)
      if (const unsigned int v = H1[i]) atomicAdd(&a.th_hist[i], v);
  if (a.trace && tid == 0) a.trace[(size_t)b * 16 + 2] = wall_clock64();
}

// test hook (hs_debug_fastmath): out[i] = {div_nr(a, b, rcp_nr(b)), a / b, sqrt_nr(a), sqrtf(a)}
__global__ void hs_k_debug_fastmath(int n, const float* a, const float* b, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = a[i], y = b[i];
  const float4 r = make_float4(div_nr(x, y, rcp_nr(y)), x / y, sqrt_nr(x), sqrtf(x));
  reinterpret_cast<float4*>(out)[i] = r;
}
