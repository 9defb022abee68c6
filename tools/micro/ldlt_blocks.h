// ldlt_blocks.h — round-4 EXPERIMENT (tools/micro/ldlt8.hip), not used by the product: a column-block LDLT of the GN
// step's scaled system (EnergyFunctional::solveSystemF's `SHS.ldlt().solve(Sb)`, Src/EnergyFunctional.cpp:799-801)
// inside one workgroup.  Correct (x within 1e-11 of a host fp64 LDLT), but not faster than hs_k_solve's panel LDLT
// (hs_ba_kernels.hip ldlt_solve_blocked): 28-34k cycles for nF = 8 against ~31k, and the solve kernel measured
// 28.3 vs 26.2 us per launch with it (gpurun_out/r04_p, r04_q).  Per 4-pivot phase: the owner's apply of the previous
// block ~500-930 cycles, its block ~650-790, the barrier ~280 (gpurun_out/r04_r).  See DESIGN.md §4 *Solve*.
//
// The system is n = 4 + 8 nF (calib rows first, then 8 rows per frame), symmetric positive definite after the
// damping, factored without pivoting (backward stable for SPD; Eigen's diagonal pivoting changes x by rounding only,
// the solve is checked against the oracle by tolerance).
//
//  1. Calib block: wave 0 forms G = A_cc^-1 (4x4), then every lane its row of A_fc G, its columns of the frame
//     block's Schur complement S = A_ff - A_fc G A_cf and (the rhs wave) b_f - A_fc G b_c: block elimination of the
//     first 4 pivots, the same factorization with the calib first.
//  2. S (8 nF <= 64 rows) = L D L^T, right-looking, lane = row.  Wave w holds the C columns C w .. C w + C - 1 of S in
//     registers.  Phase p (one s_barrier each): wave p applies block p - 1's published columns to its own, then
//     factors its block from registers — per pivot a scalar recurrence d_{k+1} = A(k+1, k+1) - A(k+1, k) A(k, k+1) /
//     d_k on readlane'd entries (the chain is the reciprocal and one fma) while the column updates run beside it —
//     and publishes each raw column u_k = S(:, k) (d_k on its diagonal) to LDS; the later waves apply block p - 1
//     beside it (after a short sleep, so the next owner's batch reads meet no burst).  The next owner also writes
//     block p - 1's L = u / d transposed for the back substitution.  The rhs is one more column of the last wave
//     (forward substitution z = L^-1 b, one block at a time).
//     Measured on gfx950 (tools/micro/ldlt8.hip, handoff.hip): an s_barrier hand-off resumes a waiting wave ~70 cycles
//     after the last arrival, an LDS flag polled by another wave ~210; one fp64 FMA issues every ~7 cycles from one
//     wave and completes in ~13.5, v_rcp_f64 in ~24.
//  3. y = D^-1 z, back substitution L^T x = y on the last wave (lane = row, x_j by readlane, the L^T rows loaded
//     ahead), then x_c = G (b_c - A_cf x_f).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <type_traits>

namespace hs_ldlt {

constexpr int MST = 64;  // Mv row stride (row k = published raw column u_k)
constexpr int TST = 65;  // MvT row stride (MvT[j][i] = L(j, i); odd: conflict-free lane-strided stores)

// LDS the solve needs beside the system (~66 KB)
struct Lds {
  double Mv[64 * MST];   // row k: the raw column u_k = S(:, k) after steps < k (d_k = u_k[k]; rows < k unused)
  double MvT[64 * TST];  // L transposed: MvT[j][i] = L(j, i) for i < j, 0 otherwise
  double G[16];          // A_cc^-1
};

#define HS_LDS __attribute__((address_space(3)))
// LDS accesses through explicit local-address-space pointers: a generic pointer compiles to flat loads
__device__ __forceinline__ const HS_LDS double* lds(const double* p) { return (const HS_LDS double*)p; }
__device__ __forceinline__ HS_LDS double* lds(double* p) { return (HS_LDS double*)p; }
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ double rdl(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// 1/d: v_rcp_f64 + one Newton step (~4e-15 relative); 0 for a (near-)zero pivot
__device__ __forceinline__ double rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  return fabs(d) > DBL_MIN ? r : 0.0;
}
// the pivots of the damped SPD system are positive: no zero guard on the factorization's chain (a non-positive
// pivot gives a non-finite x, which the solve reports as a non-finite step)
__device__ __forceinline__ double rcp_nz(double d) {
  double r = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}
// DPP move of a double (both halves), full row / bank masks
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// sum over the 64 lanes (uniform result): row sums by DPP (xor 1, xor 2, rotate 4, rotate 8 within the row of 16),
// then the four rows' sums by readlane
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x124>(v);  // row_ror:4
  v += dpp<0x128>(v);  // row_ror:8
  return (rdl(v, 0) + rdl(v, 16)) + (rdl(v, 32) + rdl(v, 48));
}

// 4x4 SPD inverse by an unpivoted LDLT (uniform)
__device__ __forceinline__ void inv4(const double a[4][4], double g[4][4]) {
  double l[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}}, d[4], di[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    double s = a[j][j];
#pragma unroll
    for (int k = 0; k < j; k++) s -= l[j][k] * l[j][k] * d[k];
    d[j] = s;
    di[j] = rcp(s);
#pragma unroll
    for (int i = j + 1; i < 4; i++) {
      double t = a[i][j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= l[i][k] * l[j][k] * d[k];
      l[i][j] = t * di[j];
    }
  }
  double li[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};  // L^-1 (unit lower)
#pragma unroll
  for (int i = 1; i < 4; i++)
#pragma unroll
    for (int j = 0; j < i; j++) {
      double s = 0.0;
#pragma unroll
      for (int k = j; k < i; k++) s -= l[i][k] * li[k][j];
      li[i][j] = s;
    }
#pragma unroll
  for (int i = 0; i < 4; i++)  // G = L^-T D^-1 L^-1
#pragma unroll
    for (int j = 0; j < 4; j++) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 4; k++) s += li[k][i] * di[k] * li[k][j];
      g[i][j] = s;
    }
}

// Solves A x = b.  A: row-major, stride n = 4 + 8 nF (nF <= 8), in LDS; yv[n]: b in, x out (LDS).  The frame block
// S is factored in 2 nF column blocks of 4; block b belongs to wave b % W (W = 8: 512 threads, each wave holding up
// to two blocks; W = 16: 1024 threads).  Every thread of the workgroup calls it (no preparation of L needed); it ends
// with a barrier.
template <int W>
__device__ void solve(const double* A_, double* yv_, int nF, Lds& L, int tid, long long* trace = nullptr,
                      long long* ltrace = nullptr) {
  constexpr int C = 4, JB = 16 / W;  // columns per block, blocks per wave
  static_assert(W == 8 || W == 16, "8 or 16 waves");
  typedef double dbl2 __attribute__((ext_vector_type(2)));
  const HS_LDS double* A = lds(A_);
  HS_LDS double* yv = lds(yv_);
  HS_LDS double* Mv = lds(L.Mv);
  HS_LDS double* MvT = lds(L.MvT);
  const int n = 4 + 8 * nF, n8 = 8 * nF, nb = n8 / C;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), i = tid & 63;  // w in an SGPR: uniform branches
  const int hold = (nb - 1) % W;  // the rhs / back-substitution wave (the last block's owner)
  const bool vrow = i < n8;
  const int r = 4 + (vrow ? i : 0);
  auto held = [&](int j) { return w + W * j < nb; };  // wave w's j-th block exists
  // ---- 1. calib block
  double ar[4], aj[JB][C], aq[4][JB][C];
#pragma unroll
  for (int p = 0; p < 4; p++) ar[p] = A[r * n + p];
#pragma unroll
  for (int j = 0; j < JB; j++)
    if (held(j))  // operands requested before G exists
#pragma unroll
      for (int c = 0; c < C; c++) {
        const int jc = 4 + C * (w + W * j) + c;
        aj[j][c] = A[r * n + jc];
#pragma unroll
        for (int q = 0; q < 4; q++) aq[q][j][c] = A[q * n + jc];
      }
  if (w == 0) {
    double acc[4][4], g[4][4];
#pragma unroll
    for (int p = 0; p < 4; p++)
#pragma unroll
      for (int q = 0; q < 4; q++) acc[p][q] = A[p * n + q];
    inv4(acc, g);
#pragma unroll
    for (int q = 0; q < 16; q++)  // static indices: g stays in registers
      if (i == q) lds(L.G)[q] = g[q >> 2][q & 3];
  }
  __syncthreads();
  double col[JB][C];
  double rhs = 0.0;
  {
    double t[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      double v = 0.0;
#pragma unroll
      for (int p = 0; p < 4; p++) v = __builtin_fma(ar[p], lds(L.G)[p * 4 + q], v);
      t[q] = vrow ? v : 0.0;
    }
#pragma unroll
    for (int j = 0; j < JB; j++)
#pragma unroll
      for (int c = 0; c < C; c++) {
        double v = held(j) ? aj[j][c] : 0.0;
#pragma unroll
        for (int q = 0; q < 4; q++) v = __builtin_fma(-t[q], held(j) ? aq[q][j][c] : 0.0, v);
        col[j][c] = vrow ? v : 0.0;
      }
    if (w == hold) {
      double v = vrow ? yv[r] : 0.0;
#pragma unroll
      for (int q = 0; q < 4; q++) v = __builtin_fma(-t[q], yv[q], v);
      rhs = vrow ? v : 0.0;
    }
  }
  if (trace && tid == 0) trace[1] = clock64();

  // ---- 2. S = L D L^T.  Mv row k: L(:, k) (rows > k), d_k on the diagonal slot (rows < k: values no one reads).
  // The holder's forward substitution over block kb: the block's z_k by readlane, a uniform unit-lower 4 x 4 solve,
  // one rank-4 update of the rows below; it also writes the block's L^T rows (lm: this lane's L entries, masked).
  auto holder_block = [&](int kb, const double (&lm)[C]) {
    const int k0 = C * kb;
#pragma unroll
    for (int kc = 0; kc < C; kc++) MvT[i * TST + k0 + kc] = lm[kc];
    double z[C];
#pragma unroll
    for (int kc = 0; kc < C; kc++) z[kc] = rdl(rhs, k0 + kc);
#pragma unroll
    for (int kc = 1; kc < C; kc++)
#pragma unroll
      for (int kp = 0; kp < kc; kp++) z[kc] = __builtin_fma(-Mv[(k0 + kp) * MST + k0 + kc], z[kp], z[kc]);
#pragma unroll
    for (int kc = 0; kc < C; kc++) rhs = __builtin_fma(-lm[kc], z[kc], rhs);
  };
  // the owner's block kb = w + W jo (its columns up to date through block kb - 1): the 4 x 4 diagonal block by
  // readlane, its LDLT uniformly (the pivot chain: 4 reciprocals), then the L columns lane-parallel from the uniform
  // factors (no further readlane)
  auto own_block = [&](int kb, auto jo_tag) {
    constexpr int jo = decltype(jo_tag)::value;
    __builtin_amdgcn_s_setprio(3);
    const int k0 = C * kb;
    double B[C][C], d[C], rr[C], Wd[C][C];  // Wd(r, c) = d_c L(r, c): the entry after the steps < c
#pragma unroll
    for (int c = 0; c < C; c++)
#pragma unroll
      for (int rr_ = c; rr_ < C; rr_++) B[rr_][c] = rdl(col[jo][c], k0 + rr_);
#pragma unroll
    for (int c = 0; c < C; c++) {
      double dc = B[c][c];
#pragma unroll
      for (int kp = 0; kp < c; kp++) dc = __builtin_fma(-Wd[c][kp] * rr[kp], Wd[c][kp], dc);
      d[c] = dc;
      rr[c] = rcp_nz(dc);
#pragma unroll
      for (int rr_ = c + 1; rr_ < C; rr_++) {
        double a = B[rr_][c];
#pragma unroll
        for (int kp = 0; kp < c; kp++) a = __builtin_fma(-Wd[rr_][kp] * rr[kp], Wd[c][kp], a);
        Wd[rr_][c] = a;
      }
    }
    double m[C], lm[C];
#pragma unroll
    for (int kc = 0; kc < C; kc++) {
      const int k = k0 + kc;
      double v = col[jo][kc];
#pragma unroll
      for (int kp = 0; kp < kc; kp++) v = __builtin_fma(-m[kp], Wd[kc][kp], v);
      m[kc] = v * rr[kc];
      Mv[k * MST + i] = i == k ? d[kc] : m[kc];
      lm[kc] = i > k ? m[kc] : 0.0;
    }
    compiler_fence();  // the block's stores are issued here
    __builtin_amdgcn_s_setprio(0);
    if (w == hold) holder_block(kb, lm);
  };
  // block kb's published columns applied to this wave's pending blocks (those after kb): one batch of LDS reads
  auto apply_block = [&](int kb) {
    const int k0 = C * kb;
    const HS_LDS dbl2* Mv2 = (const HS_LDS dbl2*)Mv;
    double mi[C], u[C];
#pragma unroll
    for (int kc = 0; kc < C; kc++) {
      mi[kc] = Mv[(k0 + kc) * MST + i];
      u[kc] = mi[kc] * Mv[(k0 + kc) * (MST + 1)];  // d_k L(i, k)
    }
#pragma unroll
    for (int j = 0; j < JB; j++) {
      const int b = w + W * j;
      if (b > kb && b < nb) {
        double mb[C][C];
#pragma unroll
        for (int kc = 0; kc < C; kc++)
#pragma unroll
          for (int c = 0; c < C; c += 2) {  // 16-byte broadcast reads of L(b's columns, k)
            const dbl2 v = Mv2[((k0 + kc) * MST + C * b + c) >> 1];
            mb[kc][c] = v.x;
            mb[kc][c + 1] = v.y;
          }
#pragma unroll
        for (int c = 0; c < C; c++)  // column 0 first: the next owner's first pivot waits on it
#pragma unroll
          for (int kc = 0; kc < C; kc++) col[j][c] = __builtin_fma(-u[kc], mb[kc][c], col[j][c]);
      }
    }
    if (w == hold && kb % W != hold) {  // (the holder's own blocks went through holder_block in own_block)
      double lm[C];
#pragma unroll
      for (int kc = 0; kc < C; kc++) lm[kc] = i > k0 + kc ? mi[kc] : 0.0;
      holder_block(kb, lm);
    }
  };
  for (int p = 0; p < nb; p++) {  // uniform over the workgroup: every wave takes every barrier
    const int owner = p % W;
    if (ltrace && w == owner && i == 0) ltrace[p * 4 + 0] = clock64();
    if (p >= 1 && (held(0) || held(JB - 1))) {
      bool pending = false;
#pragma unroll
      for (int j = 0; j < JB; j++) pending |= held(j) && w + W * j >= p;
      if (pending || w == hold) {
        if (w == owner) __builtin_amdgcn_s_setprio(2);
        else if (w != hold) __builtin_amdgcn_s_sleep(8);  // ~510 cycles: the next owner's batch reads go first
        apply_block(p - 1);
      }
    }
    if (ltrace && w == owner && i == 0) ltrace[p * 4 + 1] = clock64();
    if (w == owner) {
      if (p < W) own_block(p, std::integral_constant<int, 0>());
      else own_block(p, std::integral_constant<int, JB - 1>());
    }
    if (ltrace && w == owner && i == 0) ltrace[p * 4 + 2] = clock64();
    if (ltrace && w == hold && i == 0) ltrace[p * 4 + 3] = clock64();
    __syncthreads();
  }
  if (trace && tid == 0) trace[2] = clock64();

  // ---- 3. D^-1, back substitution (holder wave), calib
  if (w == hold) {
    double y = vrow ? rhs * rcp(Mv[min(i, n8 - 1) * (MST + 1)]) : 0.0;
    // column-oriented: x_j = y_j (lane j, final once the rows below are done), then y_i -= L(j, i) x_j on every lane.
    // Unrolled, so the L^T rows are loaded ahead of the readlane -> fma chain; rows >= n8 hold y = 0 (x_j = 0)
#pragma unroll
    for (int j = 63; j >= 1; j--) {
      const double lji = (vrow && j < n8) ? MvT[j * TST + i] : 0.0;  // rows >= n8 are never written
      y = __builtin_fma(-lji, rdl(y, j), y);
    }
    // x_c = G (b_c - A_cf x_f): four wave sums of A(q, 4 + i) x_i
    double sq[4];
#pragma unroll
    for (int q = 0; q < 4; q++) sq[q] = wave_sum(vrow ? A[q * n + 4 + i] * y : 0.0);
    double xc[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < 4; q++) v = __builtin_fma(lds(L.G)[p * 4 + q], yv[q] - sq[q], v);
      xc[p] = v;
    }
    if (vrow) yv[4 + i] = y;
    if (i < 4) yv[i] = i == 0 ? xc[0] : i == 1 ? xc[1] : i == 2 ? xc[2] : xc[3];
  }
  if (trace && tid == 0) trace[4] = clock64();
  __syncthreads();
}

}  // namespace hs_ldlt
