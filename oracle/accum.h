/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Scalar restatement of the reference's
 * numerically-blocked fp32 accumulators (Include/MatrixAccumulators.h):
 *   AccumulatorXX<i,j>   :36-89     A += (w*L)*R^T, 1 / 1k / 1m blocking
 *   AccumulatorX<i>      :177-237   A += w*L
 *   Accumulator11        :91-172    4-lane SSE partial sums
 *   AccumulatorApprox    :595-972   13x13 [calib4|xi6|a|b|r], update/TopRight/BotRight
 *   Accumulator9         :982-1345  4-lane SSE 9x9 (45 entries) for CoarseTracker (updateSSE_eighted) and
 *                                   DirectRefinement (updateSSE :1025-1087, updateSingleWeighted :1242-1331)
 * shiftUp: flush to the next level when the level holds > 1000 updates.
 * The 4-lane SSE adds are restated lane by lane (same rounding as _mm_add_ps).
 */
#pragma once
#include <cstring>

namespace hso {

template <int I, int J>
struct AccXX {
  float A[I * J], A1k[I * J], A1m[I * J];
  size_t num;
  float numIn1, numIn1k, numIn1m;
  void initialize() {
    std::memset(A, 0, sizeof(A)); std::memset(A1k, 0, sizeof(A1k)); std::memset(A1m, 0, sizeof(A1m));
    num = 0; numIn1 = numIn1k = numIn1m = 0;
  }
  void finish() { shiftUp(true); num = (size_t)(numIn1 + numIn1k + numIn1m); }
  void update(const float* L, const float* R, float w) {
    for (int r = 0; r < I; r++) {
      const float wl = w * L[r];
      for (int c = 0; c < J; c++) A[r * J + c] += wl * R[c];
    }
    numIn1++;
    shiftUp(false);
  }
  void shiftUp(bool force) {
    if (numIn1 > 1000 || force) {
      for (int k = 0; k < I * J; k++) { A1k[k] += A[k]; A[k] = 0; }
      numIn1k += numIn1; numIn1 = 0;
    }
    if (numIn1k > 1000 || force) {
      for (int k = 0; k < I * J; k++) { A1m[k] += A1k[k]; A1k[k] = 0; }
      numIn1m += numIn1k; numIn1k = 0;
    }
  }
};

template <int I>
struct AccX {
  float A[I], A1k[I], A1m[I];
  size_t num;
  float numIn1, numIn1k, numIn1m;
  void initialize() {
    std::memset(A, 0, sizeof(A)); std::memset(A1k, 0, sizeof(A1k)); std::memset(A1m, 0, sizeof(A1m));
    num = 0; numIn1 = numIn1k = numIn1m = 0;
  }
  void finish() { shiftUp(true); num = (size_t)(numIn1 + numIn1k + numIn1m); }
  void update(const float* L, float w) {
    for (int r = 0; r < I; r++) A[r] += w * L[r];
    numIn1++;
    shiftUp(false);
  }
  // updateNoWeight (Include/MatrixAccumulators.h:210-215)
  void updateNoWeight(const float* L) {
    for (int r = 0; r < I; r++) A[r] += L[r];
    numIn1++;
    shiftUp(false);
  }
  void shiftUp(bool force) {
    if (numIn1 > 1000 || force) {
      for (int k = 0; k < I; k++) { A1k[k] += A[k]; A[k] = 0; }
      numIn1k += numIn1; numIn1 = 0;
    }
    if (numIn1k > 1000 || force) {
      for (int k = 0; k < I; k++) { A1m[k] += A1k[k]; A1k[k] = 0; }
      numIn1m += numIn1k; numIn1k = 0;
    }
  }
};

// AccumulatorApprox: Data[60] (55 used: upper triangle of the 10x10 [calib|xi] block),
// TopRight[32] (30 used: 10 rows x {a,b,r}), BotRight[8] (6 used).
struct AccApprox {
  float Data[60], Data1k[60], Data1m[60];
  float TR[32], TR1k[32], TR1m[32];
  float BR[8], BR1k[8], BR1m[8];
  float H[13 * 13];
  size_t num;
  float numIn1, numIn1k, numIn1m;

  void initialize() {
    std::memset(Data, 0, sizeof(Data)); std::memset(Data1k, 0, sizeof(Data1k)); std::memset(Data1m, 0, sizeof(Data1m));
    std::memset(TR, 0, sizeof(TR)); std::memset(TR1k, 0, sizeof(TR1k)); std::memset(TR1m, 0, sizeof(TR1m));
    std::memset(BR, 0, sizeof(BR)); std::memset(BR1k, 0, sizeof(BR1k)); std::memset(BR1m, 0, sizeof(BR1m));
    num = 0; numIn1 = numIn1k = numIn1m = 0;
  }
  void finish() {
    std::memset(H, 0, sizeof(H));
    shiftUp(true);
    int idx = 0;
    for (int r = 0; r < 10; r++)
      for (int c = r; c < 10; c++) { H[r * 13 + c] = H[c * 13 + r] = Data1m[idx]; idx++; }
    idx = 0;
    for (int r = 0; r < 10; r++)
      for (int c = 0; c < 3; c++) { H[r * 13 + c + 10] = H[(c + 10) * 13 + r] = TR1m[idx]; idx++; }
    H[10 * 13 + 10] = BR1m[0];
    H[10 * 13 + 11] = H[11 * 13 + 10] = BR1m[1];
    H[10 * 13 + 12] = H[12 * 13 + 10] = BR1m[2];
    H[11 * 13 + 11] = BR1m[3];
    H[11 * 13 + 12] = H[12 * 13 + 11] = BR1m[4];
    H[12 * 13 + 12] = BR1m[5];
    num = (size_t)(numIn1 + numIn1k + numIn1m);
  }
  // update(x4,x6,y4,y6,a,b,c): Data[(r,c>=r)] += a*x_c*x_r + c*y_c*y_r + b*(x_c*y_r + y_c*x_r)
  void update(const float* x4, const float* x6, const float* y4, const float* y6, float a, float b, float c) {
    float x[10], y[10];
    for (int i = 0; i < 4; i++) { x[i] = x4[i]; y[i] = y4[i]; }
    for (int i = 0; i < 6; i++) { x[4 + i] = x6[i]; y[4 + i] = y6[i]; }
    int idx = 0;
    for (int r = 0; r < 10; r++)
      for (int cc = r; cc < 10; cc++) {
        Data[idx] += a * x[cc] * x[r] + c * y[cc] * y[r] + b * (x[cc] * y[r] + y[cc] * x[r]);
        idx++;
      }
    num++;
    numIn1++;
    shiftUp(false);
  }
  void updateTopRight(const float* x4, const float* x6, const float* y4, const float* y6, float TR00, float TR10,
                      float TR01, float TR11, float TR02, float TR12) {
    float x[10], y[10];
    for (int i = 0; i < 4; i++) { x[i] = x4[i]; y[i] = y4[i]; }
    for (int i = 0; i < 6; i++) { x[4 + i] = x6[i]; y[4 + i] = y6[i]; }
    for (int r = 0; r < 10; r++) {
      TR[3 * r + 0] += x[r] * TR00 + y[r] * TR10;
      TR[3 * r + 1] += x[r] * TR01 + y[r] * TR11;
      TR[3 * r + 2] += x[r] * TR02 + y[r] * TR12;
    }
  }
  void updateBotRight(float a00, float a01, float a02, float a11, float a12, float a22) {
    BR[0] += a00; BR[1] += a01; BR[2] += a02; BR[3] += a11; BR[4] += a12; BR[5] += a22;
  }
  void shiftUp(bool force) {
    if (numIn1 > 1000 || force) {
      for (int i = 0; i < 60; i++) { Data1k[i] = Data[i] + Data1k[i]; }
      for (int i = 0; i < 32; i++) { TR1k[i] = TR[i] + TR1k[i]; }
      for (int i = 0; i < 8; i++) { BR1k[i] = BR[i] + BR1k[i]; }
      numIn1k += numIn1; numIn1 = 0;
      std::memset(Data, 0, sizeof(Data)); std::memset(TR, 0, sizeof(TR)); std::memset(BR, 0, sizeof(BR));
    }
    if (numIn1k > 1000 || force) {
      for (int i = 0; i < 60; i++) { Data1m[i] = Data1k[i] + Data1m[i]; }
      for (int i = 0; i < 32; i++) { TR1m[i] = TR1k[i] + TR1m[i]; }
      for (int i = 0; i < 8; i++) { BR1m[i] = BR1k[i] + BR1m[i]; }
      numIn1m += numIn1k; numIn1k = 0;
      std::memset(Data1k, 0, sizeof(Data1k)); std::memset(TR1k, 0, sizeof(TR1k)); std::memset(BR1k, 0, sizeof(BR1k));
    }
  }
};

// Accumulator9: 45 upper-triangular entries x 4 SSE lanes.
struct Acc9 {
  float S[45 * 4], S1k[45 * 4], S1m[45 * 4];
  float H[81];
  size_t num;
  float numIn1, numIn1k, numIn1m;
  void initialize() {
    std::memset(S, 0, sizeof(S)); std::memset(S1k, 0, sizeof(S1k)); std::memset(S1m, 0, sizeof(S1m));
    std::memset(H, 0, sizeof(H));
    num = 0; numIn1 = numIn1k = numIn1m = 0;
  }
  void finish() {
    std::memset(H, 0, sizeof(H));
    shiftUp(true);
    int idx = 0;
    for (int r = 0; r < 9; r++)
      for (int c = r; c < 9; c++) {
        float d = S1m[idx + 0] + S1m[idx + 1] + S1m[idx + 2] + S1m[idx + 3];
        H[r * 9 + c] = H[c * 9 + r] = d;
        idx += 4;
      }
  }
  // updateSSE_eighted (Include/MatrixAccumulators.h:1091-1166): J[k][lane], w[lane]
  void updateSSE_eighted(const float J[9][4], const float w[4]) {
    float* pt = S;
    for (int r = 0; r < 9; r++) {
      float Jw[4];
      for (int l = 0; l < 4; l++) Jw[l] = J[r][l] * w[l];
      for (int c = r; c < 9; c++) {
        for (int l = 0; l < 4; l++) pt[l] = pt[l] + Jw[l] * J[c][l];
        pt += 4;
      }
    }
    num += 4;
    numIn1++;
    shiftUp(false);
  }
  // updateSSE (Include/MatrixAccumulators.h:1025-1087): J[k][lane], unweighted
  void updateSSE(const float J[9][4]) {
    float* pt = S;
    for (int r = 0; r < 9; r++)
      for (int c = r; c < 9; c++) {
        for (int l = 0; l < 4; l++) pt[l] = pt[l] + J[r][l] * J[c][l];
        pt += 4;
      }
    num += 4;
    numIn1++;
    shiftUp(false);
  }
  // updateSingleWeighted (Include/MatrixAccumulators.h:1242-1331), off = 0: lane 0 only;
  // the diagonal term is (J_r*J_r)*w, then J_r *= w for the rest of its row
  void updateSingleWeighted(const float Jin[9], float w) {
    float J[9];
    for (int k = 0; k < 9; k++) J[k] = Jin[k];
    float* pt = S;
    for (int r = 0; r < 9; r++) {
      *pt += J[r] * J[r] * w;
      pt += 4;
      J[r] *= w;
      for (int c = r + 1; c < 9; c++) {
        *pt += J[c] * J[r];
        pt += 4;
      }
    }
    num++;
    numIn1++;
    shiftUp(false);
  }
  void shiftUp(bool force) {
    if (numIn1 > 1000 || force) {
      for (int i = 0; i < 180; i++) S1k[i] = S[i] + S1k[i];
      numIn1k += numIn1; numIn1 = 0;
      std::memset(S, 0, sizeof(S));
    }
    if (numIn1k > 1000 || force) {
      for (int i = 0; i < 180; i++) S1m[i] = S1k[i] + S1m[i];
      numIn1m += numIn1k; numIn1k = 0;
      std::memset(S1k, 0, sizeof(S1k));
    }
  }
};

// Accumulator11 (Include/MatrixAccumulators.h:91-172): updateSingle adds to lane 0; finish() sets A
// from the 1m level.  Updates after finish() change num but not A (DirectRefinement relies on that).
struct Acc11 {
  float A;
  size_t num;
  float S[4], S1k[4], S1m[4];
  float numIn1, numIn1k, numIn1m;
  void initialize() {
    A = 0;
    std::memset(S, 0, sizeof(S)); std::memset(S1k, 0, sizeof(S1k)); std::memset(S1m, 0, sizeof(S1m));
    num = 0; numIn1 = numIn1k = numIn1m = 0;
  }
  void finish() {
    shiftUp(true);
    A = S1m[0] + S1m[1] + S1m[2] + S1m[3];
  }
  void updateSingle(float val) {
    S[0] += val;
    num++; numIn1++;
    shiftUp(false);
  }
  void shiftUp(bool force) {
    if (numIn1 > 1000 || force) {
      for (int l = 0; l < 4; l++) { S1k[l] = S[l] + S1k[l]; S[l] = 0; }
      numIn1k += numIn1; numIn1 = 0;
    }
    if (numIn1k > 1000 || force) {
      for (int l = 0; l < 4; l++) { S1m[l] = S1k[l] + S1m[l]; S1k[l] = 0; }
      numIn1m += numIn1k; numIn1k = 0;
    }
  }
};

}  // namespace hso
