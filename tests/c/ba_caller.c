/* A plain C99 caller of the BA boundary (include/hs_ba.h): builds a small synthetic window (3 keyframes of a
 * smooth 160x120 texture, 90 points with residuals into the other frames), then runs the calls the reference's
 * System would make per keyframe: set_window, optimize, the optimize tail (fix_linearization), the dormant
 * energies, the frame read-back.  Prints one line and exits 0 when every call returns HS_OK with finite energies.
 * Built by h-slam_amd/csrc/Makefile (gcc, no HIP headers): the header is consumable from C. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hs_ba.h"

#define W 160
#define H 120
#define NF 3
#define NPH 30 /* points per host */

static float img_at(int f, double x, double y, int ch) {
  const double sx = x + 3.0 * f, sy = y; /* frame f sees the texture shifted by 3 px */
  if (ch == 0) return (float)(128.0 + 50.0 * sin(sx / 7.0) * cos(sy / 9.0));
  if (ch == 1) return (float)(50.0 / 7.0 * cos(sx / 7.0) * cos(sy / 9.0));
  return (float)(-50.0 / 9.0 * sin(sx / 7.0) * sin(sy / 9.0));
}

#define CHECK(call)                                                        \
  do {                                                                     \
    int st_ = (call);                                                      \
    if (st_ != HS_OK) {                                                    \
      fprintf(stderr, "%s failed: %d (%s)\n", #call, st_, hs_last_error()); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(void) {
  static float imgs[NF][W * H * 3];
  for (int f = 0; f < NF; f++)
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++)
        for (int c = 0; c < 3; c++) imgs[f][(y * W + x) * 3 + c] = img_at(f, x, y, c);
  const float* img_ptrs[NF] = {imgs[0], imgs[1], imgs[2]};
  hs_camera cam = {W, H, 3, 0, 100.f, 100.f, 80.f, 60.f};
  hs_frame fr[NF];
  memset(fr, 0, sizeof(fr));
  for (int f = 0; f < NF; f++) {
    /* world -> cam: identity rotation, translation (-0.06 f, 0, 0): the 3-px shift at idepth 0.5 */
    const double q[7] = {0, 0, 0, 1, -0.06 * f, 0, 0};
    memcpy(fr[f].worldToCam_evalPT, q, sizeof(q));
    fr[f].ab_exposure = 1.f;
    fr[f].frameEnergyTH = 8 * 8 * 8;
    fr[f].id = f;
  }
  enum { NP = NF * NPH };
  static int host[NP], rp[NP * (NF - 1)], rt[NP * (NF - 1)];
  static float u[NP], v[NP], idp[NP], idz[NP], col[NP * 8], wgt[NP * 8];
  static const int pdx[8] = {0, -1, 1, -2, 0, 2, -1, 0}, pdy[8] = {-2, -1, -1, 0, 0, 0, 1, 2};
  int nr = 0;
  for (int p = 0; p < NP; p++) {
    const int h = p / NPH, k = p % NPH;
    host[p] = h;
    u[p] = 20.f + 12.f * (k % 10) + 0.37f * h;
    v[p] = 25.f + 30.f * (k / 10) + 0.21f * k;
    idp[p] = idz[p] = 0.5f;
    for (int j = 0; j < 8; j++) {
      col[p * 8 + j] = img_at(h, u[p] + pdx[j], v[p] + pdy[j], 0);
      wgt[p * 8 + j] = 1.f;
    }
    for (int t = 0; t < NF; t++)
      if (t != h) {
        rp[nr] = p;
        rt[nr] = t;
        nr++;
      }
  }
  hs_points pts = {NP, host, u, v, idp, idz, col, wgt, NULL};
  hs_residuals rs = {nr, rp, rt, NULL};
  hs_params prm;
  CHECK(hs_params_default(&prm));
  hs_ctx* ctx = NULL;
  CHECK(hs_create(&ctx, &prm, 0));
  CHECK(hs_ba_set_window(ctx, &cam, NF, fr, img_ptrs, &pts, &rs));
  double energies[16];
  int done = 0;
  CHECK(hs_ba_optimize(ctx, 15, 0, energies, &done)); /* 3 frames: 15 iterations; energies holds max_iters + 1 */
  static uint8_t drop[NP * (NF - 1)];
  static float relbl[NP], hdif[NP];
  static int ngood[NP];
  double efix = 0, eL = 0, eM = 0;
  CHECK(hs_ba_fix_linearization(ctx, &efix, drop, relbl, ngood, hdif));
  CHECK(hs_ba_calc_energies(ctx, &eL, &eM));
  double state[NF * 10], pose[NF * 7];
  CHECK(hs_ba_get_frames(ctx, state, NULL, pose, NULL));
  int ndrop = 0;
  for (int r = 0; r < nr; r++) ndrop += drop[r];
  hs_destroy(ctx);
  const int ok = isfinite(energies[0]) && isfinite(energies[done]) && isfinite(efix) && isfinite(eL) && isfinite(eM);
  printf("{\"iters\": %d, \"E0\": %.6g, \"E\": %.6g, \"E_fix\": %.6g, \"dropped\": %d, \"residuals\": %d, "
         "\"EL\": %.6g, \"EM\": %.6g}\n", done, energies[0], energies[done], efix, ndrop, nr, eL, eM);
  return ok ? 0 : 2;
}
