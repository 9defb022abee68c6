// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.h for the parity status).
// Frame::CreateDirPyrs (Src/Frame.cpp:104-181) restated: DirPyr[lvl] as (I, dx, dy) float triplets and
// absSquaredGrad[lvl]; level sizes w >> lvl, h >> lvl (CalibData wpyr / hpyr).  The reference leaves dI of the
// first and last rows uninitialised: 0 here (and on the device).  No gamma weighting (PhotoUnDistL is null).
#include <cmath>
#include <cstddef>
#include <vector>

extern "C" void hso_dir_pyramid(int W, int H, int nlev, const float* img, float* out, float* absg) {
  std::vector<std::vector<float>> I(nlev);
  size_t o3 = 0, o1 = 0;
  for (int l = 0; l < nlev; l++) {
    const int wl = W >> l, hl = H >> l;
    I[l].assign((size_t)wl * hl, 0.f);
    if (l == 0) {
      for (int i = 0; i < wl * hl; i++) I[0][i] = img[i];
    } else {
      const int wm = W >> (l - 1);
      const std::vector<float>& P = I[l - 1];
      for (int y = 0; y < hl; y++)
        for (int x = 0; x < wl; x++)
          I[l][x + y * wl] = 0.25f * (P[2 * x + 2 * y * wm] + P[2 * x + 1 + 2 * y * wm] + P[2 * x + 2 * y * wm + wm] +
                                      P[2 * x + 1 + 2 * y * wm + wm]);
    }
    const std::vector<float>& L = I[l];
    for (int i = 0; i < wl * hl; i++) {
      float dx = 0.f, dy = 0.f, g = 0.f;
      if (i >= wl && i < wl * (hl - 1)) {
        dx = 0.5f * (L[i + 1] - L[i - 1]);
        dy = 0.5f * (L[i + wl] - L[i - wl]);
        if (!std::isfinite(dx)) dx = 0;
        if (!std::isfinite(dy)) dy = 0;
        g = dx * dx + dy * dy;
      }
      if (out) {
        out[o3 + 3 * i] = L[i];
        out[o3 + 3 * i + 1] = dx;
        out[o3 + 3 * i + 2] = dy;
      }
      if (absg) absg[o1 + i] = g;
    }
    o3 += (size_t)3 * wl * hl;
    o1 += (size_t)wl * hl;
  }
}
