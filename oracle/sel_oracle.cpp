// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.h for the parity status).
// PixelSelector (Src/PixelSelector.cpp:14-418) restated: the randomPattern of the constructor (std::srand(3141592),
// rand() & 0xFF — the C library's generator, as the reference), makeHists, makeMaps (with its re-selection
// recursion and random sub-sampling) and select.  Inputs are Frame::DirPyr[0] (I, dx, dy) and absSquaredGrad of
// levels 0..2 (Src/Frame.cpp:104-181).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "oracle_common.h"

namespace hso {

struct Selector {
  hs_params P;
  int w, h;
  std::vector<unsigned char> randomPattern;
  std::vector<int> gradHist;
  std::vector<float> ths, thsSmoothed;
  int thsStep = 0, gradHistFrame = -1, currentPotential = 3;
};

// computeHistQuantil, :45-54
static int hist_quantil(const int* hist, float below) {
  int th = hist[0] * below + 0.5f;
  for (int i = 0; i < 90; i++) {
    th -= hist[i + 1];
    if (th < 0) return i;
  }
  return 90;
}

// makeHists, :57-117
static void make_hists(Selector& S, const float* const* grad, int id) {
  S.gradHistFrame = id;
  const float* mapmax0 = grad[0];
  const int w = S.w, h = S.h, w32 = w / 32, h32 = h / 32;
  S.thsStep = w32;
  for (int y = 0; y < h32; y++)
    for (int x = 0; x < w32; x++) {
      const float* map0 = mapmax0 + 32 * x + 32 * y * w;
      int* hist0 = S.gradHist.data();
      memset(hist0, 0, sizeof(int) * 50);
      for (int j = 0; j < 32; j++)
        for (int i = 0; i < 32; i++) {
          const int it = i + 32 * x, jt = j + 32 * y;
          if (it > w - 2 || jt > h - 2 || it < 1 || jt < 1) continue;
          int g = sqrtf(map0[i + j * w]);
          if (g > 48) g = 48;
          hist0[g + 1]++;
          hist0[0]++;
        }
      S.ths[x + y * w32] = hist_quantil(hist0, S.P.minGradHistCut) + S.P.minGradHistAdd;
    }
  for (int y = 0; y < h32; y++)
    for (int x = 0; x < w32; x++) {
      float sum = 0, num = 0;
      if (x > 0) {
        if (y > 0) { num++; sum += S.ths[x - 1 + (y - 1) * w32]; }
        if (y < h32 - 1) { num++; sum += S.ths[x - 1 + (y + 1) * w32]; }
        num++;
        sum += S.ths[x - 1 + (y)*w32];
      }
      if (x < w32 - 1) {
        if (y > 0) { num++; sum += S.ths[x + 1 + (y - 1) * w32]; }
        if (y < h32 - 1) { num++; sum += S.ths[x + 1 + (y + 1) * w32]; }
        num++;
        sum += S.ths[x + 1 + (y)*w32];
      }
      if (y > 0) { num++; sum += S.ths[x + (y - 1) * w32]; }
      if (y < h32 - 1) { num++; sum += S.ths[x + (y + 1) * w32]; }
      num++;
      sum += S.ths[x + y * w32];
      S.thsSmoothed[x + y * w32] = (sum / num) * (sum / num);
    }
}

static const float kDirections[16][2] = {
    {0, 1.0000},        {0.3827, 0.9239},  {0.1951, 0.9808},  {0.9239, 0.3827},  {0.7071, 0.7071},  {0.3827, -0.9239},
    {0.8315, 0.5556},   {0.8315, -0.5556}, {0.5556, -0.8315}, {0.9808, 0.1951},  {0.9239, -0.3827}, {0.7071, -0.7071},
    {0.5556, 0.8315},   {0.9808, -0.1951}, {1.0000, 0.0000},  {0.1951, -0.9808}};

// select, :265-415.  dirpyr0: (I, dx, dy) triplets; grad: absSquaredGrad levels 0..2.
static void select_px(Selector& S, const float* dirpyr0, const float* const* grad, float* map_out, int pot,
                      float thFactor, int n[3]) {
  const float* mapmax0 = grad[0];
  const float* mapmax1 = grad[1];
  const float* mapmax2 = grad[2];
  const int w = S.w, w1 = S.w >> 1, w2 = S.w >> 2, h = S.h;
  memset(map_out, 0, sizeof(float) * w * h);
  const float dw1 = S.P.gradDownweightPerLevel;
  const float dw2 = dw1 * dw1;
  int n3 = 0, n2 = 0, n4 = 0;
  auto dot = [&](int idx, const float* dir) { return dirpyr0[3 * idx + 1] * dir[0] + dirpyr0[3 * idx + 2] * dir[1]; };
  for (int y4 = 0; y4 < h; y4 += (4 * pot))
    for (int x4 = 0; x4 < w; x4 += (4 * pot)) {
      const int my3 = std::min((4 * pot), h - y4);
      const int mx3 = std::min((4 * pot), w - x4);
      int bestIdx4 = -1;
      float bestVal4 = 0;
      const float* dir4 = kDirections[S.randomPattern[n2] & 0xF];
      for (int y3 = 0; y3 < my3; y3 += (2 * pot))
        for (int x3 = 0; x3 < mx3; x3 += (2 * pot)) {
          const int x34 = x3 + x4, y34 = y3 + y4;
          const int my2 = std::min((2 * pot), h - y34);
          const int mx2 = std::min((2 * pot), w - x34);
          int bestIdx3 = -1;
          float bestVal3 = 0;
          const float* dir3 = kDirections[S.randomPattern[n2] & 0xF];
          for (int y2 = 0; y2 < my2; y2 += pot)
            for (int x2 = 0; x2 < mx2; x2 += pot) {
              const int x234 = x2 + x34, y234 = y2 + y34;
              const int my1 = std::min(pot, h - y234);
              const int mx1 = std::min(pot, w - x234);
              int bestIdx2 = -1;
              float bestVal2 = 0;
              const float* dir2 = kDirections[S.randomPattern[n2] & 0xF];
              for (int y1 = 0; y1 < my1; y1 += 1)
                for (int x1 = 0; x1 < mx1; x1 += 1) {
                  const int idx = x1 + x234 + w * (y1 + y234);
                  const int xf = x1 + x234, yf = y1 + y234;
                  if (xf < 4 || xf >= w - 5 || yf < 4 || yf > h - 4) continue;
                  const float pixelTH0 = S.thsSmoothed[(xf >> 5) + (yf >> 5) * S.thsStep];
                  const float pixelTH1 = pixelTH0 * dw1;
                  const float pixelTH2 = pixelTH1 * dw2;
                  const float ag0 = mapmax0[idx];
                  if (ag0 > pixelTH0 * thFactor) {
                    float dirNorm = fabsf((float)(dot(idx, dir2)));
                    if (!S.P.selectDirectionDistribution) dirNorm = ag0;
                    if (dirNorm > bestVal2) {
                      bestVal2 = dirNorm;
                      bestIdx2 = idx;
                      bestIdx3 = -2;
                      bestIdx4 = -2;
                    }
                  }
                  if (bestIdx3 == -2) continue;
                  const float ag1 = mapmax1[(int)(xf * 0.5f + 0.25f) + (int)(yf * 0.5f + 0.25f) * w1];
                  if (ag1 > pixelTH1 * thFactor) {
                    float dirNorm = fabsf((float)(dot(idx, dir3)));
                    if (!S.P.selectDirectionDistribution) dirNorm = ag1;
                    if (dirNorm > bestVal3) {
                      bestVal3 = dirNorm;
                      bestIdx3 = idx;
                      bestIdx4 = -2;
                    }
                  }
                  if (bestIdx4 == -2) continue;
                  const float ag2 = mapmax2[(int)(xf * 0.25f + 0.125) + (int)(yf * 0.25f + 0.125) * w2];
                  if (ag2 > pixelTH2 * thFactor) {
                    float dirNorm = fabsf((float)(dot(idx, dir4)));
                    if (!S.P.selectDirectionDistribution) dirNorm = ag2;
                    if (dirNorm > bestVal4) {
                      bestVal4 = dirNorm;
                      bestIdx4 = idx;
                    }
                  }
                }
              if (bestIdx2 > 0) {
                map_out[bestIdx2] = 1;
                bestVal3 = 1e10;
                n2++;
              }
            }
          if (bestIdx3 > 0) {
            map_out[bestIdx3] = 2;
            bestVal4 = 1e10;
            n3++;
          }
        }
      if (bestIdx4 > 0) {
        map_out[bestIdx4] = 4;
        n4++;
      }
    }
  n[0] = n2;
  n[1] = n3;
  n[2] = n4;
}

// makeMaps, :118-262 (the FAST branch is commented out in the reference)
static int make_maps(Selector& S, const float* dirpyr0, const float* const* grad, int id, float* map_out,
                     float density, int recursionsLeft, float thFactor) {
  float numHave = 0;
  const float numWant = density;
  float quotia;
  int idealPotential = S.currentPotential;
  {
    if (id != S.gradHistFrame) make_hists(S, grad, id);
    int n[3];
    select_px(S, dirpyr0, grad, map_out, S.currentPotential, thFactor, n);
    numHave = n[0] + n[1] + n[2];
    quotia = numWant / numHave;
    const float K = numHave * (S.currentPotential + 1) * (S.currentPotential + 1);
    idealPotential = sqrtf(K / numWant) - 1;
    if (idealPotential < 1) idealPotential = 1;
    if (recursionsLeft > 0 && quotia > 1.25 && S.currentPotential > 1) {
      if (idealPotential >= S.currentPotential) idealPotential = S.currentPotential - 1;
      S.currentPotential = idealPotential;
      return make_maps(S, dirpyr0, grad, id, map_out, density, recursionsLeft - 1, thFactor);
    } else if (recursionsLeft > 0 && quotia < 0.25) {
      if (idealPotential <= S.currentPotential) idealPotential = S.currentPotential + 1;
      S.currentPotential = idealPotential;
      return make_maps(S, dirpyr0, grad, id, map_out, density, recursionsLeft - 1, thFactor);
    }
  }
  int numHaveSub = numHave;
  if (quotia < 0.95) {
    const int wh = S.w * S.h;
    int rn = 0;
    const unsigned char charTH = 255 * quotia;
    for (int i = 0; i < wh; i++)
      if (map_out[i] != 0) {
        if (S.randomPattern[rn] > charTH) {
          map_out[i] = 0;
          numHaveSub--;
        }
        rn++;
      }
  }
  S.currentPotential = idealPotential;
  return numHaveSub;
}

}  // namespace hso

using namespace hso;

extern "C" {

void* hso_sel_create(const hs_params* params, int W, int H) {
  Selector* S = new Selector();
  if (params) S->P = *params;
  else params_default(&S->P);
  S->w = W;
  S->h = H;
  const int area = W * H;
  S->randomPattern.resize(area);
  std::srand(3141592);  // PixelSelector ctor, :18-20
  for (int i = 0; i < area; ++i) S->randomPattern[i] = rand() & 0xFF;
  S->gradHist.assign(100 * (1 + W / 32) * (1 + H / 32), 0);
  // the reference allocates (W/32)*(H/32)+100 floats, uninitialised (:28-29).  select reads past the w32 x h32
  // table for pixels in the last partial column / row of 32-blocks (W or H not a multiple of 32, e.g. KITTI
  // 1232x368): here those slack entries are 0 (a fresh allocation), sized to cover every index select forms.
  const size_t nths = std::max((size_t)(W / 32) * (H / 32) + 100, (size_t)(W / 32) * (H / 32 + 1) + 1);
  S->ths.assign(nths, 0.f);
  S->thsSmoothed.assign(nths, 0.f);
  return S;
}

void hso_sel_destroy(void* h) { delete (Selector*)h; }

int hso_sel_make_maps(void* h, int id, const float* dirpyr0, const float* absg0, const float* absg1,
                      const float* absg2, float density, int recursionsLeft, float thFactor, float* map_out) {
  const float* g[3] = {absg0, absg1, absg2};
  return make_maps(*(Selector*)h, dirpyr0, g, id, map_out, density, recursionsLeft, thFactor);
}

int hso_sel_potential(void* h) { return ((Selector*)h)->currentPotential; }
void hso_sel_set_potential(void* h, int p) { ((Selector*)h)->currentPotential = p; }
void hso_sel_random_pattern(void* h, unsigned char* out) {
  Selector* S = (Selector*)h;
  memcpy(out, S->randomPattern.data(), S->randomPattern.size());
}
void hso_sel_ths(void* h, float* ths, float* smoothed) {
  Selector* S = (Selector*)h;
  const int n = (S->w / 32) * (S->h / 32);
  for (int i = 0; i < n; i++) {
    ths[i] = S->ths[i];
    smoothed[i] = S->thsSmoothed[i];
  }
}

}  // extern "C"
