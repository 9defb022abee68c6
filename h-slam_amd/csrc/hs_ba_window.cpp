// hs_ba_window.cpp — the incremental keyframe window of include/hs_ba.h: EnergyFunctional::insertFrame / insertPoint /
// insertResidual / dropResidual / removePoint / marginalizeFrame / makeIDX (Src/EnergyFunctional.cpp:371-454,
// 456-543,632-646,819-840) and the System-level loops around them in AddKeyframe (Src/Mapping.cpp:12-140),
// removeOutliers (Src/FullSystemOptimize.cpp:575-598), linearizeAll(true)'s toRemove (:137-159) and marginalizeFrame
// (Src/FullSystemMarginalize.cpp:108-176).
//
// The host keeps a mirror of the window's structure only: frames (frameHessians order), each frame's point list
// (pointHessians order), each point's residual list (PointHessian::residuals order, as frame keys).  Edits change the
// mirror with the reference's own list semantics (push_back, swap-with-last removal, order-preserving frame removal).
// The device keeps every value.  A commit (makeIDX) writes the mirror's order into one pinned blob -- old position of
// every point (or its staged data), residual tables, the frame column map, HM / bM -- uploads it with one
// asynchronous copy, and one gather kernel (hs_win_kernels.hip) moves the device-resident point state into the new
// order.  No device allocation and no synchronous copy on the keyframe path.
#include <algorithm>
#include <cstring>
#include <vector>

#include "hs_ba_ctx.h"
#include "hs_pyr_kernels.h"

using namespace hs;

namespace {

int frame_index(const hs_ctx* c, int key) {
  for (int i = 0; i < (int)c->wframes.size(); i++)
    if (c->wframes[i].key == key) return i;
  return -1;
}

void set_loc(hs_ctx* c, int handle, int key, int idx) {
  if ((int)c->loc_key.size() <= handle) {
    c->loc_key.resize(handle + 1, -1);
    c->loc_idx.resize(handle + 1, -1);
  }
  c->loc_key[handle] = key;
  c->loc_idx[handle] = idx;
}

WinPoint* find_point(hs_ctx* c, int handle) {
  if (handle < 0 || handle >= (int)c->loc_key.size() || c->loc_key[handle] < 0) return nullptr;
  const int f = frame_index(c, c->loc_key[handle]);
  if (f < 0) return nullptr;
  return &c->wpts[f][c->loc_idx[handle]];
}

// the mirror of a committed window built by hs_ba_set_window (points keep the handles 0..nP-1)
void mirror_from_committed(hs_ctx* c) {
  c->wframes.assign(c->nF, WinFrame());
  c->wpts.assign(c->nF, {});
  for (int f = 0; f < c->nF; f++) {
    c->wframes[f].key = f;
    c->wframes[f].slot = c->img_slot[f];
    c->wframes[f].committed = f;
  }
  c->next_frame_key = c->nF;
  c->loc_key.assign(c->nP, -1);
  c->loc_idx.assign(c->nP, -1);
  int maxh = -1;
  for (int p = 0; p < c->nP; p++) {
    WinPoint w;
    w.handle = c->pt_handle[p];
    w.src = p;
    for (int q = 0; q < HS_MAXF; q++) {
      const int t = c->res_order[(size_t)p * 8 + q];
      if (t < 0) break;
      w.tgt[w.nres] = t;
      w.st[w.nres] = (uint8_t)HS_WIN_KEEP;
      w.nres++;
    }
    const int h = c->pt_host[p];
    set_loc(c, w.handle, h, (int)c->wpts[h].size());
    c->wpts[h].push_back(w);
    maxh = std::max(maxh, w.handle);
  }
  c->next_handle = maxh + 1;
  c->staged.clear();
  c->incremental = true;
}

int ensure_incremental(hs_ctx* c) {
  if (!c || !c->d_state || !c->haveCam) return fail(HS_ERR_STATE, "no capacity: hs_ba_reserve or hs_ba_set_window first");
  if (!c->incremental) mirror_from_committed(c);
  HS_HIP(hipSetDevice(c->device));
  return HS_OK;
}

// PointHessian::residuals: remove entry q by moving the last one into its place (EnergyFunctional::dropResidual)
void drop_at(WinPoint& w, int q) {
  w.tgt[q] = w.tgt[w.nres - 1];
  w.st[q] = w.st[w.nres - 1];
  w.nres--;
}

// flagPointsForRemoval / removeOutliers compaction of one frame's point list: a removed entry takes the list's last
// one, which is tested again (Src/Mapping.cpp:318-326, Src/FullSystemOptimize.cpp:587-595)
template <typename Pred>
void compact_list(hs_ctx* c, int f, Pred removed, std::vector<int>* out) {
  auto& v = c->wpts[f];
  const int key = c->wframes[f].key;
  for (int i = 0; i < (int)v.size(); i++) {
    while (i < (int)v.size() && removed(v[i])) {
      if (out) out->push_back(v[i].handle);
      c->loc_key[v[i].handle] = -1;
      v[i] = v.back();
      v.pop_back();
      if (i < (int)v.size()) set_loc(c, v[i].handle, key, i);
    }
  }
}

size_t align16(size_t b) { return (b + 15) & ~(size_t)15; }

}  // namespace

namespace hs {
size_t stage_bytes(int capP) {
  const size_t n = (size_t)capP;
  return align16(4 * n) + align16(32 * n) + align16(4 * n) + align16(8 * n) + align16(8 * n) + 64 +
         align16(sizeof(HsStagedPoint) * n) + align16(8 * (size_t)HS_MAXDIM * HS_MAXDIM) + align16(8 * HS_MAXDIM) + 256;
}

// makeIDX: the mirror's order onto the device (see the file comment)
int commit(hs_ctx* c) {
  if (!c->dirty) return HS_OK;
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(wait_uploads(c));
  const int nF = (int)c->wframes.size();
  int nP = 0;
  for (auto& l : c->wpts) nP += (int)l.size();
  if (nP > c->cap_P) return fail(HS_ERR_NOMEM, "window exceeds the reserved point capacity (hs_ba_reserve)");
  for (int f = 0; f < nF; f++)
    if (c->wframes[f].slot < 0) return fail(HS_ERR_STATE, "a window frame has no image");

  // ---- frames
  bool frames_changed = nF != c->nF;
  int col_src[HS_MAXF];
  float th_init[HS_MAXF];
  for (int f = 0; f < HS_MAXF; f++) {
    col_src[f] = f < nF ? c->wframes[f].committed : -1;
    th_init[f] = f < nF ? c->wframes[f].init.frameEnergyTH : 0.f;
    if (f < nF && col_src[f] != f) frames_changed = true;
  }
  if (frames_changed) {
    if (c->nF > 0 && !c->h_state_valid) HS_TRY(fetch_state(c));
    static thread_local HsDevState old;
    std::memcpy((void*)&old, (const void*)c->h_state, sizeof(HsDevState));
    HsDevState& S = *c->h_state;
    for (int f = 0; f < HS_MAXF; f++) {
      FrameH& F = S.frames[f];
      F = FrameH();
      if (f >= nF) continue;
      if (col_src[f] >= 0) {
        F = old.frames[col_src[f]];
      } else {  // EnergyFunctional::insertFrame: FrameOptimizationData::takeData on the inserted frame
        const hs_frame& in = c->wframes[f].init;
        F.id = in.id;
        F.ab_exposure = in.ab_exposure;
        F.frameEnergyTH = in.frameEnergyTH;
        F.evalPT = SE3::fromData(in.worldToCam_evalPT);
        F.setState(in.state);
        F.setStateZero(in.state_zero);
        F.takeData(c->P);
      }
      F.idx = f;
    }
    // a new window dimension: the solve's loop state starts fresh (as hs_ba_set_window's)
    std::memset(S.lastX, 0, sizeof(S.lastX));
    std::memset(S.cstep, 0, sizeof(S.cstep));
    S.iteration = S.status = S.log_count = S.canbreak = 0;
    c->nF = nF;
    HS_TRY(upload_frames(c));
    for (int f = 0; f < nF; f++) {
      c->img_slot[f] = c->wframes[f].slot;
      c->wframes[f].committed = f;
    }
    // the system vector's layout changed: no stale entry of the old layout stays in its (unread) lower triangle
    HS_HIP(hipMemsetAsync(c->d_sys, 0, sizeof(double) * ((size_t)HS_MAXDIM * HS_MAXDIM + HS_MAXDIM + 3 + HS_MAXF * 64),
                          c->stream));
  }

  // ---- points: the blob
  const int n = c->dim(), k = (int)c->staged.size();
  const size_t need = stage_bytes(c->cap_P);
  if (need > c->h_stage_cap) return fail(HS_ERR_STATE, "staging buffer not reserved");
  uint8_t* b = c->h_stage;
  size_t off = 0;
  auto take = [&](size_t bytes) { uint8_t* p = b + off; off += align16(bytes); return p; };
  int* src = (int*)take(4 * (size_t)nP);
  int* ros = (int*)take(32 * (size_t)nP);
  int* pth = (int*)take(4 * (size_t)nP);
  int8_t* rord = (int8_t*)take(8 * (size_t)nP);
  uint8_t* nres = take(8 * (size_t)nP);
  int* hpb = (int*)take(64);
  HsStagedPoint* stg = (HsStagedPoint*)take(sizeof(HsStagedPoint) * (size_t)std::max(k, 1));
  double* hm = (double*)take(8 * (size_t)n * n);
  double* bm = (double*)take(8 * (size_t)n);
  std::vector<int> key_idx(c->next_frame_key + 1, -1);
  for (int f = 0; f < nF; f++) key_idx[c->wframes[f].key] = f;
  c->pt_host.resize(nP);
  c->pt_handle.resize(nP);
  c->res_of_slot.assign((size_t)nP * 8, -1);
  c->res_order.assign((size_t)nP * 8, (int8_t)-1);
  c->res_point.clear();
  c->res_target.clear();
  c->host_pt_begin.assign(nF + 1, nP);
  int p = 0, r = 0;
  for (int f = 0; f < nF; f++) {
    c->host_pt_begin[f] = p;
    auto& v = c->wpts[f];
    for (int i = 0; i < (int)v.size(); i++, p++) {
      WinPoint& w = v[i];
      src[p] = w.src;
      pth[p] = f;
      for (int s = 0; s < 8; s++) {
        ros[p * 8 + s] = -1;
        rord[p * 8 + s] = -1;
        nres[p * 8 + s] = (uint8_t)HS_WIN_NONE;
      }
      for (int q = 0; q < w.nres; q++) {
        const int t = key_idx[w.tgt[q]];
        rord[p * 8 + q] = (int8_t)t;
        ros[p * 8 + t] = r;
        nres[p * 8 + t] = w.st[q];
        c->res_point.push_back(p);
        c->res_target.push_back(t);
        r++;
        w.st[q] = (uint8_t)HS_WIN_KEEP;
      }
      w.src = p;
      c->pt_host[p] = f;
      c->pt_handle[p] = w.handle;
      c->loc_idx[w.handle] = i;
    }
  }
  c->host_pt_begin[nF] = nP;
  for (int f = 0; f <= HS_MAXF; f++) hpb[f] = f <= nF ? c->host_pt_begin[f] : nP;
  std::memcpy(c->res_of_slot.data(), ros, sizeof(int) * 8 * (size_t)nP);
  std::memcpy(c->res_order.data(), rord, 8 * (size_t)nP);
  if (k > 0) std::memcpy(stg, c->staged.data(), sizeof(HsStagedPoint) * k);
  HS_TRY(sync_hm(c));
  if ((int)c->HM.size() != n * n) c->HM.assign((size_t)n * n, 0.0);
  if ((int)c->bM.size() != n) c->bM.assign(n, 0.0);
  std::memcpy(hm, c->HM.data(), 8 * (size_t)n * n);
  std::memcpy(bm, c->bM.data(), 8 * (size_t)n);
  c->hm_zero = std::all_of(c->HM.begin(), c->HM.end(), [](double x) { return x == 0.0; });
  const size_t bytes = off;
  HS_HIP(hipMemcpyAsync(c->d_stage, b, bytes, hipMemcpyHostToDevice, c->stream));
  HS_HIP(hipEventRecord(c->ev_upload, c->stream));
  const uint8_t* db = c->d_stage;
  auto dptr = [&](const void* hp) { return db + ((const uint8_t*)hp - b); };

  // ---- the gather (+ the index tables, HM / bM into place)
  HsWinGatherArgs a;
  std::memset(&a, 0, sizeof(a));
  a.n = nP;
  a.nF = nF;
  for (int f = 0; f < HS_MAXF; f++) {
    a.col_src[f] = frames_changed ? col_src[f] : f;
    a.th_init[f] = th_init[f];
  }
  a.src = (const int*)dptr(src);
  a.newres = dptr(nres);
  a.staged = (const HsStagedPoint*)dptr(stg);
  const PointSet& F = c->ps[c->cur];
  const PointSet& T = c->ps[c->cur ^ 1];
  a.from = {F.u, F.v, F.idepth, F.idepth_zero, F.priorF, F.color, F.weight, F.relBL, F.nGood, F.r_state, F.r_center};
  a.to = {T.u, T.v, T.idepth, T.idepth_zero, T.priorF, T.color, T.weight, T.relBL, T.nGood, T.r_state, T.r_center};
  float* hdif_dst = c->hdif_solved == c->d_p_HdiF ? c->d_p_HdiF_alt : c->d_p_HdiF;
  a.hdif_from = c->hdif_solved;
  a.hdif_to = hdif_dst;
  a.frameTH = c->d_frameTH;
  const int grid = std::max(1, (nP * 8 + 255) / 256);
  hipLaunchKernelGGL(hs_k_win_gather, dim3(grid), dim3(256), 0, c->stream, a);
  HS_HIP(hipGetLastError());
  HS_HIP(hipMemcpyAsync(c->d_res_of_slot, dptr(ros), 32 * (size_t)nP, hipMemcpyDeviceToDevice, c->stream));
  HS_HIP(hipMemcpyAsync(c->d_res_order, dptr(rord), 8 * (size_t)nP, hipMemcpyDeviceToDevice, c->stream));
  HS_HIP(hipMemcpyAsync(c->d_pt_host, dptr(pth), 4 * (size_t)nP, hipMemcpyDeviceToDevice, c->stream));
  HS_HIP(hipMemcpyAsync(c->d_host_pt_begin, dptr(hpb), 4 * (HS_MAXF + 1), hipMemcpyDeviceToDevice, c->stream));
  HS_HIP(hipMemcpyAsync(c->d_HM, dptr(hm), 8 * (size_t)n * n, hipMemcpyDeviceToDevice, c->stream));
  HS_HIP(hipMemcpyAsync(c->d_bM, dptr(bm), 8 * (size_t)n, hipMemcpyDeviceToDevice, c->stream));
  if (nP < c->nP || c->cand_stride != c->cap_stride)  // this rank's stale newest-frame candidates -> none (NaN)
    HS_HIP(hipMemsetAsync(c->d_cand + (size_t)c->rank * c->cap_stride + nP, 0xff,
                          sizeof(float) * (size_t)(c->cap_stride - nP), c->stream));
  c->cur ^= 1;
  bind_point_set(c);
  c->d_p_HdiF_alt = c->hdif_solved;
  c->d_p_HdiF = hdif_dst;
  c->hdif_solved = hdif_dst;
  c->staged.clear();
  c->nP = nP;
  c->nR = r;
  c->cand_stride = c->cap_stride;
  HS_TRY(make_partition(c));
  drop_graph(c);
  c->haveSystem = false;
  c->sepValid = false;
  c->tail_valid = false;
  c->dirty = false;
  return HS_OK;
}

}  // namespace hs

extern "C" {

int hs_ba_reserve(hs_ctx* c, const hs_camera* cam, int max_points) {
  if (!c || !cam) return fail(HS_ERR_INVALID, "null argument");
  if (cam->width < 8 || cam->height < 8 || max_points < 1) return fail(HS_ERR_INVALID, "bad camera size / capacity");
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(wait_stream(c));
  HS_TRY(ensure_capacity(c, cam->width, cam->height, max_points, max_blocks_for(max_points)));
  drop_graph(c);
  c->cam = *cam;
  c->haveCam = true;
  c->nF = c->nP = c->nR = 0;
  c->blk_begin.assign(1, 0);
  c->host_pt_begin.assign(1, 0);
  c->pt_host.clear(); c->pt_handle.clear(); c->res_point.clear(); c->res_target.clear();
  c->res_of_slot.clear(); c->res_order.clear();
  c->nblk = 0;
  c->wframes.clear(); c->wpts.clear(); c->staged.clear(); c->loc_key.clear(); c->loc_idx.clear();
  c->next_handle = 0;
  c->next_frame_key = 0;
  c->incremental = true;
  c->dirty = false;
  c->haveSystem = false;
  c->sepValid = false;
  c->HM.clear();
  c->bM.clear();
  c->hm_zero = true;
  c->hm_host_stale = false;
  c->cand_stride = c->cap_stride;
  c->cur = 0;
  bind_point_set(c);
  c->hdif_solved = c->d_p_HdiF;
  // the calibration of the (empty) window: CalibData's ctor (setValueScaled, value_zero = value)
  HS_TRY(wait_uploads(c));
  HsDevState& S = *c->h_state;
  std::memset((void*)&S, 0, sizeof(HsDevState));
  CalibH& cal = S.calib;
  cal.W = cam->width;
  cal.H = cam->height;
  double vs[4] = {cam->fx, cam->fy, cam->cx, cam->cy};
  cal.setValueScaled(vs);
  for (int i = 0; i < 4; i++) {
    cal.value_zero[i] = cal.value[i];
    cal.value_minus_value_zero[i] = 0;
    cal.step[i] = 0;
    cal.value_backup[i] = cal.value[i];
  }
  S.dcal = cal.device();
  c->h_state_valid = true;
  c->tail_pending = false;
  HS_HIP(hipMemsetAsync(c->d_cand, 0xff, sizeof(float) * (size_t)c->cap_stride * c->nranks, c->stream));
  HS_TRY(wait_stream(c));
  return HS_OK;
}

int hs_ba_insert_frame(hs_ctx* c, const hs_frame* frame, const float* image) {
  if (!frame) return fail(HS_ERR_INVALID, "null frame");
  HS_TRY(ensure_incremental(c));
  if ((int)c->wframes.size() >= HS_MAXF) return fail(HS_ERR_INVALID, "window is full (HS_MAX_FRAMES frames)");
  bool used[HS_MAXF] = {false};
  for (auto& f : c->wframes) used[f.slot] = true;
  int slot = 0;
  while (slot < HS_MAXF && used[slot]) slot++;
  WinFrame w;
  w.key = c->next_frame_key++;
  w.slot = slot;
  w.committed = -1;
  w.init = *frame;
  c->wframes.push_back(w);
  c->wpts.emplace_back();
  // HM.conservativeResize + zero the new rows / columns (Src/EnergyFunctional.cpp:389-394)
  HS_TRY(sync_hm(c));
  const int n1 = 4 + 8 * ((int)c->wframes.size() - 1), n2 = n1 + 8;
  std::vector<double> HM((size_t)n2 * n2, 0.0), bM(n2, 0.0);
  if ((int)c->HM.size() == n1 * n1)
    for (int i = 0; i < n1; i++)
      for (int j = 0; j < n1; j++) HM[(size_t)i * n2 + j] = c->HM[(size_t)i * n1 + j];
  if ((int)c->bM.size() == n1)
    for (int i = 0; i < n1; i++) bM[i] = c->bM[i];
  c->HM.swap(HM);
  c->bM.swap(bM);
  c->dirty = true;
  if (image) HS_TRY(hs_ba_set_frame_image(c, (int)c->wframes.size() - 1, image));
  return HS_OK;
}

static int frame_slot_ptr(hs_ctx* c, int frame, float4** dst) {
  HS_TRY(ensure_incremental(c));
  if (frame < 0 || frame >= (int)c->wframes.size()) return fail(HS_ERR_INVALID, "frame index out of range");
  *dst = c->d_img_all + (size_t)c->wframes[frame].slot * c->img_px;
  return HS_OK;
}

int hs_ba_set_frame_image(hs_ctx* c, int frame, const float* image) {
  float4* dst = nullptr;
  if (!image) return fail(HS_ERR_INVALID, "null image");
  HS_TRY(frame_slot_ptr(c, frame, &dst));
  // (I, dI/dx, dI/dy) triplets -> float4 texels on the host, one synchronous copy (the host-image path; the raw and
  // device paths below avoid both)
  std::vector<float4> tex(c->img_px);
  for (size_t i = 0; i < c->img_px; i++) tex[i] = make_float4(image[3 * i], image[3 * i + 1], image[3 * i + 2], 0.f);
  HS_HIP(hipMemcpyAsync(dst, tex.data(), c->img_px * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HS_TRY(pack_slot(c, c->wframes[frame].slot));
  HS_TRY(wait_stream(c));
  return HS_OK;
}

int hs_ba_set_frame_image_raw(hs_ctx* c, int frame, const float* raw) {
  float4* dst = nullptr;
  if (!raw) return fail(HS_ERR_INVALID, "null image");
  HS_TRY(frame_slot_ptr(c, frame, &dst));
  if (!c->h_raw || !c->d_raw) return fail(HS_ERR_STATE, "no raw staging (hs_ba_reserve)");
  HS_TRY(wait_uploads(c));
  std::memcpy(c->h_raw, raw, sizeof(float) * c->img_px);  // pinned: the upload below is asynchronous
  HS_HIP(hipMemcpyAsync(c->d_raw, c->h_raw, sizeof(float) * c->img_px, hipMemcpyHostToDevice, c->stream));
  HS_HIP(hipEventRecord(c->ev_upload, c->stream));
  float4* lv[1] = {dst};
  HS_HIP(hs_build_dir_pyramid(c->stream, c->d_raw, c->cam.width, c->cam.height, 1, lv, nullptr));
  return pack_slot(c, c->wframes[frame].slot);
}

}  // extern "C"

namespace hs {
// window frame `frame`'s image from device texels, ordered on the context's stream; no host synchronisation
int copy_frame_image_device(hs_ctx* c, int frame, const void* d_texels) {
  float4* dst = nullptr;
  if (!d_texels) return fail(HS_ERR_INVALID, "null texels");
  HS_TRY(frame_slot_ptr(c, frame, &dst));
  HS_HIP(hipMemcpyAsync(dst, d_texels, c->img_px * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
  return pack_slot(c, c->wframes[frame].slot);
}
}  // namespace hs

extern "C" {

int hs_ba_set_frame_image_device(hs_ctx* c, int frame, const void* d_texels) {
  HS_TRY(hs::copy_frame_image_device(c, frame, d_texels));
  // the source is foreign memory whose producer this context cannot order against: the copy must have read it
  // before this call returns (hs_tracker_frame_to_ba orders the tracker's hand-off on the device instead)
  HS_TRY(wait_stream(c));
  return HS_OK;
}

int hs_ba_insert_points(hs_ctx* c, const hs_points* pts, const float* relBL, const int* nGood, int* handles_out) {
  if (!pts || pts->n < 0 || (pts->n > 0 && (!pts->host || !pts->u || !pts->v || !pts->idepth || !pts->idepth_zero ||
                                           !pts->color || !pts->weights)))
    return fail(HS_ERR_INVALID, "bad points");
  HS_TRY(ensure_incremental(c));
  const int nF = (int)c->wframes.size();
  for (int i = 0; i < pts->n; i++)
    if (pts->host[i] < 0 || pts->host[i] >= nF) return fail(HS_ERR_INVALID, "bad point host");
  if ((int)c->staged.size() + pts->n > c->cap_P) return fail(HS_ERR_NOMEM, "too many points staged");
  for (int i = 0; i < pts->n; i++) {
    HsStagedPoint s;
    s.u = pts->u[i];
    s.v = pts->v[i];
    s.idepth = pts->idepth[i];
    s.idepth_zero = pts->idepth_zero[i];
    // MapPointOptimizationData::takeData: priorF = hasDepthPrior ? setting_idepthFixPrior * SCALE_IDEPTH^2 : 0
    s.priorF = (pts->has_depth_prior && pts->has_depth_prior[i]) ? c->P.idepthFixPrior * 1.0f * 1.0f : 0.f;
    s.relBL = relBL ? relBL[i] : 0.f;
    s.nGood = nGood ? nGood[i] : 0;
    for (int q = 0; q < 8; q++) {
      s.color[q] = pts->color[i * 8 + q];
      s.weight[q] = pts->weights[i * 8 + q];
    }
    WinPoint w;
    w.handle = c->next_handle++;
    w.src = -(1 + (int)c->staged.size());
    c->staged.push_back(s);
    const int f = pts->host[i];
    set_loc(c, w.handle, c->wframes[f].key, (int)c->wpts[f].size());
    c->wpts[f].push_back(w);
    if (handles_out) handles_out[i] = w.handle;
  }
  if (pts->n > 0) c->dirty = true;
  return HS_OK;
}

static int add_residual(hs_ctx* c, WinPoint* w, int host_key, int t, uint8_t st) {
  if (!w) return fail(HS_ERR_INVALID, "unknown point handle");
  if (t < 0 || t >= (int)c->wframes.size()) return fail(HS_ERR_INVALID, "bad residual target");
  const int key = c->wframes[t].key;
  if (key == host_key) return fail(HS_ERR_INVALID, "residual target == host");
  for (int q = 0; q < w->nres; q++)
    if (w->tgt[q] == key) return fail(HS_ERR_INVALID, "duplicate (point, target) residual");
  if (w->nres >= HS_MAXF - 1) return fail(HS_ERR_INVALID, "residual list full");
  if (st > HS_RES_OUT) return fail(HS_ERR_INVALID, "bad residual state");
  w->tgt[w->nres] = key;
  w->st[w->nres] = st;
  w->nres++;
  c->dirty = true;
  return HS_OK;
}

int hs_ba_insert_residuals(hs_ctx* c, int n, const int* handles, const int* targets, const uint8_t* states) {
  if (n < 0 || (n > 0 && (!handles || !targets))) return fail(HS_ERR_INVALID, "bad residual list");
  HS_TRY(ensure_incremental(c));
  for (int i = 0; i < n; i++) {
    WinPoint* w = find_point(c, handles[i]);
    HS_TRY(add_residual(c, w, w ? c->loc_key[handles[i]] : -1, targets[i], states ? states[i] : (uint8_t)HS_RES_IN));
  }
  return HS_OK;
}

int hs_ba_add_residuals_to_newest(hs_ctx* c, int* n_added) {
  HS_TRY(ensure_incremental(c));
  const int nF = (int)c->wframes.size();
  if (nF < 1) return fail(HS_ERR_STATE, "empty window");
  int cnt = 0;
  for (int f = 0; f < nF - 1; f++)
    for (auto& w : c->wpts[f]) {
      HS_TRY(add_residual(c, &w, c->wframes[f].key, nF - 1, (uint8_t)HS_RES_IN));
      cnt++;
    }
  if (n_added) *n_added = cnt;
  return HS_OK;
}

int hs_ba_drop_residuals(hs_ctx* c, int n, const int* handles, const int* targets) {
  if (n < 0 || (n > 0 && (!handles || !targets))) return fail(HS_ERR_INVALID, "bad residual list");
  HS_TRY(ensure_incremental(c));
  for (int i = 0; i < n; i++) {
    WinPoint* w = find_point(c, handles[i]);
    if (!w) return fail(HS_ERR_INVALID, "unknown point handle");
    if (targets[i] < 0 || targets[i] >= (int)c->wframes.size()) return fail(HS_ERR_INVALID, "bad target");
    const int key = c->wframes[targets[i]].key;
    int q = 0;
    while (q < w->nres && w->tgt[q] != key) q++;
    if (q == w->nres) return fail(HS_ERR_INVALID, "no such residual");
    drop_at(*w, q);
    c->dirty = true;
  }
  return HS_OK;
}

int hs_ba_drop_inactive_residuals(hs_ctx* c, int* n_dropped) {
  HS_TRY(ensure_incremental(c));
  if (c->dirty) return fail(HS_ERR_STATE, "the window changed since hs_ba_fix_linearization");
  if (!c->tail_valid) return fail(HS_ERR_STATE, "hs_ba_fix_linearization must run first");
  // the tail's active flags through the context's pinned staging (a pageable copy is a synchronous staged one)
  HS_HIP(c->rb_stage((size_t)std::max(c->nP, 1) * 8));
  const uint8_t* act = c->h_rb;
  if (c->nP > 0) {
    c->rb_pending = true;
    HS_HIP(hipMemcpyAsync(c->h_rb, c->d_r_active, (size_t)c->nP * 8, hipMemcpyDeviceToHost, c->stream));
    HS_TRY(wait_stream(c));
    c->rb_pending = false;
  }
  // toRemove in activeResiduals order (points in window order, each list in order), then dropResidual one by one
  int cnt = 0, p = 0;
  for (int f = 0; f < (int)c->wframes.size(); f++)
    for (auto& w : c->wpts[f]) {
      int rm[HS_MAXF], m = 0;
      for (int q = 0; q < w.nres; q++) {
        int t = -1;
        for (int g = 0; g < (int)c->wframes.size(); g++)
          if (c->wframes[g].key == w.tgt[q]) t = g;
        if (!act[(size_t)p * 8 + t]) rm[m++] = w.tgt[q];
      }
      for (int i = 0; i < m; i++) {
        int q = 0;
        while (w.tgt[q] != rm[i]) q++;
        drop_at(w, q);
      }
      cnt += m;
      p++;
    }
  if (cnt > 0) c->dirty = true;
  if (n_dropped) *n_dropped = cnt;
  return HS_OK;
}

int hs_ba_remove_points(hs_ctx* c, int n, const int* handles) {
  if (n < 0 || (n > 0 && !handles)) return fail(HS_ERR_INVALID, "bad point list");
  HS_TRY(ensure_incremental(c));
  std::vector<uint8_t> mark(c->loc_key.size(), 0);
  for (int i = 0; i < n; i++) {
    if (!find_point(c, handles[i])) return fail(HS_ERR_INVALID, "unknown point handle");
    mark[handles[i]] = 1;
  }
  for (int f = 0; f < (int)c->wframes.size(); f++)
    compact_list(c, f, [&](const WinPoint& w) { return mark[w.handle] != 0; }, nullptr);
  if (n > 0) c->dirty = true;
  return HS_OK;
}

int hs_ba_remove_points_without_residuals(hs_ctx* c, int* handles_out, int* n_out) {
  HS_TRY(ensure_incremental(c));
  std::vector<int> out;
  for (int f = 0; f < (int)c->wframes.size(); f++)
    compact_list(c, f, [](const WinPoint& w) { return w.nres == 0; }, &out);
  if (!out.empty()) c->dirty = true;
  if (handles_out && !out.empty()) std::memcpy(handles_out, out.data(), sizeof(int) * out.size());
  if (n_out) *n_out = (int)out.size();
  return HS_OK;
}

int hs_ba_remove_frame(hs_ctx* c, int frame, int marginalize) {
  HS_TRY(ensure_incremental(c));
  if (frame < 0 || frame >= (int)c->wframes.size()) return fail(HS_ERR_INVALID, "frame index out of range");
  if (!c->wpts[frame].empty()) return fail(HS_ERR_STATE, "the frame still hosts points (remove them first)");
  // The prior's Schur complement needs the committed frame state and HM / bM.  Pending point-only changes (removed
  // points, dropped residuals, staged points) leave both as committed and the frame order unchanged, so they stay
  // pending: the next commit takes them together with this removal (one commit per keyframe instead of two).
  bool frames_pending = (int)c->wframes.size() != c->nF;
  for (int f = 0; f < (int)c->wframes.size() && !frames_pending; f++) frames_pending = c->wframes[f].committed != f;
  if (frames_pending) HS_TRY(commit_if_dirty(c));
  if (marginalize && !c->h_state_valid) HS_TRY(fetch_state(c));  // one read-back for the state and HM / bM
  HS_TRY(sync_hm(c));
  const int od = c->dim(), nd = od - 8, f0 = 4 + 8 * frame;
  std::vector<double> HMn, bMn;
  if (marginalize) {
    HS_TRY(marginalize_frame_prior(c, frame, HMn, bMn));
  } else {  // the frame's rows / columns dropped
    HMn.assign((size_t)nd * nd, 0.0);
    bMn.assign(nd, 0.0);
    for (int i = 0, ii = 0; i < od; i++) {
      if (i >= f0 && i < f0 + 8) continue;
      bMn[ii] = c->bM[i];
      for (int j = 0, jj = 0; j < od; j++) {
        if (j >= f0 && j < f0 + 8) continue;
        HMn[(size_t)ii * nd + jj] = c->HM[(size_t)i * od + j];
        jj++;
      }
      ii++;
    }
  }
  // drop all observations of existing points in that frame (window order; one residual per point)
  const int key = c->wframes[frame].key;
  for (int f = 0; f < (int)c->wframes.size(); f++) {
    if (f == frame) continue;
    for (auto& w : c->wpts[f])
      for (int q = 0; q < w.nres; q++)
        if (w.tgt[q] == key) {
          drop_at(w, q);
          break;
        }
  }
  c->wframes.erase(c->wframes.begin() + frame);
  c->wpts.erase(c->wpts.begin() + frame);
  c->HM.swap(HMn);
  c->bM.swap(bMn);
  c->dirty = true;
  return HS_OK;
}

int hs_ba_make_idx(hs_ctx* c, int* nF, int* nP, int* nR) {
  HS_TRY(ensure_incremental(c));
  HS_TRY(commit_if_dirty(c));
  if (nF) *nF = c->nF;
  if (nP) *nP = c->nP;
  if (nR) *nR = c->nR;
  return HS_OK;
}

int hs_ba_get_structure(hs_ctx* c, int* handles, int* pt_host, int* nres, int* res_target) {
  HS_TRY(ensure_incremental(c));
  HS_TRY(commit_if_dirty(c));
  for (int p = 0; p < c->nP; p++) {
    if (handles) handles[p] = c->pt_handle[p];
    if (pt_host) pt_host[p] = c->pt_host[p];
    if (nres) {
      int m = 0;
      while (m < 8 && c->res_order[(size_t)p * 8 + m] >= 0) m++;
      nres[p] = m;
    }
  }
  if (res_target)
    for (int r = 0; r < c->nR; r++) res_target[r] = c->res_target[r];
  return HS_OK;
}

}  // extern "C"

extern "C" {

int hs_ba_synchronize(hs_ctx* c) {
  if (!c) return fail(HS_ERR_INVALID, "null context");
  HS_HIP(hipSetDevice(c->device));
  HS_TRY(wait_stream(c));
  return HS_OK;
}

int hs_ba_get_marginal_prior(hs_ctx* c, double* HM, double* bM) {
  HS_TRY(ensure_incremental(c));
  HS_TRY(commit_if_dirty(c));
  HS_TRY(sync_hm(c));
  const int n = c->dim();
  if (HM) {
    if ((int)c->HM.size() == n * n) std::memcpy(HM, c->HM.data(), sizeof(double) * n * n);
    else std::memset(HM, 0, sizeof(double) * n * n);
  }
  if (bM) {
    if ((int)c->bM.size() == n) std::memcpy(bM, c->bM.data(), sizeof(double) * n);
    else std::memset(bM, 0, sizeof(double) * n);
  }
  return HS_OK;
}

int hs_ba_get_point_state(hs_ctx* c, float* idepth, float* idepth_zero, float* relBL, int* nGood, float* HdiF) {
  HS_TRY(ensure_incremental(c));
  HS_TRY(commit_if_dirty(c));
  const size_t n = c->nP;
  if (n == 0) return HS_OK;
  // through the context's pinned staging: asynchronous copies, one sync, then host copies
  HS_HIP(c->rb_stage(5 * n * 4));
  void* dst[5] = {idepth, idepth_zero, relBL, nGood, HdiF};
  const void* src[5] = {c->d_idepth, c->d_idepth_zero, c->d_fix_relBL, c->d_fix_nGood, c->hdif_solved};
  c->rb_pending = true;
  for (int k = 0; k < 5; k++)
    if (dst[k]) HS_HIP(hipMemcpyAsync(c->h_rb + k * n * 4, src[k], n * 4, hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  c->rb_pending = false;
  for (int k = 0; k < 5; k++)
    if (dst[k]) std::memcpy(dst[k], c->h_rb + k * n * 4, n * 4);
  return HS_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- test hooks (not part of include/hs_ba.h)
// The device window state (HsDevState: frames, calib, loop state) as a blob: tests/test_gpu_window.py transplants
// it into a context rebuilt with hs_ba_set_window, so both run from the same fp64 frame state; setting it re-runs
// setAdjointsF / setPrecalcValues / the projector on it, as a commit does.
extern "C" int hs_debug_state_size(void) { return (int)sizeof(HsDevState); }
extern "C" int hs_debug_get_state(hs_ctx* c, void* out) {
  if (!c || !out) return fail(HS_ERR_INVALID, "null");
  HS_TRY(commit_if_dirty(c));
  HS_TRY(fetch_state(c));
  std::memcpy(out, c->h_state, sizeof(HsDevState));
  return HS_OK;
}
// The largest |difference| between the nullspaces the DEVICE state holds for each frame and setStateZero's
// (Include/Frame.h:166-190) recomputed from that frame's evalPT: 0 when no frame's device copy is stale.
extern "C" int hs_debug_nullspace_error(hs_ctx* c, double* err_out) {
  if (!c || !err_out || c->nF == 0) return fail(HS_ERR_INVALID, "null / no window");
  HS_TRY(commit_if_dirty(c));
  if (c->tail_pending) HS_TRY(fetch_state(c));  // settles the moved newest frame (host and device copies)
  HsDevState dev;
  HS_HIP(hipMemcpyAsync(&dev, c->d_state, sizeof(HsDevState), hipMemcpyDeviceToHost, c->stream));
  HS_TRY(wait_stream(c));
  double e = 0;
  for (int f = 0; f < c->nF; f++) {
    hs::FrameH r = dev.frames[f];
    double sz[10];
    std::memcpy(sz, r.state_zero, sizeof(sz));
    r.setStateZero(sz);
    for (int i = 0; i < 6; i++) {
      e = std::max(e, std::fabs(r.nullspaces_scale[i] - dev.frames[f].nullspaces_scale[i]));
      for (int k = 0; k < 6; k++) e = std::max(e, std::fabs(r.nullspaces_pose[i][k] - dev.frames[f].nullspaces_pose[i][k]));
    }
  }
  *err_out = e;
  return HS_OK;
}
extern "C" int hs_debug_set_state(hs_ctx* c, const void* in) {
  if (!c || !in || c->nF == 0) return fail(HS_ERR_INVALID, "null / no window");
  HS_TRY(commit_if_dirty(c));
  HS_TRY(wait_uploads(c));
  std::memcpy((void*)c->h_state, in, sizeof(HsDevState));
  if (c->h_state->nF != c->nF) return fail(HS_ERR_INVALID, "state of a different window size");
  HS_TRY(upload_frames(c));
  HS_TRY(wait_stream(c));
  return HS_OK;
}
