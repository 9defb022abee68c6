// hs_track.cpp — C-ABI implementation of the CoarseTracker boundary (include/hs_track.h): tracker context,
// device pyramids / reference points, makeCoarseDepthL0 launches, the hypothesis kernel and the exact
// host replay of trackNewestCoarse's early abort and System::trackNewCoarse's try loop.
#include <hip/hip_runtime.h>

#include <cmath>
#include <algorithm>
#include <cstring>
#include <string>
#include <chrono>
#include <vector>

#include "../../include/hs_ba.h"
#include "../../include/hs_track.h"
#include "hs_ba_ctx.h"
#include "hs_track_kernels.h"
#include "hs_pyr_kernels.h"

namespace {
int tfail(int code, const std::string& msg) {
  hs::g_err = msg;
  return code;
}
}  // namespace

#define TS_HIP(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return tfail(HS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define TS_TRY(x)        \
  do {                   \
    int rc_ = (x);       \
    if (rc_) return rc_; \
  } while (0)

// a captured makeCoarseDepthL0 (make_depth_l0 from a device count): ~32 launches and copies, replayed as one graph;
// keyed by everything its launches bake in (the reference pyramid's level pointers swap on a promoted frame)
struct DepthGraph {
  const int* d_n = nullptr;
  const float* pts = nullptr;
  int stride = 0;
  const void* ref[HS_TRK_MAXLEV] = {};
  hipGraphExec_t exec = nullptr;
};

struct hs_tracker {
  hs_params P;
  int device = 0;
  DepthGraph dg[2];
  int dg_next = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;  // the per-call event pair (hs_tracker_set_event_timing, off by default)
  hipEvent_t ev_handoff = nullptr;        // cross-stream hand-offs with a BA context (set_ref_ba, frame_to_ba)
  int evt = 0;                            // hs_tracker_set_event_timing
  int W = 0, H = 0, nlev = 0;
  int w[HS_TRK_MAXLEV], h[HS_TRK_MAXLEV];
  float fx[HS_TRK_MAXLEV], fy[HS_TRK_MAXLEV], cx[HS_TRK_MAXLEV], cy[HS_TRK_MAXLEV], Ki[HS_TRK_MAXLEV][9];
  float4* d_ref[HS_TRK_MAXLEV] = {nullptr};
  float4* d_new[HS_TRK_MAXLEV] = {nullptr};
  float *d_id[HS_TRK_MAXLEV] = {nullptr}, *d_ws[HS_TRK_MAXLEV] = {nullptr}, *d_bak[HS_TRK_MAXLEV] = {nullptr};
  float *d_pu[HS_TRK_MAXLEV] = {nullptr}, *d_pv[HS_TRK_MAXLEV] = {nullptr}, *d_pid[HS_TRK_MAXLEV] = {nullptr},
        *d_pcol[HS_TRK_MAXLEV] = {nullptr};
  int* d_pcn = nullptr;
  int *d_bcnt = nullptr, *d_boff = nullptr;
  float *d_pts = nullptr;  // cu | cv | cid | hdi
  float* d_raw = nullptr;  // staging of a raw level-0 frame (hs_tracker_set_frame_raw)
  int pts_cap = 0;
  double* d_Tin = nullptr;
  HsTryOut* d_out = nullptr;
  double* d_part = nullptr;       // [try_cap][2][HS_TRK_MAXG][HS_TRK_NRED] pass partials of the member workgroups
  unsigned int* d_cnt = nullptr;  // [try_cap] timeout flags, then (cnt_bytes on) the outputs d_out: one read-back
  HsTryOut* h_out = nullptr;      // pinned mirror: h_cnt, then h_out
  double* h_in = nullptr;         // pinned staging of the hypotheses (T | aff), so their upload is asynchronous
  unsigned int* h_cnt = nullptr;
  unsigned int* dh_cnt = nullptr;  // device aliases of h_cnt / h_out (mapped pinned memory)
  HsTryOut* dh_out = nullptr;
  unsigned int* h_done = nullptr;  // pinned done words [try_cap] (HsTrackArgs.hdone) and their device alias
  unsigned int* dh_done = nullptr;
  unsigned int seq = 0;            // launch sequence number (the done words' value)
  unsigned int epoch = 0;         // the last member-meeting launch's granule epoch (hs_track_kernels.h)
  double* d_lmlog = nullptr;
  int* d_lmlvl = nullptr;
  int try_cap = 0, last_n_tries = 0;
  float refExposure = 1, newExposure = 1;
  double refAff[2] = {0, 0};
  bool haveRef = false, haveFrame = false;
  double last_ms = 0;
  long long* d_trace = nullptr;
  int last_G = 1;                 // workgroups per hypothesis of the last track launch
  int n_cu = 256;                 // the device's compute units (hipDeviceAttributeMultiprocessorCount)
  int wclk_khz = 100000;          // the constant wall clock the meetings' timeout reads (hipDeviceAttributeWallClockRate)
  int fallbacks = 0;              // launches rerun with G = 1 after a member-meeting timeout
  int trace_cap = 0;              // HS_KTRACE=1: per-hypothesis phase cycles of hs_k_track (stderr)
};

static int upload_pyr(hs_tracker* t, float4** dst, const float* const* pyr) {
  for (int l = 0; l < t->nlev; l++) {
    const size_t n = (size_t)t->w[l] * t->h[l];
    std::vector<float4> tex(n);
    const float* s = pyr[l];
    if (!s) return tfail(HS_ERR_INVALID, "null pyramid level");
    for (size_t i = 0; i < n; i++) tex[i] = make_float4(s[3 * i], s[3 * i + 1], s[3 * i + 2], 0.f);
    TS_HIP(hipMemcpyAsync(dst[l], tex.data(), n * sizeof(float4), hipMemcpyHostToDevice, t->stream));
    TS_HIP(hipStreamSynchronize(t->stream));  // tex is a temporary
  }
  return HS_OK;
}

// the member workgroups' pass granules of n hypotheses: [n][2][HS_TRK_MAXG][HS_TRK_NRED][2] u64
constexpr int kTrkOneMemberPoints = 2048;  // hs_k_track: 512 threads x 4 points in flight
static size_t meet_bytes(int n) { return sizeof(unsigned long long) * 2 * HS_TRK_MAXG * HS_TRK_NRED * 2 * (size_t)n; }
// the pass meetings' granules, then the level-end records (hs_track_kernels.h: lvrec), zeroed together
static size_t part_bytes(int n) { return meet_bytes(n) + sizeof(unsigned long long) * HS_TRK_MAXLVSEQ * 32 * (size_t)n; }
// the timeout flags in front of the outputs, padded to 256 B
static size_t cnt_bytes(int n) { return (sizeof(unsigned int) * (size_t)n + 255) & ~(size_t)255; }
static size_t done_bytes(int n) { return cnt_bytes(n); }  // the pinned done words after the pinned records

static int ensure_tries(hs_tracker* t, int n) {
  if (n <= t->try_cap) return HS_OK;
  if (t->d_Tin) (void)hipFree(t->d_Tin);
  if (t->d_cnt) (void)hipFree(t->d_cnt);
  if (t->h_cnt) (void)hipHostFree(t->h_cnt);
  if (t->d_lmlog) (void)hipFree(t->d_lmlog);
  if (t->d_part) (void)hipFree(t->d_part);
  if (t->h_in) (void)hipHostFree(t->h_in);
  t->d_part = nullptr; t->d_cnt = nullptr; t->h_in = nullptr; t->h_cnt = nullptr;
  if (t->d_lmlvl) (void)hipFree(t->d_lmlvl);
  t->d_Tin = nullptr; t->d_out = nullptr; t->h_out = nullptr; t->d_lmlog = nullptr; t->d_lmlvl = nullptr;
  TS_HIP(hipMalloc((void**)&t->d_Tin, sizeof(double) * 9 * n));  // T (7) | aff (2)
  TS_HIP(hipMalloc((void**)&t->d_cnt, cnt_bytes(n) + sizeof(HsTryOut) * n));
  t->d_out = reinterpret_cast<HsTryOut*>(reinterpret_cast<char*>(t->d_cnt) + cnt_bytes(n));
  TS_HIP(hipMalloc((void**)&t->d_lmlog, sizeof(double) * 3 * HS_TRK_MAXLOG * n));
  TS_HIP(hipMalloc((void**)&t->d_lmlvl, sizeof(int) * HS_TRK_MAXLOG * n));
  TS_HIP(hipMalloc((void**)&t->d_part, part_bytes(n)));
  // mapped, coherent: the kernel may write the flags and records straight into it (HS_TRK_ZC, run_tries)
  TS_HIP(hipHostMalloc((void**)&t->h_cnt, cnt_bytes(n) + sizeof(HsTryOut) * n + done_bytes(n),
                       hipHostMallocMapped | hipHostMallocCoherent));
  t->h_out = reinterpret_cast<HsTryOut*>(reinterpret_cast<char*>(t->h_cnt) + cnt_bytes(n));
  t->h_done = reinterpret_cast<unsigned int*>(reinterpret_cast<char*>(t->h_out) + sizeof(HsTryOut) * n);
  std::memset(t->h_cnt, 0, cnt_bytes(n) + sizeof(HsTryOut) * n + done_bytes(n));
  TS_HIP(hipHostGetDevicePointer((void**)&t->dh_cnt, t->h_cnt, 0));
  t->dh_out = reinterpret_cast<HsTryOut*>(reinterpret_cast<char*>(t->dh_cnt) + cnt_bytes(n));
  t->dh_done = reinterpret_cast<unsigned int*>(reinterpret_cast<char*>(t->dh_out) + sizeof(HsTryOut) * n);
  TS_HIP(hipHostMalloc((void**)&t->h_in, sizeof(double) * 9 * n));
  t->try_cap = n;
  t->epoch = 0;  // fresh granules and flags: zeroed at the next member-meeting launch
  return HS_OK;
}

static HsTrackArgs make_args(hs_tracker* t) {
  HsTrackArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int l = 0; l < t->nlev; l++) {
    HsTrkLevel& L = a.lv[l];
    L.w = t->w[l]; L.h = t->h[l];
    L.fx = t->fx[l]; L.fy = t->fy[l]; L.cx = t->cx[l]; L.cy = t->cy[l];
    for (int q = 0; q < 9; q++) L.Ki[q] = t->Ki[l][q];
    L.img = t->d_new[l];
    L.pc_u = t->d_pu[l]; L.pc_v = t->d_pv[l]; L.pc_id = t->d_pid[l]; L.pc_col = t->d_pcol[l];
    L.pc_n = t->d_pcn + l;
  }
  a.huberTH = t->P.huberTH;
  a.coarseCutoffTH = t->P.coarseCutoffTH;
  a.affineOptModeA = t->P.affineOptModeA;
  a.affineOptModeB = t->P.affineOptModeB;
  a.refExposure = t->refExposure;
  a.newExposure = t->newExposure;
  a.refAff[0] = t->refAff[0];
  a.refAff[1] = t->refAff[1];
  return a;
}

// n hypotheses (T | aff per row in h_in), run to completion without abort.  force_g1: the one-workgroup LM loop
// (the rerun after a G-member meeting timed out)
static int run_tries(hs_tracker* t, int n, const double* h_in, int coarsest, int single_pass, int lvl, float cutoff,
                     bool force_g1 = false) {
  TS_TRY(ensure_tries(t, n));
  HsTrackArgs a = make_args(t);
  a.n_inl = 0;
  if (n <= HS_TRK_INL) {  // a few hypotheses travel in the kernel arguments: no upload
    a.n_inl = n;
    std::memcpy(a.inl, h_in, sizeof(double) * 9 * n);
  } else {
    std::memcpy(t->h_in, h_in, sizeof(double) * 9 * n);
    TS_HIP(hipMemcpyAsync(t->d_Tin, t->h_in, sizeof(double) * 9 * n, hipMemcpyHostToDevice, t->stream));
  }
  a.coarsest = coarsest;
  a.T_in = t->d_Tin;
  a.aff_in = t->d_Tin + 7 * n;
  a.out = t->d_out;
  a.lm_log = t->d_lmlog;
  a.lm_lvl = t->d_lmlvl;
  a.single_pass = single_pass;
  a.pass_lvl = lvl;
  a.pass_cutoff = cutoff;
  // workgroups per hypothesis: the device's CUs shared by the hypotheses, one member per CU (every member must be
  // resident at once: they meet once per pass), at most HS_TRK_MAXG; env HS_TRK_G caps it (1 = the one-workgroup LM
  // loop).  16 measured best at C2 (r04_trk5: G = 4 / 8 / 12 / 16: 0.287 / 0.260 / 0.258 / 0.254 ms per track; in
  // round 3, with a costlier point loop and meeting, 8 was: more members shorten the point loop but lengthen the
  // per-pass meeting).  Members that are not co-resident after all (a smaller partition, kernels of other streams on
  // the CUs) make a meeting time out: the launch is then rerun with G = 1, which needs no co-residency.
  const int cap = std::max(1, t->n_cu / std::max(1, n));
  int G = std::max(1, std::min(16, cap));
  if (const char* e = std::getenv("HS_TRK_G")) G = std::max(1, std::min({HS_TRK_MAXG, cap, std::atoi(e)}));
  if (const char* e = std::getenv("HS_TRK_G_UNCHECKED"))  // test hook: G without the co-residency cap
    G = std::max(1, std::min(HS_TRK_MAXG, std::atoi(e)));
  if (single_pass || force_g1) G = 1;
  // a meeting's time bound: 20 ms of the device's wall clock (a healthy meeting takes a few us); after the first
  // timeout the launch's members skip every later meeting and leave the LM loop (hs_k_track, S.dead), so a launch
  // with a missing member costs ~20 ms per member before the G = 1 rerun, not 20 ms per pass
  a.spin_limit = (unsigned int)std::min<long long>(0xffffffffll, (long long)t->wclk_khz * 20);
  if (const char* e = std::getenv("HS_TRK_SPIN")) a.spin_limit = (unsigned int)std::max(1, std::atoi(e));  // ticks (test hook)
  a.G = G;
  a.nhyp = n;
  const int nblk = n * G;
  a.part = t->d_part;
  a.lvrec = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(t->d_part) + meet_bytes(t->try_cap));
  // levels below one workgroup's batch of points run on one member (r05_trk1 at C2: level 4's 936 points, 8 passes:
  // 0.232 -> 0.226 ms per track; a larger threshold, or fewer members at the finer levels, measured slower: the
  // point loop outweighs the meeting there).  Env HS_TRK_GMIN, 0 = every level on all G members.
  a.gmin = kTrkOneMemberPoints;
  if (const char* e = std::getenv("HS_TRK_GMIN")) a.gmin = std::max(0, std::atoi(e));
  // zero-copy results (default; env HS_TRK_ZC=0: a read-back copy behind the kernel): the lead workgroups write
  // their records, and timed-out members their flags, into mapped pinned memory: no copy is queued behind the kernel
  // (r04_trk5: 0.260 against 0.270 ms per track).  Polling the launch's end event instead of the blocking
  // synchronize gained nothing measurable here and cost activation 12 % (r04_sync1), so the synchronize stays.
  const char* zce = std::getenv("HS_TRK_ZC");
  const bool zc = !(zce && zce[0] == '0');
  a.cnt = zc ? t->dh_cnt : t->d_cnt;
  a.hout = zc ? t->dh_out : nullptr;
  a.hdone = zc ? t->dh_done : nullptr;
  a.seq = ++t->seq;
  t->last_G = G;
  // a new granule epoch per member-meeting launch; the granules and the timeout flags are zeroed only when the
  // epoch starts over (a fresh allocation, or 2^20 - 1 launches)
  if (G > 1) {
    if (t->epoch == 0 || t->epoch >= (1u << (32 - HS_TRK_PASS_BITS)) - 1) {
      TS_HIP(hipMemsetAsync(t->d_part, 0, part_bytes(t->try_cap), t->stream));
      TS_HIP(hipMemsetAsync(t->d_cnt, 0, sizeof(unsigned int) * t->try_cap, t->stream));
      std::memset(t->h_cnt, 0, sizeof(unsigned int) * t->try_cap);  // (no launch in flight: every call waits)
      t->epoch = 0;
    }
    t->epoch++;
  }
  a.epoch = t->epoch;
  a.solve = 0;
  if (const char* e = std::getenv("HS_TRK_SOLVE")) a.solve = std::atoi(e) == 1 ? 1 : 0;  // A/B: 1 = the LDLT
  const char* kt = std::getenv("HS_KTRACE");
  if (kt && kt[0] == '1' && !single_pass) {
    const int nb = nblk;
    if (nb > t->trace_cap) {  // grown once to the largest block count (freed by hs_tracker_destroy)
      if (t->d_trace) (void)hipFree(t->d_trace);
      t->d_trace = nullptr;
      TS_HIP(hipMalloc((void**)&t->d_trace, sizeof(long long) * 16 * nb));
      t->trace_cap = nb;
    }
    TS_HIP(hipMemsetAsync(t->d_trace, 0, sizeof(long long) * 16 * nb, t->stream));
    a.trace = t->d_trace;
  }
  // the launch's device time (hs_tracker_last_ms) from an event pair around it, only with event timing on
  // (hs_tracker_set_event_timing; ~3-4 us of host time per call, r05_trk14): by default the host takes the results
  // from the hypotheses' done words and last_ms stays 0.  Env HS_TRK_NOEVT=0 / 1 (read per call) forces either.
  const char* ne = std::getenv("HS_TRK_NOEVT");
  const bool no_evt = ne ? ne[0] == '1' : !t->evt;
  if (!no_evt) TS_HIP(hipEventRecord(t->e0, t->stream));
  hipLaunchKernelGGL(hs_k_track, dim3(nblk), dim3(512), 0, t->stream, a);
  TS_HIP(hipGetLastError());
  if (!no_evt) TS_HIP(hipEventRecord(t->e1, t->stream));
  if (!zc)  // the timeout flags and the outputs of the n hypotheses, in one read-back
    TS_HIP(hipMemcpyAsync(t->h_cnt, t->d_cnt, cnt_bytes(t->try_cap) + sizeof(HsTryOut) * n, hipMemcpyDeviceToHost,
                          t->stream));
  // zero-copy without the event pair or a trace: wait for every hypothesis' done word (its record and flags are in
  // place before it) instead of the launch's end; bounded, then the synchronize as before.  Otherwise the synchronize.
  bool waited = false;
  if (zc && no_evt && !a.trace) {
    const auto t_start = std::chrono::steady_clock::now();
    for (int spins = 0;; spins++) {
      bool all = true;
      for (int i = 0; i < n && all; i++) all = __atomic_load_n(&t->h_done[i], __ATOMIC_ACQUIRE) == a.seq;
      if (all) {
        waited = true;
        break;
      }
      if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t_start > std::chrono::seconds(2)) break;
    }
  }
  if (!waited) TS_HIP(hipStreamSynchronize(t->stream));  // (zero-copy: the records are in place once the launch completed)
  for (int i = 0; G > 1 && i < n; i++)
    if (t->h_cnt[i] == t->epoch) {  // a meeting timed out: the launch's results are void, rerun every hypothesis with G = 1
      t->fallbacks++;
      return run_tries(t, n, h_in, coarsest, single_pass, lvl, cutoff, true);
    }
  float ms = 0;
  if (!no_evt) TS_HIP(hipEventElapsedTime(&ms, t->e0, t->e1));
  t->last_ms = ms;
  t->last_n_tries = single_pass ? 0 : n;
  if (a.trace) {
    long long h[16];
    TS_HIP(hipMemcpy(h, t->d_trace, sizeof(h), hipMemcpyDeviceToHost));
    {  // placement probe: block -> xcd / cu (h, g)
      std::vector<long long> pl((size_t)nblk * 16);
      TS_HIP(hipMemcpy(pl.data(), t->d_trace, sizeof(long long) * pl.size(), hipMemcpyDeviceToHost));
      std::fprintf(stderr, "[trk place]");
      for (int b = 0; b < nblk && b < 64; b++) {
        const long long v = pl[(size_t)b * 16 + 14];
        if (pl[(size_t)b * 16] == 0) continue;  // an idle block
        std::fprintf(stderr, " %d:x%lld/c%lld(h%lld g%lld)", b, v & 15, (v >> 4) & 15, (v >> 8) & 255, (v >> 16) & 255);
      }
      std::fprintf(stderr, "\n");
    }
    std::fprintf(stderr, "[trk trace] %.3f ms: point loop %lld, reductions %lld (wave reduce %lld, barrier wait %lld, "
                 "meetings %lld over %lld), LM steps %lld (LDLT %lld, exp + product %lld) cycles over %lld passes "
                 "(G %d, n %d, fallbacks so far %d); wave-0 tail: tree %lld, meeting + results %lld, bookkeeping %lld\n",
                 ms, h[4], h[5], h[8], h[9], h[12], h[13], h[6], h[10], h[11], h[7], G, n, t->fallbacks, h[1], h[2], h[3]);
  }
  return HS_OK;
}

// trackNewestCoarse's per-level abort (Src/CoarseTracker.cpp:647-651) replayed on a hypothesis' log:
// returns the reference's return value and its lastResiduals / lastFlowIndicators at return
static bool replay_abort(const HsTryOut& o, const double minRes[5], double lastRes[5], double flow[3]) {
  for (int i = 0; i < 5; i++) lastRes[i] = NAN;
  for (int i = 0; i < 3; i++) flow[i] = 1000;
  for (int c = 0; c < o.n_checks; c++) {
    const int l = o.check_lvl[c];
    if (l < 5) lastRes[l] = o.check_res[c];
    for (int i = 0; i < 3; i++) flow[i] = o.check_flow[c][i];
    if (l < 5 && o.check_res[c] > 1.5 * minRes[l]) return false;
  }
  return o.ok != 0;
}

// CoarseTracker::makeCoarseDepthL0 (Src/CoarseTracker.cpp:105-263) on the device: the reference points (cu | cv | cid |
// HdiF at pts + stride * {0,1,2,3}; their count n_host, or *d_n on the device) scattered into the level-0 idepth /
// weight maps in point order, summed up the pyramid, dilated, normalised and compacted into the pc_* arrays.
static int make_depth_l0(hs_tracker* t, int n_host, const int* d_n, const float* pts, int stride) {
  const size_t n0 = (size_t)t->w[0] * t->h[0];
  TS_HIP(hipMemsetAsync(t->d_id[0], 0, n0 * sizeof(float), t->stream));
  TS_HIP(hipMemsetAsync(t->d_ws[0], 0, n0 * sizeof(float), t->stream));
  if (d_n || n_host > 0)
    hipLaunchKernelGGL(hs_k_trk_scatter_sorted, dim3(1), dim3(1024), sizeof(unsigned long long) * HS_TRK_SCAT_CAP,
                       t->stream, d_n, n_host, pts, pts + stride, pts + 2 * (size_t)stride, pts + 3 * (size_t)stride,
                       t->w[0], t->h[0], t->d_id[0], t->d_ws[0]);
  TS_HIP(hipGetLastError());
  for (int l = 1; l < t->nlev; l++) {
    const int np = t->w[l] * t->h[l];
    hipLaunchKernelGGL(hs_k_trk_down, dim3((np + 255) / 256), dim3(256), 0, t->stream, t->w[l], t->h[l], t->w[l - 1],
                       t->d_id[l - 1], t->d_ws[l - 1], t->d_id[l], t->d_ws[l]);
    TS_HIP(hipGetLastError());
  }
  for (int l = 0; l < t->nlev; l++) {
    const int np = t->w[l] * t->h[l];
    TS_HIP(hipMemcpyAsync(t->d_bak[l], t->d_ws[l], np * sizeof(float), hipMemcpyDeviceToDevice, t->stream));
    const int inner = np - 2 * t->w[l];
    hipLaunchKernelGGL(hs_k_trk_dilate, dim3((inner + 255) / 256), dim3(256), 0, t->stream, t->w[l], t->h[l],
                       l < 2 ? 1 : 0, t->d_bak[l], t->d_id[l], t->d_ws[l]);
    TS_HIP(hipGetLastError());
  }
  for (int l = 0; l < t->nlev; l++) {
    const int np = t->w[l] * t->h[l], nb = (np + 255) / 256;
    hipLaunchKernelGGL(hs_k_trk_count, dim3(nb), dim3(256), 0, t->stream, t->w[l], t->h[l], t->d_id[l], t->d_ws[l],
                       t->d_ref[l], t->d_bcnt);
    hipLaunchKernelGGL(hs_k_trk_scan, dim3(1), dim3(1024), 0, t->stream, nb, t->d_bcnt, t->d_boff, t->d_pcn + l);
    hipLaunchKernelGGL(hs_k_trk_compact, dim3(nb), dim3(256), 0, t->stream, t->w[l], t->h[l], t->d_id[l], t->d_ws[l],
                       t->d_ref[l], t->d_boff, t->d_pu[l], t->d_pv[l], t->d_pid[l], t->d_pcol[l]);
    TS_HIP(hipGetLastError());
  }
  return HS_OK;
}

// make_depth_l0 from a device count (hs_tracker_set_ref_ba) as a replayed hipGraph: the host cost of ~32 launches
// and copies per keyframe becomes one graph launch.  HS_TRK_GRAPH=0 launches them one by one.
static int make_depth_l0_dev(hs_tracker* t, const int* d_n, const float* pts, int stride) {
  static const bool off = getenv("HS_TRK_GRAPH") && getenv("HS_TRK_GRAPH")[0] == '0';
  if (off) return make_depth_l0(t, 0, d_n, pts, stride);
  auto same = [&](const DepthGraph& g) {
    if (!g.exec || g.d_n != d_n || g.pts != pts || g.stride != stride) return false;
    for (int l = 0; l < t->nlev; l++)
      if (g.ref[l] != t->d_ref[l]) return false;
    return true;
  };
  DepthGraph* hit = same(t->dg[0]) ? &t->dg[0] : same(t->dg[1]) ? &t->dg[1] : nullptr;
  if (!hit) {
    DepthGraph& g = t->dg[t->dg_next];
    t->dg_next ^= 1;
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    g.exec = nullptr;
    TS_HIP(hipStreamBeginCapture(t->stream, hipStreamCaptureModeThreadLocal));
    const int rc = make_depth_l0(t, 0, d_n, pts, stride);
    hipGraph_t graph = nullptr;
    const hipError_t ec = hipStreamEndCapture(t->stream, &graph);
    if (rc != HS_OK) {
      if (graph) (void)hipGraphDestroy(graph);
      return rc;
    }
    if (ec != hipSuccess) return tfail(HS_ERR_HIP, "makeCoarseDepthL0 capture failed");
    const hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ei != hipSuccess) {
      g.exec = nullptr;
      return tfail(HS_ERR_HIP, "makeCoarseDepthL0 graph instantiation failed");
    }
    g.d_n = d_n;
    g.pts = pts;
    g.stride = stride;
    for (int l = 0; l < HS_TRK_MAXLEV; l++) g.ref[l] = l < t->nlev ? t->d_ref[l] : nullptr;
    hit = &g;
  }
  TS_HIP(hipGraphLaunch(hit->exec, t->stream));
  return HS_OK;
}

extern "C" {

int hs_tracker_create(hs_tracker** out, const hs_params* params, int device_id, int width, int height,
                      int n_levels, const float K4[4]) {
  if (!out || !K4) return tfail(HS_ERR_INVALID, "null argument");
  *out = nullptr;
  if (n_levels < 1 || n_levels > HS_TRK_MAXLEV) return tfail(HS_ERR_INVALID, "n_levels out of range");
  if (width < 16 || height < 16 || (width >> (n_levels - 1)) < 8 || (height >> (n_levels - 1)) < 8)
    return tfail(HS_ERR_INVALID, "image too small for the pyramid");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return tfail(HS_ERR_HIP, "no HIP device");
  if (device_id < 0 || device_id >= ndev) return tfail(HS_ERR_INVALID, "bad device id");
  hs_tracker* t = new hs_tracker();
  if (params) t->P = *params;
  else hs_params_default(&t->P);
  t->device = device_id;
  t->W = width; t->H = height; t->nlev = n_levels;
  // CoarseTracker::makeK (Src/CoarseTracker.cpp:73-101)
  t->w[0] = width; t->h[0] = height;
  t->fx[0] = K4[0]; t->fy[0] = K4[1]; t->cx[0] = K4[2]; t->cy[0] = K4[3];
  for (int l = 1; l < n_levels; l++) {
    t->w[l] = t->w[0] >> l;
    t->h[l] = t->h[0] >> l;
    t->fx[l] = t->fx[l - 1] * 0.5;
    t->fy[l] = t->fy[l - 1] * 0.5;
    t->cx[l] = (t->cx[0] + 0.5) / ((int)1 << l) - 0.5;
    t->cy[l] = (t->cy[0] + 0.5) / ((int)1 << l) - 0.5;
  }
  for (int l = 0; l < n_levels; l++) {
    const float K[9] = {t->fx[l], 0, t->cx[l], 0, t->fy[l], t->cy[l], 0, 0, 1};
    hs::inv3f(K, t->Ki[l]);
  }
  if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&t->e0) != hipSuccess || hipEventCreate(&t->e1) != hipSuccess ||
      hipEventCreateWithFlags(&t->ev_handoff, hipEventDisableTiming) != hipSuccess) {
    delete t;
    return tfail(HS_ERR_HIP, "stream / event creation failed");
  }
  if (hipDeviceGetAttribute(&t->n_cu, hipDeviceAttributeMultiprocessorCount, device_id) != hipSuccess || t->n_cu < 1)
    t->n_cu = 1;
  if (hipDeviceGetAttribute(&t->wclk_khz, hipDeviceAttributeWallClockRate, device_id) != hipSuccess || t->wclk_khz < 1)
    t->wclk_khz = 100000;
  int maxBlocks = 1;
  for (int l = 0; l < n_levels; l++) {
    const size_t n = (size_t)t->w[l] * t->h[l];
    TS_HIP(hipMalloc((void**)&t->d_ref[l], n * sizeof(float4)));
    TS_HIP(hipMalloc((void**)&t->d_new[l], n * sizeof(float4)));
    TS_HIP(hipMalloc((void**)&t->d_id[l], n * sizeof(float)));
    TS_HIP(hipMalloc((void**)&t->d_ws[l], n * sizeof(float)));
    TS_HIP(hipMalloc((void**)&t->d_bak[l], n * sizeof(float)));
    TS_HIP(hipMalloc((void**)&t->d_pu[l], n * sizeof(float)));
    TS_HIP(hipMalloc((void**)&t->d_pv[l], n * sizeof(float)));
    TS_HIP(hipMalloc((void**)&t->d_pid[l], n * sizeof(float)));
    TS_HIP(hipMalloc((void**)&t->d_pcol[l], n * sizeof(float)));
    maxBlocks = std::max(maxBlocks, (int)((n + 255) / 256));
  }
  TS_HIP(hipMalloc((void**)&t->d_pcn, sizeof(int) * HS_TRK_MAXLEV));
  TS_HIP(hipMemsetAsync(t->d_pcn, 0, sizeof(int) * HS_TRK_MAXLEV, t->stream));  // on the kernels' stream
  TS_HIP(hipMalloc((void**)&t->d_bcnt, sizeof(int) * maxBlocks));
  TS_HIP(hipMalloc((void**)&t->d_boff, sizeof(int) * maxBlocks));
  *out = t;
  return HS_OK;
}

void hs_tracker_destroy(hs_tracker* t) {
  if (!t) return;
  (void)hipSetDevice(t->device);
  if (t->stream) (void)hipStreamSynchronize(t->stream);
  for (auto& g : t->dg)
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
  for (int l = 0; l < HS_TRK_MAXLEV; l++) {
    void* ps[] = {t->d_ref[l], t->d_new[l], t->d_id[l], t->d_ws[l], t->d_bak[l], t->d_pu[l], t->d_pv[l], t->d_pid[l],
                  t->d_pcol[l]};
    for (void* p : ps)
      if (p) (void)hipFree(p);
  }
  void* ps[] = {t->d_pcn, t->d_bcnt, t->d_boff, t->d_pts, t->d_Tin, t->d_cnt, t->d_lmlog, t->d_lmlvl, t->d_raw,
                t->d_trace, t->d_part};  // d_out lives in d_cnt's allocation, h_out in h_cnt's
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (t->h_in) (void)hipHostFree(t->h_in);
  if (t->h_cnt) (void)hipHostFree(t->h_cnt);
  if (t->e0) (void)hipEventDestroy(t->e0);
  if (t->e1) (void)hipEventDestroy(t->e1);
  if (t->ev_handoff) (void)hipEventDestroy(t->ev_handoff);
  if (t->stream) (void)hipStreamDestroy(t->stream);
  delete t;
}

int hs_tracker_set_ref(hs_tracker* t, const float* const* ref_pyr, float ab_exposure, const double aff_g2l[2], int n,
                       const float* cu, const float* cv, const float* cid, const float* hdi) {
  if (!t || !ref_pyr || !aff_g2l || n < 0 || (n > 0 && (!cu || !cv || !cid || !hdi)))
    return tfail(HS_ERR_INVALID, "null argument");
  TS_HIP(hipSetDevice(t->device));
  TS_TRY(upload_pyr(t, t->d_ref, ref_pyr));
  t->refExposure = ab_exposure;
  t->refAff[0] = aff_g2l[0];
  t->refAff[1] = aff_g2l[1];
  if (n > t->pts_cap) {
    if (t->d_pts) (void)hipFree(t->d_pts);
    t->d_pts = nullptr;
    TS_HIP(hipMalloc((void**)&t->d_pts, sizeof(float) * 4 * n));
    t->pts_cap = n;
  }
  std::vector<float> h((size_t)4 * std::max(n, 0));  // lives until the stream synchronize below
  if (n > 0) {
    std::memcpy(h.data(), cu, 4 * n);
    std::memcpy(h.data() + n, cv, 4 * n);
    std::memcpy(h.data() + 2 * n, cid, 4 * n);
    std::memcpy(h.data() + 3 * n, hdi, 4 * n);
    TS_HIP(hipMemcpyAsync(t->d_pts, h.data(), sizeof(float) * 4 * n, hipMemcpyHostToDevice, t->stream));
  }
  TS_TRY(make_depth_l0(t, n, nullptr, t->d_pts, n));
  TS_HIP(hipStreamSynchronize(t->stream));
  t->haveRef = true;
  return HS_OK;
}

int hs_tracker_frame_texels(hs_tracker* t, int lvl, const void** d_texels) {
  if (!t || !d_texels) return tfail(HS_ERR_INVALID, "null argument");
  if (lvl < 0 || lvl >= t->nlev) return tfail(HS_ERR_INVALID, "bad level");
  if (!t->haveFrame) return tfail(HS_ERR_STATE, "no frame set");
  *d_texels = t->d_new[lvl];
  return HS_OK;
}

// setCoarseTrackingRef(frameHessians) after AddKeyframe's optimize (Src/Mapping.cpp:93-100), fed from the BA context
// on the device: the points whose residual into the newest frame is IN, in window order (hs_k_win_newest on the BA
// stream), then makeCoarseDepthL0 on the tracker stream after an event -- no host round trip, no host sync.
int hs_tracker_set_ref_ba(hs_tracker* t, hs_ctx* ba, int promote_frame, float ab_exposure, const double aff_g2l[2]) {
  if (!t || !ba || !aff_g2l) return tfail(HS_ERR_INVALID, "null argument");
  if (ba->device != t->device) return tfail(HS_ERR_INVALID, "tracker and BA context on different devices");
  TS_HIP(hipSetDevice(t->device));
  HS_TRY(hs::commit_if_dirty(ba));
  if (ba->nF < 1) return tfail(HS_ERR_STATE, "empty BA window");
  if (ba->cam.width != t->W || ba->cam.height != t->H) return tfail(HS_ERR_INVALID, "image size mismatch");
  if (promote_frame && !t->haveFrame) return tfail(HS_ERR_STATE, "no frame to promote");
  // the hand-off buffer: points of the BA window (capacity), compacted on the BA's stream
  hipLaunchKernelGGL(hs_k_win_newest, dim3(1), dim3(1024), 0, ba->stream, ba->nP, ba->nF - 1, ba->d_res_of_slot,
                     ba->d_r_state, ba->d_r_center, ba->hdif_solved, ba->d_ref_pts, ba->cap_P, ba->d_ref_n);
  TS_HIP(hipGetLastError());
  if (!promote_frame)  // the reference pyramid's level 0 is the BA's newest frame image
    TS_HIP(hipMemcpyAsync(t->d_ref[0], ba->d_img_all + (size_t)ba->img_slot[ba->nF - 1] * ba->img_px,
                          sizeof(float4) * (size_t)t->W * t->H, hipMemcpyDeviceToDevice, ba->stream));
  TS_HIP(hipEventRecord(ba->ev_ready, ba->stream));
  TS_HIP(hipStreamWaitEvent(t->stream, ba->ev_ready, 0));
  if (promote_frame) {
    for (int l = 0; l < t->nlev; l++) std::swap(t->d_ref[l], t->d_new[l]);
    t->haveFrame = false;  // d_new now holds the old reference: the next frame to track must be set
  } else {
    TS_HIP(hs_build_dir_pyramid_upper(t->stream, t->W, t->H, t->nlev, t->d_ref));
  }
  t->refExposure = ab_exposure;
  t->refAff[0] = aff_g2l[0];
  t->refAff[1] = aff_g2l[1];
  TS_TRY(make_depth_l0_dev(t, ba->d_ref_n, ba->d_ref_pts, ba->cap_P));
  // the BA stream must not rewrite the hand-off buffer before the tracker consumed it
  TS_HIP(hipEventRecord(t->ev_handoff, t->stream));
  TS_HIP(hipStreamWaitEvent(ba->stream, t->ev_handoff, 0));
  t->haveRef = true;
  return HS_OK;
}

// AddKeyframe's image hand-off (Src/Mapping.cpp:22, the keyframe's Frame::DirPyr[0] into the window): the level-0
// texels of the frame last set here become window frame `frame`'s image, ordered on the device both ways -- the BA
// stream waits for the tracker's stream (the frame's pyramid), the copy and the packed slot run on the BA stream,
// and the tracker's stream waits for the copy, so its next set_frame cannot rewrite d_new before the copy read it.
int hs_tracker_frame_to_ba(hs_tracker* t, hs_ctx* ba, int frame) {
  if (!t || !ba) return tfail(HS_ERR_INVALID, "null argument");
  if (ba->device != t->device) return tfail(HS_ERR_INVALID, "tracker and BA context on different devices");
  if (ba->cam.width != t->W || ba->cam.height != t->H) return tfail(HS_ERR_INVALID, "image size mismatch");
  if (!t->haveFrame) return tfail(HS_ERR_STATE, "no frame set");
  TS_HIP(hipSetDevice(t->device));
  TS_HIP(hipEventRecord(t->ev_handoff, t->stream));
  TS_HIP(hipStreamWaitEvent(ba->stream, t->ev_handoff, 0));
  if (const int rc = hs::copy_frame_image_device(ba, frame, t->d_new[0]))
    return tfail(rc, std::string("hs_tracker_frame_to_ba: ") + hs::g_err);
  TS_HIP(hipEventRecord(ba->ev_ready, ba->stream));
  TS_HIP(hipStreamWaitEvent(t->stream, ba->ev_ready, 0));
  return HS_OK;
}

int hs_tracker_set_event_timing(hs_tracker* t, int on) {
  if (!t) return tfail(HS_ERR_INVALID, "null tracker");
  t->evt = on ? 1 : 0;
  return HS_OK;
}

int hs_tracker_get_ref(hs_tracker* t, int lvl, int* n, float* u, float* v, float* idepth, float* color) {
  if (!t || !n) return tfail(HS_ERR_INVALID, "null argument");
  if (lvl < 0 || lvl >= t->nlev) return tfail(HS_ERR_INVALID, "bad level");
  if (!t->haveRef) return tfail(HS_ERR_STATE, "no reference set");
  TS_HIP(hipSetDevice(t->device));
  TS_HIP(hipStreamSynchronize(t->stream));
  TS_HIP(hipMemcpy(n, t->d_pcn + lvl, sizeof(int), hipMemcpyDeviceToHost));
  const size_t b = sizeof(float) * (size_t)*n;
  if (*n > 0) {
    if (u) TS_HIP(hipMemcpy(u, t->d_pu[lvl], b, hipMemcpyDeviceToHost));
    if (v) TS_HIP(hipMemcpy(v, t->d_pv[lvl], b, hipMemcpyDeviceToHost));
    if (idepth) TS_HIP(hipMemcpy(idepth, t->d_pid[lvl], b, hipMemcpyDeviceToHost));
    if (color) TS_HIP(hipMemcpy(color, t->d_pcol[lvl], b, hipMemcpyDeviceToHost));
  }
  return HS_OK;
}

int hs_tracker_set_frame(hs_tracker* t, const float* const* new_pyr, float ab_exposure) {
  if (!t || !new_pyr) return tfail(HS_ERR_INVALID, "null argument");
  TS_HIP(hipSetDevice(t->device));
  TS_TRY(upload_pyr(t, t->d_new, new_pyr));
  t->newExposure = ab_exposure;
  t->haveFrame = true;
  return HS_OK;
}

int hs_tracker_set_frame_raw(hs_tracker* t, const float* img, float ab_exposure) {
  if (!t || !img) return tfail(HS_ERR_INVALID, "null argument");
  TS_HIP(hipSetDevice(t->device));
  if (!t->d_raw) TS_HIP(hipMalloc((void**)&t->d_raw, sizeof(float) * t->W * t->H));
  TS_HIP(hipMemcpyAsync(t->d_raw, img, sizeof(float) * t->W * t->H, hipMemcpyHostToDevice, t->stream));
  TS_HIP(hs_build_dir_pyramid(t->stream, t->d_raw, t->W, t->H, t->nlev, t->d_new, nullptr));
  TS_HIP(hipStreamSynchronize(t->stream));  // the caller's buffer may go away after return
  t->newExposure = ab_exposure;
  t->haveFrame = true;
  return HS_OK;
}

int hs_tracker_calc_res(hs_tracker* t, int lvl, const double T7[7], const double aff[2], float cutoffTH, double res6[6],
                        double H64[64], double b8[8], int* n_warped) {
  if (!t || !T7 || !aff || !res6) return tfail(HS_ERR_INVALID, "null argument");
  if (lvl < 0 || lvl >= t->nlev) return tfail(HS_ERR_INVALID, "bad level");
  if (!t->haveRef || !t->haveFrame) return tfail(HS_ERR_STATE, "reference and frame must be set");
  TS_HIP(hipSetDevice(t->device));
  double in[9];
  std::memcpy(in, T7, sizeof(double) * 7);
  in[7] = aff[0];
  in[8] = aff[1];
  TS_TRY(run_tries(t, 1, in, lvl, 1, lvl, cutoffTH));
  const HsTryOut& o = t->h_out[0];
  std::memcpy(res6, o.res6, sizeof(double) * 6);
  if (H64) std::memcpy(H64, o.H, sizeof(double) * 64);
  if (b8) std::memcpy(b8, o.b, sizeof(double) * 8);
  if (n_warped) *n_warped = o.n_warped;
  return HS_OK;
}

int hs_tracker_track(hs_tracker* t, double T_inout[7], double aff_inout[2], int coarsest_lvl,
                     const double minResForAbort[5], double lastResiduals[5], double flow[3], int* ok) {
  if (!t || !T_inout || !aff_inout || !minResForAbort || !lastResiduals || !flow || !ok)
    return tfail(HS_ERR_INVALID, "null argument");
  if (coarsest_lvl < 0 || coarsest_lvl >= t->nlev || coarsest_lvl >= 5)
    return tfail(HS_ERR_INVALID, "coarsest level must be < min(5, n_levels)");
  if (!t->haveRef || !t->haveFrame) return tfail(HS_ERR_STATE, "reference and frame must be set");
  TS_HIP(hipSetDevice(t->device));
  double in[9];
  std::memcpy(in, T_inout, sizeof(double) * 7);
  in[7] = aff_inout[0];
  in[8] = aff_inout[1];
  TS_TRY(run_tries(t, 1, in, coarsest_lvl, 0, 0, 0.f));
  const HsTryOut& o = t->h_out[0];
  const bool good = replay_abort(o, minResForAbort, lastResiduals, flow);
  *ok = good ? 1 : 0;
  bool completed = true;  // the abort returns before "set!": the outputs keep their inputs
  for (int c = 0; c < o.n_checks; c++)
    if (o.check_lvl[c] < 5 && o.check_res[c] > 1.5 * minResForAbort[o.check_lvl[c]]) completed = false;
  if (completed) {
    std::memcpy(T_inout, o.T, sizeof(double) * 7);
    aff_inout[0] = o.aff[0];
    aff_inout[1] = o.aff[1];
  }
  return HS_OK;
}

int hs_tracker_track_tries(hs_tracker* t, int n_tries, const double* tries7, const double aff_last[2],
                           const double lastCoarseRMSE[5], float reTrackThreshold, double T_out[7], double aff_out[2],
                           double achievedRes[5], double flowVecs[3], int* have_one_good, int* n_tried) {
  if (!t || n_tries < 1 || !tries7 || !aff_last || !lastCoarseRMSE || !T_out || !aff_out || !achievedRes || !flowVecs ||
      !have_one_good || !n_tried)
    return tfail(HS_ERR_INVALID, "null argument");
  if (!t->haveRef || !t->haveFrame) return tfail(HS_ERR_STATE, "reference and frame must be set");
  TS_HIP(hipSetDevice(t->device));
  const int coarsest = std::min(t->nlev - 1, 4);
  std::vector<double> in((size_t)9 * n_tries);
  std::memcpy(in.data(), tries7, sizeof(double) * 7 * n_tries);
  for (int i = 0; i < n_tries; i++) {
    in[7 * n_tries + 2 * i] = aff_last[0];
    in[7 * n_tries + 2 * i + 1] = aff_last[1];
  }
  TS_TRY(run_tries(t, n_tries, in.data(), coarsest, 0, 0, 0.f));
  // System::trackNewCoarse try loop (Src/System.cpp:413-481), replayed in the reference's order
  double ach[5];
  for (int k = 0; k < 5; k++) ach[k] = NAN;
  bool haveOneGood = false;
  double flow[3] = {100, 100, 100};
  int best = -1, tried = 0;
  for (int i = 0; i < n_tries; i++) {
    const HsTryOut& o = t->h_out[i];
    double lastRes[5], lf[3];
    const bool good = replay_abort(o, ach, lastRes, lf);
    tried++;
    if (good && std::isfinite((float)lastRes[0]) && !(lastRes[0] >= ach[0])) {
      for (int k = 0; k < 3; k++) flow[k] = lf[k];
      best = i;
      haveOneGood = true;
    }
    if (haveOneGood)
      for (int k = 0; k < 5; k++)
        if (!std::isfinite((float)ach[k]) || ach[k] > lastRes[k]) ach[k] = lastRes[k];
    if (haveOneGood && ach[0] < lastCoarseRMSE[0] * reTrackThreshold) break;
  }
  if (haveOneGood) {
    std::memcpy(T_out, t->h_out[best].T, sizeof(double) * 7);
    aff_out[0] = t->h_out[best].aff[0];
    aff_out[1] = t->h_out[best].aff[1];
  } else {
    flow[0] = flow[1] = flow[2] = 0;
    std::memcpy(T_out, tries7, sizeof(double) * 7);
    aff_out[0] = aff_last[0];
    aff_out[1] = aff_last[1];
  }
  for (int k = 0; k < 5; k++) achievedRes[k] = ach[k];
  for (int k = 0; k < 3; k++) flowVecs[k] = flow[k];
  *have_one_good = haveOneGood ? 1 : 0;
  *n_tried = tried;
  return HS_OK;
}

int hs_tracker_get_lm_log(hs_tracker* t, int try_idx, int cap, int* n, int* lvl, double* new_ratio,
                          double* old_ratio, double* inc_norm) {
  if (!t || !n) return tfail(HS_ERR_INVALID, "null argument");
  if (try_idx < 0 || try_idx >= t->last_n_tries) return tfail(HS_ERR_INVALID, "no such hypothesis in the last call");
  TS_HIP(hipSetDevice(t->device));
  TS_HIP(hipStreamSynchronize(t->stream));
  const int iters = t->h_out[try_idx].iters;
  *n = iters;
  const int m = std::min(std::min(iters, cap), HS_TRK_MAXLOG);
  if (m > 0) {
    std::vector<double> lg((size_t)3 * m);
    TS_HIP(hipMemcpy(lg.data(), t->d_lmlog + (size_t)try_idx * HS_TRK_MAXLOG * 3, sizeof(double) * 3 * m,
                     hipMemcpyDeviceToHost));
    if (lvl)
      TS_HIP(hipMemcpy(lvl, t->d_lmlvl + (size_t)try_idx * HS_TRK_MAXLOG, sizeof(int) * m, hipMemcpyDeviceToHost));
    for (int i = 0; i < m; i++) {
      if (new_ratio) new_ratio[i] = lg[3 * i];
      if (old_ratio) old_ratio[i] = lg[3 * i + 1];
      if (inc_norm) inc_norm[i] = lg[3 * i + 2];
    }
  }
  return HS_OK;
}

int hs_tracker_last_stats(hs_tracker* t, int try_idx, double* ms, int* passes, long long* point_passes) {
  if (!t) return tfail(HS_ERR_INVALID, "null tracker");
  if (try_idx < 0 || try_idx >= t->last_n_tries) return tfail(HS_ERR_INVALID, "no such hypothesis in the last call");
  if (ms) *ms = t->last_ms;
  if (passes) *passes = t->h_out[try_idx].passes;
  if (point_passes) *point_passes = t->h_out[try_idx].point_passes;
  return HS_OK;
}

int hs_tracker_launch_info(hs_tracker* t, int* G, int* fallbacks) {
  if (!t) return tfail(HS_ERR_INVALID, "null tracker");
  if (G) *G = t->last_G;
  if (fallbacks) *fallbacks = t->fallbacks;
  return HS_OK;
}

int hs_tracker_last_ms(hs_tracker* t, double* ms) {
  if (!t || !ms) return tfail(HS_ERR_INVALID, "null argument");
  *ms = t->last_ms;
  return HS_OK;
}

}  // extern "C"
