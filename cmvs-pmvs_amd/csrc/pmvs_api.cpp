// pmvs_api.cpp -- the C-ABI (include/pmvs_amd.h) on top of the HIP kernels.
//
// Host responsibilities (C++, no torch types): scene validation, camera setup restated from
// the reference's CCamera (camera.cpp:56-173) and COptim::setAxesScales (optim.cpp:43-64),
// device allocation of the pyramid / camera / visibility tables, kernel launches on one HIP
// stream per scene, HIP-event timing, and error mapping (never exit(); PMVS_EDEVICE + message).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pmvs_amd.h"
#include "pmvs_features.h"
#include "pmvs_launch.h"

using namespace pmvsdev;

namespace {

thread_local std::string g_err = "";

pmvs_status fail(pmvs_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return st;
}

}  // namespace

pmvs_status pmvs_io_fail(pmvs_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return st;
}

namespace {

#define HIPCHK(expr)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(PMVS_EDEVICE, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

// ---- host restatement of the reference camera setup (CONTOUR projection given as 12 floats)
static inline float dot4f(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3]; }
static inline float dot3f(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void cross3f(const float* u, const float* v, float* o) {
  o[0] = u[1] * v[2] - v[1] * u[2];
  o[1] = -u[0] * v[2] + v[0] * u[2];
  o[2] = u[0] * v[1] - v[0] * u[1];
}
static inline void unitize3f(float* v) {
  const float l = dot3f(v, v);
  if (l != 1.0 && l != 0.0) {
    const float d = (float)std::sqrt((double)l);
    v[0] /= d; v[1] /= d; v[2] /= d;
  }
}

// CCamera::updateProjection / updateCamera / getOpticalCenter (camera.cpp:56-173), txtType 0.
void setup_camera(DView& v, const float* p12, int maxLevel) {
  for (int i = 0; i < 12; ++i) v.P[0][i] = p12[i];
  for (int level = 1; level < maxLevel; ++level) {
    for (int i = 0; i < 12; ++i) v.P[level][i] = v.P[level - 1][i];
    for (int x = 0; x < 4; ++x) {
      v.P[level][x] /= 2.0f;
      v.P[level][4 + x] /= 2.0f;
    }
  }
  for (int level = maxLevel; level < MAXL; ++level) std::memcpy(v.P[level], v.P[maxLevel - 1], sizeof(v.P[0]));
  float oa[4] = {v.P[0][8], v.P[0][9], v.P[0][10], 0.0f};
  const float ftmp = (float)std::sqrt((double)dot4f(oa, oa));
  oa[3] = v.P[0][11];
  for (int i = 0; i < 4; ++i) oa[i] /= ftmp;
  for (int i = 0; i < 4; ++i) v.oaxis[i] = oa[i];
  if (v.P[0][8] == 0.0 && v.P[0][9] == 0.0 && v.P[0][10] == 0.0) {
    float a[3] = {v.P[0][0], v.P[0][1], v.P[0][2]}, b[3] = {v.P[0][4], v.P[0][5], v.P[0][6]}, c[3];
    cross3f(a, b, c);
    unitize3f(c);
    v.center[0] = c[0]; v.center[1] = c[1]; v.center[2] = c[2]; v.center[3] = 0.0f;
  } else {
    double A[3][3], b[3];
    for (int y = 0; y < 3; ++y) {
      for (int x = 0; x < 3; ++x) A[y][x] = v.P[0][4 * y + x];
      b[y] = -(double)v.P[0][4 * y + 3];
    }
    auto cr = [](const double* u, const double* w, double* o) {
      o[0] = u[1] * w[2] - w[1] * u[2];
      o[1] = -u[0] * w[2] + w[0] * u[2];
      o[2] = u[0] * w[1] - w[0] * u[1];
    };
    double ad[3][3];
    cr(A[1], A[2], ad[0]);
    cr(A[2], A[0], ad[1]);
    cr(A[0], A[1], ad[2]);
    const double det = ad[0][0] * A[0][0] + ad[0][1] * A[0][1] + ad[0][2] * A[0][2];
    double inv[3][3] = {{0}};
    if (det != 0.0)
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) inv[r][c] = ad[c][r] / det;
    for (int r = 0; r < 3; ++r) v.center[r] = (float)(inv[r][0] * b[0] + inv[r][1] * b[1] + inv[r][2] * b[2]);
    v.center[3] = 1.0f;
  }
  // COptim::setAxesScales (optim.cpp:43-64)
  float z[3] = {oa[0], oa[1], oa[2]}, x[3] = {v.P[0][0], v.P[0][1], v.P[0][2]}, y[3];
  cross3f(z, x, y);
  unitize3f(y);
  cross3f(y, z, x);
  for (int i = 0; i < 3; ++i) { v.xaxis[i] = x[i]; v.yaxis[i] = y[i]; v.zaxis[i] = z[i]; }
  const float xa[4] = {x[0], x[1], x[2], 0.0f}, ya[4] = {y[0], y[1], y[2], 0.0f};
  const float p0[4] = {v.P[0][0], v.P[0][1], v.P[0][2], v.P[0][3]}, p1[4] = {v.P[0][4], v.P[0][5], v.P[0][6], v.P[0][7]};
  const float fx = dot4f(xa, p0), fy = dot4f(ya, p1);
  v.ipscale = fx + fy;
}

// CImage::buildMask / buildEdge (image.cpp:327-405) on the host (binary maps are optional).
void build_binary(std::vector<uint8_t>* pyr, const int* w, const int* h, int maxLevel) {
  for (int level = 1; level < maxLevel; ++level) {
    pyr[level].assign((size_t)w[level] * h[level], 0);
    for (int y = 0; y < h[level]; ++y) {
      const int ys[2] = {2 * y, std::min(h[level - 1] - 1, 2 * y + 1)};
      for (int x = 0; x < w[level]; ++x) {
        const int xs[2] = {2 * x, std::min(w[level - 1] - 1, 2 * x + 1)};
        int in = 0;
        for (int j = 0; j < 2; ++j)
          for (int i = 0; i < 2; ++i)
            if (pyr[level - 1][ys[j] * w[level - 1] + xs[i]]) in++;
        pyr[level][y * w[level] + x] = (0 < in) ? 255 : 0;
      }
    }
  }
}

// PMVS_POISON_ALLOC=<byte>: fill new device allocations with that byte (uninitialised-read hunting).
inline void poison_alloc(void* p, size_t bytes) {
  static const int v = [] {
    const char* e = getenv("PMVS_POISON_ALLOC");
    return e ? atoi(e) : -1;
  }();
  if (v >= 0 && p && bytes) {
    (void)hipMemset(p, v & 0xff, bytes);
    (void)hipDeviceSynchronize();
  }
}

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t alloc(size_t count) {
    release();
    n = count;
    if (count == 0) return hipSuccess;
    const hipError_t e = hipMalloc((void**)&p, count * sizeof(T));
    if (e == hipSuccess) poison_alloc(p, count * sizeof(T));
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

}  // namespace

struct pmvs_scene {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t kev[4] = {nullptr, nullptr, nullptr, nullptr};  // around pre / refine / post kernels
  bool last_refine = false;
  DScene ds{};
  int maxLevel = 0;
  std::vector<DView> hviews;
  DBuf<DView> views;
  DBuf<uint32_t> pyr;
  DBuf<uint8_t> masks, edges;
  DBuf<int> vis_off, vis, bindexes;
  DBuf<float> scratch;
  DBuf<DevStats> stats;
  DBuf<RefineJob> jobs;
  FilterBuffers fbuf;
  ExpandBuffers xbuf;
  DBuf<pmvs_patch> fpatches;
  DBuf<int> fkeep;
  DBuf<unsigned long long> digest;  // pmvs_loop_hash
  int grid = 0, refine_grid = 0, tslots = 226014;
  // batches below small_n candidates run the lane form, one candidate per wavefront with its BOBYQA
  // state over the lanes (tslots_small, pmvs_refine_lane.hip): their length is one chain's latency,
  // not the chip's throughput (the C3 loop, gpurun r06d: small launches 1029 -> 687 ms
  // per step against the workgroup form 132042, split point 7000 against 5000 / 10000)
  int tslots_small = 300000, small_n = 7000;
  int refine_cfg(int n) const { return n < small_n ? tslots_small : tslots; }
  // expansion sharding (pmvs_scene_set_shard) and the kept result of pmvs_expand_run(out = NULL)
  int shard_rank = 0, shard_world = 1;
  pmvs_allgather_fn shard_fn = nullptr;
  void* shard_ctx = nullptr;
  pmvs_rccl* shard_rccl = nullptr;  // set: the records go device to device (pmvs_scene_set_shard_rccl)
  // cluster boundary exchange (pmvs_scene_set_cluster)
  int cl_rank = 0, cl_world = 1;
  pmvs_allgather_fn cl_fn = nullptr;
  void* cl_ctx = nullptr;
  pmvs_rccl* cl_rccl = nullptr;
  DBuf<unsigned char> cl_shared;
  DBuf<int> cl_ids, cl_id2idx;
  int cl_maxid = -1;
  ClusterBuffers cbuf;
  RefineHost rhost;             // host libm step of every refine batch (launch_refine)
  int xkept = -1, lkept = -1;   // models kept on the device for pmvs_expand_fetch / pmvs_loop_fetch
  std::vector<pmvs_patch> skept; // seeds kept for pmvs_seed_fetch (pmvs_seed_run with out = NULL, cap = 0)
  bool seeds_kept = false;
  std::vector<int> xalive;
  DBuf<pmvs_patch> fpatches2;   // compaction target of pmvs_run_loop
  FeatBuffers feat;             // feature-detection scratch (pmvs_detect_features)
  // host copies the seed phase's control logic reads (canAdd masks, collectImages inputs)
  std::vector<std::vector<uint8_t>> hmask_level;  // per view, the binary mask at the scene level (empty = none)
  std::vector<int> hvis_off, hvis;
  int sequence = -1;
  // staging for host-pointer calls
  DBuf<pmvs_candidate> cand;
  DBuf<pmvs_refined> res;
  DBuf<pmvs_eval_query> evq;
  DBuf<double> evout;
  DBuf<pmvs_tex_query> tq;
  DBuf<float> tout;
  DBuf<int> tvalid;
  ~pmvs_scene() {
    cl_shared.release(); cl_ids.release(); cl_id2idx.release();
    fpatches2.release(); views.release(); pyr.release(); masks.release(); edges.release(); vis_off.release(); vis.release();
    bindexes.release(); scratch.release(); stats.release(); jobs.release(); fpatches.release(); fkeep.release(); digest.release(); cand.release(); res.release(); evq.release();
    evout.release(); tq.release(); tout.release(); tvalid.release();
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    for (hipEvent_t e : kev)
      if (e) (void)hipEventDestroy(e);
    if (stream) d2h_stage_release(stream);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {
template <class T>
pmvs_status ensure(DBuf<T>& b, size_t n) {
  if (b.n >= n) return PMVS_OK;
  hipError_t e = b.alloc(n);
  if (e != hipSuccess) return fail(PMVS_ENOMEM, "hipMalloc(%zu bytes): %s", n * sizeof(T), hipGetErrorString(e));
  return PMVS_OK;
}
int grow_alive(pmvs_scene* sc, int n) {
  ExpandBuffers& X = sc->xbuf;
  if ((size_t)n <= X.cap_alive && X.alive) return 0;
  if (X.alive) (void)hipFree(X.alive);
  X.alive = nullptr;
  X.cap_alive = (size_t)n;
  if (hipMalloc((void**)&X.alive, (size_t)n * sizeof(int)) != hipSuccess) return 1;
  poison_alloc(X.alive, (size_t)n * sizeof(int));
  return 0;
}
}  // namespace

extern "C" {

const char* pmvs_last_error(void) { return g_err.c_str(); }

int32_t pmvs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

pmvs_status pmvs_scene_create(const pmvs_scene_desc* d, int32_t device, pmvs_scene** out) {
  if (!d || !out) return fail(PMVS_EINVAL, "null argument");
  *out = nullptr;
  if (d->num_views < 1 || d->num_targets < 1 || d->num_targets > d->num_views)
    return fail(PMVS_EINVAL, "num_views=%d num_targets=%d", d->num_views, d->num_targets);
  if (d->level < 0 || d->level > PMVS_MAX_LEVEL) return fail(PMVS_EUNSUPPORTED, "level %d outside 0..%d", d->level, PMVS_MAX_LEVEL);
  if (d->wsize != 5 && d->wsize != 7 && d->wsize != 9) return fail(PMVS_EUNSUPPORTED, "wsize %d (supported: 5, 7, 9)", d->wsize);
  if (d->csize < 1) return fail(PMVS_EINVAL, "csize %d", d->csize);
  if (d->min_image_num < 1) return fail(PMVS_EINVAL, "minImageNum %d", d->min_image_num);
  const int tau = std::min(d->min_image_num * 2, d->num_views);
  if (tau > PMVS_MAX_TAU) return fail(PMVS_EUNSUPPORTED, "tau = min(2*minImageNum, num) = %d > %d", tau, PMVS_MAX_TAU);
  if (!d->views || !d->visdata2_offsets) return fail(PMVS_EINVAL, "views / visdata2 missing");
  {  // the organizer and commit records index target cells (pgrids) with 32-bit ints
    long long cells = 0;
    for (int t = 0; t < d->num_targets; ++t) {
      long long w = d->views[t].width, h = d->views[t].height;
      for (int l = 0; l < d->level; ++l) { w /= 2; h /= 2; }
      const long long gw = (w + d->csize - 1) / d->csize, gh = (h + d->csize - 1) / d->csize;
      // pmvs_patch keeps cell coordinates as int16 (include/pmvs_amd.h)
      if (gw > 32767 || gh > 32767) return fail(PMVS_EUNSUPPORTED, "view %d: %lld x %lld cells (at most 32767 a side)", t, gw, gh);
      cells += gw * gh;
    }
    if (cells > INT_MAX) return fail(PMVS_EUNSUPPORTED, "%lld target cells at level %d exceed 2^31 - 1", cells, d->level);
  }
  if (d->num_views > 32767) return fail(PMVS_EUNSUPPORTED, "%d views (pmvs_patch image indexes are 16-bit)", d->num_views);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PMVS_EDEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(PMVS_EINVAL, "device %d of %d", device, ndev);
  HIPCHK(hipSetDevice(device));

  (void)hipGetLastError();  // launches below are checked with hipGetLastError: start from a clean slate
  pmvs_scene* sc = new pmvs_scene();
  sc->device = device;
  const int num = d->num_views;
  const int maxLevel = std::max(1, d->level + 3);
  sc->maxLevel = maxLevel;
  auto bail = [&](pmvs_status st) {
    delete sc;
    return st;
  };
  if (hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&sc->ev0) != hipSuccess || hipEventCreate(&sc->ev1) != hipSuccess ||
      hipEventCreate(&sc->kev[0]) != hipSuccess || hipEventCreate(&sc->kev[1]) != hipSuccess ||
      hipEventCreate(&sc->kev[2]) != hipSuccess || hipEventCreate(&sc->kev[3]) != hipSuccess)
    return bail(fail(PMVS_EDEVICE, "stream/event creation failed"));

  // ---- views: sizes, cameras, pyramid offsets
  sc->hviews.assign(num, DView{});
  long long words = 0;
  bool anyMask = false, anyEdge = false;
  for (int i = 0; i < num; ++i) {
    const pmvs_view_desc& vd = d->views[i];
    if (vd.width < 8 || vd.height < 8 || !vd.rgb) return bail(fail(PMVS_EINVAL, "view %d: bad image", i));
    DView& v = sc->hviews[i];
    v.w[0] = vd.width;
    v.h[0] = vd.height;
    for (int l = 1; l < MAXL; ++l) {
      v.w[l] = l < maxLevel ? v.w[l - 1] / 2 : 0;
      v.h[l] = l < maxLevel ? v.h[l - 1] / 2 : 0;
    }
    for (int l = 0; l < MAXL; ++l) {
      v.pyr_off[l] = words;
      if (l < maxLevel) words += (long long)v.w[l] * v.h[l] + 1;  // +1 pad word: bilinear reads lx+1
      v.mask_off[l] = -1;
      v.edge_off[l] = -1;
    }
    setup_camera(v, vd.projection, maxLevel);
    anyMask |= vd.mask != nullptr;
    anyEdge |= vd.edge != nullptr;
  }
  if (hipMalloc((void**)&sc->pyr.p, words * sizeof(uint32_t)) != hipSuccess)
    return bail(fail(PMVS_ENOMEM, "pyramid: %lld words", words));
  sc->pyr.n = words;
  if (memset_big(sc->pyr.p, 0, words * sizeof(uint32_t), sc->stream) != hipSuccess)
    return bail(fail(PMVS_EDEVICE, "pyramid: clearing %lld words", words));

  // ---- pyramids on device: RGB level chain (CImage::buildImage) then RGBA packing
  {
    size_t maxrgb = 0;
    for (int i = 0; i < num; ++i) maxrgb = std::max(maxrgb, (size_t)d->views[i].width * d->views[i].height * 3);
    uint8_t *a = nullptr, *b = nullptr, *pin = nullptr;
    // host images go up through a pinned bounce buffer, in pieces: a direct pageable copy out of a
    // multi-GB host array (70 views x 8K = 7 GB, sliced per view) failed with "invalid resource
    // handle" (gpurun r03q), and pinned pieces also keep the copy at full PCIe rate
    constexpr size_t kPin = size_t(32) << 20;
    if (hipMalloc((void**)&a, maxrgb) != hipSuccess || hipMalloc((void**)&b, maxrgb) != hipSuccess ||
        hipHostMalloc((void**)&pin, 2 * kPin, hipHostMallocDefault) != hipSuccess) {
      if (a) (void)hipFree(a);
      if (b) (void)hipFree(b);
      return bail(fail(PMVS_ENOMEM, "pyramid staging"));
    }
    hipEvent_t piece_done[2];
    bool ev_ok = hipEventCreate(&piece_done[0]) == hipSuccess;
    ev_ok = hipEventCreate(&piece_done[1]) == hipSuccess && ev_ok;
    // double-buffered: piece k is copied into half k % 2 once that half's previous upload finished
    auto upload = [&](uint8_t* dst, const uint8_t* src, size_t bytes) -> hipError_t {
      if (!ev_ok) return hipErrorOutOfMemory;
      bool used[2] = {false, false};
      for (size_t off = 0, k = 0; off < bytes; off += kPin, ++k) {
        const int h = (int)(k & 1);
        const size_t m = bytes - off < kPin ? bytes - off : kPin;
        if (used[h]) {
          const hipError_t e = hipEventSynchronize(piece_done[h]);
          if (e != hipSuccess) return e;
        }
        std::memcpy(pin + h * kPin, src + off, m);
        hipError_t e = hipMemcpyAsync(dst + off, pin + h * kPin, m, hipMemcpyHostToDevice, sc->stream);
        if (e == hipSuccess) e = hipEventRecord(piece_done[h], sc->stream);
        if (e != hipSuccess) return e;
        used[h] = true;
      }
      return hipSuccess;
    };
    pmvs_status st = PMVS_OK;
    for (int i = 0; i < num && st == PMVS_OK; ++i) {
      const DView& v = sc->hviews[i];
      const size_t bytes0 = (size_t)v.w[0] * v.h[0] * 3;
      const char* step = "upload";
      int lv = 0;
      hipError_t e = upload(a, d->views[i].rgb, bytes0);
      if (e == hipSuccess && (step = "pack")) e = launch_pack_rgba(a, sc->pyr.p + v.pyr_off[0], (long long)v.w[0] * v.h[0], sc->stream);
      uint8_t* src = a;
      uint8_t* dst = b;
      for (int l = 1; l < maxLevel && e == hipSuccess; ++l) {
        lv = l;
        step = "downsample";
        e = launch_build_level(src, v.w[l - 1], v.h[l - 1], dst, v.w[l], v.h[l], sc->stream);
        if (e == hipSuccess && (step = "pack")) e = launch_pack_rgba(dst, sc->pyr.p + v.pyr_off[l], (long long)v.w[l] * v.h[l], sc->stream);
        std::swap(src, dst);
      }
      if (e == hipSuccess && (step = "sync")) e = hipStreamSynchronize(sc->stream);  // staging reused per view
      if (e != hipSuccess)
        st = fail(PMVS_EDEVICE, "pyramid build (view %d, level %d, %s): %s", i, lv, step, hipGetErrorString(e));
    }
    (void)hipStreamSynchronize(sc->stream);
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipHostFree(pin);
    if (ev_ok) {
      (void)hipEventDestroy(piece_done[0]);
      (void)hipEventDestroy(piece_done[1]);
    }
    if (st != PMVS_OK) return bail(st);
  }

  // ---- optional masks / edges (binary pyramids built on the host)
  auto upload_binary = [&](bool any, bool isMask, DBuf<uint8_t>& buf) -> pmvs_status {
    if (!any) return PMVS_OK;
    std::vector<uint8_t> all;
    for (int i = 0; i < num; ++i) {
      const pmvs_view_desc& vd = d->views[i];
      const uint8_t* m0 = isMask ? vd.mask : vd.edge;
      DView& v = sc->hviews[i];
      if (!m0) continue;
      std::vector<uint8_t> pyr[MAXL];
      pyr[0].resize((size_t)v.w[0] * v.h[0]);
      for (size_t k = 0; k < pyr[0].size(); ++k)
        pyr[0][k] = isMask ? ((127 < (int)m0[k]) ? 255 : 0) : ((1 < m0[k]) ? 255 : 0);  // image.cpp:159-180
      build_binary(pyr, v.w, v.h, maxLevel);
      if (isMask) sc->hmask_level[i] = pyr[d->level];
      for (int l = 0; l < maxLevel; ++l) {
        (isMask ? v.mask_off[l] : v.edge_off[l]) = (long long)all.size();
        all.insert(all.end(), pyr[l].begin(), pyr[l].end());
      }
    }
    if (buf.alloc(all.size()) != hipSuccess) return fail(PMVS_ENOMEM, "mask/edge upload");
    if (hipMemcpy(buf.p, all.data(), all.size(), hipMemcpyHostToDevice) != hipSuccess)
      return fail(PMVS_EDEVICE, "mask/edge copy");
    return PMVS_OK;
  };
  sc->hmask_level.assign(num, std::vector<uint8_t>());
  pmvs_status st = upload_binary(anyMask, true, sc->masks);
  if (st == PMVS_OK) st = upload_binary(anyEdge, false, sc->edges);
  if (st != PMVS_OK) return bail(st);

  // ---- tables
  std::vector<int> voff(d->visdata2_offsets, d->visdata2_offsets + num + 1);
  const int nvis = voff[num];
  sc->hvis_off = voff;
  sc->hvis.assign(d->visdata2, d->visdata2 + nvis);
  sc->sequence = d->sequence;
  for (int k = 0; k < nvis; ++k)
    if (d->visdata2[k] < 0 || d->visdata2[k] >= num) return bail(fail(PMVS_EINVAL, "visdata2[%d] = %d", k, d->visdata2[k]));
  for (int k = 0; k < d->num_bindexes; ++k)
    if (d->bindexes[k] < 0 || d->bindexes[k] >= num) return bail(fail(PMVS_EINVAL, "bindexes[%d]", k));
  if (sc->views.alloc(num) != hipSuccess || sc->vis_off.alloc(num + 1) != hipSuccess ||
      sc->vis.alloc(std::max(1, nvis)) != hipSuccess || sc->bindexes.alloc(std::max(1, d->num_bindexes)) != hipSuccess ||
      sc->stats.alloc(1) != hipSuccess)
    return bail(fail(PMVS_ENOMEM, "scene tables"));
  if (hipMemcpy(sc->views.p, sc->hviews.data(), num * sizeof(DView), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(sc->vis_off.p, voff.data(), (num + 1) * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
      (nvis && hipMemcpy(sc->vis.p, d->visdata2, nvis * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) ||
      (d->num_bindexes && hipMemcpy(sc->bindexes.p, d->bindexes, d->num_bindexes * sizeof(int), hipMemcpyHostToDevice) != hipSuccess))
    return bail(fail(PMVS_EDEVICE, "scene table copy"));

  // ---- persistent grid: enough single-wave workgroups to fill every CU
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return bail(fail(PMVS_EDEVICE, "device properties"));
  int gpc = 8;  // persistent single-wave workgroups per CU (pre/post, organizer and filter kernels)
  if (const char* e = getenv("PMVS_GRID_WAVES_PER_CU")) gpc = std::max(1, std::min(32, atoi(e)));
  sc->grid = std::max(1, prop.multiProcessorCount) * gpc;
  // tuning knobs (defaults measured on MI355X): refine wavefronts per CU and the
  // number of texture slots one cooperative objective chunk packs
  int wpc = 8;  // 1206: 19.5 KB LDS, <= 256 registers -> 8 resident per CU
  if (const char* e = getenv("PMVS_REFINE_WAVES_PER_CU")) wpc = std::max(1, std::min(32, atoi(e)));
  if (const char* e = getenv("PMVS_REFINE_CONFIG")) {  // one layout for every batch size
    sc->tslots = atoi(e);
    if (!refine_config_supported(sc->tslots)) sc->tslots = 1206;
    sc->tslots_small = sc->tslots;
  }
  if (const char* e = getenv("PMVS_REFINE_LARGE_CONFIG")) {  // the layout of the batches >= small_n only
    const int v = atoi(e);
    if (refine_config_supported(v)) sc->tslots = v;
  }
  if (const char* e = getenv("PMVS_REFINE_SMALL_CONFIG")) {  // the layout of the batches < small_n only
    const int v = atoi(e);
    if (refine_config_supported(v)) sc->tslots_small = v;
  }
  if (const char* e = getenv("PMVS_REFINE_SMALL_N")) sc->small_n = std::max(0, atoi(e));
  sc->refine_grid = std::max(1, prop.multiProcessorCount) * wpc;
  // per-workgroup global scratch: the scene grid, or pre / post's larger grid (prepost_waves)
  const size_t scratch_blocks = (size_t)sc->grid * std::max(2, prepost_waves()) / 2;
  if (sc->scratch.alloc(scratch_blocks * PMVS_MAX_IMAGES * PMVS_MAX_IMAGES) != hipSuccess)
    return bail(fail(PMVS_ENOMEM, "scratch"));

  DScene& s = sc->ds;
  s.views = sc->views.p;
  s.pyr = sc->pyr.p;
  s.masks = sc->masks.p;
  s.edges = sc->edges.p;
  s.vis_off = sc->vis_off.p;
  s.vis = sc->vis.p;
  s.bindexes = sc->bindexes.p;
  s.scratch = sc->scratch.p;
  s.nb = d->num_bindexes;
  s.num = num;
  s.tnum = d->num_targets;
  s.level = d->level;
  s.csize = d->csize;
  s.wsize = d->wsize;
  s.minImageNum = d->min_image_num;
  s.tau = tau;
  s.anyMask = anyMask ? 1 : 0;
  // CFindMatch::init thresholds (findMatch.cpp:92-106)
  s.nccThreshold = d->threshold;
  s.nccThresholdBefore = d->threshold - 0.3f;
  s.maxAngle = d->max_angle;
  const float angle0 = (float)(60.0f * M_PI / 180.0f);
  s.angle1 = (float)(60.0f * M_PI / 180.0f);
  s.athreshold = (float)std::cos((double)angle0);
  s.cosAngle1 = std::cos((double)s.angle1);
  s.sortThreshold = (float)(1.0f - std::cos(10.0 * M_PI / 180.0));
  s.ascale = (float)(M_PI / 48.0f);
  s.log2f = (float)std::log(2.0);
  s.quad = d->quad_threshold;
  s.depth = 0;
  if (hipStreamSynchronize(sc->stream) != hipSuccess) return bail(fail(PMVS_EDEVICE, "scene upload"));
  *out = sc;
  return PMVS_OK;
}

void pmvs_scene_destroy(pmvs_scene* scene) {
  if (!scene) return;
  (void)hipSetDevice(scene->device);
  (void)hipStreamSynchronize(scene->stream);
  delete scene;
}

pmvs_status pmvs_set_thresholds(pmvs_scene* sc, float ncc, float ncc_before, int32_t depth) {
  if (!sc) return fail(PMVS_EINVAL, "null scene");
  if (depth < 0) return fail(PMVS_EINVAL, "depth %d", depth);
  sc->ds.depth = depth;
  sc->ds.nccThreshold = ncc;
  sc->ds.nccThresholdBefore = ncc_before;
  return PMVS_OK;
}

pmvs_status pmvs_scene_get_level(pmvs_scene* sc, int32_t view, int32_t level, uint8_t* out, int32_t* width,
                                 int32_t* height) {
  if (!sc) return fail(PMVS_EINVAL, "null scene");
  if (view < 0 || view >= sc->ds.num || level < 0 || level >= sc->maxLevel) return fail(PMVS_EINVAL, "view/level");
  const DView& v = sc->hviews[view];
  if (width) *width = v.w[level];
  if (height) *height = v.h[level];
  if (!out) return PMVS_OK;
  HIPCHK(hipSetDevice(sc->device));
  const long long npix = (long long)v.w[level] * v.h[level];
  uint8_t* tmp = nullptr;
  HIPCHK(hipMalloc((void**)&tmp, npix * 3));
  hipError_t e = launch_unpack_rgba(sc->pyr.p + v.pyr_off[level], tmp, npix, sc->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, tmp, npix * 3, hipMemcpyDeviceToHost, sc->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(sc->stream);
  (void)hipFree(tmp);
  if (e != hipSuccess) return fail(PMVS_EDEVICE, "get_level: %s", hipGetErrorString(e));
  return PMVS_OK;
}

// ---- feature detection (CDetectFeatures::run, detectFeatures.cpp:47-124)
namespace {

// CDetector::setGaussI (detector.cpp:29-49): float weights, exp() of a float argument evaluated
// by the double C exp (unqualified exp(float) in that TU; probed), float normalisation.
FeatFilter gauss_i(float sigma) {
  FeatFilter f{};
  const int m = (int)std::ceil((double)(2 * sigma));
  f.n = 2 * m + 1;
  float denom = 0.0f;
  for (int x = 0; x < f.n; ++x) {
    const int xt = x - m;
    const float arg = (float)(-(xt * xt)) / (2 * sigma * sigma);
    const float d = (float)std::exp((double)arg);
    f.w[x] = d;
    denom += d;
  }
  for (int x = 0; x < f.n; ++x) f.w[x] /= denom;
  return f;
}

// The result multisets of one detector (harris.cpp:251-261 / dog.cpp:192-202) read from the
// largest element (detectFeatures.cpp:84-88, 103-107): blocks are inserted in raster order, each
// block's points in ascending order, so equal responses come out in reverse insertion order.
void order_points(const FeatPoint* pts, const int* cnt, int nb, int type, std::vector<pmvs_point>& out) {
  struct Item { float r; int64_t seq; float x, y; };
  std::vector<Item> v;
  int64_t seq = 0;
  for (int b = 0; b < nb; ++b)
    for (int k = 0; k < cnt[b]; ++k) {
      const FeatPoint& p = pts[4 * b + k];
      v.push_back({p.response, seq++, p.x, p.y});
    }
  std::sort(v.begin(), v.end(), [](const Item& a, const Item& b) {
    if (a.r != b.r) return a.r > b.r;
    return a.seq > b.seq;
  });
  for (const Item& it : v) out.push_back(pmvs_point{it.x, it.y, it.r, type});
}

}  // namespace

pmvs_status pmvs_detect_features(pmvs_scene* sc, int32_t view, int32_t fcsize, pmvs_point* out, int32_t cap,
                                 int32_t* n_out) {
  if (!sc || !n_out || (cap > 0 && !out)) return fail(PMVS_EINVAL, "null argument");
  if (view < 0 || view >= sc->ds.num) return fail(PMVS_EINVAL, "view %d", view);
  if (fcsize < 1) return fail(PMVS_EINVAL, "fcsize %d", fcsize);
  HIPCHK(hipSetDevice(sc->device));
  const int level = sc->ds.level;
  const DView& v = sc->hviews[view];
  FeatJob j{};
  j.W = v.w[level];
  j.H = v.h[level];
  j.pyr = sc->pyr.p + v.pyr_off[level];
  j.mask = v.mask_off[level] >= 0 ? sc->masks.p + v.mask_off[level] : nullptr;
  j.edge = v.edge_off[level] >= 0 ? sc->edges.p + v.edge_off[level] : nullptr;
  // CHarris::run: gridsize = gspeedup * 2 (harris.cpp:216-221), gspeedup = fcsize (16 in findMatch.cpp:81)
  j.gsize = fcsize * 2;
  j.bw = (j.W + j.gsize - 1) / j.gsize;
  j.bh = (j.H + j.gsize - 1) / j.gsize;
  const float sigma = 4.0f;  // detectFeatures.cpp:73
  j.harris_margin = ((2 * (int)std::ceil((double)(2 * sigma)) + 1)) / 2;  // (int)_gaussD.size() / 2
  j.dfilter.n = 3;
  j.dfilter.w[0] = -0.5f; j.dfilter.w[1] = 0.0f; j.dfilter.w[2] = 0.5f;  // harris.cpp:151
  j.ifilter.n = 3;
  j.ifilter.w[0] = j.ifilter.w[1] = j.ifilter.w[2] = (float)(1.0 / 3.0);  // harris.cpp:153
  j.gaussI = gauss_i(sigma);
  // CDifferenceOfGaussians::run (dog.cpp:130-160), firstScale 1, lastScale 3 (detectFeatures.cpp:75-76)
  const float first = 1.0f, last = 3.0f;
  const float step = (float)std::pow(2.0, 0.5);  // pow(2.0f, 1 / 2.0f): the double C pow
  const int steps = std::max(4, (int)std::ceil(std::log((double)(last / first)) / std::log((double)step)));
  if (steps != 4) return fail(PMVS_EUNSUPPORTED, "DoG with %d steps", steps);
  const float scales[5] = {first, first * step, first * step * step, (float)(first * std::pow((double)step, 3.0)),
                           (float)(first * std::pow((double)step, 4.0))};
  for (int k = 0; k < 5; ++k) j.dog_gauss[k] = gauss_i(scales[k]);
  for (int k = 0; k < 2; ++k) j.dog_margin[k] = (int)std::ceil((double)(2 * scales[3 + k]));
  for (const FeatFilter* f : {&j.gaussI, &j.dog_gauss[4]})
    if (f->n > 32) return fail(PMVS_EUNSUPPORTED, "filter with %d taps", f->n);
  HIPCHK(detect_features(j, sc->feat, sc->stream));
  const int nb = j.bw * j.bh;
  std::vector<FeatPoint> pts((size_t)nb * 8);
  std::vector<int> cnt((size_t)nb * 2);
  HIPCHK(hipMemcpyAsync(pts.data(), sc->feat.pts, pts.size() * sizeof(FeatPoint), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipMemcpyAsync(cnt.data(), sc->feat.cnt, cnt.size() * sizeof(int), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipStreamSynchronize(sc->stream));
  std::vector<pmvs_point> all;
  order_points(pts.data(), cnt.data(), nb, 0, all);
  order_points(pts.data() + 4 * (size_t)nb, cnt.data() + nb, nb, 1, all);
  *n_out = (int32_t)all.size();
  if (out) std::memcpy(out, all.data(), std::min<size_t>(all.size(), (size_t)std::max(cap, 0)) * sizeof(pmvs_point));
  return PMVS_OK;
}

pmvs_status pmvs_seed_run(pmvs_scene* sc, const pmvs_point* points, const int32_t* num_points, int32_t batch,
                          pmvs_patch* out, int32_t cap, int32_t* n_out, pmvs_seed_stats* stats) {
  if (!sc || !num_points || !n_out || cap < 0 || (cap > 0 && !out)) return fail(PMVS_EINVAL, "null argument");
  const bool keep = !out && cap == 0;  // the scene keeps the seeds; pmvs_seed_fetch copies them out
  sc->seeds_kept = false;
  std::vector<pmvs_patch>().swap(sc->skept);
  if (sc->ds.depth != 0) return fail(PMVS_EINVAL, "the seed phase runs at depth 0 (scene depth %d)", sc->ds.depth);
  long long np = 0;
  for (int i = 0; i < sc->ds.num; ++i) {
    if (num_points[i] < 0) return fail(PMVS_EINVAL, "num_points[%d] = %d", i, num_points[i]);
    np += num_points[i];
  }
  if (np > 0 && !points) return fail(PMVS_EINVAL, "null points");
  for (long long k = 0; k < np; ++k)
    if (!(points[k].x >= 0.0f && points[k].y >= 0.0f)) return fail(PMVS_EINVAL, "point %lld outside the image", k);
  *n_out = 0;
  if (stats) std::memset(stats, 0, sizeof(*stats));
  HIPCHK(hipSetDevice(sc->device));
  SeedInput in;
  in.points = points;
  in.npts = num_points;
  in.vis_off = sc->hvis_off.data();
  in.vis = sc->hvis.data();
  in.sequence = sc->sequence;
  in.angle0 = (float)(60.0f * M_PI / 180.0f);  // findMatch.cpp:92
  for (int i = 0; i < sc->ds.num; ++i) in.mask_level.push_back(sc->hmask_level[i].empty() ? nullptr : sc->hmask_level[i].data());
  in.batch = batch > 0 ? batch : 16384;
  in.per_cell = 4;
  if (const char* e = getenv("PMVS_SEED_PER_CELL")) in.per_cell = std::max(1, atoi(e));
  in.lookahead = 1;  // speculation into the next images: measured no fewer rounds
  if (const char* e = getenv("PMVS_SEED_LOOKAHEAD")) in.lookahead = std::max(1, atoi(e));
  in.spec_near = 2048;
  if (const char* e = getenv("PMVS_SEED_NEAR")) in.spec_near = std::max(1, atoi(e));
  HIPCHK(hipMemsetAsync(sc->stats.p, 0, sizeof(DevStats), sc->stream));
  sc->rhost.prof = false;
  RefineFn refine = [&](const pmvs_candidate* d_in, int m, pmvs_refined* d_out) -> hipError_t {
    if (ensure(sc->jobs, m)) return hipErrorOutOfMemory;
    hipError_t e = hipMemsetAsync(&sc->stats.p->queue, 0, 3 * sizeof(unsigned long long), sc->stream);
    if (e != hipSuccess) return e;
    return launch_refine(sc->ds, d_in, sc->jobs.p, d_out, m, sc->stats.p, sc->grid, sc->refine_grid, sc->refine_cfg(m),
                         sc->stream, sc->kev, sc->rhost);
  };
  SeedOutput so;
  const hipError_t e = seed_pass(sc->ds, sc->hviews, in, sc->stream, refine, so);
  if (e == hipErrorOutOfMemory) return fail(PMVS_ENOMEM, "seed phase: device memory");
  if (e == hipErrorNotSupported)
    return fail(PMVS_EUNSUPPORTED, "seed phase: a candidate's image list exceeds %d entries", PMVS_MAX_IMAGES);
  HIPCHK(e);
  sc->last_refine = false;
  const int ns = (int)so.seeds.size();
  *n_out = ns;
  if (stats) {
    stats->trial = so.stats[0]; stats->pass = so.stats[1]; stats->fail0 = so.stats[2]; stats->fail1 = so.stats[3];
    stats->refined = so.stats[4]; stats->rounds = so.stats[5]; stats->candidates = so.stats[6];
    stats->wall_ms = so.wall_ms; stats->gen_ms = so.gen_ms; stats->refine_ms = so.refine_ms;
  }
  if (keep) {
    sc->skept.swap(so.seeds);
    sc->seeds_kept = true;
    return PMVS_OK;
  }
  if (ns > cap) return fail(PMVS_EINVAL, "seed phase: %d seeds, capacity %d", ns, cap);
  if (ns) std::memcpy(out, so.seeds.data(), (size_t)ns * sizeof(pmvs_patch));
  return PMVS_OK;
}

pmvs_status pmvs_seed_fetch(pmvs_scene* sc, pmvs_patch* out, int32_t n) {
  if (!sc || n < 0 || (n > 0 && !out)) return fail(PMVS_EINVAL, "invalid argument");
  if (!sc->seeds_kept || (size_t)n != sc->skept.size())
    return fail(PMVS_EINVAL, "seed_fetch: %d seeds kept, %d asked", sc->seeds_kept ? (int)sc->skept.size() : -1, n);
  if (n) std::memcpy(out, sc->skept.data(), (size_t)n * sizeof(pmvs_patch));
  sc->seeds_kept = false;
  std::vector<pmvs_patch>().swap(sc->skept);
  return PMVS_OK;
}

pmvs_status pmvs_grab_tex(pmvs_scene* sc, const pmvs_tex_query* q, int32_t n, float* out_tex, int32_t* out_valid) {
  if (!sc || (n > 0 && (!q || !out_tex || !out_valid))) return fail(PMVS_EINVAL, "null argument");
  if (n <= 0) return PMVS_OK;
  for (int i = 0; i < n; ++i)
    if (q[i].view < 0 || q[i].view >= sc->ds.num) return fail(PMVS_EINVAL, "query %d: view %d", i, q[i].view);
  HIPCHK(hipSetDevice(sc->device));
  const int len = 3 * sc->ds.wsize * sc->ds.wsize;
  pmvs_status st;
  if ((st = ensure(sc->tq, n)) || (st = ensure(sc->tout, (size_t)n * len)) || (st = ensure(sc->tvalid, n))) return st;
  HIPCHK(hipMemcpyAsync(sc->tq.p, q, n * sizeof(pmvs_tex_query), hipMemcpyHostToDevice, sc->stream));
  HIPCHK(launch_grab_tex(sc->ds, sc->tq.p, n, sc->tout.p, sc->tvalid.p, sc->stream));
  HIPCHK(hipMemcpyAsync(out_tex, sc->tout.p, (size_t)n * len * sizeof(float), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipMemcpyAsync(out_valid, sc->tvalid.p, n * sizeof(int), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipStreamSynchronize(sc->stream));
  return PMVS_OK;
}

static void fill_stats(const DevStats& d, int64_t n, float ms, pmvs_stats* st) {
  if (!st) return;
  st->candidates = n;
  st->accepted = (int64_t)d.accepted;
  st->fail_pre = (int64_t)d.fail_pre;
  st->fail_post = (int64_t)d.fail_post;
  st->refine_failed = (int64_t)d.refine_failed;
  st->evals = (int64_t)d.evals;
  st->tex_valid = (int64_t)d.tex_valid;
  st->tex_grabs = (int64_t)d.tex_grabs;
  st->kernel_ms = ms;
  st->opt_cycles = (int64_t)d.cyc_opt;
  st->objective_cycles = (int64_t)d.cyc_eval;
  st->rounds = (int64_t)d.rounds;
  st->chunks = (int64_t)d.chunks;
  for (int i = 0; i < 8; ++i) st->prof[i] = (int64_t)d.prof[i];
}

pmvs_status pmvs_incc_eval(pmvs_scene* sc, const pmvs_eval_query* q, int32_t n, double* out_f, pmvs_stats* stats) {
  if (!sc || (n > 0 && (!q || !out_f))) return fail(PMVS_EINVAL, "null argument");
  if (n <= 0) return PMVS_OK;
  for (int i = 0; i < n; ++i) {
    if (q[i].num_images < 1 || q[i].num_images > PMVS_MAX_TAU) return fail(PMVS_EINVAL, "query %d: num_images", i);
    for (int k = 0; k < q[i].num_images; ++k)
      if (q[i].images[k] < 0 || q[i].images[k] >= sc->ds.num) return fail(PMVS_EINVAL, "query %d: image", i);
  }
  HIPCHK(hipSetDevice(sc->device));
  pmvs_status st;
  if ((st = ensure(sc->evq, n)) || (st = ensure(sc->evout, n))) return st;
  HIPCHK(hipMemcpyAsync(sc->evq.p, q, n * sizeof(pmvs_eval_query), hipMemcpyHostToDevice, sc->stream));
  HIPCHK(hipMemsetAsync(sc->stats.p, 0, sizeof(DevStats), sc->stream));
  HIPCHK(hipEventRecord(sc->ev0, sc->stream));
  HIPCHK(launch_incc_eval(sc->ds, sc->evq.p, n, sc->evout.p, sc->stats.p, sc->stream));
  HIPCHK(hipEventRecord(sc->ev1, sc->stream));
  HIPCHK(hipMemcpyAsync(out_f, sc->evout.p, n * sizeof(double), hipMemcpyDeviceToHost, sc->stream));
  DevStats ds{};
  HIPCHK(hipMemcpyAsync(&ds, sc->stats.p, sizeof(DevStats), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipStreamSynchronize(sc->stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, sc->ev0, sc->ev1));
  fill_stats(ds, n, ms, stats);
  return PMVS_OK;
}

static pmvs_status check_candidates(const pmvs_scene* sc, const pmvs_candidate* in, int n) {
  for (int i = 0; i < n; ++i) {
    if (in[i].num_images < 1 || in[i].num_images > PMVS_MAX_IMAGES) return fail(PMVS_EINVAL, "candidate %d: num_images %d", i, in[i].num_images);
    for (int k = 0; k < in[i].num_images; ++k)
      if (in[i].images[k] < 0 || in[i].images[k] >= sc->ds.num) return fail(PMVS_EINVAL, "candidate %d: image %d", i, in[i].images[k]);
  }
  return PMVS_OK;
}

pmvs_status pmvs_refine_batch_device(pmvs_scene* sc, const pmvs_candidate* d_in, int32_t n, pmvs_refined* d_out) {
  if (!sc || (n > 0 && (!d_in || !d_out))) return fail(PMVS_EINVAL, "null argument");
  if (sc->ds.depth != 0)
    return fail(PMVS_EUNSUPPORTED, "refine at depth %d: the depth >= 1 postProcess steps (setVImagesVGrids, check) "
                "are not part of pmvs_refine_batch in this release", sc->ds.depth);
  if (n <= 0) return PMVS_OK;
  HIPCHK(hipSetDevice(sc->device));
  pmvs_status st;
  if ((st = ensure(sc->jobs, n))) return st;
  HIPCHK(hipMemsetAsync(sc->stats.p, 0, sizeof(DevStats), sc->stream));
  HIPCHK(hipEventRecord(sc->ev0, sc->stream));
  HIPCHK(launch_refine(sc->ds, d_in, sc->jobs.p, d_out, n, sc->stats.p, sc->grid, sc->refine_grid, sc->refine_cfg(n), sc->stream,
                       sc->kev, sc->rhost));
  HIPCHK(hipEventRecord(sc->ev1, sc->stream));
  sc->last_refine = true;
  return PMVS_OK;
}

pmvs_status pmvs_scene_sync(pmvs_scene* sc, pmvs_stats* stats) {
  if (!sc) return fail(PMVS_EINVAL, "null scene");
  HIPCHK(hipSetDevice(sc->device));
  DevStats ds{};
  HIPCHK(hipMemcpyAsync(&ds, sc->stats.p, sizeof(DevStats), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipStreamSynchronize(sc->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, sc->ev0, sc->ev1) != hipSuccess) ms = 0;
  fill_stats(ds, (int64_t)(ds.queue > 0 ? ds.queue : 0), ms, stats);
  if (stats && sc->last_refine) {
    float a = 0, b = 0, c = 0;
    if (hipEventElapsedTime(&a, sc->kev[0], sc->kev[1]) == hipSuccess) stats->pre_ms = a;
    if (hipEventElapsedTime(&b, sc->kev[1], sc->kev[2]) == hipSuccess) stats->refine_ms = b;
    if (hipEventElapsedTime(&c, sc->kev[2], sc->kev[3]) == hipSuccess) stats->post_ms = c;
  }
  if (stats) {
    // queue overshoots by one dequeue per workgroup: the candidate count is recorded by the caller
    stats->candidates = (int64_t)(ds.accepted + ds.fail_pre + ds.fail_post);
  }
  return PMVS_OK;
}

pmvs_status pmvs_refine_batch(pmvs_scene* sc, const pmvs_candidate* in, int32_t n, pmvs_refined* out,
                              pmvs_stats* stats) {
  if (!sc || (n > 0 && (!in || !out))) return fail(PMVS_EINVAL, "null argument");
  if (n <= 0) {
    if (stats) std::memset(stats, 0, sizeof(*stats));
    return PMVS_OK;
  }
  pmvs_status st = check_candidates(sc, in, n);
  if (st) return st;
  HIPCHK(hipSetDevice(sc->device));
  if ((st = ensure(sc->cand, n)) || (st = ensure(sc->res, n))) return st;
  HIPCHK(hipMemcpyAsync(sc->cand.p, in, n * sizeof(pmvs_candidate), hipMemcpyHostToDevice, sc->stream));
  if ((st = pmvs_refine_batch_device(sc, sc->cand.p, n, sc->res.p))) return st;
  HIPCHK(hipMemcpyAsync(out, sc->res.p, n * sizeof(pmvs_refined), hipMemcpyDeviceToHost, sc->stream));
  return pmvs_scene_sync(sc, stats);
}

pmvs_status pmvs_selftest_math(int32_t device, int32_t op, const double* in, double* out, int32_t n) {
  if (!in || !out || n <= 0) return fail(PMVS_EINVAL, "null argument");
  HIPCHK(hipSetDevice(device));
  double *di = nullptr, *dout = nullptr;
  HIPCHK(hipMalloc((void**)&di, n * sizeof(double)));
  hipError_t e = hipMalloc((void**)&dout, n * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(di, in, n * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_math_selftest(op, di, dout, n, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, dout, n * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(di);
  if (dout) (void)hipFree(dout);
  if (e != hipSuccess) return fail(PMVS_EDEVICE, "math selftest: %s", hipGetErrorString(e));
  return PMVS_OK;
}

pmvs_status pmvs_selftest_lls(int32_t device, const float* A, const float* b, const int32_t* offsets, int32_t nsys,
                              float* x) {
  if (!A || !b || !offsets || !x || nsys <= 0) return fail(PMVS_EINVAL, "null argument");
  for (int k = 0; k < nsys; ++k)
    if (offsets[k + 1] - offsets[k] < 5) return fail(PMVS_EINVAL, "system %d has fewer than 5 rows", k);
  HIPCHK(hipSetDevice(device));
  HIPCHK(lls_selftest(A, b, offsets, nsys, offsets[nsys], x));
  return PMVS_OK;
}

pmvs_status pmvs_selftest_bobyqa(int32_t device, int32_t mode, int32_t kind, const double* x0, int32_t n,
                                 int32_t maxeval, double* out, double* ms) {
  if (!x0 || !out || n <= 0) return fail(PMVS_EINVAL, "null argument");
  HIPCHK(hipSetDevice(device));
  double *dx = nullptr, *dout = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIPCHK(hipMalloc((void**)&dx, 3 * n * sizeof(double)));
  hipError_t e = hipMalloc((void**)&dout, 6 * n * sizeof(double));
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = hipMemcpy(dx, x0, 3 * n * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipEventRecord(e0, nullptr);
  if (e == hipSuccess) e = launch_bobyqa_selftest(mode, kind, dx, n, maxeval, dout, nullptr);
  if (e == hipSuccess) e = hipEventRecord(e1, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, dout, 6 * n * sizeof(double), hipMemcpyDeviceToHost);
  float t = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
  if (ms) *ms = t;
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(dx);
  if (dout) (void)hipFree(dout);
  if (e != hipSuccess) return fail(PMVS_EDEVICE, "bobyqa selftest: %s", hipGetErrorString(e));
  return PMVS_OK;
}

}  // extern "C"

pmvs_status pmvs_patch_colors(pmvs_scene* sc, int32_t n, const float* coords4, const int32_t* nimg,
                              const int32_t* images_flat, int32_t* colors_out) {
  if (!sc || n < 0 || (n > 0 && (!coords4 || !nimg || !images_flat || !colors_out))) return fail(PMVS_EINVAL, "null argument");
  if (n == 0) return PMVS_OK;
  std::vector<int> off(n + 1, 0);
  for (int i = 0; i < n; ++i) {
    if (nimg[i] < 1) return fail(PMVS_EINVAL, "patch %d: no images", i);
    off[i + 1] = off[i] + nimg[i];
  }
  for (int k = 0; k < off[n]; ++k)
    if (images_flat[k] < 0 || images_flat[k] >= sc->ds.num) return fail(PMVS_EINVAL, "image index %d", images_flat[k]);
  HIPCHK(hipSetDevice(sc->device));
  float* dc = nullptr;
  int *doff = nullptr, *dimg = nullptr, *dout = nullptr;
  hipError_t e = hipMalloc((void**)&dc, (size_t)n * 4 * sizeof(float));
  if (e == hipSuccess) e = hipMalloc((void**)&doff, (size_t)(n + 1) * sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&dimg, (size_t)off[n] * sizeof(int));
  if (e == hipSuccess) e = hipMalloc((void**)&dout, (size_t)n * 3 * sizeof(int));
  if (e == hipSuccess) e = hipMemcpyAsync(dc, coords4, (size_t)n * 4 * sizeof(float), hipMemcpyHostToDevice, sc->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(doff, off.data(), (size_t)(n + 1) * sizeof(int), hipMemcpyHostToDevice, sc->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dimg, images_flat, (size_t)off[n] * sizeof(int), hipMemcpyHostToDevice, sc->stream);
  if (e == hipSuccess) e = launch_patch_colors(sc->ds, n, dc, doff, dimg, dout, sc->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(colors_out, dout, (size_t)n * 3 * sizeof(int), hipMemcpyDeviceToHost, sc->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(sc->stream);
  (void)hipFree(dc);
  (void)hipFree(doff);
  (void)hipFree(dimg);
  (void)hipFree(dout);
  if (e != hipSuccess) return fail(PMVS_EDEVICE, "patch colours: %s", hipGetErrorString(e));
  return PMVS_OK;
}

pmvs_status pmvs_filter_run(pmvs_scene* sc, pmvs_patch* patches, int32_t n, int32_t* keep, pmvs_filter_stats* stats) {
  if (!sc || n < 0 || (n > 0 && (!patches || !keep))) return fail(PMVS_EINVAL, "null argument");
  if (sc->ds.tnum > PMVS_MAX_TARGETS) return fail(PMVS_EUNSUPPORTED, "filter pass: more than %d target images", PMVS_MAX_TARGETS);
  for (int i = 0; i < n; ++i) {
    const pmvs_patch& p = patches[i];
    if (p.num_images < 1 || p.num_images > PMVS_MAX_IMAGES || p.num_vimages < 0 || p.num_vimages > PMVS_MAX_IMAGES)
      return fail(PMVS_EINVAL, "patch %d: image counts", i);
    for (int k = 0; k < p.num_images; ++k)
      if (p.images[k] < 0 || p.images[k] >= sc->ds.num) return fail(PMVS_EINVAL, "patch %d: image %d", i, p.images[k]);
    for (int k = 0; k < p.num_vimages; ++k)
      if (p.vimages[k] < 0 || p.vimages[k] >= sc->ds.tnum) return fail(PMVS_EINVAL, "patch %d: vimage", i);
  }
  if (stats) std::memset(stats, 0, sizeof(*stats));
  if (n == 0) return PMVS_OK;
  HIPCHK(hipSetDevice(sc->device));
  pmvs_status st;
  if ((st = ensure(sc->fpatches, n)) || (st = ensure(sc->fkeep, n))) return st;
  std::vector<long long> tgoff(sc->ds.tnum + 1, 0);
  for (int t = 0; t < sc->ds.tnum; ++t) {
    const DView& v = sc->hviews[t];
    const long long gw = (v.w[sc->ds.level] + sc->ds.csize - 1) / sc->ds.csize;
    const long long gh = (v.h[sc->ds.level] + sc->ds.csize - 1) / sc->ds.csize;
    tgoff[t + 1] = tgoff[t] + gw * gh;
  }
  HIPCHK(hipMemcpyAsync(sc->fpatches.p, patches, (size_t)n * sizeof(pmvs_patch), hipMemcpyHostToDevice, sc->stream));
  HIPCHK(hipEventRecord(sc->ev0, sc->stream));
  int counts[4], overflow = 0;
  const hipError_t fe = filter_pass(sc->ds, sc->fbuf, sc->fpatches.p, n, tgoff[sc->ds.tnum], tgoff.data(), sc->grid,
                                    sc->stream, counts, &overflow, sc->fkeep.p);
  if (fe == hipErrorNotSupported)
    return fail(PMVS_EUNSUPPORTED, "filter pass: a patch is visible in more than %d target images", PMVS_MAX_IMAGES);
  HIPCHK(fe);
  HIPCHK(hipEventRecord(sc->ev1, sc->stream));
  HIPCHK(hipMemcpyAsync(patches, sc->fpatches.p, (size_t)n * sizeof(pmvs_patch), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipMemcpyAsync(keep, sc->fkeep.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipStreamSynchronize(sc->stream));
  if (overflow) return fail(PMVS_EUNSUPPORTED, "filterNeighbor: %d patches with more than 16384 neighbours", overflow);
  if (stats) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, sc->ev0, sc->ev1);
    stats->input = n;
    stats->removed_outside = counts[0];
    stats->removed_exact = counts[1];
    stats->removed_neighbor = counts[2];
    stats->removed_groups = counts[3];
    int64_t k = 0;
    for (int i = 0; i < n; ++i) k += keep[i];
    stats->kept = k;
    stats->kernel_ms = ms;
  }
  sc->last_refine = false;
  return PMVS_OK;
}

namespace {

// validation of a caller's patch set (image counts and indexes)
pmvs_status check_patches(const pmvs_scene* sc, const pmvs_patch* patches, int n) {
  for (int i = 0; i < n; ++i) {
    const pmvs_patch& p = patches[i];
    if (p.num_images < 1 || p.num_images > PMVS_MAX_IMAGES || p.num_vimages < 0 || p.num_vimages > PMVS_MAX_IMAGES)
      return fail(PMVS_EINVAL, "patch %d: image counts", i);
    for (int k = 0; k < p.num_images; ++k)
      if (p.images[k] < 0 || p.images[k] >= sc->ds.num) return fail(PMVS_EINVAL, "patch %d: image %d", i, p.images[k]);
    for (int k = 0; k < p.num_vimages; ++k)
      if (p.vimages[k] < 0 || p.vimages[k] >= sc->ds.tnum) return fail(PMVS_EINVAL, "patch %d: vimage", i);
  }
  return PMVS_OK;
}

// The scene's shard (pmvs_scene_set_shard / _rccl) as the organizer code takes it.
Shard make_shard(const pmvs_scene* sc) {
  Shard sh;
  if (sc->shard_fn && sc->shard_world > 1) {
    sh.rank = sc->shard_rank;
    sh.world = sc->shard_world;
    pmvs_allgather_fn fn = sc->shard_fn;
    void* ctx = sc->shard_ctx;
    sh.exchange = [fn, ctx](const void* send, size_t bytes, void* recv) { return fn(ctx, send, (int64_t)bytes, recv); };
    if (pmvs_rccl* comm = sc->shard_rccl)
      sh.exchange_dev = [comm](const void* dsend, size_t bytes, void* drecv, hipStream_t st) {
        return pmvs_rccl_allgather_device(comm, dsend, (int64_t)bytes, drecv, st);
      };
  }
  return sh;
}

// The scene's cluster exchange channel (pmvs_scene_set_cluster / _rccl).
Shard make_cluster_shard(const pmvs_scene* sc) {
  Shard sh;
  if (sc->cl_fn && sc->cl_world > 1) {
    sh.rank = sc->cl_rank;
    sh.world = sc->cl_world;
    pmvs_allgather_fn fn = sc->cl_fn;
    void* ctx = sc->cl_ctx;
    sh.exchange = [fn, ctx](const void* send, size_t bytes, void* recv) { return fn(ctx, send, (int64_t)bytes, recv); };
    if (pmvs_rccl* comm = sc->cl_rccl)
      sh.exchange_dev = [comm](const void* dsend, size_t bytes, void* drecv, hipStream_t st) {
        return pmvs_rccl_allgather_device(comm, dsend, (int64_t)bytes, drecv, st);
      };
  }
  return sh;
}

// Loop-level 8-byte header {error, 0} of the sharded loop: a rank that fails outside the
// expansion's / filter's own exchanges sends it once (its peers receive it in place of their next
// expansion batch header), and every rank sends {0} when the loop ends.  Returns 0 = every rank
// OK, 1 = some rank failed, -1 = the exchange itself failed.
int loop_header(const Shard& sh, int err) {
  int h[2] = {err, 0};
  std::vector<int> all(2 * (size_t)sh.world, 0);
  if (sh.exchange(h, sizeof(h), all.data()) != 0) return -1;
  for (int r = 0; r < sh.world; ++r)
    if (all[2 * r] != 0) return 1;
  return 0;
}

std::vector<long long> target_cells(pmvs_scene* sc) {
  std::vector<long long> tgoff(sc->ds.tnum + 1, 0);
  sc->xbuf.gw.assign(sc->ds.tnum, 0);
  sc->xbuf.gh.assign(sc->ds.tnum, 0);
  for (int t = 0; t < sc->ds.tnum; ++t) {
    const DView& v = sc->hviews[t];
    sc->xbuf.gw[t] = (v.w[sc->ds.level] + sc->ds.csize - 1) / sc->ds.csize;
    sc->xbuf.gh[t] = (v.h[sc->ds.level] + sc->ds.csize - 1) / sc->ds.csize;
    tgoff[t + 1] = tgoff[t] + (long long)sc->xbuf.gw[t] * sc->xbuf.gh[t];
  }
  return tgoff;
}

// One expansion run on the device-resident model sc->fpatches[0, n0) with alive flags
// sc->xbuf.alive; *n_out patches afterwards.
// Test hook (tests/test_gpu_expand.py): PMVS_TEST_SHARD_FAIL="rank:0:x" (after the expansion's last
// exchange) or "rank:0:s" (after the filter pass's last exchange) makes that rank fail locally there,
// as an asynchronous kernel fault surfacing at the stream synchronisation would.
bool test_local_fail(const pmvs_scene* sc, char where) {
  const char* e = getenv("PMVS_TEST_SHARD_FAIL");
  int r = -1, w = -1;
  char c = 0;
  if (!e || sscanf(e, "%d:%d:%c", &r, &w, &c) != 3 || c != where) return false;
  return (sc->shard_world > 1 && r == sc->shard_rank) || (sc->cl_world > 1 && r == sc->cl_rank);
}

// *handled (sharded loop): whether the peers already know of a failure returned here -- true only
// for failures expand_pass reported through its own header exchanges.
pmvs_status expand_device(pmvs_scene* sc, int n0, int wave, int min_cands, int cthr, int flags, int cap, int* n_out,
                          pmvs_expand_stats* stats, bool* handled = nullptr) {
  if (handled) *handled = false;
  const std::vector<long long> tgoff = target_cells(sc);
  // refine-work accounting: device counters accumulate over the run (only the work-queue heads
  // are reset per launch); the refine-kernel time of each launch is read at the next one, when
  // the host has synchronised in between.
  double refine_ms = 0.0, refine_ms_small = 0.0;
  int64_t refined = 0, launches = 0, launches_small = 0;
  bool pending = false, pending_small = false;
  auto take_time = [&]() {
    if (!pending) return;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, sc->kev[1], sc->kev[2]) == hipSuccess) {
      refine_ms += ms;
      if (pending_small) refine_ms_small += ms;
    }
    pending = false;
  };
  HIPCHK(hipMemsetAsync(sc->stats.p, 0, sizeof(DevStats), sc->stream));
  sc->rhost.prof = getenv("PMVS_EXPAND_PROFILE") != nullptr;
  sc->rhost.trip_ms = 0.0;
  sc->rhost.trips = 0;
  RefineFn refine = [&](const pmvs_candidate* d_in, int m, pmvs_refined* d_out) -> hipError_t {
    if (ensure(sc->jobs, m)) return hipErrorOutOfMemory;
    take_time();
    hipError_t e = hipMemsetAsync(&sc->stats.p->queue, 0, 3 * sizeof(unsigned long long), sc->stream);
    if (e != hipSuccess) return e;
    refined += m;
    ++launches;
    pending = true;
    const int cfg = sc->refine_cfg(m);
    pending_small = m < sc->small_n;  // the small batches (refine_cfg: tslots_small)
    launches_small += pending_small ? 1 : 0;
    return launch_refine(sc->ds, d_in, sc->jobs.p, d_out, m, sc->stats.p, sc->grid, sc->refine_grid, cfg, sc->stream,
                         sc->kev, sc->rhost);
  };
  const Shard sh = make_shard(sc);
  long long sv[8];
  const auto t0 = std::chrono::steady_clock::now();
  const hipError_t e = expand_pass(sc->ds, sc->fbuf, sc->xbuf, sc->fpatches.p, sc->fpatches.n, n0, sc->xbuf.alive, cap,
                                   tgoff[sc->ds.tnum], tgoff.data(), wave, cthr, flags, sc->grid, sc->stream, refine, sh,
                                   sv, n_out, min_cands);
  if (handled) *handled = e != hipSuccess;  // expand_pass ends every failure with a header all ranks see
  if (e == kCapacityOverflow)
    return fail(PMVS_EUNSUPPORTED,
                "expansion: capacity %d exceeded, a patch has more than 16384 neighbours, or a patch's image / "
                "visible-target list exceeds %d entries", cap, PMVS_MAX_IMAGES);
  if (e == hipErrorOutOfMemory) return fail(PMVS_ENOMEM, "expansion: device memory");
  if (e == hipErrorUnknown && sh.world > 1) return fail(PMVS_EDEVICE, "expansion: the shard exchange or another rank failed");
  HIPCHK(e);
  if (handled) *handled = false;  // from here on a failure is this rank's alone
  if (test_local_fail(sc, 'x')) return fail(PMVS_EDEVICE, "expansion: injected local failure (test)");
  HIPCHK(hipStreamSynchronize(sc->stream));
  take_time();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  DevStats ds{};
  HIPCHK(hipMemcpy(&ds, sc->stats.p, sizeof(DevStats), hipMemcpyDeviceToHost));
  if (sc->rhost.prof)
    fprintf(stderr, "[refine round trip] batches=%lld device_ms=%.1f (pre_kernel end -> refine start: start points "
                    "down, host libm asin/acos, angles up)\n", sc->rhost.trips, sc->rhost.trip_ms);
  if (getenv("PMVS_REFINE_TAIL"))  // diagnostics: the refine launches' tails (s_memrealtime: 100 MHz)
    for (int f = 0; f < 2; ++f)
      if (ds.tail_launches[f])
        fprintf(stderr, "[refine tail] form=%s launches=%llu span_ms=%.2f tail_ms=%.2f tail_frac=%.3f\n",
                f ? "workgroup" : "wavefront", ds.tail_launches[f], ds.span_t[f] / 1e5, ds.tail_t[f] / 1e5,
                ds.span_t[f] ? (double)ds.tail_t[f] / (double)ds.span_t[f] : 0.0);
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->parents = sv[0]; stats->candidates = sv[1]; stats->fail_prep = sv[2]; stats->fail_pre = sv[3];
    stats->fail_post = sv[4]; stats->fail_commit = sv[5]; stats->added = sv[6]; stats->waves = sv[7];
    stats->wall_ms = ms;
    stats->refined = refined;
    stats->evals = (int64_t)ds.evals;
    stats->tex_valid = (int64_t)ds.tex_valid;
    stats->refine_ms = refine_ms;
    stats->refine_launches = launches;
    stats->tex_valid_small = (int64_t)ds.tex_valid_wg;
    stats->refine_ms_small = refine_ms_small;
    stats->refine_launches_small = launches_small;
  }
  sc->last_refine = false;
  return PMVS_OK;
}

// One filter pass on the device-resident model sc->fpatches[0, n); keep flags in sc->fkeep.
// *handled (sharded loop): whether the peers already know of a failure returned here.
pmvs_status filter_device(pmvs_scene* sc, int n, pmvs_filter_stats* stats, bool* handled = nullptr) {
  if (handled) *handled = false;
  if (stats) std::memset(stats, 0, sizeof(*stats));
  if (n == 0) return PMVS_OK;
  pmvs_status st;
  if ((st = ensure(sc->fkeep, n))) return st;
  std::vector<long long> tgoff = target_cells(sc);
  HIPCHK(hipEventRecord(sc->ev0, sc->stream));
  int counts[4], overflow = 0;
  const Shard sh = make_shard(sc);
  bool fh = true;
  const hipError_t fe = filter_pass(sc->ds, sc->fbuf, sc->fpatches.p, n, tgoff[sc->ds.tnum], tgoff.data(), sc->grid,
                                    sc->stream, counts, &overflow, sc->fkeep.p, &sh, &fh);
  if (fe != hipSuccess) {
    if (handled) *handled = fh;
    if (fe == hipErrorNotSupported)
      return fail(PMVS_EUNSUPPORTED, "filter pass: a patch is visible in more than %d target images", PMVS_MAX_IMAGES);
    return fail(PMVS_EDEVICE, "filter pass: %s", hipGetErrorString(fe));
  }
  // kernels launched after the pass's last exchange (small groups, collect, keep) fault only at
  // this synchronisation, on this rank alone: *handled stays false so the loop announces it
  HIPCHK(hipEventRecord(sc->ev1, sc->stream));
  if (test_local_fail(sc, 's')) return fail(PMVS_EDEVICE, "filter pass: injected local failure (test)");
  HIPCHK(hipStreamSynchronize(sc->stream));
  if (handled) *handled = true;  // overflow is all-gathered: every rank returns it together
  if (overflow) return fail(PMVS_EUNSUPPORTED, "filterNeighbor: %d patches with more than 16384 neighbours", overflow);
  if (stats) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, sc->ev0, sc->ev1);
    stats->input = n;
    stats->removed_outside = counts[0];
    stats->removed_exact = counts[1];
    stats->removed_neighbor = counts[2];
    stats->removed_groups = counts[3];
    stats->kept = n - counts[0] - counts[1] - counts[2] - counts[3];
    stats->kernel_ms = ms;
  }
  sc->last_refine = false;
  return PMVS_OK;
}

}  // namespace

pmvs_status pmvs_expand_run(pmvs_scene* sc, const pmvs_patch* patches, const int32_t* alive, int32_t n, int32_t wave,
                            int32_t min_candidates, int32_t count_threshold, int32_t flags, pmvs_patch* out, int32_t* alive_out, int32_t cap,
                            int32_t* n_out, pmvs_expand_stats* stats) {
  const bool keep = !out && !alive_out;
  if (!sc || n < 0 || (n > 0 && (!patches || !alive)) || (!keep && (!out || !alive_out)) || !n_out || cap < n)
    return fail(PMVS_EINVAL, "invalid argument");
  if (wave < 1 || wave > kMaxWave) return fail(PMVS_EINVAL, "wave must be in [1, %d]", kMaxWave);
  if (sc->ds.tnum > PMVS_MAX_TARGETS) return fail(PMVS_EUNSUPPORTED, "expansion: more than %d target images", PMVS_MAX_TARGETS);
  pmvs_status st;
  if ((st = check_patches(sc, patches, n))) return st;
  if (stats) std::memset(stats, 0, sizeof(*stats));
  *n_out = 0;
  sc->xkept = keep ? 0 : -1;
  sc->xalive.clear();
  if (n == 0) return PMVS_OK;
  HIPCHK(hipSetDevice(sc->device));
  if ((st = ensure(sc->fpatches, n))) return st;
  if (grow_alive(sc, n)) return fail(PMVS_ENOMEM, "alive flags");
  HIPCHK(hipMemcpyAsync(sc->fpatches.p, patches, (size_t)n * sizeof(pmvs_patch), hipMemcpyHostToDevice, sc->stream));
  HIPCHK(hipMemcpyAsync(sc->xbuf.alive, alive, (size_t)n * sizeof(int), hipMemcpyHostToDevice, sc->stream));
  int nn = 0;
  if (min_candidates < 0) return fail(PMVS_EINVAL, "min_candidates %d", min_candidates);
  if ((st = expand_device(sc, n, wave, min_candidates, count_threshold, flags, cap, &nn, stats))) return st;
  *n_out = nn;
  std::vector<int> al(alive, alive + n);
  al.resize(nn, 1);
  if (keep) {
    sc->xkept = nn;
    sc->xalive.swap(al);
    return PMVS_OK;
  }
  HIPCHK(hipMemcpy(out, sc->fpatches.p, (size_t)nn * sizeof(pmvs_patch), hipMemcpyDeviceToHost));
  std::memcpy(alive_out, al.data(), (size_t)nn * sizeof(int));
  return PMVS_OK;
}

pmvs_status pmvs_expand_fetch(pmvs_scene* sc, pmvs_patch* out, int32_t* alive_out, int32_t n) {
  if (!sc || n < 0 || (n > 0 && (!out || !alive_out))) return fail(PMVS_EINVAL, "invalid argument");
  if (n != sc->xkept) return fail(PMVS_EINVAL, "expand_fetch: %d patches kept, %d asked", sc->xkept, n);
  if (n) {
    HIPCHK(hipSetDevice(sc->device));
    HIPCHK(hipMemcpy(out, sc->fpatches.p, (size_t)n * sizeof(pmvs_patch), hipMemcpyDeviceToHost));
    if (alive_out) std::memcpy(alive_out, sc->xalive.data(), (size_t)n * sizeof(int));
  }
  sc->xkept = -1;
  std::vector<int>().swap(sc->xalive);
  return PMVS_OK;
}

pmvs_status pmvs_run_loop(pmvs_scene* sc, const pmvs_patch* seeds, int32_t n, float threshold, int32_t iterations,
                          int32_t wave, int32_t min_candidates, int32_t flags, int32_t cap, int32_t* n_out, pmvs_loop_iter* iters) {
  if (!sc || n < 0 || (n > 0 && !seeds) || !n_out || iterations < 0 || cap < n || min_candidates < 0)
    return fail(PMVS_EINVAL, "invalid argument");
  if (wave < 1 || wave > kMaxWave) return fail(PMVS_EINVAL, "wave must be in [1, %d]", kMaxWave);
  if (sc->ds.tnum > PMVS_MAX_TARGETS) return fail(PMVS_EUNSUPPORTED, "expansion: more than %d target images", PMVS_MAX_TARGETS);
  pmvs_status st;
  if ((st = check_patches(sc, seeds, n))) return st;
  *n_out = 0;
  sc->lkept = -1;
  if (iters) std::memset(iters, 0, sizeof(pmvs_loop_iter) * (size_t)iterations);
  HIPCHK(hipSetDevice(sc->device));
  if ((st = ensure(sc->fpatches, std::max(n, 1)))) return st;
  if (n) HIPCHK(hipMemcpyAsync(sc->fpatches.p, seeds, (size_t)n * sizeof(pmvs_patch), hipMemcpyHostToDevice, sc->stream));
  // CFindMatch::run after the seed phase (findMatch.cpp:196-217); updateThreshold in float
  // (findMatch.cpp:23-28): before = threshold - 0.3f (findMatch.cpp:104)
  float ncc = threshold, before = threshold - 0.3f;
  int cthr = 4, depth = 1, cur = n;
  // Sharded: a failure the peers have not seen is announced with one loop header (loop_header).
  const Shard lsh = make_shard(sc);
  const Shard csh = make_cluster_shard(sc);  // cluster boundary exchange (pmvs_scene_set_cluster)
  if (lsh.world > 1 && csh.world > 1) return fail(PMVS_EINVAL, "a scene is either sharded or a cluster, not both");
  const Shard& hsh = (csh.world > 1) ? csh : lsh;  // the channel of the loop's error headers
  auto fail_loop = [&](pmvs_status s0, bool peers_know) {
    if (hsh.world > 1 && !peers_know) (void)loop_header(hsh, 1);
    return s0;
  };
  // Compaction targets (fpatches2) are sized by the kept records: the source's capacity (the
  // expansion's, up to twice its model) would hold two full-size models at once -- at C5 scale
  // (50 M patches of 1608 B after one expansion) more than the GPU has.  The source buffer is
  // released after the swap when it is much larger than the model.
  bool dst_oom = false;
  auto dst_for = [&](int k, pmvs_patch** d) -> hipError_t {
    if (sc->fpatches2.n > 2 * (size_t)std::max(k, 1)) sc->fpatches2.release();
    if (ensure(sc->fpatches2, std::max(k, 1))) {
      dst_oom = true;
      return hipErrorOutOfMemory;
    }
    *d = sc->fpatches2.p;
    return hipSuccess;
  };
  auto swap_models = [&](int kept) {
    std::swap(sc->fpatches.p, sc->fpatches2.p);
    std::swap(sc->fpatches.n, sc->fpatches2.n);
    if (sc->fpatches2.n > 2 * (size_t)std::max(kept, 1)) sc->fpatches2.release();
  };
  // the model without foreign patches, compacted through fpatches2
  auto drop = [&](int n, int* kept) -> pmvs_status {
    if (n == 0) { *kept = 0; return PMVS_OK; }
    if (drop_foreign(sc->fbuf, sc->fpatches.p, n, dst_for, kept, sc->stream) != hipSuccess)
      return dst_oom ? fail(PMVS_ENOMEM, "model (%d patches)", *kept) : fail(PMVS_EDEVICE, "foreign patches");
    swap_models(*kept);
    return PMVS_OK;
  };
  for (int it = 0; it < iterations; ++it) {
    sc->ds.depth = depth;
    sc->ds.nccThreshold = ncc;
    sc->ds.nccThresholdBefore = before;
    if (grow_alive(sc, std::max(cur, 1))) return fail_loop(fail(PMVS_ENOMEM, "alive flags"), false);
    if (fill_int(sc->xbuf.alive, cur, 1, sc->stream) != hipSuccess) return fail_loop(fail(PMVS_EDEVICE, "alive flags"), false);
    pmvs_loop_iter li{};
    li.depth = depth;
    int nn = cur;
    // expand_device / filter_device report failures their own exchanges announced (*handled); those
    // exchanges run on the shard channel, so in a cluster scene (loop headers on the cluster
    // channel) no peer has seen them and the loop header must carry them
    bool xhandled = true;
    const int xflags = (flags & ~PMVS_EXPAND_AFTER_SEEDS) | ((it == 0 && (flags & PMVS_EXPAND_AFTER_SEEDS)) ? 1 : 0);
    if (cur > 0 && (st = expand_device(sc, cur, wave, min_candidates, cthr, xflags, cap, &nn, &li.expand, &xhandled)))
      return fail_loop(st, xhandled && &hsh == &lsh);
    bool handled = true;
    if ((st = filter_device(sc, nn, &li.filter, &handled))) return fail_loop(st, handled && &hsh == &lsh);
    int kept = 0;
    if (nn > 0) {
      if (compact_model(sc->fbuf, sc->fpatches.p, nn, sc->fkeep.p, dst_for, &kept, sc->stream) != hipSuccess)
        return fail_loop(dst_oom ? fail(PMVS_ENOMEM, "model (%d patches)", kept) : fail(PMVS_EDEVICE, "model compaction"),
                         false);
      swap_models(kept);
    }
    cur = kept;
    li.patches = kept;
    if (csh.world > 1 && it + 1 < iterations) {  // cluster boundary exchange before the next iteration
      int own = 0;
      if ((st = drop(cur, &own))) return fail_loop(st, false);
      li.patches = own;
      // PMVS_LOOP_LEAN=1: the pass buffers go back to the device while this rank waits for its peers
      // (several 8K clusters sharing one GPU, tests/test_gpu_c5_exchange.py); the next pass reserves
      // them again
      if (getenv("PMVS_LOOP_LEAN")) {
        if (hipStreamSynchronize(sc->stream) != hipSuccess) return fail_loop(fail(PMVS_EDEVICE, "loop synchronisation"), false);
        sc->fbuf.release();
        sc->xbuf.release();
      }
      const ClusterMaps cm{sc->cl_shared.p, sc->cl_ids.p, sc->cl_id2idx.p, sc->cl_maxid};
      long long xs[3] = {0, 0, 0};
      bool agreed = false;
      int nn2 = own;
      const hipError_t xe = cluster_exchange(sc->ds, sc->cbuf, cm, sc->fpatches.p, own, sc->fpatches.p, sc->fpatches.n, &nn2,
                                             csh, sc->stream, xs, agreed);
      if (xe != hipSuccess) return fail_loop(fail(PMVS_EDEVICE, "cluster exchange: %s", hipGetErrorString(xe)), agreed);
      cur = nn2;
      li.boundary_sent = xs[0];
      li.boundary_received = xs[1];
      li.boundary_inserted = xs[2];
    }
    if (iters) iters[it] = li;
    ncc -= 0.05f;
    before -= 0.05f;
    cthr = 2;
    ++depth;
  }
  if (csh.world > 1) {  // the cluster's own patches only
    int own = 0;
    if ((st = drop(cur, &own))) return fail_loop(st, false);
    cur = own;
  }
  if (hipStreamSynchronize(sc->stream) != hipSuccess) return fail_loop(fail(PMVS_EDEVICE, "loop synchronisation"), false);
  if (hsh.world > 1 && loop_header(hsh, 0) != 0) return fail(PMVS_EDEVICE, "sharded loop: another rank failed");
  *n_out = cur;
  sc->lkept = cur;
  return PMVS_OK;
}

pmvs_status pmvs_loop_fetch(pmvs_scene* sc, pmvs_patch* out, int32_t n) {
  if (!sc || n < 0 || (n > 0 && !out)) return fail(PMVS_EINVAL, "invalid argument");
  if (n != sc->lkept) return fail(PMVS_EINVAL, "loop_fetch: %d patches kept, %d asked", sc->lkept, n);
  if (n) {
    HIPCHK(hipSetDevice(sc->device));
    HIPCHK(hipMemcpy(out, sc->fpatches.p, (size_t)n * sizeof(pmvs_patch), hipMemcpyDeviceToHost));
  }
  sc->lkept = -1;
  return PMVS_OK;
}

pmvs_status pmvs_loop_hash(pmvs_scene* sc, uint64_t* hash) {
  if (!sc || !hash) return fail(PMVS_EINVAL, "invalid argument");
  if (sc->lkept < 0) return fail(PMVS_EINVAL, "loop_hash: no loop result on the device");
  HIPCHK(hipSetDevice(sc->device));
  if (ensure(sc->digest, 1)) return fail(PMVS_ENOMEM, "digest");
  HIPCHK(hipMemsetAsync(sc->digest.p, 0, sizeof(unsigned long long), sc->stream));
  static_assert(sizeof(pmvs_patch) % 4 == 0, "record words");
  HIPCHK(launch_model_digest(sc->fpatches.p, sc->lkept, (int)sizeof(pmvs_patch), sc->digest.p, sc->stream));
  unsigned long long h = 0;
  HIPCHK(hipMemcpyAsync(&h, sc->digest.p, sizeof(h), hipMemcpyDeviceToHost, sc->stream));
  HIPCHK(hipStreamSynchronize(sc->stream));
  *hash = h ^ (unsigned long long)sc->lkept;
  return PMVS_OK;
}

pmvs_status pmvs_scene_set_shard(pmvs_scene* sc, int32_t rank, int32_t world, pmvs_allgather_fn fn, void* ctx) {
  if (!sc || world < 1 || rank < 0 || rank >= world || (world > 1 && !fn)) return fail(PMVS_EINVAL, "invalid shard");
  sc->shard_rank = rank;
  sc->shard_world = world;
  sc->shard_fn = fn;
  sc->shard_ctx = ctx;
  sc->shard_rccl = nullptr;
  return PMVS_OK;
}

pmvs_status pmvs_scene_set_cluster(pmvs_scene* sc, int32_t rank, int32_t world, const int32_t* image_ids,
                                   pmvs_allgather_fn fn, void* ctx) {
  if (!sc || world < 1 || rank < 0 || rank >= world || (world > 1 && (!fn || !image_ids)))
    return fail(PMVS_EINVAL, "invalid cluster");
  sc->cl_world = 1;
  sc->cl_fn = nullptr;
  sc->cl_rccl = nullptr;
  if (world == 1) return PMVS_OK;
  const int num = sc->ds.num, tnum = sc->ds.tnum;
  // Local validation first; its outcome travels in the all-gather (mine[0] < 0), so a rank with a
  // bad argument fails together with its peers instead of leaving them in the collective.
  pmvs_status bad = PMVS_OK;
  int maxid = -1;
  std::vector<int> id2idx;
  if (tnum > PMVS_MAX_TARGETS) bad = fail(PMVS_EUNSUPPORTED, "cluster: more than %d target images", PMVS_MAX_TARGETS);
  for (int i = 0; i < num && !bad; ++i) {
    if (image_ids[i] < 0) bad = fail(PMVS_EINVAL, "image_ids[%d] = %d", i, image_ids[i]);
    maxid = std::max(maxid, image_ids[i]);
  }
  if (!bad && maxid > (1 << 26)) bad = fail(PMVS_EUNSUPPORTED, "image number %d", maxid);
  if (!bad) {
    id2idx.assign((size_t)maxid + 1, -1);
    for (int i = 0; i < num && !bad; ++i) {
      if (id2idx[image_ids[i]] >= 0) bad = fail(PMVS_EINVAL, "image number %d appears twice", image_ids[i]);
      id2idx[image_ids[i]] = i;
    }
  }
  // all-gather of the target image numbers (collective): a target is shared when another cluster
  // has it as a target too
  std::vector<int> mine(1 + PMVS_MAX_TARGETS, -1), all((size_t)(1 + PMVS_MAX_TARGETS) * world, -1);
  mine[0] = bad ? -1 : tnum;
  for (int t = 0; t < tnum && !bad; ++t) mine[1 + t] = image_ids[t];
  if (fn(ctx, mine.data(), (int64_t)(mine.size() * sizeof(int)), all.data()) != 0)
    return fail(PMVS_EDEVICE, "cluster setup: the all-gather failed");
  if (bad) return bad;
  for (int r = 0; r < world; ++r)
    if (all[(size_t)r * (1 + PMVS_MAX_TARGETS)] < 0) return fail(PMVS_EINVAL, "cluster setup: rank %d failed its validation", r);
  std::vector<unsigned char> shared(std::max(tnum, 1), 0);
  for (int r = 0; r < world; ++r) {
    if (r == rank) continue;
    const int* o = all.data() + (size_t)r * (1 + PMVS_MAX_TARGETS);
    for (int k = 0; k < std::min(o[0], PMVS_MAX_TARGETS); ++k) {
      const int id = o[1 + k];
      if (0 <= id && id <= maxid && id2idx[id] >= 0 && id2idx[id] < tnum) shared[id2idx[id]] = 1;
    }
  }
  HIPCHK(hipSetDevice(sc->device));
  pmvs_status st;
  if ((st = ensure(sc->cl_shared, shared.size())) || (st = ensure(sc->cl_ids, (size_t)num)) ||
      (st = ensure(sc->cl_id2idx, id2idx.size())))
    return st;
  HIPCHK(hipMemcpy(sc->cl_shared.p, shared.data(), shared.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(sc->cl_ids.p, image_ids, (size_t)num * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(sc->cl_id2idx.p, id2idx.data(), id2idx.size() * sizeof(int), hipMemcpyHostToDevice));
  sc->cl_maxid = maxid;
  sc->cl_rank = rank;
  sc->cl_world = world;
  sc->cl_fn = fn;
  sc->cl_ctx = ctx;
  return PMVS_OK;
}

pmvs_status pmvs_scene_set_cluster_rccl(pmvs_scene* sc, int32_t rank, int32_t world, const int32_t* image_ids,
                                        pmvs_rccl* comm) {
  if (!sc || !comm) return fail(PMVS_EINVAL, "invalid cluster");
  const pmvs_status st = pmvs_scene_set_cluster(sc, rank, world, image_ids, &pmvs_rccl_allgather, comm);
  if (st == PMVS_OK && world > 1) sc->cl_rccl = comm;
  return st;
}

pmvs_status pmvs_scene_set_shard_rccl(pmvs_scene* sc, int32_t rank, int32_t world, pmvs_rccl* comm) {
  if (!sc || !comm || world < 1 || rank < 0 || rank >= world) return fail(PMVS_EINVAL, "invalid shard");
  const pmvs_status st = pmvs_scene_set_shard(sc, rank, world, &pmvs_rccl_allgather, comm);
  if (st == PMVS_OK) sc->shard_rccl = comm;
  return st;
}

// ---- in-process all-gather among threads (generation-counted barrier)
struct pmvs_thread_exchange {
  int world = 1;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0, leaving = 0;
  long long gen = 0;
  std::vector<const void*> send;
  int64_t bytes = -1;
  bool bad = false;
  std::vector<std::pair<pmvs_thread_exchange*, int>> ctx;
};

pmvs_thread_exchange* pmvs_thread_exchange_create(int32_t world) {
  if (world < 1) return nullptr;
  auto* g = new pmvs_thread_exchange();
  g->world = world;
  g->send.assign(world, nullptr);
  for (int r = 0; r < world; ++r) g->ctx.push_back({g, r});
  return g;
}

void* pmvs_thread_exchange_ctx(pmvs_thread_exchange* g, int32_t rank) {
  if (!g || rank < 0 || rank >= g->world) return nullptr;
  return &g->ctx[rank];
}

int pmvs_thread_allgather(void* ctx, const void* send, int64_t bytes, void* recv) {
  auto* c = static_cast<std::pair<pmvs_thread_exchange*, int>*>(ctx);
  if (!c) return -1;
  pmvs_thread_exchange* g = c->first;
  const int r = c->second;
  std::unique_lock<std::mutex> lk(g->mu);
  g->cv.wait(lk, [&] { return g->leaving == 0; });  // the previous round has fully drained
  if (g->arrived == 0) { g->bytes = bytes; g->bad = false; }
  if (bytes != g->bytes) g->bad = true;
  g->send[r] = send;
  const long long my = g->gen;
  if (++g->arrived == g->world) {
    g->leaving = g->world;
    g->arrived = 0;
    ++g->gen;
    g->cv.notify_all();
  } else {
    g->cv.wait(lk, [&] { return g->gen != my; });
  }
  const bool bad = g->bad;
  if (!bad)
    for (int k = 0; k < g->world; ++k) std::memcpy((char*)recv + (size_t)k * bytes, g->send[k], (size_t)bytes);
  if (--g->leaving == 0) g->cv.notify_all();  // nobody returns before every copy is done
  else g->cv.wait(lk, [&] { return g->leaving == 0; });
  return bad ? -1 : 0;
}

void pmvs_thread_exchange_destroy(pmvs_thread_exchange* g) { delete g; }
