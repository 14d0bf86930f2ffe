// pmvs_launch.h -- host-side launchers of the kernels in pmvs_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "pmvs_device.h"
#include <functional>
#include <vector>

namespace pmvsdev {

// hipMemsetAsync in pieces of at most 1 GiB: the C5-scale buffers (a 70-view 8K pyramid is 12 GB,
// its cell tables 2-5 GB) exceed what one fill launch takes (a 12 GB pyramid clear failed with
// "invalid resource handle", gpurun r03p).
inline hipError_t memset_big(void* p, int value, size_t bytes, hipStream_t st) {
  constexpr size_t kPiece = size_t(1) << 30;
  char* c = static_cast<char*>(p);
  for (size_t off = 0; off < bytes; off += kPiece) {
    const hipError_t e = hipMemsetAsync(c + off, value, bytes - off < kPiece ? bytes - off : kPiece, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
bool refine_config_supported(int tslots);  // PMVS_REFINE_CONFIG values this build instantiates
// Host staging of the refine batches' start-point angles (encode_angles_host, pmvs_kernels.hip).
struct RefineHost {
  float4* d_enc = nullptr;
  double2* d_ang = nullptr;
  float4* h_enc = nullptr;   // pinned
  double2* h_ang = nullptr;  // pinned
  size_t cap = 0;
  // PMVS_EXPAND_PROFILE: the round trip's share of the device timeline (pre_kernel's end to the
  // refine kernel's start: start points down, host libm, angles up), summed over the batches
  bool prof = false;
  hipEvent_t ev_pre = nullptr;
  double trip_ms = 0.0;
  long long trips = 0;
  hipError_t ensure(size_t n);
  void release();
  ~RefineHost() { release(); }
};
// Waves per SIMD pre_kernel / post_kernel are built for (PMVS_PREPOST_WPE, default 3: pmvs_kernels.hip); their
// persistent grid is the scene grid x this / 2, and the per-workgroup global scratch is sized for it.
int prepost_waves();
hipError_t launch_refine(const DScene& s, const pmvs_candidate* d_in, RefineJob* d_jobs, pmvs_refined* d_out, int n,
                         DevStats* d_st, int grid, int refine_grid, int tslots, hipStream_t stream, hipEvent_t* ev,
                         RefineHost& rh);
// split-form refine kernel alone (pmvs_refine_split.hip), config 200000 + optimizer wavefronts * 1000 +
// chains per optimizer wavefront, wsize 5 or 7
bool refine_split_supported(int config);
hipError_t launch_refine_split(int config, const DScene& s, RefineJob* d_jobs, int n, DevStats* d_st, hipStream_t stream);
// lane-form refine kernel (pmvs_refine_lane.hip): one candidate per wavefront, BOBYQA state spread over
// the lanes; config 300000 (lanes per texture from tau), 300004, 300008
bool refine_lane_supported(int config);
hipError_t launch_refine_lane(int config, const DScene& s, RefineJob* d_jobs, int n, DevStats* d_st, hipStream_t stream);
hipError_t launch_incc_eval(const DScene& s, const pmvs_eval_query* d_q, int n, double* d_out, DevStats* d_st,
                            hipStream_t stream);
hipError_t launch_grab_tex(const DScene& s, const pmvs_tex_query* d_q, int n, float* d_out, int* d_valid,
                           hipStream_t stream);
hipError_t launch_build_level(const uint8_t* d_src, int Wp, int Hp, uint8_t* d_dst, int W, int H, hipStream_t stream);
hipError_t launch_pack_rgba(const uint8_t* d_rgb, uint32_t* d_out, long long npix, hipStream_t stream);
hipError_t launch_unpack_rgba(const uint32_t* d_in, uint8_t* d_rgb, long long npix, hipStream_t stream);
hipError_t launch_math_selftest(int op, const double* d_in, double* d_out, int n, hipStream_t stream);
hipError_t launch_bobyqa_selftest(int mode, int kind, const double* d_x0, int n, int maxeval, double* d_out,
                                  hipStream_t stream);
hipError_t launch_model_digest(const void* recs, int n, int record_bytes, unsigned long long* d_out, hipStream_t stream);
hipError_t launch_patch_colors(const DScene& s, int n, const float* coords, const int* off, const int* images, int* out,
                               hipStream_t stream);

// ---- filter pass (pmvs_filter.hip)
// Page-locked host staging (hipHostMalloc), grown on demand: the large per-pass downloads
// (filterSmallGroups' edge lists, the expansion queue's initial order) at full PCIe rate.
struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t c = bytes + bytes / 4 + 4096;
    const hipError_t e = hipHostMalloc(&p, c, hipHostMallocDefault);
    if (e == hipSuccess) cap = c;
    return e;
  }
  template <class T>
  T* as(size_t offset_bytes = 0) const { return reinterpret_cast<T*>(static_cast<char*>(p) + offset_bytes); }
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
};
// The fields of a patch that neighbour and visibility tests read from OTHER patches (isNeighbor,
// computeGain, isVisible), one 64-B line per patch instead of 2-3 lines of its 1.6-KB record;
// rebuilt by every collect and written by the expansion's commit (coord / normal / dscale / ncc
// never change after a patch is created; unit0 = getUnit(images[0], coord) follows setRefImage).
struct alignas(64) PHot {
  float coord[4];
  float normal[4];
  float dscale, ncc, unit0, pad[5];
};
struct FilterBuffers {
  PinnedBuf pin;  // host staging of the small-groups BFS inputs
  Reg *preg = nullptr, *vreg = nullptr, *safe = nullptr;  // per patch: registered / filterExact-safe list entries
  unsigned long long *keys = nullptr, *keys2 = nullptr, *dpkey = nullptr;
  long long* tgoff = nullptr;
  int *cnt = nullptr, *off = nullptr, *cellcnt = nullptr, *pg_off = nullptr, *pg_items = nullptr, *vp_off = nullptr,
      *vp_items = nullptr, *order = nullptr, *rank = nullptr, *flags = nullptr, *need = nullptr, *list = nullptr,
      *counters = nullptr, *edge_off = nullptr, *edges = nullptr;
  PHot* hot = nullptr;
  double* scratch = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0, edges_cap = 0;
  unsigned* rbits = nullptr;  // sharded filterNeighbor: packed reject flags
  float4* coordc = nullptr;   // collected patches' coordinates in collect order (depth maps)
  size_t cap_rbits = 0;
  // setVImagesVGrids' visibility rows (target-major bits), the collected patches' normals and used
  // targets; owner-partitioned pass (world > 1): setRefImage outcomes and the all-gathered payloads
  unsigned long long *vrows = nullptr, *used = nullptr;
  float4* normalc = nullptr;
  int* refpos = nullptr;
  char* xr = nullptr;
  size_t cap_vrows = 0, cap_used = 0, cap_normalc = 0, cap_refpos = 0, cap_xr = 0;
  // filterNeighbor's deferred quadric fits (pmvs_filter.hip QuadJobs)
  float* qf = nullptr;
  double* qrows = nullptr;
  int4* qjobs = nullptr;
  unsigned long long* qctr = nullptr;  // [0] rows used, [1] low 32 bits: jobs, [2] low 32 bits: quad_split_kernel's kb
  unsigned long long *qkeys = nullptr, *qkeys2 = nullptr;  // jobs by descending row count
  int *qcrows = nullptr, *qoff = nullptr;                  // per 64-job chunk: pool rows, offsets
  size_t cap_qrows = 0;
  // the neighbour walks' NB_CAP_BIG re-walks (pmvs_filter.hip NbOverflow): overflowed work items
  // and the big form's global scratch
  int* ovf_items = nullptr;
  double* scratch_big = nullptr;
  size_t cap_ovf = 0;
  int cap_n = 0, cap_grid = 0;
  long long cap_cells = 0;
  size_t cap_e = 0, cap_pi = 0, cap_vi = 0;  // entries of keys/keys2, pg_items, vp_items: grown to the lists' size
  hipError_t reserve(int n, long long ncells, int tnum, int grid);
  hipError_t ensure_entries(size_t e, int vis);
  void release();  // frees every buffer; the next pass reserves again (PMVS_LOOP_LEAN)
  ~FilterBuffers();
};

// setRefImage + setGrids for the patches list[0, m) (filterExact); with refpos, only the entries whose
// reference image rank owns (of world) are evaluated, their outcomes written to refpos (see the kernel)
hipError_t launch_filter_refimage(const DScene& s, pmvs_patch* P, const int* list, int m, int grid, hipStream_t stream,
                                  int* refpos = nullptr, int rank = 0, int world = 1);
hipError_t launch_apply_refpos(const DScene& s, pmvs_patch* P, const int* list, int m, const int* allpos, int world,
                               hipStream_t stream);

// ---- expansion run (pmvs_filter.hip)
constexpr int kMaxWave = 65536;  // parents per expansion wave (device slot arrays are sized by it)
struct CommitWork;  // device commit scratch (pmvs_filter.hip)
// Pinned staging of the per-wave host -> device index lists, with the event of its last copy
// (recorded on the scene's stream; owned by the scene, so never waited on after that stream is gone)
struct H2DStage {
  PinnedBuf pin;
  hipEvent_t done = nullptr;
  bool pending = false;
  ~H2DStage() {
    if (done) (void)hipEventDestroy(done);
  }
};
// The expansion's logical capacity overflows (more than NB_CAP_BIG neighbours, a list past
// PMVS_MAX_IMAGES, the model cap) return this code, so the API tells them from a device allocation
// that failed (hipErrorOutOfMemory: PMVS_ENOMEM).
constexpr hipError_t kCapacityOverflow = hipErrorNotSupported;

struct ExpandBuffers {
  CommitWork* cm = nullptr;
  long long ncells = 0;  // target cells of the pass (the commit sorts only the cell bits of its keys)
  // (the initial queue run is built on the device: qkeep / qpos / qitems)
  H2DStage h2d;
  unsigned char* occ = nullptr;  // per target cell: pgrids holds a patch (device commit)
  size_t cap_occ = 0;
  int *parents = nullptr, *cand_ok = nullptr, *status = nullptr, *slots = nullptr, *ostatus = nullptr, *alive = nullptr;
  float* cand_coord = nullptr;
  pmvs_candidate *cand = nullptr, *cand2 = nullptr;
  pmvs_patch *prep = nullptr, *prep2 = nullptr, *outp = nullptr;
  pmvs_refined* res = nullptr;
  unsigned char* counts = nullptr;
  // registrations committed during the run: per-cell chain heads + entry pool (FilterDev delta)
  // d_ent: the pool, {item, next} per entry (one 8-B load per chain step; round 6, separate item / next
  // arrays made every step touch two cache lines)
  int *pg_head = nullptr, *vp_head = nullptr, *pool_used = nullptr;
  int2* d_ent = nullptr;
  int* tcells = nullptr;        // cells whose counts a commit changed, and their values
  unsigned short* cellinit = nullptr;  // per-cell {count, occupied} staged for the host mirror
  float* qtmp = nullptr;        // _tmp of the collected patches (queue)
  float* qkey = nullptr;        // the initial queue sorted on the device: keys, collect ranks, temp
  int *qrank = nullptr, *qrank2 = nullptr;
  int *qkeep = nullptr, *qpos = nullptr;  // the initial run built on the device (queue_items_kernel)
  int *sflag = nullptr, *spos = nullptr, *slot2 = nullptr;  // survivor compaction (surv_*_kernel)
  size_t cap_sflag = 0, cap_spos = 0, cap_slot2 = 0;
  char* qitems = nullptr;
  size_t cap_qkeep = 0, cap_qpos = 0, cap_qitems = 0;
  void* qsort_tmp = nullptr;
  size_t cap_qkey = 0, cap_qrank = 0, cap_qrank2 = 0, cap_qsort = 0;
  char *xsd = nullptr, *xrd = nullptr;  // device payload of the sharded exchange (send, all ranks)
  size_t cap_xsd = 0, cap_xrd = 0;
  int* cidx = nullptr;  // wave slot -> compact index of its free direction (candidate / prep records)
  size_t cap_cidx = 0;
  int *crec = nullptr, *acc = nullptr;  // commit records; committed record indexes
  int2* dupd = nullptr;         // (parent, failed-direction bits) of a wave
  unsigned char* tvals = nullptr;
  size_t pool_host = 0;
  size_t cap_coord = 0, cap_ok = 0, cap_cand = 0, cap_prep = 0, cap_slots = 0, cap_prep2 = 0, cap_res = 0, cap_outp = 0,
         cap_ost = 0, cap_par = 0, cap_status = 0, cap_cand2 = 0, cap_alive = 0, cap_cnt = 0, cap_pghead = 0,
         cap_vphead = 0, cap_ent = 0, cap_pused = 0, cap_tcells = 0, cap_tvals = 0,
         cap_qtmp = 0, cap_crec = 0, cap_acc = 0, cap_dupd = 0, cap_cellinit = 0;
  std::vector<int> gw, gh;  // grid sizes of the target images
  void release();  // frees every buffer; the next pass grows them again (PMVS_LOOP_LEAN)
  ~ExpandBuffers();
};
using RefineFn = std::function<hipError_t(const pmvs_candidate* d_in, int n, pmvs_refined* d_out)>;
// All-gather of `bytes` per rank into recv (world * bytes, rank order); 0 = OK.
using ExchangeFn = std::function<int(const void* send, size_t bytes, void* recv)>;
// Device all-gather on the given stream (RCCL); empty = the payload goes through `exchange`.
using ExchangeDevFn = std::function<int(const void* dsend, size_t bytes, void* drecv, hipStream_t st)>;
struct Shard {
  int rank = 0, world = 1;
  ExchangeFn exchange;
  ExchangeDevFn exchange_dev;
};
// dP[0, n0): the device-resident model (grown in place, contents kept); d_alive[0, n0) marks the
// patches the organizer holds; cap bounds the result size *n_out.
// One CFilter::run pass on the device model; sharded (sh->world > 1) filterNeighbor runs on the
// patches this rank owns and the flags are all-gathered (one exchange per pass).
hipError_t filter_pass(const DScene& s, FilterBuffers& B, pmvs_patch* dP, int n, long long ncells, const long long* h_tgoff,
                       int grid, hipStream_t st, int counts[4], int* overflow, int* keep_dev, const Shard* sh = nullptr,
                       bool* handled = nullptr);
hipError_t expand_pass(const DScene& s, FilterBuffers& B, ExpandBuffers& X, pmvs_patch*& dP, size_t& dP_cap, int n0,
                       const int* d_alive, int cap, long long ncells, const long long* h_tgoff, int wave, int cthr,
                       int flags, int grid, hipStream_t st, const RefineFn& refine, const Shard& sh, long long stats[8],
                       int* n_out, int min_cands = 0);
// dst_for(kept, &dst) supplies the target once the number of kept records is known
using CompactDst = std::function<hipError_t(int, pmvs_patch**)>;
hipError_t compact_model(FilterBuffers& B, const pmvs_patch* src, int n, const int* keep, const CompactDst& dst_for,
                         int* nkept, hipStream_t st);
hipError_t fill_int(int* a, int n, int v, hipStream_t st);
// frees the device-to-host staging buffers of a scene's stream (pmvs_scene_destroy)
void d2h_stage_release(hipStream_t st);

// ---- CMVS cluster boundary exchange (pmvs_scene_set_cluster)
struct ClusterMaps {              // device tables of one cluster scene
  const unsigned char* shared_t;  // per local target index: its image is a target of another cluster too
  const int* ids;                 // per local view index: the global image number
  const int* id2idx;              // global image number (0 .. maxid) -> local view index, or -1
  int maxid;
};
struct ClusterBuffers {
  BRec *send = nullptr, *recv = nullptr;
  pmvs_patch* ins = nullptr;
  int *flags = nullptr, *pos = nullptr, *cnts = nullptr;
  void* temp = nullptr;
  size_t cap_send = 0, cap_recv = 0, cap_ins = 0, cap_flags = 0, cap_pos = 0, temp_bytes = 0;
  int cap_cnts = 0;
  ~ClusterBuffers();
};
// The model without other clusters' boundary patches (fix != PMVS_FIX_FOREIGN), compacted into dst.
hipError_t drop_foreign(FilterBuffers& B, const pmvs_patch* src, int n, const CompactDst& dst_for, int* n_out,
                        hipStream_t st);
// One boundary exchange: src[0, n) is this rank's model without foreign patches.  Its boundary
// patches (registered in a target image another cluster also has as a target) are all-gathered
// (header {error, count} first, the "visibility counts"; then the records), and every other rank's
// records whose reference image is one of this scene's views and that project into one of its
// targets are appended to dst (= src's contents + the inserted patches; grown as needed) as fixed,
// never-expanded patches (fix = PMVS_FIX_FOREIGN), with grids from CPatchOrganizerS::setGrids.
// xstats: [0] own boundary patches, [1] records received, [2] inserted.  agreed: the failure (if
// any) was seen by every rank.
hipError_t cluster_exchange(const DScene& s, ClusterBuffers& CB, const ClusterMaps& cm, const pmvs_patch* src, int n,
                            pmvs_patch*& dst, size_t& dst_cap, int* n_out, const Shard& sh, hipStream_t st,
                            long long xstats[3], bool& agreed);
hipError_t lls_selftest(const float* A, const float* b, const int* off, int nsys, int total, float* x);

// ---- seed phase (pmvs_seed.hip)
struct SeedInput {
  const pmvs_point* points;  // every view's feature points, view 0 first
  const int* npts;           // per view
  const int* vis_off;        // visdata2 CSR (host)
  const int* vis;
  int sequence;
  float angle0;              // _angleThreshold0
  std::vector<const uint8_t*> mask_level;  // per view: binary mask at the scene level (host), or null
  int batch, per_cell;       // speculative refine batch size / unknown candidates requested per cell
  int lookahead;             // images (current + next) the speculation may request candidates of
  int spec_near;             // cells from the replay cursor every speculation walk re-visits
};
struct SeedOutput {
  std::vector<pmvs_patch> seeds;  // addPatch order
  long long stats[8];             // trial, pass, fail0, fail1, refined, rounds, candidates
  double gen_ms = 0, refine_ms = 0, wall_ms = 0;
};
hipError_t seed_pass(const DScene& s, const std::vector<DView>& hv, const SeedInput& in, hipStream_t st,
                     const RefineFn& refine, SeedOutput& out);
}  // namespace pmvsdev
