/*
 * pmvs_amd.h -- C-ABI of the MI355X-native PMVS2 dense-matching core.
 *
 * The reference (robjermy/CMVS-PMVS) has no plugin/FFI surface for its hot path: the stages
 * share one CFindMatch& (reference include/pmvs/findMatch.hpp:150-163).  This ABI is the
 * boundary SURVEY.md §8(b) defines; each entry point names the reference interface it
 * replaces.  Plain pointers and sizes only; no exceptions cross it; errors are status codes
 * with a message from pmvs_last_error().  Never calls exit().
 *
 * Index convention: every image number below is an *index* into the scene's view list
 * (targets first, then other images), exactly like the reference's internal _images
 * (CPatchOrganizerS::image2index / index2image, patchOrganizerS.cpp:16-52).
 *
 * Ownership: all input/output arrays belong to the caller (host memory); a scene owns its
 * device memory.  Threading: calls on one scene are serialised on that scene's HIP stream;
 * different scenes (one per GPU) may be driven from different host threads.
 */
#ifndef PMVS_AMD_H
#define PMVS_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Capacity of one patch's image list and of its visible-target list (reference: unbounded
 * std::vector, patch.hpp:38,42).  A patch's images are distinct views and its vimages distinct
 * targets, so both lists always fit for scenes of up to PMVS_MAX_IMAGES views; larger scenes are
 * supported, and a list that would overflow fails the call with PMVS_EUNSUPPORTED (never a clamp). */
#define PMVS_MAX_IMAGES 128
#define PMVS_MAX_TARGETS 256 /* target images (timages) per scene: a C5 cluster is maximage 70 plus overlap */
#define PMVS_MAX_TAU 16    /* max textures in the objective: tau = min(2*minImageNum, num) */
#define PMVS_MAX_LEVEL 4   /* reference MyPow2 table limits level to <= 4 (optim.cpp:808-811) */
/* Unique neighbours one findNeighbors walk may hold (filterNeighbor, findEmptyBlocks, the depth >= 2
 * check; reference: unbounded std::vector).  Walks past 1024 are redone with a 16384-entry form;
 * beyond this the call fails with PMVS_EUNSUPPORTED. */
#define PMVS_MAX_NEIGHBOURS 16384

typedef enum pmvs_status {
  PMVS_OK = 0,
  PMVS_EINVAL = 1,      /* invalid argument */
  PMVS_EDEVICE = 2,     /* HIP runtime error */
  PMVS_ENOMEM = 3,      /* allocation failure */
  PMVS_EUNSUPPORTED = 4 /* configuration outside the supported envelope */
} pmvs_status;

/* Outcome of one candidate in pmvs_refine_batch (CSeed::initialMatchSub seed.cpp:387-414,
 * CExpand::expandSub expand.cpp:225-237: preProcess -> refinePatch -> postProcess). */
typedef enum pmvs_candidate_status {
  PMVS_ACCEPTED = 0,      /* postProcess returned 0 */
  PMVS_FAIL_PRE = 1,      /* COptim::preProcess returned 1 */
  PMVS_FAIL_POST = 2,     /* COptim::postProcess returned 1 */
  PMVS_FAIL_OVERFLOW = 3  /* image list exceeded PMVS_MAX_IMAGES (not a reference outcome; the loop entry
                             points turn it into a PMVS_EUNSUPPORTED error) */
} pmvs_candidate_status;

/* One view: CPhoto = CImage (pyramid) + CCamera (projection), reference include/image/photo.hpp. */
typedef struct pmvs_view_desc {
  int32_t width, height;    /* level-0 size */
  const uint8_t* rgb;       /* width*height*3 interleaved RGB8, row-major (CImage::_images[0]) */
  const uint8_t* mask;      /* optional width*height, 0 = outside; NULL = no mask */
  const uint8_t* edge;      /* optional width*height; NULL = no edge map */
  float projection[12];     /* level-0 3x4 projection, row-major (txt/%08d.txt, CCamera::init) */
} pmvs_view_desc;

/* Scene: SOption (option.cpp:10-28,30-158) + CFindMatch::init (findMatch.cpp:30-107). */
typedef struct pmvs_scene_desc {
  int32_t num_views;          /* _num = |timages| + |oimages| */
  int32_t num_targets;        /* _tnum = |timages| */
  int32_t level;              /* option level (0..PMVS_MAX_LEVEL) */
  int32_t csize;              /* option csize */
  int32_t wsize;              /* option wsize (odd) */
  int32_t min_image_num;      /* option minImageNum */
  float threshold;            /* option threshold (initial _nccThreshold) */
  float max_angle;            /* SOption::_maxAngleThreshold in radians (maxAngle * M_PI/180) */
  float quad_threshold;       /* option quad */
  int32_t sequence;           /* option sequence (-1 = off) */
  const int32_t* visdata2_offsets; /* CSR row starts, num_views+1 entries (SOption::_visdata2) */
  const int32_t* visdata2;         /* CSR column indexes */
  int32_t num_bindexes;            /* SOption::_bindexes (useBound) */
  const int32_t* bindexes;
  const pmvs_view_desc* views;     /* num_views entries */
} pmvs_scene_desc;

/* A patch candidate before preProcess (Patch::CPatch, reference include/pmvs/patch.hpp:10-77). */
typedef struct pmvs_candidate {
  float coord[4];  /* _coord, w = 1 */
  float normal[4]; /* _normal, w = 0 */
  float dscale;    /* initial _dscale (0 for a freshly constructed CPatch) */
  int32_t num_images;
  int32_t images[PMVS_MAX_IMAGES]; /* _images (indexes); [0] is the reference image */
} pmvs_candidate;

/* A candidate after preProcess -> refinePatch -> postProcess. */
typedef struct pmvs_refined {
  int32_t status;      /* pmvs_candidate_status */
  int32_t refine_code; /* optimizer result, NLopt numbering (4 = XTOL_REACHED, 5 = MAXEVAL, -4 = ROUNDOFF) */
  int32_t evals;       /* objective evaluations (COptim::my_f calls) in refinePatch */
  int32_t num_images;
  float coord[4];
  float normal[4];
  float ncc;           /* _ncc (stays -1 if refinement failed, as in the reference) */
  float dscale;
  float ascale;
  float tmp;           /* _tmp = score2(nccThreshold) */
  int32_t timages;
  int32_t reserved;
  int32_t images[PMVS_MAX_IMAGES];
  int32_t grids[PMVS_MAX_IMAGES][2]; /* _grids (cell x, cell y) per image */
} pmvs_refined;

/* Objective query: the refine state of refinePatchBFGS (optim.cpp:580-599) for a patch, and
 * an optimizer point x at which COptim::my_f (optim.cpp:507-578) is evaluated. */
typedef struct pmvs_eval_query {
  float coord[4];
  float normal[4];
  float dscale;
  int32_t num_images;
  int32_t images[PMVS_MAX_TAU]; /* first min(tau, num_images) are used */
  double x[3];
} pmvs_eval_query;

/* One texture grab: COptim::grabTex (optim.cpp:815-863) followed by COptim::normalize
 * (optim.cpp:1031-1067) when valid. */
typedef struct pmvs_tex_query {
  float coord[4];
  float pxaxis[4];
  float pyaxis[4];
  float normal[4];
  int32_t view;
  int32_t normalize; /* 1 = apply normalize() to a valid texture */
} pmvs_tex_query;

typedef struct pmvs_stats {
  int64_t candidates;
  int64_t accepted;
  int64_t fail_pre;
  int64_t fail_post;
  int64_t refine_failed;  /* optimizer result not in {SUCCESS, STOPVAL, FTOL, XTOL} */
  int64_t evals;          /* my_f evaluations inside refinePatch */
  int64_t tex_valid;      /* sum over those evaluations of valid textures (algorithmic bytes = 588*this for wsize 7) */
  int64_t tex_grabs;      /* every grabTex executed (incl. pre/post-processing) */
  double kernel_ms;       /* device time of the last call's kernels (HIP events on the scene stream) */
  /* refine-kernel phase profile (diagnostics; summed over wavefronts, shader clock cycles) */
  int64_t opt_cycles;       /* BOBYQA steps, refill and request publication */
  int64_t objective_cycles; /* cooperative my_f / computeINCC evaluation */
  int64_t rounds;           /* optimizer rounds (all lanes step once) */
  int64_t chunks;           /* cooperative objective chunks */
  int64_t prof[8];          /* cycles: refill, optimizer step, publish, chunk setup, gather, normalize, dot, reduce */
  double pre_ms, refine_ms, post_ms; /* per-kernel device time of the last refine batch (HIP events) */
} pmvs_stats;

typedef struct pmvs_scene pmvs_scene;

/* Last error message of the calling thread (never NULL). */
const char* pmvs_last_error(void);

/* Number of visible HIP devices (0 if none). */
int32_t pmvs_device_count(void);

/* Replaces CFindMatch::init's image/camera setup (findMatch.cpp:30-107): CPhotoSetS::init
 * (photoSetS.cpp:12-80) + CImage::buildImage pyramids (image.cpp:228-325, built ON DEVICE),
 * CCamera::updateCamera (camera.cpp:109-138), COptim::setAxesScales (optim.cpp:43-64) and the
 * threshold defaults (findMatch.cpp:92-106).  Copies everything to device `device`. */
pmvs_status pmvs_scene_create(const pmvs_scene_desc* desc, int32_t device, pmvs_scene** out);

void pmvs_scene_destroy(pmvs_scene* scene);

/* CFindMatch::updateThreshold semantics (findMatch.cpp:23-28) made explicit, plus _depth. */
pmvs_status pmvs_set_thresholds(pmvs_scene* scene, float ncc, float ncc_before, int32_t depth);

/* Read back one pyramid level of one view (parity of CImage::buildImage). */
pmvs_status pmvs_scene_get_level(pmvs_scene* scene, int32_t view, int32_t level, uint8_t* out,
                                 int32_t* width, int32_t* height);

/* A feature point (PMVS3::CPoint, point.hpp): image coordinates at the option level, detector
 * response, type 0 = Harris, 1 = DoG. */
typedef struct pmvs_point {
  float x, y, response;
  int32_t type;
} pmvs_point;

/* PMVS3::CDetectFeatures::run for one view (detectFeatures.cpp:47-124; the caller is
 * CFindMatch::init, findMatch.cpp:79-82 with fcsize 16): CHarris (sigma 4) then
 * CDifferenceOfGaussians (scales 1..3) on the view's pyramid at the scene level with its mask and
 * edge images, at most 4 points per 2*fcsize block, computed on the device.  Points come in the
 * reference's order: Harris points by decreasing response, then DoG points by decreasing response
 * (each detector's std::multiset read from its end).  *n_out = the number of points; at most cap
 * are written (call with cap = 0 to size the array). */
pmvs_status pmvs_detect_features(pmvs_scene* scene, int32_t view, int32_t fcsize, pmvs_point* out, int32_t cap,
                                 int32_t* n_out);

/* Batched COptim::grabTex + normalize: out_tex is n * 3*wsize*wsize floats, out_valid n ints
 * (1 = texture grabbed, 0 = grabTex returned 1 / empty texture). */
pmvs_status pmvs_grab_tex(pmvs_scene* scene, const pmvs_tex_query* q, int32_t n, float* out_tex,
                          int32_t* out_valid);

/* Batched COptim::my_f: out_f[i] = my_f(q[i].x) after the refinePatchBFGS setup of q[i]. */
pmvs_status pmvs_incc_eval(pmvs_scene* scene, const pmvs_eval_query* q, int32_t n, double* out_f,
                           pmvs_stats* stats);

/* Batched preProcess -> refinePatch -> postProcess (optim.cpp:95-190, 496-658) for n candidates
 * at the scene's current thresholds, as the seed phase calls them (CSeed at _depth 0,
 * findMatch.cpp:187-194; seed.cpp:385-395).  The expansion's calls (expand.cpp:225-237, _depth >= 1)
 * also run postProcess's organizer steps (setVImagesVGrids, check(); optim.cpp:178-188) against the
 * model, so they run inside pmvs_expand_run / pmvs_run_loop, where the organizer lives on the
 * device; this call returns PMVS_EUNSUPPORTED when the scene's depth is >= 1. */
pmvs_status pmvs_refine_batch(pmvs_scene* scene, const pmvs_candidate* in, int32_t n,
                              pmvs_refined* out, pmvs_stats* stats);

/* Device-resident variant for benchmarking: candidates/results already on the device
 * (pointers from hipMalloc / torch).  Runs on the scene stream and waits once mid-call (after
 * preProcess, for the start points' angles, which the host's libm computes as the reference's
 * encode does); returns with the refine and postProcess kernels queued: call pmvs_scene_sync()
 * and read stats afterwards. */
pmvs_status pmvs_refine_batch_device(pmvs_scene* scene, const pmvs_candidate* d_in, int32_t n,
                                     pmvs_refined* d_out);
pmvs_status pmvs_scene_sync(pmvs_scene* scene, pmvs_stats* stats);


/* Self-test: evaluates the device libm function `op` (0 sqrt, 1 sin, 2 cos, 3 asin, 4 acos,
 * 5 atan, 6 log, 7 f32 sqrt, 8 f32 divide in[i]/in[i+1], 9 floor) on n doubles. */
pmvs_status pmvs_selftest_math(int32_t device, int32_t op, const double* in, double* out, int32_t n);

/* Self-test: the device Cmylapack::lls (filterQuad's least squares, Eigen JacobiSVD semantics) on
 * nsys n_k x 5 systems: rows offsets[k] .. offsets[k+1]-1 of A (5 floats per row) and b; x: 5 floats
 * per system. */
pmvs_status pmvs_selftest_lls(int32_t device, const float* A, const float* b, const int32_t* offsets, int32_t nsys,
                              float* x);

/* Self-test: device BOBYQA on analytic objective `kind` (0 quadratic, 1 Rosenbrock-3, 2 bound
 * active) from n start points x0 (3 doubles each).  mode 0 = one problem per lane, 1 = one per
 * wavefront.  out: 6 doubles per problem (x[3], minf, nevals, result code); *ms kernel time. */
pmvs_status pmvs_selftest_bobyqa(int32_t device, int32_t mode, int32_t kind, const double* x0, int32_t n,
                                 int32_t maxeval, double* out, double* ms);

/* ---------------------------------------------------------------------------------------
 * Filter pass over a patch set (PMVS3::CFilter::run, filter.cpp:13-27): the cell organizer
 * (CPatchOrganizerS pgrids / vpgrids / depth maps) is built on the device from the patch
 * array; insertion order = array index.  Runs at the scene's thresholds and depth
 * (pmvs_set_thresholds; the reference runs filters at depth >= 1).
 * The model record (CPatch, patch.hpp:10-77) keeps its lists as 16-bit view indexes and 16-bit
 * cell coordinates (scenes of < 32768 views, cell grids < 32768 wide and high: checked by
 * pmvs_scene_create), so 128-entry lists cost the bytes 64 32-bit entries did. */
typedef struct pmvs_patch {
  float coord[4], normal[4];
  float ncc, dscale, ascale, tmp;
  int32_t timages, flag, fix, num_images, num_vimages, dflag; /* dflag: CPatch::_dflag (failed expansion directions) */
  int16_t images[PMVS_MAX_IMAGES];
  int16_t grids[PMVS_MAX_IMAGES][2];
  int16_t vimages[PMVS_MAX_IMAGES];
  int16_t vgrids[PMVS_MAX_IMAGES][2];
} pmvs_patch;

/* pmvs_patch.fix: 0 = a patch of this scene, 1 = fixed (CPatch::_fix, patchOrganizerS.cpp:175-197: never
 * filtered), PMVS_FIX_FOREIGN = another cluster's boundary patch inserted by the cluster exchange
 * (pmvs_scene_set_cluster): fixed, and never expanded or returned by this scene. */
#define PMVS_FIX_FOREIGN 2

typedef struct pmvs_filter_stats {
  int64_t input, removed_outside, removed_exact, removed_neighbor, removed_groups, kept;
  double kernel_ms;
} pmvs_filter_stats;

/* patches are updated in place (images/grids/timages/vimages/vgrids as the reference leaves
 * them); keep[i] = 1 when patch i is still in the organizer (the model) after the pass. */
pmvs_status pmvs_filter_run(pmvs_scene* scene, pmvs_patch* patches, int32_t n, int32_t* keep,
                            pmvs_filter_stats* stats);

/* One expansion run (PMVS3::CExpand::run, expand.cpp:17-406) on a model = patches[i] with
 * alive[i] (the state a filter pass leaves: pgrids/vpgrids/depth maps are rebuilt from it).  The
 * max-_tmp queue is expanded in waves of `wave` parents (1 = the reference's single-thread
 * schedule), candidates are refined with preProcess -> refinePatch ->
 * postProcess including the depth >= 1 steps (setVImagesVGrids; check() at depth >= 2) and
 * committed in (parent priority, direction) order; with min_candidates > 0 (and wave > 1) a wave
 * takes further chunks of `wave` parents until its parents have that many free directions
 * (findEmptyBlocks against the start-of-wave model).  count_threshold = _countThreshold1 (4 at the
 * first expansion, 2 after updateThreshold).  The result is the old patches (with updated
 * _flag/_dflag) followed by the new ones, at most `cap` in all; *n_out is their number.
 * out/alive_out receive it when non-NULL; with out == alive_out == NULL the scene keeps it and
 * pmvs_expand_fetch copies it out (so the caller can size its arrays after the run).
 * With a shard set (pmvs_scene_set_shard) the call is collective: every rank passes the same
 * model and arguments and gets the same result. */
#define PMVS_EXPAND_AFTER_SEEDS 1 /* model straight from the seed phase: no depth maps yet (findMatch.cpp:193-202) */
/* flags bits 8..31: stop after that many waves (0 = run until the queue is empty).  Not a reference
 * behaviour: it bounds full-size parity samples against the CPU oracle, which has the same bound. */
#define PMVS_EXPAND_MAX_WAVES(n) ((int32_t)((uint32_t)(n) << 8))
typedef struct pmvs_expand_stats {
  int64_t parents, candidates, fail_prep, fail_pre, fail_post, fail_commit, added, waves;
  double wall_ms;
  /* this rank's refine work (preProcess -> refinePatch -> postProcess of its candidate share):
   * candidates refined, my_f + computeINCC evaluations, valid textures over them, summed
   * refine-kernel time (HIP events) */
  int64_t refined, evals, tex_valid;
  double refine_ms;
  int64_t refine_launches;
  /* the part of tex_valid / refine_ms / refine_launches that ran the small-batch refine layout
   * (batches below the scene's small-batch size: the workgroup-form kernel) */
  int64_t tex_valid_small;
  double refine_ms_small;
  int64_t refine_launches_small;
} pmvs_expand_stats;
pmvs_status pmvs_expand_run(pmvs_scene* scene, const pmvs_patch* patches, const int32_t* alive, int32_t n,
                            int32_t wave, int32_t min_candidates, int32_t count_threshold, int32_t flags, pmvs_patch* out, int32_t* alive_out,
                            int32_t cap, int32_t* n_out, pmvs_expand_stats* stats);
/* Copies the result the last pmvs_expand_run kept (out == NULL) and releases it; n = *n_out. */
pmvs_status pmvs_expand_fetch(pmvs_scene* scene, pmvs_patch* out, int32_t* alive_out, int32_t n);

/* The dense-matching loop after the seed phase, PMVS3::CFindMatch::run (findMatch.cpp:196-217):
 * `iterations` x (CExpand::run, CFilter::run, updateThreshold) from the seed patches, with the
 * model resident in HBM between the passes (only the final model crosses PCIe).  Thresholds as
 * the reference: depth 1 upwards, ncc = threshold and before = threshold - 0.3f, both -= 0.05f
 * and _countThreshold1 4 -> 2 after each iteration (findMatch.cpp:23-28, 104).  flags:
 * PMVS_EXPAND_AFTER_SEEDS for the first expansion; PMVS_EXPAND_MAX_WAVES(n) bounds every
 * iteration's expansion to n waves (not a reference behaviour: full-size parity samples of the
 * whole loop against the CPU oracle, which has the same bound).  cap bounds the model size.  *n_out = the final
 * model's size; pmvs_loop_fetch copies it out.  iters (may be NULL) receives per-iteration stats.
 * Collective when a shard is set. */
typedef struct pmvs_loop_iter {
  int32_t depth, patches; /* patches kept after the filter pass */
  pmvs_expand_stats expand;
  pmvs_filter_stats filter;
  /* cluster exchange after this iteration (pmvs_scene_set_cluster; 0 otherwise): this rank's boundary
   * patches sent, the other ranks' records received, the records inserted as foreign patches */
  int64_t boundary_sent, boundary_received, boundary_inserted;
} pmvs_loop_iter;
pmvs_status pmvs_run_loop(pmvs_scene* scene, const pmvs_patch* seeds, int32_t n, float threshold, int32_t iterations,
                          int32_t wave, int32_t min_candidates, int32_t flags, int32_t cap, int32_t* n_out, pmvs_loop_iter* iters);
pmvs_status pmvs_loop_fetch(pmvs_scene* scene, pmvs_patch* out, int32_t n);
/* (new) A 64-bit digest of pmvs_run_loop's result while it is still on the device (no PCIe
 * transfer): every record's bytes mixed with its position, so equal models give equal digests
 * (identical-repetition checks of a device-resident pipeline).  pmvs_loop_fetch still works after it. */
pmvs_status pmvs_loop_hash(pmvs_scene* scene, uint64_t* hash);

/* The seed phase, PMVS3::CSeed::init + run (seed.cpp:11-107) at CPU 1: target images in the
 * reference's std::shuffle(mt19937(42)) order, cells in raster order, the feature points of every
 * view (points: num_points[0] of view 0, then view 1, ..., as pmvs_detect_features returns them)
 * matched along epipolar lines on the device, and the candidates of a point refined in order of
 * _response (the reference sorts them by heap address, seed.cpp:322: documented deviation) until
 * two succeed (preProcess -> refinePatch -> postProcess, seed.cpp:387-414).  Refinement is batched
 * and speculative; the result equals the sequential one for any batch size.  Runs at depth 0 with
 * the scene's current thresholds (CFindMatch::init values).  Writes the seed patches in addPatch
 * order (at most cap; *n_out = their number) -- the `seeds` input of pmvs_run_loop.  With out = NULL
 * and cap = 0 the scene keeps the seeds and pmvs_seed_fetch copies them out (size the array from
 * *n_out first). */
typedef struct pmvs_seed_stats {
  int64_t trial, pass, fail0, fail1; /* initialMatchSub calls and outcomes (seed.cpp:94-100) */
  int64_t refined;                   /* candidates refined on the device (incl. speculative ones) */
  int64_t rounds;                    /* refine launches */
  int64_t candidates;                /* epipolar candidates collected */
  int64_t reserved;
  double wall_ms, gen_ms, refine_ms; /* whole call, candidate generation, refine batches (wall) */
} pmvs_seed_stats;
pmvs_status pmvs_seed_run(pmvs_scene* scene, const pmvs_point* points, const int32_t* num_points, int32_t batch,
                          pmvs_patch* out, int32_t cap, int32_t* n_out, pmvs_seed_stats* stats);
/* Copies the seeds the last pmvs_seed_run kept (out = NULL, cap = 0) and releases them; n = *n_out. */
pmvs_status pmvs_seed_fetch(pmvs_scene* scene, pmvs_patch* out, int32_t n);

/* Multi-GPU sharding of the expansion: one scene per GPU/rank, all holding the
 * same model.  Each wave's candidates are split into contiguous rank ranges for the refine and
 * the per-candidate results are all-gathered through `fn` before the (replicated) commit.
 * fn(ctx, send, bytes, recv): all-gather of `bytes` from every rank into recv (world * bytes, in
 * rank order), host memory, returns 0 on success; it is called from the thread that called
 * pmvs_expand_run.  world = 1 (or fn = NULL) turns sharding off. */
typedef int (*pmvs_allgather_fn)(void* ctx, const void* send, int64_t bytes, void* recv);
pmvs_status pmvs_scene_set_shard(pmvs_scene* scene, int32_t rank, int32_t world, pmvs_allgather_fn fn, void* ctx);

/* Native RCCL communicator (one process per GPU; librccl.so.1 opened at run time).  Rank 0 calls
 * pmvs_rccl_unique_id and shares the 128 bytes with every rank (any channel); each rank calls
 * pmvs_rccl_create on its device, then pmvs_scene_set_shard_rccl: the expansion's per-wave
 * records are then all-gathered device to device on the scene's stream (ncclAllGather), and the
 * 8-byte error headers through pmvs_rccl_allgather (a pmvs_allgather_fn on host buffers). */
typedef struct pmvs_rccl pmvs_rccl;
pmvs_status pmvs_rccl_unique_id(uint8_t* id128);
pmvs_status pmvs_rccl_create(int32_t device, int32_t rank, int32_t world, const uint8_t* id128, pmvs_rccl** out);
void pmvs_rccl_destroy(pmvs_rccl* comm);
int pmvs_rccl_allgather(void* comm, const void* send, int64_t bytes, void* recv);
int pmvs_rccl_allgather_device(void* comm, const void* dsend, int64_t bytes, void* drecv, void* hip_stream);
pmvs_status pmvs_scene_set_shard_rccl(pmvs_scene* scene, int32_t rank, int32_t world, pmvs_rccl* comm);

/* CMVS cluster per GPU with a boundary exchange.  The reference runs one
 * pmvs2 per cluster option file (genOption.cpp:73-108) and CMVS clusters overlap in their target images
 * (bundle.cpp:1003-1160, ske.dat).  With a cluster set, pmvs_run_loop on this scene (one rank of
 * `world`, one scene per GPU) all-gathers after every iteration but the last, through `fn` (or the
 * native RCCL communicator, device to device), the patches it holds in target images that another
 * rank also has as targets -- a {error, record count} header per rank first, then the records with
 * image NUMBERS.  (CExpand's per-cell _counts are not exchanged: every expansion run starts by clearing
 * them, expand.cpp:32, and the exchange happens between runs; the inserted patches carry the cell
 * occupancy the next run's checkCounts reads.)  Every rank inserts the other ranks' records whose reference
 * image is one of its views as the reference's readPatches inserts another run's patches
 * (patchOrganizerS.cpp:133-197: image numbers mapped to indexes, _vimages cleared, setGrids, addPatch),
 * as fixed patches that are never expanded (fix = PMVS_FIX_FOREIGN): they fill their cells, so the
 * rank does not reconstruct the surface the others already hold there, and they take part in the
 * filters' visibility tests.  Foreign patches are never returned: the final model is this cluster's
 * own patches, and the merged reconstruction is the concatenation of the ranks' models (as the
 * reference's per-cluster .ply files are merged).  image_ids: num_views global image numbers of the
 * scene's views (the option file's timages then oimages).  Collective: every rank calls it (it
 * all-gathers the target lists once).  world = 1 turns it off.  Not combined with a shard. */
pmvs_status pmvs_scene_set_cluster(pmvs_scene* scene, int32_t rank, int32_t world, const int32_t* image_ids,
                                   pmvs_allgather_fn fn, void* ctx);
pmvs_status pmvs_scene_set_cluster_rccl(pmvs_scene* scene, int32_t rank, int32_t world, const int32_t* image_ids,
                                        pmvs_rccl* comm);

/* A host all-gather over TCP among `world` processes (pmvs_hostcomm.cpp): rank 0 listens on addr:port,
 * the other ranks connect (retrying until timeout_ms); pmvs_tcp_allgather is a pmvs_allgather_fn with
 * ctx = the pmvs_tcp.  The multi-rank pmvs2 job's bootstrap (the RCCL unique id travels on it) and its
 * exchange channel when the ranks share one GPU (PMVS_EXCHANGE=tcp).  A rank that exits closes its
 * connection, so its peers' exchanges fail instead of blocking. */
typedef struct pmvs_tcp pmvs_tcp;
pmvs_status pmvs_tcp_create(int32_t rank, int32_t world, const char* addr, int32_t port, int32_t timeout_ms,
                            pmvs_tcp** out);
int pmvs_tcp_allgather(void* ctx, const void* send, int64_t bytes, void* recv);
void pmvs_tcp_destroy(pmvs_tcp* comm);

/* An in-process all-gather among `world` threads (one scene per thread, e.g. several scenes on
 * one GPU): pmvs_thread_allgather with ctx = pmvs_thread_exchange_ctx(group, rank). */
typedef struct pmvs_thread_exchange pmvs_thread_exchange;
pmvs_thread_exchange* pmvs_thread_exchange_create(int32_t world);
void* pmvs_thread_exchange_ctx(pmvs_thread_exchange* group, int32_t rank);
int pmvs_thread_allgather(void* ctx, const void* send, int64_t bytes, void* recv);
void pmvs_thread_exchange_destroy(pmvs_thread_exchange* group);

/* ---------------------------------------------------------------------------------------
 * pmvs2 input / output surface (SURVEY.md §8(b) external boundary, §8 row a19).  Host code;
 * errors are status codes (the reference exits). */

/* Image::CCamera::init + setProjection (camera.cpp:13-54, 256-360): reads a CONTOUR /
 * CONTOUR2 / CONTOUR3 txt file and writes the level-0 3x4 projection (row-major). */
pmvs_status pmvs_camera_load(const char* txt_path, float projection[12]);

/* Binary 8-bit PPM (P6) reader: the PNM path of CImage::readAnyImage (image.cpp:473-506).
 * rgb may be NULL to query the size; otherwise width*height*3 bytes are written. */
pmvs_status pmvs_ppm_load(const char* path, int32_t* width, int32_t* height, uint8_t* rgb);

/* CImage::readAnyImage (image.cpp:473-506) by extension: binary PPM, or JPEG decoded with the
 * image's libjpeg (loaded at run time, as CImg's cimg_use_jpeg path).  rgb may be NULL (size query). */
pmvs_status pmvs_image_load(const char* path, int32_t* width, int32_t* height, uint8_t* rgb);

/* CImage::readPGMImage / readPBMImage (image.cpp:508-670): binary P5 / P4 mask or edge image, raw
 * bytes (P4 bits: 1 -> 0, 0 -> 255).  out may be NULL (size query). */
pmvs_status pmvs_pnm_mask_load(const char* path, int32_t* width, int32_t* height, uint8_t* out);

/* CImage::setEdge (image.cpp:407-460): the edge map the option `setEdge threshold` derives from the
 * level-0 image (width*height bytes, 0/255). */
pmvs_status pmvs_set_edge(const uint8_t* rgb, int32_t width, int32_t height, float threshold, uint8_t* edge_out);

/* PMVS3::SOption (option.cpp:10-307): option file keys and defaults, timages/oimages
 * (enumeration, -1 range, -2 from vis.dat, -3 none), useVisData (vis.dat), useBound
 * (bimages.dat).  Image lists are image NUMBERS; visdata2 is CSR over view indexes
 * (timages first, then oimages); bindexes are target indexes. */
typedef struct pmvs_options {
  int32_t level, csize, wsize, min_image_num, cpu, use_bound, use_vis_data, sequence, tflag, oflag;
  float threshold, set_edge, max_angle /* radians */, quad;
  int32_t num_timages, num_oimages, num_bindexes;
  const int32_t* timages;
  const int32_t* oimages;
  const int32_t* bindexes;
  const int32_t* visdata2_offsets; /* num_timages + num_oimages + 1 */
  const int32_t* visdata2;
} pmvs_options;
pmvs_status pmvs_options_load(const char* prefix, const char* option_file, pmvs_options** out);
void pmvs_options_free(pmvs_options* options);

/* Patch fields for the writers: 11 floats per patch = coord[4], normal[4], ncc, dscale, ascale. */
/* .patch text exactly as CPatchOrganizerS::writePatches2 + Patch::operator<< (patchOrganizerS.cpp:98-116,
 * patch.cpp:31-48); ids/vids are image numbers (index2image applied by the caller). */
pmvs_status pmvs_write_patches(const char* path, int32_t n, const float* fields, const int32_t* nimg,
                               const int32_t* ids, const int32_t* nvimg, const int32_t* vids);
/* .pset text (patchOrganizerS.cpp:118-131). */
pmvs_status pmvs_write_pset(const char* path, int32_t n, const float* fields);
/* ASCII .ply with colour and quality (CPatchOrganizerS::writePLY, patchOrganizerS.cpp:687-776). */
pmvs_status pmvs_write_ply(const char* path, int32_t n, const float* fields, const int32_t* colors);
/* writePLY colour mode 0 on the device: mean of CPhotoSetS::getColor over the patch's images at
 * the scene level, floor(c + 0.5) clamped to 255.  images_flat holds nimg[i] view indexes per patch. */
pmvs_status pmvs_patch_colors(pmvs_scene* scene, int32_t n, const float* coords4, const int32_t* nimg,
                              const int32_t* images_flat, int32_t* colors_out);

/* ---------------------------------------------------------------------------------------
 * Synthetic workload generator (NOT a reference interface: the reference ships no data).
 * Textured unit sphere seen by a ring of pinhole cameras. */
typedef struct pmvs_synth_params {
  int32_t num_views;     /* ring cameras */
  int32_t num_targets;   /* candidate reference images are drawn from the first num_targets */
  int32_t width, height; /* level-0 image size */
  int32_t supersample;   /* per-axis supersampling (1..4) */
  int32_t level;         /* option level the candidates are meant for (depth perturbation scale) */
  uint64_t seed;         /* texture seed */
  double ring_radius;    /* camera distance from the sphere centre (4.0) */
  double height_offset;  /* alternating camera height (0.3) */
  double focal_scale;    /* f = focal_scale * width */
  double arc_step_deg;   /* angular spacing of the cameras on the ring (0 = 360/num_views) */
  /* photometrically hard mode (all 0 = the plain scene): per-view gain N(1, gain_sigma) and bias
   * N(0, bias_sigma), per-pixel sensor noise of std noise_sigma (intensities in [0, 1]), low-texture
   * regions where a low-frequency noise field is below `lowtex` (texture contrast x 0.05), and a
   * textured occluding sphere of radius occluder_radius between the ring and the main sphere. */
  double gain_sigma, bias_sigma, noise_sigma, lowtex, occluder_radius;
  /* render only the render_count views render_first, render_first + 1, ... (mod num_views) into rgb
   * (count 0 = all views); projections are written for every view */
  int32_t render_first, render_count;
} pmvs_synth_params;

/* Renders num_views RGB8 images (rgb: num_views*width*height*3 bytes, may be NULL to get only
 * the projections) and writes num_views 3x4 projections (proj: 12 floats per view). */
pmvs_status pmvs_synth_ring(const pmvs_synth_params* p, uint8_t* rgb, float* proj, int32_t nthreads);

/* n seed-path candidates (images = [most frontal target, next most frontal view]). */
pmvs_status pmvs_synth_candidates(const pmvs_synth_params* p, const float* proj, int32_t n, uint64_t seed,
                                  float depth_sigma_px, float max_tilt_deg, pmvs_candidate* out);

#ifdef __cplusplus
}
#endif
#endif /* PMVS_AMD_H */
