// pmvs2_main.cpp -- the `pmvs2 prefix option_file [PATCH] [PSET]` executable (reference
// source/pmvs.cpp:7-63 with CFindMatch::init / run / write, findMatch.cpp:30-224), driving the
// MI355X-native core through its C-ABI (include/pmvs_amd.h).  A drop-in for the program
// genOption's pmvs.sh calls (genOption.cpp:73): same arguments, same input tree
// (prefix/visualize, prefix/txt, prefix/masks, prefix/edges, vis.dat, bimages.dat), same outputs
// (prefix/models/<option>.ply always, .patch / .pset on request).
//
// Pipeline: option file -> images (PPM / JPEG), masks, edges, cameras -> pmvs_scene_create (device
// pyramids) -> pmvs_detect_features (Harris + DoG on the device) -> pmvs_seed_run (seed phase) ->
// pmvs_run_loop (3 x expand / filter, model resident in HBM) -> writers (colours on the device).
//
// Multi-rank jobs (CMVS cluster per GPU): with WORLD_SIZE > 1 in the environment
// (torchrun-style: RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT; genOption --gpus N writes
// the script that sets them) the WORLD_SIZE pmvs2 processes of one job -- one cluster option file
// each -- find each other over TCP (pmvs_tcp), and their loops exchange the clusters' boundary
// patches after every iteration (pmvs_scene_set_cluster): device to device over RCCL on GPU LOCAL_RANK
// (the unique id travels on the TCP channel), or over the TCP channel itself with
// PMVS_EXCHANGE=tcp (several ranks on one GPU).  Each rank writes its own cluster's outputs.
//
// Expansion schedule: option `CPU 1` selects the reference's single-thread schedule exactly
// (wave = 1); any other value the production wave schedule (the reference's own
// multi-threaded schedule is nondeterministic).  PMVS_WAVE / PMVS_MIN_CANDIDATES override it.
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pmvs_amd.h"

namespace {

bool exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

[[noreturn]] void die(const char* what, pmvs_status st) {
  std::cerr << "pmvs2: " << what << ": " << pmvs_last_error() << " (status " << (int)st << ")" << std::endl;
  std::exit(1);
}

#define CHECK(what, expr)                     \
  do {                                        \
    pmvs_status st_ = (expr);                 \
    if (st_ != PMVS_OK) die(what, st_);       \
  } while (0)

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

const char* env_str(const char* name, const char* dflt) {
  const char* e = std::getenv(name);
  return (e && *e) ? e : dflt;
}

// The job's channels (WORLD_SIZE > 1): TCP between the processes, and RCCL unless PMVS_EXCHANGE=tcp.
struct Job {
  int rank = 0, world = 1, device = 0;
  bool rccl = true;
  pmvs_tcp* tcp = nullptr;
  pmvs_rccl* comm = nullptr;
  ~Job() {
    pmvs_rccl_destroy(comm);
    pmvs_tcp_destroy(tcp);
  }
  // every rank's `ok` flag; false when some rank failed (or has exited: its connection is closed)
  bool all_ok(bool ok) {
    if (world == 1) return ok;
    int32_t mine = ok ? 1 : 0;
    std::vector<int32_t> all(world, 0);
    if (pmvs_tcp_allgather(tcp, &mine, sizeof(mine), all.data()) != 0) return false;
    for (int32_t a : all)
      if (!a) return false;
    return true;
  }
};

// CImage::completeName (image.cpp:40-84): the first existing extension, else the bare name.
std::string complete_name(const std::string& base, bool color) {
  const char* ext_c[] = {".ppm", ".jpg"};
  const char* ext_m[] = {".pgm", ".pbm"};
  for (const char* e : (color ? ext_c : ext_m))
    if (exists(base + e)) return base + e;
  return base;
}

struct View {
  std::vector<uint8_t> rgb, mask, edge;
  int w = 0, h = 0;
  float proj[12];
};

void usage(const char* argv0) {
  std::cerr << "Usage: " << argv0 << " prefix option_file [Optional export]" << std::endl
            << std::endl
            << "--------------------------------------------------" << std::endl
            << "level       1    csize    2" << std::endl
            << "threshold   0.7  wsize    7" << std::endl
            << "minImageNum 3    CPU      4" << std::endl
            << "useVisData  0    sequence -1" << std::endl
            << "quad        2.5  maxAngle 10.0" << std::endl
            << "--------------------------------------------------" << std::endl
            << "2 ways to specify targetting images" << std::endl
            << "timages  5  1 3 5 7 9 (enumeration)" << std::endl
            << "        -1  0 24 (range specification)" << std::endl
            << "--------------------------------------------------" << std::endl
            << "4 ways to specify other images" << std::endl
            << "oimages  5  0 2 4 6 8 (enumeration)" << std::endl
            << "        -1  24 48 (range specification)" << std::endl
            << std::endl
            << "[Optional export] PATCH PSET" << std::endl
            << " i.e export patch and pset: prefix option_file PATCH PSET"
            << " i.e export patch only: prefix option_file PATCH" << std::endl;
}

}  // namespace

int main(int argc, char* argv[]) {
  if (argc < 3) {
    usage(argv[0]);
    return 1;
  }
  for (int i = 0; i < argc; ++i) std::cout << std::endl << argv[i];
  std::cout << std::endl;
  const std::string prefix = argv[1], option = argv[2];
  bool export_patch = false, export_pset = false;
  for (int i = 3; i < argc; ++i) {
    if (std::string(argv[i]) == "PATCH") export_patch = true;
    if (std::string(argv[i]) == "PSET") export_pset = true;
  }
  const double t0 = now_s();

  // ---- the job (WORLD_SIZE > 1: one rank per cluster option file)
  Job job;
  job.world = env_int("WORLD_SIZE", 1);
  job.rank = env_int("RANK", 0);
  job.device = env_int("PMVS_DEVICE", env_int("LOCAL_RANK", 0));
  job.rccl = std::string(env_str("PMVS_EXCHANGE", "rccl")) != "tcp";
  if (job.world < 1 || job.rank < 0 || job.rank >= job.world) {
    std::cerr << "pmvs2: RANK " << job.rank << " / WORLD_SIZE " << job.world << " out of range" << std::endl;
    return 1;
  }
  if (job.world > 1) {
    CHECK("job", pmvs_tcp_create(job.rank, job.world, env_str("MASTER_ADDR", "127.0.0.1"), env_int("MASTER_PORT", 29533),
                                 env_int("PMVS_JOIN_TIMEOUT_MS", 600000), &job.tcp));
    std::cerr << "pmvs2: rank " << job.rank << " of " << job.world << ", GPU " << job.device << ", exchange "
              << (job.rccl ? "rccl" : "tcp") << std::endl;
  }

  // ---- SOption::init (option.cpp:30-160)
  pmvs_options* opt = nullptr;
  CHECK("option file", pmvs_options_load(prefix.c_str(), option.c_str(), &opt));
  std::vector<int> images(opt->timages, opt->timages + opt->num_timages);
  images.insert(images.end(), opt->oimages, opt->oimages + opt->num_oimages);
  const int num = (int)images.size(), tnum = opt->num_timages;
  if (tnum == 0) {
    std::cerr << "pmvs2: no target images" << std::endl;
    return 1;
  }

  // ---- CPhotoSetS::init (photoSetS.cpp:12-80): 8-digit names, else 4-digit.  The reference decodes
  // the views one after the other; here a pool of host threads decodes them (PMVS_IO_THREADS, default
  // min(16, cores)), and failures are reported in view order as the serial loop would.
  std::vector<View> views(num);
  std::vector<std::string> errors(num);
  std::vector<pmvs_status> status(num, PMVS_OK);
  std::cerr << "Reading images: " << std::flush;
  {
    std::atomic<int> next{0};
    auto load_one = [&](int index) -> pmvs_status {
      const int image = images[index];
      char b8[64], b4[64];
      std::snprintf(b8, sizeof(b8), "%08d", image);
      std::snprintf(b4, sizeof(b4), "%04d", image);
      const std::string v8 = prefix + "visualize/" + b8;
      const std::string id = (exists(v8 + ".ppm") || exists(v8 + ".jpg")) ? b8 : b4;
      View& v = views[index];
      const std::string name = complete_name(prefix + "visualize/" + id, true);
      pmvs_status st;
      errors[index] = "image";
      if ((st = pmvs_image_load(name.c_str(), &v.w, &v.h, nullptr))) return st;
      v.rgb.resize((size_t)v.w * v.h * 3);
      if ((st = pmvs_image_load(name.c_str(), &v.w, &v.h, v.rgb.data()))) return st;
      errors[index] = "camera";
      if ((st = pmvs_camera_load((prefix + "txt/" + id + ".txt").c_str(), v.proj))) return st;
      for (int k = 0; k < 2; ++k) {
        const std::string m = complete_name(prefix + (k == 0 ? "masks/" : "edges/") + id, false);
        if (m.size() < 4 || (m.compare(m.size() - 4, 4, ".pgm") && m.compare(m.size() - 4, 4, ".pbm"))) continue;
        int mw = 0, mh = 0;
        std::vector<uint8_t>& dst = k == 0 ? v.mask : v.edge;
        errors[index] = "mask/edge";
        if ((st = pmvs_pnm_mask_load(m.c_str(), &mw, &mh, nullptr))) return st;
        if (mw != v.w || mh != v.h) {
          errors[index] = m + " is " + std::to_string(mw) + "x" + std::to_string(mh) + ", image " + std::to_string(v.w) +
                          "x" + std::to_string(v.h);
          return PMVS_EINVAL;
        }
        dst.resize((size_t)mw * mh);
        if ((st = pmvs_pnm_mask_load(m.c_str(), &mw, &mh, dst.data()))) return st;
      }
      // CFindMatch::init: _pss.setEdge(_setEdge) replaces the edge maps (findMatch.cpp:74-76)
      if (opt->set_edge != 0.0f) {
        v.edge.resize((size_t)v.w * v.h);
        errors[index] = "setEdge";
        if ((st = pmvs_set_edge(v.rgb.data(), v.w, v.h, opt->set_edge, v.edge.data()))) return st;
      }
      return PMVS_OK;
    };
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int nthreads = std::max(1, std::min({num, env_int("PMVS_IO_THREADS", std::min(16, hw))}));
    std::vector<std::thread> pool;
    for (int t = 0; t < nthreads; ++t)
      pool.emplace_back([&]() {
        for (int index; (index = next.fetch_add(1)) < num;) {
          status[index] = load_one(index);
          if (status[index] != PMVS_OK && errors[index].find(' ') == std::string::npos)
            errors[index] += std::string(": ") + pmvs_last_error();  // the worker's own last error
        }
      });
    for (auto& t : pool) t.join();
  }
  for (int index = 0; index < num; ++index) {
    if (status[index] != PMVS_OK) {
      std::cerr << std::endl << "pmvs2: " << errors[index] << " (status " << (int)status[index] << ")" << std::endl;
      return 1;
    }
    std::cerr << '*';
  }
  std::cerr << std::endl;
  const double t_read = now_s();

  // ---- the device scene (CFindMatch::init, findMatch.cpp:30-107)
  std::vector<pmvs_view_desc> vd(num);
  for (int i = 0; i < num; ++i) {
    vd[i].width = views[i].w;
    vd[i].height = views[i].h;
    vd[i].rgb = views[i].rgb.data();
    vd[i].mask = views[i].mask.empty() ? nullptr : views[i].mask.data();
    vd[i].edge = views[i].edge.empty() ? nullptr : views[i].edge.data();
    std::memcpy(vd[i].projection, views[i].proj, sizeof(views[i].proj));
  }
  pmvs_scene_desc d{};
  d.num_views = num;
  d.num_targets = tnum;
  d.level = opt->level;
  d.csize = opt->csize;
  d.wsize = opt->wsize;
  d.min_image_num = opt->min_image_num;
  d.threshold = opt->threshold;
  d.max_angle = opt->max_angle;
  d.quad_threshold = opt->quad;
  d.sequence = opt->sequence;
  d.visdata2_offsets = opt->visdata2_offsets;
  d.visdata2 = opt->visdata2;
  d.num_bindexes = opt->num_bindexes;
  d.bindexes = opt->bindexes;
  d.views = vd.data();
  pmvs_scene* sc = nullptr;
  CHECK("scene", pmvs_scene_create(&d, job.device, &sc));
  // every rank has its scene before any collective (a rank that failed has exited, which its
  // peers see here instead of blocking in the RCCL bootstrap)
  if (!job.all_ok(true)) {
    std::cerr << "pmvs2: another rank of the job failed before the cluster exchange was set up" << std::endl;
    return 1;
  }
  if (job.world > 1) {
    if (job.rccl) {
      uint8_t id[128] = {0};
      if (job.rank == 0) CHECK("rccl", pmvs_rccl_unique_id(id));
      std::vector<uint8_t> ids((size_t)128 * job.world);
      if (pmvs_tcp_allgather(job.tcp, id, 128, ids.data()) != 0) {
        std::cerr << "pmvs2: the RCCL id exchange failed" << std::endl;
        return 1;
      }
      CHECK("rccl", pmvs_rccl_create(job.device, job.rank, job.world, ids.data(), &job.comm));
      CHECK("cluster", pmvs_scene_set_cluster_rccl(sc, job.rank, job.world, images.data(), job.comm));
    } else {
      CHECK("cluster", pmvs_scene_set_cluster(sc, job.rank, job.world, images.data(), &pmvs_tcp_allgather, job.tcp));
    }
  }
  std::vector<int> gwidth(num);  // _gwidths (patchOrganizerS.cpp:54-87)
  for (int i = 0; i < num; ++i) {
    int w = views[i].w;
    for (int l = 0; l < opt->level; ++l) w /= 2;
    gwidth[i] = (w + opt->csize - 1) / opt->csize;
  }
  std::vector<View>().swap(views);  // level-0 images live on the device now
  const double t_init = now_s();

  // ---- CDetectFeatures::run (detectFeatures.cpp:14-124, fcsize 16): skipped for an image whose
  // prefix/models/%08d.affin<level> exists, as the reference does
  std::vector<pmvs_point> points;
  std::vector<int32_t> npts(num, 0);
  for (int index = 0; index < num; ++index) {
    char buf[64];
    std::snprintf(buf, sizeof(buf), "%08d.affin%d", images[index], opt->level);
    if (exists(prefix + "models/" + buf)) continue;
    int32_t n = 0;
    CHECK("features", pmvs_detect_features(sc, index, 16, nullptr, 0, &n));
    const size_t at = points.size();
    points.resize(at + n);
    CHECK("features", pmvs_detect_features(sc, index, 16, points.data() + at, n, &n));
    npts[index] = n;
  }
  const double t_feat = now_s();

  // ---- seed phase (CSeed::run, findMatch.cpp:193)
  int32_t nseeds = 0;
  pmvs_seed_stats sst{};
  CHECK("seeds", pmvs_seed_run(sc, points.data(), npts.data(), env_int("PMVS_SEED_BATCH", 0), nullptr, 0, &nseeds,
                               &sst));
  std::vector<pmvs_patch> seeds(std::max(nseeds, 1));
  CHECK("seeds", pmvs_seed_fetch(sc, seeds.data(), nseeds));
  seeds.resize(nseeds);
  std::cerr << "Total pass fail0 fail1 refinepatch: " << sst.trial << ' ' << sst.pass << ' ' << sst.fail0 << ' '
            << sst.fail1 << ' ' << sst.pass + sst.fail1 << std::endl;
  const double t_seed = now_s();

  // every rank reaches the loop (a rank whose features or seeds failed has exited, which its peers
  // see on the TCP channel here rather than inside an RCCL collective); failures inside the loop
  // reach every rank through the loop's error headers
  if (!job.all_ok(true)) {
    std::cerr << "pmvs2: another rank of the job failed before the loop" << std::endl;
    return 1;
  }

  // ---- expansion / filtering (findMatch.cpp:196-217)
  const int wave = env_int("PMVS_WAVE", opt->cpu == 1 ? 1 : 32768);
  const int min_cands = env_int("PMVS_MIN_CANDIDATES", wave == 1 ? 0 : 131072);
  const int iterations = 3;
  std::vector<pmvs_loop_iter> it(iterations);
  int32_t nmodel = 0;
  CHECK("expand/filter", pmvs_run_loop(sc, seeds.data(), nseeds, opt->threshold, iterations, wave, min_cands,
                                       PMVS_EXPAND_AFTER_SEEDS, INT_MAX / 2, &nmodel, it.data()));
  std::vector<pmvs_patch> model(std::max(nmodel, 1));
  CHECK("fetch", pmvs_loop_fetch(sc, model.data(), nmodel));
  model.resize(nmodel);
  for (int t = 0; t < iterations; ++t)
    std::cerr << "depth " << it[t].depth << ": expanded " << it[t].expand.added << ", kept " << it[t].patches
              << (job.world > 1 ? ", boundary sent " + std::to_string(it[t].boundary_sent) + " received " +
                                      std::to_string(it[t].boundary_received) + " inserted " +
                                      std::to_string(it[t].boundary_inserted)
                                : std::string())
              << std::endl;
  const double t_loop = now_s();

  // ---- CPatchOrganizerS::writePatches2 (patchOrganizerS.cpp:89-132): collectPatches(1)
  // (patchOrganizerS.cpp:207-236) walks target images, their cells in raster order and each cell's
  // list in insertion (= model) order, taking every patch at its first registration: the key is
  // (lowest target image holding the patch, its cell there), ties in model order.
  std::vector<long long> key(nmodel);
  for (int p = 0; p < nmodel; ++p) {
    const pmvs_patch& q = model[p];
    int bt = INT_MAX, k0 = -1;
    for (int k = 0; k < q.num_images; ++k)
      if (q.images[k] < tnum && q.images[k] < bt) { bt = q.images[k]; k0 = k; }
    key[p] = k0 < 0 ? LLONG_MAX
                    : ((long long)bt << 40) + (long long)q.grids[k0][1] * gwidth[bt] + q.grids[k0][0];
  }
  std::vector<int> order(nmodel);
  for (int p = 0; p < nmodel; ++p) order[p] = p;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key[a] < key[b]; });
  std::vector<float> fields((size_t)nmodel * 11);
  std::vector<int32_t> nimg(nmodel), nvimg(nmodel), ids, vids, idx;
  for (int r = 0; r < nmodel; ++r) {
    const pmvs_patch& q = model[order[r]];
    float* f = fields.data() + (size_t)r * 11;
    for (int k = 0; k < 4; ++k) { f[k] = q.coord[k]; f[4 + k] = q.normal[k]; }
    f[8] = q.ncc; f[9] = q.dscale; f[10] = q.ascale;
    nimg[r] = q.num_images;
    nvimg[r] = q.num_vimages;
    for (int k = 0; k < q.num_images; ++k) {
      ids.push_back(images[q.images[k]]);  // index2image
      idx.push_back(q.images[k]);
    }
    for (int k = 0; k < q.num_vimages; ++k) vids.push_back(images[q.vimages[k]]);
  }
  const std::string out = prefix + "models/" + option;
  std::vector<float> coords((size_t)std::max(nmodel, 1) * 4);
  for (int r = 0; r < nmodel; ++r)
    for (int k = 0; k < 4; ++k) coords[(size_t)4 * r + k] = fields[(size_t)r * 11 + k];
  std::vector<int32_t> colors((size_t)std::max(nmodel, 1) * 3);
  if (nmodel) CHECK("colours", pmvs_patch_colors(sc, nmodel, coords.data(), nimg.data(), idx.data(), colors.data()));
  CHECK("ply", pmvs_write_ply((out + ".ply").c_str(), nmodel, fields.data(), colors.data()));
  if (export_patch)
    CHECK("patch", pmvs_write_patches((out + ".patch").c_str(), nmodel, fields.data(), nimg.data(), ids.data(),
                                      nvimg.data(), vids.data()));
  if (export_pset) CHECK("pset", pmvs_write_pset((out + ".pset").c_str(), nmodel, fields.data()));
  pmvs_scene_destroy(sc);
  pmvs_options_free(opt);
  const double t_end = now_s();
  std::fprintf(stderr,
               "---- pmvs2: %d seeds, %d patches | init %.2f s, features %.2f s, seeds %.2f s, loop %.2f s, write %.2f s "
               "----\n",
               nseeds, nmodel, t_init - t0, t_feat - t_init, t_seed - t_feat, t_loop - t_seed, t_end - t_loop);
  return 0;
}
