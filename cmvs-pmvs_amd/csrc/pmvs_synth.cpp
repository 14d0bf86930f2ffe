// pmvs_synth.cpp -- deterministic synthetic workload generator.
//
// Not a reference interface: the reference ships no data (its .gitignore drops data/), so the
// benchmark and parity inputs are generated here.  A textured unit sphere at the origin
// (albedo = 3 octaves of 3-D value noise, lattice 8/16/32 per unit) seen by a ring of pinhole
// cameras (radius 4, heights alternating +-0.3, looking at the origin), rendered with analytic
// ray-sphere hits and ss x ss supersampling into RGB8; background = per-view low-contrast
// noise (NCC-poor).  Projections are CONTOUR 3x4 rows (K[R|t]).  Only +,-,*,/,sqrt and
// integer hashing inside the renderer, so the bytes are identical on every x86-64 host.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/pmvs_amd.h"

namespace {

static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline double lattice(int64_t x, int64_t y, int64_t z, uint64_t seed) {
  uint64_t h = mix64(seed ^ mix64((uint64_t)x * 0x8CB92BA72F3D8DD7ull ^ mix64((uint64_t)y * 0x9E3779B97F4A7C15ull ^ mix64((uint64_t)z))));
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

static inline double smooth(double t) { return t * t * (3.0 - 2.0 * t); }

static double value_noise(double x, double y, double z, uint64_t seed) {
  const double fx = std::floor(x), fy = std::floor(y), fz = std::floor(z);
  const int64_t ix = (int64_t)fx, iy = (int64_t)fy, iz = (int64_t)fz;
  const double tx = smooth(x - fx), ty = smooth(y - fy), tz = smooth(z - fz);
  double c[2][2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int e = 0; e < 2; ++e) c[a][b][e] = lattice(ix + a, iy + b, iz + e, seed);
  const double x00 = c[0][0][0] + (c[1][0][0] - c[0][0][0]) * tx, x10 = c[0][1][0] + (c[1][1][0] - c[0][1][0]) * tx;
  const double x01 = c[0][0][1] + (c[1][0][1] - c[0][0][1]) * tx, x11 = c[0][1][1] + (c[1][1][1] - c[0][1][1]) * tx;
  const double y0 = x00 + (x10 - x00) * ty, y1 = x01 + (x11 - x01) * ty;
  return y0 + (y1 - y0) * tz;
}

static void albedo(const double* p, uint64_t seed, double* rgb, double lowtex = 0.0) {
  const double freqs[3] = {8.0, 16.0, 32.0};
  const double amps[3] = {0.5, 0.3, 0.2};
  // low-texture regions (hard mode): contrast x 0.05 where a low-frequency field is below `lowtex`,
  // with a short linear transition
  double contrast = 1.0;
  if (lowtex > 0.0) {
    const double lf = value_noise(p[0] * 2.5 + 11.0, p[1] * 2.5 - 7.0, p[2] * 2.5 + 2.0, seed ^ 0x10E7E7ull);
    const double c = std::min(1.0, std::max(0.0, (lf - lowtex) / 0.04 + 0.5));
    contrast = 0.05 + 0.95 * c;
  }
  for (int c = 0; c < 3; ++c) {
    double v = 0.0;
    for (int o = 0; o < 3; ++o)
      v += amps[o] * value_noise(p[0] * freqs[o] + 17.0 * c, p[1] * freqs[o] - 5.0 * c, p[2] * freqs[o] + 3.0 * c, seed + 101 * c + o);
    v = (v - 0.5) * 2.2 * contrast + 0.5;  // stretch towards full range
    rgb[c] = std::min(1.0, std::max(0.0, v));
  }
}

// Hard-mode helpers: a uniform in [0, 1) from a hash, approximately Gaussian noise (sum of four
// uniforms), the per-view gain/bias, the occluder's centre.
static inline double hash_unit(uint64_t h) { return (double)(mix64(h) >> 11) * (1.0 / 9007199254740992.0); }
static inline double hash_gauss(uint64_t h) {
  double u = 0.0;
  for (int k = 0; k < 4; ++k) u += hash_unit(h * 4 + (uint64_t)k);
  return (u - 2.0) * 1.7320508075688772;  // variance 4/12 -> 1
}
static void occluder_centre(const pmvs_synth_params& p, double* oc) {
  // on the ring's arc a third of the way round the cameras, at radius 2.2, slightly above the plane
  const double step = p.arc_step_deg > 0.0 ? p.arc_step_deg * M_PI / 180.0 : 2.0 * M_PI / (double)p.num_views;
  const double th = step * (double)(p.num_views - 1) / 3.0;
  oc[0] = 2.2 * std::cos(th);
  oc[1] = 2.2 * std::sin(th);
  oc[2] = 0.1;
}

struct Cam {
  double C[3], R[3][3], f, cx, cy;
};

static void make_camera(const pmvs_synth_params& p, int i, Cam& cam, float* P) {
  const double step = p.arc_step_deg > 0.0 ? p.arc_step_deg * M_PI / 180.0 : 2.0 * M_PI / (double)p.num_views;
  const double th = step * (double)i;
  const double zc = (i % 2 == 0) ? p.height_offset : -p.height_offset;
  cam.C[0] = p.ring_radius * std::cos(th);
  cam.C[1] = p.ring_radius * std::sin(th);
  cam.C[2] = zc;
  double fwd[3] = {-cam.C[0], -cam.C[1], -cam.C[2]};
  double n = std::sqrt(fwd[0] * fwd[0] + fwd[1] * fwd[1] + fwd[2] * fwd[2]);
  for (double& v : fwd) v /= n;
  const double up[3] = {0, 0, 1};
  double right[3] = {fwd[1] * up[2] - fwd[2] * up[1], fwd[2] * up[0] - fwd[0] * up[2], fwd[0] * up[1] - fwd[1] * up[0]};
  n = std::sqrt(right[0] * right[0] + right[1] * right[1] + right[2] * right[2]);
  for (double& v : right) v /= n;
  double down[3] = {fwd[1] * right[2] - fwd[2] * right[1], fwd[2] * right[0] - fwd[0] * right[2], fwd[0] * right[1] - fwd[1] * right[0]};
  for (int k = 0; k < 3; ++k) { cam.R[0][k] = right[k]; cam.R[1][k] = down[k]; cam.R[2][k] = fwd[k]; }
  cam.f = p.focal_scale * p.width;
  cam.cx = 0.5 * (p.width - 1);
  cam.cy = 0.5 * (p.height - 1);
  double t[3];
  for (int r = 0; r < 3; ++r) t[r] = -(cam.R[r][0] * cam.C[0] + cam.R[r][1] * cam.C[1] + cam.R[r][2] * cam.C[2]);
  const double K[3][3] = {{cam.f, 0, cam.cx}, {0, cam.f, cam.cy}, {0, 0, 1}};
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) P[4 * r + c] = (float)(K[r][0] * cam.R[0][c] + K[r][1] * cam.R[1][c] + K[r][2] * cam.R[2][c]);
    P[4 * r + 3] = (float)(K[r][0] * t[0] + K[r][1] * t[1] + K[r][2] * t[2]);
  }
}

static void render_view(const pmvs_synth_params& p, int i, const Cam& cam, uint8_t* rgb) {
  const int W = p.width, H = p.height, ss = std::max(1, std::min(4, p.supersample));
  const uint64_t bgseed = p.seed * 7919ull + (uint64_t)i * 104729ull + 17;
  const uint64_t vseed = mix64(p.seed ^ (0xB1A5ull + (uint64_t)i * 0x9E37ull));
  const double gain = 1.0 + p.gain_sigma * hash_gauss(vseed), bias = p.bias_sigma * hash_gauss(vseed ^ 0x5A5Aull);
  double oc[3] = {0, 0, 0};
  const double orad = p.occluder_radius;
  if (orad > 0.0) occluder_centre(p, oc);
  const double oC[3] = {cam.C[0] - oc[0], cam.C[1] - oc[1], cam.C[2] - oc[2]};
  for (int y = 0; y < H; ++y) {
    for (int x = 0; x < W; ++x) {
      double acc[3] = {0, 0, 0};
      int hits = 0;
      for (int sy = 0; sy < ss; ++sy) {
        for (int sx = 0; sx < ss; ++sx) {
          const double u = x + ((sx + 0.5) / ss - 0.5), v = y + ((sy + 0.5) / ss - 0.5);
          double dc[3] = {(u - cam.cx) / cam.f, (v - cam.cy) / cam.f, 1.0};
          double d[3];
          for (int k = 0; k < 3; ++k) d[k] = cam.R[0][k] * dc[0] + cam.R[1][k] * dc[1] + cam.R[2][k] * dc[2];
          const double dn = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
          for (double& q : d) q /= dn;
          const double b = cam.C[0] * d[0] + cam.C[1] * d[1] + cam.C[2] * d[2];
          const double c = cam.C[0] * cam.C[0] + cam.C[1] * cam.C[1] + cam.C[2] * cam.C[2] - 1.0;
          const double disc = b * b - c;
          double tt = disc > 0.0 ? -b - std::sqrt(disc) : -1.0;
          bool occ = false;
          if (orad > 0.0) {  // the occluding sphere, when nearer
            const double ob = oC[0] * d[0] + oC[1] * d[1] + oC[2] * d[2];
            const double odisc = ob * ob - (oC[0] * oC[0] + oC[1] * oC[1] + oC[2] * oC[2] - orad * orad);
            if (odisc > 0.0) {
              const double ot = -ob - std::sqrt(odisc);
              if (ot > 0.0 && (tt < 0.0 || ot < tt)) { tt = ot; occ = true; }
            }
          }
          if (tt > 0.0) {
            const double hp[3] = {cam.C[0] + tt * d[0], cam.C[1] + tt * d[1], cam.C[2] + tt * d[2]};
            double col[3];
            if (occ) {
              const double q[3] = {(hp[0] - oc[0]) / orad, (hp[1] - oc[1]) / orad, (hp[2] - oc[2]) / orad};
              albedo(q, p.seed ^ 0x0CC1ull, col);
            } else {
              albedo(hp, p.seed, col, p.lowtex);
            }
            for (int k = 0; k < 3; ++k) acc[k] += col[k];
            hits++;
          } else {
            const double g = 0.45 + 0.06 * value_noise(u * 0.05, v * 0.05, 0.5, bgseed);
            for (int k = 0; k < 3; ++k) acc[k] += g;
          }
        }
      }
      (void)hits;
      uint8_t* o = rgb + ((size_t)y * W + x) * 3;
      for (int k = 0; k < 3; ++k) {
        double lin = acc[k] / (ss * ss);
        if (p.noise_sigma > 0.0) lin += p.noise_sigma * hash_gauss(vseed ^ (((uint64_t)y * W + x) * 3 + k) * 0x2545F491ull);
        lin = lin * gain + bias;
        const double val = lin * 255.0;
        o[k] = (uint8_t)std::min(255.0, std::max(0.0, std::floor(val + 0.5)));
      }
    }
  }
}

}  // namespace

extern "C" {

pmvs_status pmvs_synth_ring(const pmvs_synth_params* p, uint8_t* rgb, float* proj, int32_t nthreads) {
  if (!p || !proj) return PMVS_EINVAL;
  if (p->num_views < 2 || p->width < 16 || p->height < 16) return PMVS_EINVAL;
  std::vector<Cam> cams(p->num_views);
  for (int i = 0; i < p->num_views; ++i) make_camera(*p, i, cams[i], proj + 12 * i);
  if (!rgb) return PMVS_OK;
  const size_t per = (size_t)p->width * p->height * 3;
  const int first = p->render_count > 0 ? p->render_first : 0;
  const int count = p->render_count > 0 ? p->render_count : p->num_views;
  if (first < 0 || first >= p->num_views || count > p->num_views) return PMVS_EINVAL;
  int nt = std::max(1, std::min((int)nthreads, count));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t]() {
      for (int i = t; i < count; i += nt) {
        const int v = (first + i) % p->num_views;  // a cluster's views may wrap round the ring
        render_view(*p, v, cams[v], rgb + per * i);
      }
    });
  for (auto& t : th) t.join();
  return PMVS_OK;
}

// Seed-path candidates (CSeed::initialMatchSub, seed.cpp:387-414 shape): a point on the visible
// sphere, reference image = the most frontal camera, second image = the next most frontal one,
// depth perturbed along the reference ray by N(0, depth_sigma_px pixel footprints), normal =
// true surface normal tilted by a uniform 0..max_tilt_deg angle.  Deterministic (splitmix64).
pmvs_status pmvs_synth_candidates(const pmvs_synth_params* p, const float* proj, int32_t n, uint64_t seed,
                                  float depth_sigma_px, float max_tilt_deg, pmvs_candidate* out) {
  if (!p || !proj || !out || n < 0) return PMVS_EINVAL;
  std::vector<Cam> cams(p->num_views);
  std::vector<float> P(12 * p->num_views);
  for (int i = 0; i < p->num_views; ++i) make_camera(*p, i, cams[i], P.data() + 12 * i);
  uint64_t state = seed;
  auto next = [&]() {
    state += 0x9E3779B97F4A7C15ull;
    return (double)(mix64(state) >> 11) * (1.0 / 9007199254740992.0);
  };
  const int ntarget = p->num_targets > 0 ? std::min(p->num_targets, p->num_views) : p->num_views;
  for (int i = 0; i < n; ++i) {
    for (int attempt = 0; attempt < 1000; ++attempt) {
      // uniform direction
      const double z = 2.0 * next() - 1.0, phi = 2.0 * M_PI * next();
      const double r = std::sqrt(std::max(0.0, 1.0 - z * z));
      const double X[3] = {r * std::cos(phi), r * std::sin(phi), z};
      // rank cameras by frontality (normal . view direction)
      int best = -1, second = -1;
      double bv = -2, sv = -2;
      for (int c = 0; c < p->num_views; ++c) {
        double v[3] = {cams[c].C[0] - X[0], cams[c].C[1] - X[1], cams[c].C[2] - X[2]};
        const double vn = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        const double cosv = (X[0] * v[0] + X[1] * v[1] + X[2] * v[2]) / vn;
        if (c < ntarget && cosv > bv) {
          if (best >= 0 && bv > sv) { sv = bv; second = best; }
          bv = cosv;
          best = c;
        } else if (cosv > sv) {
          sv = cosv;
          second = c;
        }
      }
      if (best < 0 || second < 0 || bv < 0.6 || sv < 0.5) continue;
      const Cam& cr = cams[best];
      double ray[3] = {X[0] - cr.C[0], X[1] - cr.C[1], X[2] - cr.C[2]};
      const double dist = std::sqrt(ray[0] * ray[0] + ray[1] * ray[1] + ray[2] * ray[2]);
      for (double& q : ray) q /= dist;
      // Box-Muller
      const double u1 = std::max(1e-12, next()), u2 = next();
      const double g = std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
      const double foot = dist / cr.f;  // world size of one level-0 pixel at the point
      const double dd = g * depth_sigma_px * foot * (double)(1 << std::max(0, p->level));
      double Y[3] = {X[0] + dd * ray[0], X[1] + dd * ray[1], X[2] + dd * ray[2]};
      // tilt the normal
      double nrm[3] = {X[0], X[1], X[2]};
      double a[3] = {std::fabs(nrm[0]) < 0.9 ? 1.0 : 0.0, std::fabs(nrm[0]) < 0.9 ? 0.0 : 1.0, 0.0};
      double t1[3] = {nrm[1] * a[2] - nrm[2] * a[1], nrm[2] * a[0] - nrm[0] * a[2], nrm[0] * a[1] - nrm[1] * a[0]};
      double tn = std::sqrt(t1[0] * t1[0] + t1[1] * t1[1] + t1[2] * t1[2]);
      for (double& q : t1) q /= tn;
      double t2[3] = {nrm[1] * t1[2] - nrm[2] * t1[1], nrm[2] * t1[0] - nrm[0] * t1[2], nrm[0] * t1[1] - nrm[1] * t1[0]};
      const double tilt = max_tilt_deg * M_PI / 180.0 * next(), az = 2.0 * M_PI * next();
      double nn[3];
      for (int k = 0; k < 3; ++k)
        nn[k] = std::cos(tilt) * nrm[k] + std::sin(tilt) * (std::cos(az) * t1[k] + std::sin(az) * t2[k]);
      pmvs_candidate& c = out[i];
      std::memset(&c, 0, sizeof(c));
      for (int k = 0; k < 3; ++k) { c.coord[k] = (float)Y[k]; c.normal[k] = (float)nn[k]; }
      c.coord[3] = 1.0f;
      c.normal[3] = 0.0f;
      c.dscale = 0.0f;
      c.num_images = 2;
      c.images[0] = best;
      c.images[1] = second;
      break;
    }
  }
  return PMVS_OK;
}

}  // extern "C"
