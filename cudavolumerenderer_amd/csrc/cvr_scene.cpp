// cvr_scene.cpp - scene ingestion (the reference's SceneBuilder family) and
// the synthetic stand-ins for its missing data blobs.
//
//   Raw   RawSceneBuilder.h:35-160  (32^3 uchar, normalise by max, transfer
//         function albedo, scale 40, max_density 1, unit AABB)
//   Vdb   VDBSceneBuilder.h:40-80 + vdb_adapter/VDBAdapter.cpp (cvr_vdb.cpp)
//   Mhd   scripts/convert-mhd/mhd_to_vdb.py semantics (cvr_mhd.cpp)
//   synthetic proxies: SURVEY.md §8(d) (bucky / manix / hetvol)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "cvr.h"
#include "cvr_scene.h"

namespace cvr {

// -------------------------------------------------------------- Raw -------
// RawSceneBuilder::getAlbedoFromDensity (RawSceneBuilder.h:95-140)
// The table is two colour ramps, green->red over 20 entries then red->blue
// over 80; entry i of a ramp is a + i*(b - a)/100 (fp32, that operation
// order), alpha 1.  A voxel takes entry ceil(density * 99).
static void tf_ramp(std::vector<float>& tf, const float (&a)[3], const float (&b)[3], int entries) {
  for (int i = 0; i < entries; ++i) {
    for (int c = 0; c < 3; ++c) tf.push_back(a[c] + ((float)i * (b[c] - a[c]) / 100.F));
    tf.push_back(1.F);
  }
}

static std::vector<float> raw_transfer_albedo(const std::vector<float>& density) {
  static const float green[3] = {0.02f, 0.2f, 0.02f}, red[3] = {1.F, 0.02f, 0.02f}, blue[3] = {0.F, 0.02f, 1.F};
  std::vector<float> tf;
  tf_ramp(tf, green, red, 20);
  tf_ramp(tf, red, blue, 80);
  const float last = (float)(tf.size() / 4 - 1);
  std::vector<float> albedo(density.size() * 4);
  for (size_t i = 0; i < density.size(); ++i)
    memcpy(&albedo[4 * i], &tf[4 * (size_t)std::ceil(density[i] * last)], 4 * sizeof(float));
  return albedo;
}

int scene_from_raw_bytes(const std::vector<uint8_t>& raw, const std::string& name, cvr_scene* s) {
  const uint32_t n = 32;  // RawSceneBuilder.h:36: volume_size_ = 32^3, uchar
  if (raw.size() != (size_t)n * n * n) return CVR_ERR_IO;
  s->name = name;
  s->dims[0] = s->dims[1] = s->dims[2] = n;
  s->raw = raw;
  s->density.resize(raw.size());
  float mx = 0;
  for (size_t i = 0; i < raw.size(); ++i) {
    s->density[i] = raw[i];
    mx = std::fmax(s->density[i], mx);
  }
  for (auto& v : s->density) v /= mx;
  s->albedo = raw_transfer_albedo(s->density);
  s->max_density = 1;
  s->scale = 40;
  for (int k = 0; k < 3; ++k) {
    s->box_min[k] = -0.5f;
    s->box_max[k] = 0.5f;
  }
  return CVR_OK;
}

// VDBSceneBuilder.h:54-77: max_density = max voxel, scale 100, unit AABB,
// albedo (r,g,b,1).
void finish_vdb_like(cvr_scene* s) {
  float mx = 0.f;
  for (float v : s->density) mx = std::max(mx, v);
  s->max_density = mx;
  s->scale = 100.F;
  for (int k = 0; k < 3; ++k) {
    s->box_min[k] = -0.5f;
    s->box_max[k] = 0.5f;
  }
}

// ------------------------------------------------------ synthetic fields --
static inline uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}
static inline double lattice(int x, int y, int z, uint32_t seed) {
  uint32_t h = mix32((uint32_t)x * 0x8da6b343u ^ mix32((uint32_t)y * 0xd8163841u ^ mix32((uint32_t)z * 0xcb1ab31fu ^ seed)));
  return (h >> 8) * (1.0 / 16777216.0);
}
static inline double fade(double t) { return t * t * (3.0 - 2.0 * t); }
// trilinear value noise in [0,1]
static double vnoise(double x, double y, double z, uint32_t seed) {
  const double fx = std::floor(x), fy = std::floor(y), fz = std::floor(z);
  const int ix = (int)fx, iy = (int)fy, iz = (int)fz;
  const double tx = fade(x - fx), ty = fade(y - fy), tz = fade(z - fz);
  double c[2][2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int d = 0; d < 2; ++d) c[a][b][d] = lattice(ix + d, iy + b, iz + a, seed);
  auto L = [](double p, double q, double t) { return p + (q - p) * t; };
  const double z0 = L(L(c[0][0][0], c[0][0][1], tx), L(c[0][1][0], c[0][1][1], tx), ty);
  const double z1 = L(L(c[1][0][0], c[1][0][1], tx), L(c[1][1][0], c[1][1][1], tx), ty);
  return L(z0, z1, tz);
}
static double fbm(double x, double y, double z, int octaves, uint32_t seed) {
  double sum = 0, amp = 0.5, norm = 0, f = 1;
  for (int o = 0; o < octaves; ++o) {
    sum += amp * vnoise(x * f, y * f, z * f, seed + 977u * (uint32_t)o);
    norm += amp;
    amp *= 0.5;
    f *= 2.0;
  }
  return sum / norm;
}
// mhd_to_vdb.py:7-10 / Utilities.h:24-29
static inline double smooth_step(double e0, double e1, double x) {
  double t = (x - e0) / (e1 - e0);
  t = t < 0 ? 0 : (t > 1 ? 1 : t);
  return t * t * (3.0 - 2.0 * t);
}

// C60 (truncated icosahedron) vertices: cyclic permutations of
// (0, ±1, ±3φ), (±1, ±(2+φ), ±2φ), (±φ, ±2, ±(2φ+1)).
static std::vector<double> c60_vertices() {
  const double p = (1.0 + std::sqrt(5.0)) / 2.0;
  const double base[3][3] = {{0, 1, 3 * p}, {1, 2 + p, 2 * p}, {p, 2, 2 * p + 1}};
  std::vector<double> v;
  for (int b = 0; b < 3; ++b) {
    for (int sx = -1; sx <= 1; sx += 2)
      for (int sy = -1; sy <= 1; sy += 2)
        for (int sz = -1; sz <= 1; sz += 2) {
          double q[3] = {base[b][0] * sx, base[b][1] * sy, base[b][2] * sz};
          if ((base[b][0] == 0 && sx < 0)) continue;  // +-0 duplicates
          for (int r = 0; r < 3; ++r) {
            v.push_back(q[r % 3]);
            v.push_back(q[(r + 1) % 3]);
            v.push_back(q[(r + 2) % 3]);
          }
        }
  }
  return v;  // 60 * 3
}

// Bucky proxy: 60 Gaussian atoms (sigma 1.2 voxels) on C60
// vertices scaled to radius 11 voxels about the centre, value
// round(255*min(1, sum)).
std::vector<uint8_t> synth_bucky_bytes() {
  const int n = 32;
  std::vector<double> v = c60_vertices();
  const double p = (1.0 + std::sqrt(5.0)) / 2.0;
  const double R = std::sqrt(9.0 * p + 10.0);
  const double s = 11.0 / R, c = 15.5, sig2 = 2.0 * 1.2 * 1.2;
  std::vector<uint8_t> out((size_t)n * n * n);
  for (int z = 0; z < n; ++z)
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) {
        double sum = 0;
        for (size_t a = 0; a + 2 < v.size(); a += 3) {
          const double dx = x - (c + s * v[a]), dy = y - (c + s * v[a + 1]), dz = z - (c + s * v[a + 2]);
          sum += std::exp(-(dx * dx + dy * dy + dz * dz) / sig2);
        }
        out[((size_t)z * n + y) * n + x] = (uint8_t)std::lround(255.0 * std::min(1.0, sum));
      }
  return out;
}

// Manix proxy: CT-like field = soft ellipsoidal skull
// shell (8 voxels thick) + inner ellipsoid at 0.35 + 4-octave value noise
// (amplitude 0.15), normalised to [0,1]; density = smoothstep(0.2, 0.6, f)
// (mhd_to_vdb.py:51-53), albedo = (d, 0, 0) (mhd_to_vdb.py:62-64).
static void synth_manix(cvr_scene* s, uint32_t seed, const uint32_t* dims) {
  const uint32_t nx = dims ? dims[0] : 256, ny = dims ? dims[1] : 230, nz = dims ? dims[2] : 256;
  s->name = "manix";
  s->dims[0] = nx;
  s->dims[1] = ny;
  s->dims[2] = nz;
  const size_t n = (size_t)nx * ny * nz;
  std::vector<double> f(n);
  const double cx = 0.5 * (nx - 1), cy = 0.5 * (ny - 1), cz = 0.5 * (nz - 1);
  const double rx = 0.43 * nx, ry = 0.45 * ny, rz = 0.45 * nz;
  const double rmean = (rx + ry + rz) / 3.0, shell_half = 4.0 / rmean;
  const double nscale = 1.0 / 16.0;  // 16-voxel noise cells
  double fmin = 1e300, fmax = -1e300;
  for (uint32_t z = 0; z < nz; ++z)
    for (uint32_t y = 0; y < ny; ++y)
      for (uint32_t x = 0; x < nx; ++x) {
        const double qx = (x - cx) / rx, qy = (y - cy) / ry, qz = (z - cz) / rz;
        const double r = std::sqrt(qx * qx + qy * qy + qz * qz);
        const double shell = std::max(0.0, 1.0 - std::fabs(r - 0.92) / shell_half);
        const double inner = 0.35 * (1.0 - smooth_step(0.70, 0.80, r));
        const double noise = 0.15 * fbm(x * nscale, y * nscale, z * nscale, 4, seed);
        const double v = shell + inner + noise;
        f[((size_t)z * ny + y) * nx + x] = v;
        fmin = std::min(fmin, v);
        fmax = std::max(fmax, v);
      }
  s->density.resize(n);
  s->albedo.assign(n * 4, 0.0f);
  for (size_t i = 0; i < n; ++i) {
    const float d = (float)smooth_step(0.2, 0.6, (f[i] - fmin) / (fmax - fmin));
    s->density[i] = d;
    s->albedo[4 * i + 0] = d;
    s->albedo[4 * i + 3] = 1.0f;
  }
  finish_vdb_like(s);
}

// hetvol proxy: Mitsuba smoke grid 128x128x50, seeded fBm
// plume, ~40 % empty voxels, albedo (0.9, 0.9, 0.9).
static void synth_hetvol(cvr_scene* s, uint32_t seed, const uint32_t* dims) {
  const uint32_t nx = dims ? dims[0] : 128, ny = dims ? dims[1] : 128, nz = dims ? dims[2] : 50;
  s->name = "hetvol";
  s->dims[0] = nx;
  s->dims[1] = ny;
  s->dims[2] = nz;
  const size_t n = (size_t)nx * ny * nz;
  s->density.resize(n);
  s->albedo.assign(n * 4, 0.9f);
  float mx = 0.f;
  for (uint32_t z = 0; z < nz; ++z)
    for (uint32_t y = 0; y < ny; ++y)
      for (uint32_t x = 0; x < nx; ++x) {
        const double u = (x + 0.5) / nx, v = (y + 0.5) / ny, w = (z + 0.5) / nz;
        // plume: rising column widening with height (y), turbulent fBm
        const double rad = std::sqrt((u - 0.5) * (u - 0.5) + (w - 0.5) * (w - 0.5) * 0.5);
        const double width = 0.18 + 0.25 * v;
        const double envelope = 1.0 - smooth_step(0.6 * width, width, rad);
        const double turb = fbm(u * 6.0, v * 6.0, w * 6.0, 5, seed);
        const double d = std::max(0.0, envelope * (turb * 1.6 - 0.35));
        const float df = (float)d;
        s->density[((size_t)z * ny + y) * nx + x] = df;
        mx = std::max(mx, df);
      }
  if (mx > 0)
    for (auto& d : s->density) d /= mx;
  for (size_t i = 0; i < n; ++i) s->albedo[4 * i + 3] = 1.0f;
  finish_vdb_like(s);
}

// Cloud proxy: a sparse seeded fBm cumulus in a
// 2048x1024x2048 index box, albedo (1,1,1), VDB-like (scale 100, unit AABB,
// max_density = max voxel).  Stored sparse only: 8^3 leaves, the ones
// holding a non-zero voxel.  In normalised coordinates p = (i + 0.5) / n the
// density is clamp(2.5 (c(p) + 0.6 (fbm(6 p) - 0.5) - 0.1), 0, 1), where
// c(p) = max_k (1 - |p - c_k| / r_k) over 28 seeded blobs; the fBm (4
// octaves) is evaluated at the leaf corners and trilinearly interpolated
// inside each leaf (its finest wavelength is ~5 leaves).
struct CloudBlob {
  double c[3], r;
};

static void synth_cloud(cvr_scene* s, uint32_t seed, const uint32_t* dims) {
  const uint32_t nx = dims ? dims[0] : 2048, ny = dims ? dims[1] : 1024, nz = dims ? dims[2] : 2048;
  s->name = "cloud";
  s->dims[0] = nx;
  s->dims[1] = ny;
  s->dims[2] = nz;
  const uint32_t lnx = (nx + 7) / 8, lny = (ny + 7) / 8, lnz = (nz + 7) / 8;
  s->leaf_dims[0] = lnx;
  s->leaf_dims[1] = lny;
  s->leaf_dims[2] = lnz;
  std::vector<CloudBlob> blobs(28);
  uint32_t h = mix32(seed ^ 0x9e3779b9u);
  auto uni = [&h](double a, double b) {
    h = mix32(h + 0x6d2b79f5u);
    return a + (b - a) * ((h >> 8) * (1.0 / 16777216.0));
  };
  for (auto& b : blobs) {
    b.c[0] = uni(0.22, 0.78);
    b.c[1] = uni(0.38, 0.62);
    b.c[2] = uni(0.22, 0.78);
    b.r = uni(0.07, 0.16);
  }
  const double leaf_rad = 0.5 * std::sqrt(std::pow(8.0 / nx, 2) + std::pow(8.0 / ny, 2) + std::pow(8.0 / nz, 2));
  const unsigned nthreads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  struct Part {
    std::vector<uint32_t> leaf;
    std::vector<float> vals;
    float mx = 0.0f;
  };
  std::vector<Part> parts(nthreads);
  auto work = [&](unsigned t) {
    Part& P = parts[t];
    const uint32_t z0 = (uint32_t)((uint64_t)lnz * t / nthreads), z1 = (uint32_t)((uint64_t)lnz * (t + 1) / nthreads);
    std::vector<const CloudBlob*> near;
    float v[512];
    for (uint32_t lz = z0; lz < z1; ++lz)
      for (uint32_t ly = 0; ly < lny; ++ly)
        for (uint32_t lx = 0; lx < lnx; ++lx) {
          const double pc[3] = {(lx * 8.0 + 4.0) / nx, (ly * 8.0 + 4.0) / ny, (lz * 8.0 + 4.0) / nz};
          near.clear();
          for (const auto& b : blobs) {
            const double dx = pc[0] - b.c[0], dy = pc[1] - b.c[1], dz = pc[2] - b.c[2];
            if (std::sqrt(dx * dx + dy * dy + dz * dz) < 1.2 * b.r + leaf_rad) near.push_back(&b);
          }
          if (near.empty()) continue;
          double cn[2][2][2];  // fBm at the leaf corners
          for (int a = 0; a < 2; ++a)
            for (int bb = 0; bb < 2; ++bb)
              for (int d = 0; d < 2; ++d)
                cn[a][bb][d] = fbm(6.0 * (lx * 8.0 + 8 * d + 0.5) / nx, 6.0 * (ly * 8.0 + 8 * bb + 0.5) / ny,
                                   6.0 * (lz * 8.0 + 8 * a + 0.5) / nz, 4, seed);
          bool any = false;
          for (uint32_t k = 0; k < 512; ++k) {
            const uint32_t x = lx * 8 + (k & 7), y = ly * 8 + ((k >> 3) & 7), z = lz * 8 + (k >> 6);
            float dv = 0.0f;
            if (x < nx && y < ny && z < nz) {
              const double p[3] = {(x + 0.5) / nx, (y + 0.5) / ny, (z + 0.5) / nz};
              double cov = -1e30;
              for (const CloudBlob* b : near) {
                const double dx = p[0] - b->c[0], dy = p[1] - b->c[1], dz = p[2] - b->c[2];
                cov = std::max(cov, 1.0 - std::sqrt(dx * dx + dy * dy + dz * dz) / b->r);
              }
              const double tx = (k & 7) / 8.0, ty = ((k >> 3) & 7) / 8.0, tz = (k >> 6) / 8.0;
              auto L = [](double a, double b, double t) { return a + (b - a) * t; };
              const double n = L(L(L(cn[0][0][0], cn[0][0][1], tx), L(cn[0][1][0], cn[0][1][1], tx), ty),
                                 L(L(cn[1][0][0], cn[1][0][1], tx), L(cn[1][1][0], cn[1][1][1], tx), ty), tz);
              const double d = 2.5 * (cov + 0.6 * (n - 0.5) - 0.1);
              dv = (float)(d < 0 ? 0 : (d > 1 ? 1 : d));
            }
            v[k] = dv;
            any |= dv != 0.0f;
          }
          if (!any) continue;
          P.leaf.push_back((lz * lny + ly) * lnx + lx);
          P.vals.insert(P.vals.end(), v, v + 512);
          for (float x : v) P.mx = std::max(P.mx, x);
        }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nthreads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
  s->leaf_table.assign((size_t)lnx * lny * lnz, CVR_NO_LEAF);
  size_t total = 0;
  for (const auto& P : parts) total += P.leaf.size();
  s->leaf_density.clear();
  s->leaf_density.reserve(total * 512);
  float mx = 0.0f;
  uint32_t slot = 0;
  for (auto& P : parts) {  // threads own ascending z ranges: slots follow the leaf index
    for (uint32_t li : P.leaf) s->leaf_table[li] = slot++;
    s->leaf_density.insert(s->leaf_density.end(), P.vals.begin(), P.vals.end());
    mx = std::max(mx, P.mx);
    std::vector<float>().swap(P.vals);
  }
  s->leaf_albedo.clear();
  for (int k = 0; k < 4; ++k) s->albedo_bg[k] = 1.0f;
  s->sparse_only = true;
  s->have_leaves = true;
  s->max_density = mx;
  s->scale = 100.0f;
  for (int k = 0; k < 3; ++k) {
    s->box_min[k] = -0.5f;
    s->box_max[k] = 0.5f;
  }
}

// Dense grid -> 8^3 leaves: a leaf is stored when one of its voxels has a
// density other than 0 or an albedo other than voxel (0,0,0)'s (the
// background); the rest read as (0, background), exactly their values.
static void build_leaves(cvr_scene* s) {
  const uint32_t nx = s->dims[0], ny = s->dims[1], nz = s->dims[2];
  const uint32_t lnx = (nx + 7) / 8, lny = (ny + 7) / 8, lnz = (nz + 7) / 8;
  s->leaf_dims[0] = lnx;
  s->leaf_dims[1] = lny;
  s->leaf_dims[2] = lnz;
  const float* bg = s->albedo.data();
  memcpy(s->albedo_bg, bg, sizeof(s->albedo_bg));
  s->leaf_table.assign((size_t)lnx * lny * lnz, CVR_NO_LEAF);
  s->leaf_density.clear();
  s->leaf_albedo.clear();
  bool albedo_varies = false;
  uint32_t slot = 0;
  for (uint32_t lz = 0; lz < lnz; ++lz)
    for (uint32_t ly = 0; ly < lny; ++ly)
      for (uint32_t lx = 0; lx < lnx; ++lx) {
        bool any = false;
        for (uint32_t k = 0; k < 512 && !any; ++k) {
          const uint32_t x = lx * 8 + (k & 7), y = ly * 8 + ((k >> 3) & 7), z = lz * 8 + (k >> 6);
          if (x >= nx || y >= ny || z >= nz) continue;
          const size_t i = ((size_t)z * ny + y) * nx + x;
          any = s->density[i] != 0.0f || memcmp(&s->albedo[4 * i], bg, 16) != 0;
        }
        if (!any) continue;
        s->leaf_table[((size_t)lz * lny + ly) * lnx + lx] = slot++;
        for (uint32_t k = 0; k < 512; ++k) {
          const uint32_t x = lx * 8 + (k & 7), y = ly * 8 + ((k >> 3) & 7), z = lz * 8 + (k >> 6);
          const bool in = x < nx && y < ny && z < nz;
          const size_t i = in ? ((size_t)z * ny + y) * nx + x : 0;
          s->leaf_density.push_back(in ? s->density[i] : 0.0f);
          for (int c = 0; c < 4; ++c) s->leaf_albedo.push_back(in ? s->albedo[4 * i + c] : bg[c]);
          albedo_varies |= in && memcmp(&s->albedo[4 * i], bg, 16) != 0;
        }
      }
  if (!albedo_varies) std::vector<float>().swap(s->leaf_albedo);
  s->have_leaves = true;
}

}  // namespace cvr

using namespace cvr;

extern "C" {

int cvr_scene_synthetic(const char* name, uint32_t seed, const uint32_t* dims, cvr_scene** out) {
  if (!name || !out) return CVR_ERR_INVALID;
  *out = nullptr;
  cvr_scene* s = new cvr_scene();
  const std::string nm(name);
  int r = CVR_OK;
  if (nm == "bucky") {
    r = scene_from_raw_bytes(synth_bucky_bytes(), "bucky", s);
  } else if (nm == "manix") {
    synth_manix(s, seed ? seed : 1234u, dims);
  } else if (nm == "hetvol") {
    synth_hetvol(s, seed ? seed : 800u, dims);
  } else if (nm == "cloud") {
    synth_cloud(s, seed ? seed : 5u, dims);
  } else {
    r = CVR_ERR_INVALID;
  }
  if (r != CVR_OK) {
    delete s;
    set_last_error("unknown synthetic scene " + nm);
    return r;
  }
  *out = s;
  return CVR_OK;
}

int cvr_scene_load(const char* path, int scene_type, cvr_scene** out) {
  return cvr_scene_load_ex(path, scene_type, nullptr, out);
}

int cvr_scene_load_ex(const char* path, int scene_type, const cvr_load_options* opts, cvr_scene** out) {
  if (!path || !out) return CVR_ERR_INVALID;
  if (opts && (opts->flags & ~(uint32_t)CVR_LOAD_DEFAULT_ALBEDO)) {
    set_last_error("unknown load option flags");
    return CVR_ERR_INVALID;
  }
  const float* default_albedo = (opts && (opts->flags & CVR_LOAD_DEFAULT_ALBEDO)) ? opts->default_albedo : nullptr;
  *out = nullptr;
  std::string p(path);
  int type = scene_type;
  if (type == CVR_SCENE_AUTO) {  // ConfigParser.cpp:79-97 (+ .mhd)
    std::string ext;
    const size_t dot = p.find_last_of('.');
    if (dot != std::string::npos) ext = p.substr(dot + 1);
    for (auto& ch : ext) ch = (char)tolower((unsigned char)ch);
    if (ext == "xml") type = CVR_SCENE_MITSUBA_XML;
    else if (ext == "vdb") type = CVR_SCENE_VDB;
    else if (ext == "mhd") type = CVR_SCENE_MHD;
    else type = CVR_SCENE_RAW;
  }
  cvr_scene* s = new cvr_scene();
  int r = CVR_OK;
  if (type == CVR_SCENE_RAW) {
    FILE* fp = fopen(path, "rb");
    if (!fp) {
      r = CVR_ERR_IO;
    } else {
      std::vector<uint8_t> raw(32 * 32 * 32);
      const size_t got = fread(raw.data(), 1, raw.size(), fp);
      fclose(fp);
      r = (got == raw.size()) ? scene_from_raw_bytes(raw, p, s) : CVR_ERR_IO;  // Q16: report short files
    }
  } else if (type == CVR_SCENE_VDB || type == CVR_SCENE_VDB_SPARSE) {
    r = load_vdb_scene(p, s, type == CVR_SCENE_VDB_SPARSE, default_albedo);
  } else if (type == CVR_SCENE_MHD) {
    r = load_mhd_scene(p, s);
  } else if (type == CVR_SCENE_MITSUBA_XML) {
    r = load_xml_scene(p, s);
  } else {
    r = CVR_ERR_UNSUPPORTED;
  }
  if (r != CVR_OK) {
    delete s;
    if ((type == CVR_SCENE_VDB || type == CVR_SCENE_VDB_SPARSE) && r == CVR_ERR_IO)
      set_last_error(std::string("VDB: ") + vdb_last_error());
    else if (type != CVR_SCENE_MITSUBA_XML)
      set_last_error("cannot load scene " + p + (r == CVR_ERR_UNSUPPORTED ? " (unsupported)" : ""));
    return r;
  }
  *out = s;
  return CVR_OK;
}

int cvr_scene_medium(const cvr_scene* s, cvr_medium_desc* m) {
  if (!s || !m) return CVR_ERR_INVALID;
  memset(m, 0, sizeof(*m));
  if (s->sparse_only) {
    set_last_error("scene " + s->name + " is stored sparse only: use cvr_scene_sparse_medium");
    return CVR_ERR_UNSUPPORTED;
  }
  for (int k = 0; k < 3; ++k) {
    m->res[k] = s->dims[k];
    m->box_min[k] = s->box_min[k];
    m->box_max[k] = s->box_max[k];
  }
  m->density = s->density.data();
  m->albedo = s->albedo.data();
  m->scale = s->scale;
  m->max_density = s->max_density;
  m->g = 0.0f;                // HG g is never uploaded (Q7)
  m->roughness[0] = 0.1f;     // GGX defaults (Bsdf.h:17-30)
  m->roughness[1] = 0.1f;
  m->eta = 1.05f / 1.01f;
  return CVR_OK;
}

int cvr_scene_sparse_medium(cvr_scene* s, cvr_sparse_medium_desc* m) {
  if (!s || !m) return CVR_ERR_INVALID;
  memset(m, 0, sizeof(*m));
  if (!s->have_leaves) {
    if (s->density.empty() || s->albedo.size() != 4 * s->density.size()) return CVR_ERR_INVALID;
    build_leaves(s);
  }
  for (int k = 0; k < 3; ++k) {
    m->res[k] = s->dims[k];
    m->leaf_dims[k] = s->leaf_dims[k];
    m->box_min[k] = s->box_min[k];
    m->box_max[k] = s->box_max[k];
  }
  m->leaf_table = s->leaf_table.data();
  m->n_leaves = (uint32_t)(s->leaf_density.size() / 512);
  m->leaf_density = s->leaf_density.data();
  m->leaf_albedo = s->leaf_albedo.empty() ? nullptr : s->leaf_albedo.data();
  memcpy(m->albedo_background, s->albedo_bg, sizeof(m->albedo_background));
  m->scale = s->scale;
  m->max_density = s->max_density;
  m->g = 0.0f;
  m->roughness[0] = 0.1f;
  m->roughness[1] = 0.1f;
  m->eta = 1.05f / 1.01f;
  return CVR_OK;
}

int cvr_scene_is_sparse(const cvr_scene* s) { return s && s->sparse_only ? 1 : 0; }

int cvr_scene_camera(const cvr_scene* s, uint32_t w, uint32_t h, float inv_view[12], float r2v[2]) {
  if (!s || !inv_view || !r2v || w == 0 || h == 0) return CVR_ERR_INVALID;
  cvr::camera_for_fov(s->fov_x, w, h, inv_view, r2v);
  return CVR_OK;
}

int cvr_scene_raw_bytes(const cvr_scene* s, const uint8_t** bytes, size_t* n) {
  if (!s || !bytes || !n) return CVR_ERR_INVALID;
  *bytes = s->raw.empty() ? nullptr : s->raw.data();
  *n = s->raw.size();
  return CVR_OK;
}

void cvr_scene_destroy(cvr_scene* s) { delete s; }

// stbi_write_hdr semantics (Image.cpp:58-62): RGB of an RGBA float buffer,
// Radiance RGBE, top row first.  Written as flat (non-RLE) scanlines.
int cvr_write_hdr(const char* path, const float* rgba, uint32_t w, uint32_t h) {
  if (!path || !rgba || !w || !h) return CVR_ERR_INVALID;
  FILE* fp = fopen(path, "wb");
  if (!fp) return CVR_ERR_IO;
  fprintf(fp, "#?RADIANCE\n# Written by cudavolumerenderer_amd\nFORMAT=32-bit_rle_rgbe\nEXPOSURE=1.0\n\n-Y %u +X %u\n",
          h, w);
  std::vector<unsigned char> line((size_t)w * 4);
  for (uint32_t y = 0; y < h; ++y) {
    for (uint32_t x = 0; x < w; ++x) {
      const float* px = rgba + ((size_t)y * w + x) * 4;
      unsigned char* e = &line[(size_t)x * 4];
      const float mx = std::max(px[0], std::max(px[1], px[2]));
      if (!(mx >= 1e-32f) || !std::isfinite(mx) || px[0] != px[0] || px[1] != px[1] || px[2] != px[2]) {
        // black for empty, negative and non-finite pixels (quirk Q22 NaNs)
        e[0] = e[1] = e[2] = e[3] = 0;
      } else {
        int ex;
        const float nrm = (float)std::frexp(mx, &ex) * 256.0f / mx;
        e[0] = (unsigned char)(px[0] * nrm);
        e[1] = (unsigned char)(px[1] * nrm);
        e[2] = (unsigned char)(px[2] * nrm);
        e[3] = (unsigned char)(ex + 128);
      }
    }
    fwrite(line.data(), 1, line.size(), fp);
  }
  fclose(fp);
  return CVR_OK;
}

}  // extern "C"
