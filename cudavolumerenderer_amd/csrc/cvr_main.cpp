// cvr_main.cpp - command-line front end with the reference's flags
// (ConfigParser.cpp:10-165, Main.cpp:46-146), driving libcvr through its C
// ABI only.
//
//   cvr [--scene-file|-s] FILE [--scene-type Auto|MitsubaXml|Vdb|Raw|Mhd]
//       [--kernel|-k naiveSK|regenerationSK|...] [--algorithm|-a cudaVolPath]
//       [--iterations|-i N] [--resolution|-r W [H]] [--number-of-tiles X [Y]]
//       [--trials N] [--output|-o NAME] [--interactive BOOL]
//       [--use-unified-memory BOOL]
//   extensions: --synthetic bucky|manix|hetvol|cloud, --device N, --seed S,
//   --devices N|d0,d1,... (one context per device, each on its own host
//   thread: tile k -> device k mod N for --number-of-tiles, else 8x8-block
//   shards of the one tile; every device stores its pixels straight into one
//   pinned host image), --pfm (also write the float image as <output>.pfm)
//
// Differences from the reference, on purpose: the timer is wall clock (the
// reference uses clock(), i.e. CPU time, Main.cpp:51-77); main does not wait
// for Enter; --interactive true has no GL viewer here (out of scope, SURVEY
// §2.1) and falls back to the headless path with a notice.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "cvr.h"

namespace {

struct Options {
  std::string scene_file, scene_type = "Auto", algorithm = "cudaVolPath", kernel = "regenerationSK";
  std::string output, synthetic, rng_binding = "path", world_to_aabb = "reference", mk_compaction = "fixed";
  std::string devices;  // --devices: a count or a comma list of device ids
  bool pfm = false;
  std::vector<float> default_albedo;
  bool interactive = true, unified = false;
  unsigned trials = 1, iterations = 20, device = 0, seed = 0;
  std::vector<unsigned> tiles{1, 1}, resolution{1024, 1024};
};

bool parse_bool(const std::string& v) { return v == "1" || v == "true" || v == "on" || v == "yes"; }

void usage() {
  printf(
      "Generic:\n"
      "  -h [ --help ]                      produce help message\n"
      "  -s [ --scene-file ] arg            scene file to parse\n"
      "  --scene-type arg (=Auto)           Auto, MitsubaXml, Vdb, Raw, Mhd (+ VdbSparse)\n"
      "  --interactive arg (=1)             (no GL viewer in this build: runs headless)\n"
      "  --trials arg (=1)                  number of times to run the algorithm\n"
      "  -a [ --algorithm ] arg (=cudaVolPath)\n"
      "  -k [ --kernel ] arg (=regenerationSK)\n"
      "  --number-of-tiles arg (=1 1)\n"
      "  --use-unified-memory arg (=0)      1: upload the grid as sparse 8^3 leaves\n"
      "Scene configuration override:\n"
      "  -i [ --iterations ] arg (=20)\n"
      "  -o [ --output ] arg\n"
      "  -r [ --resolution ] arg (=1024 1024)\n"
      "Extensions:\n"
      "  --synthetic bucky|manix|hetvol|cloud  use a built-in proxy scene\n"
      "  --device N, --seed S\n"
      "  --devices N|d0,d1,...              render on several devices at once (one context and host\n"
      "                                     thread each; ids may repeat): tile k -> device k mod N\n"
      "                                     with --number-of-tiles, else 8x8-block shards of the image;\n"
      "                                     one value is a count (pick one device with --device)\n"
      "  --pfm                              also write the float image as <output>.pfm\n"
      "  --rng-binding path|thread (=path)  regenerationSK: thread = the reference's Rng(seed + tid)\n"
      "                                     per persistent thread (non-deterministic, SURVEY Q2)\n"
      "  --default-albedo r g b             VDB files without an albedo grid load with this albedo\n"
      "                                     (the reference refuses them, SURVEY Q17)\n"
      "  --world-to-aabb reference|fixed (=reference)  Woodcock density coordinate: the reference's\n"
      "                                     p - min/extent, or (p - min)/extent (SURVEY Q4)\n"
      "  --mk-compaction fixed|reference (=fixed)  naiveMK: keep every live path, or the reference's\n"
      "                                     end - begin - 1 (drops one per bounce, SURVEY Q11)\n");
}

bool is_flag(const char* a) { return a[0] == '-' && !(a[1] >= '0' && a[1] <= '9'); }

int parse(int argc, char** argv, Options& o) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto need = [&](const char* name) -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "[ConfigParser] Error: the required argument for option '%s' is missing\n", name);
        exit(2);
      }
      return argv[++i];
    };
    auto multi = [&](std::vector<unsigned>& dst) {
      dst.clear();
      while (i + 1 < argc && !is_flag(argv[i + 1])) dst.push_back((unsigned)strtoul(argv[++i], nullptr, 10));
      if (dst.empty()) {
        fprintf(stderr, "[ConfigParser] Error: option '%s' needs a value\n", a.c_str());
        exit(2);
      }
    };
    if (a == "-h" || a == "--help") return 1;
    else if (a == "-s" || a == "--scene-file") o.scene_file = need("scene-file");
    else if (a == "--scene-type") o.scene_type = need("scene-type");
    else if (a == "--interactive") o.interactive = parse_bool(need("interactive"));
    else if (a == "--trials") o.trials = (unsigned)strtoul(need("trials").c_str(), nullptr, 10);
    else if (a == "-a" || a == "--algorithm") o.algorithm = need("algorithm");
    else if (a == "-k" || a == "--kernel") o.kernel = need("kernel");
    else if (a == "--number-of-tiles") multi(o.tiles);
    else if (a == "--use-unified-memory") o.unified = parse_bool(need("use-unified-memory"));
    else if (a == "-i" || a == "--iterations") o.iterations = (unsigned)strtoul(need("iterations").c_str(), nullptr, 10);
    else if (a == "-o" || a == "--output") o.output = need("output");
    else if (a == "-r" || a == "--resolution") multi(o.resolution);
    else if (a == "--synthetic") o.synthetic = need("synthetic");
    else if (a == "--device") o.device = (unsigned)strtoul(need("device").c_str(), nullptr, 10);
    else if (a == "--devices") o.devices = need("devices");
    else if (a == "--pfm") o.pfm = true;
    else if (a == "--rng-binding") o.rng_binding = need("rng-binding");
    else if (a == "--seed") o.seed = (unsigned)strtoul(need("seed").c_str(), nullptr, 10);
    else if (a == "--world-to-aabb") o.world_to_aabb = need("world-to-aabb");
    else if (a == "--mk-compaction") o.mk_compaction = need("mk-compaction");
    else if (a == "--default-albedo") {
      o.default_albedo.clear();
      while (i + 1 < argc && o.default_albedo.size() < 3 && !(argv[i + 1][0] == '-' && argv[i + 1][1] == '-'))
        o.default_albedo.push_back(strtof(argv[++i], nullptr));
      if (o.default_albedo.size() == 1) o.default_albedo.resize(3, o.default_albedo[0]);
      if (o.default_albedo.size() != 3) {
        fprintf(stderr, "[ConfigParser] Error: --default-albedo needs 1 or 3 values\n");
        return 2;
      }
    }
    else if (!is_flag(a.c_str()) && o.scene_file.empty()) o.scene_file = a;  // positional
    else {
      fprintf(stderr, "[ConfigParser] Error: unrecognised option '%s'\n", a.c_str());
      return 2;
    }
  }
  if (o.tiles.size() == 1) o.tiles.push_back(o.tiles[0]);
  if (o.resolution.size() == 1) o.resolution.push_back(o.resolution[0]);
  return 0;
}

// --devices: "N" (devices first..first+N-1; a single value is always a count: one
// device is chosen with --device) or "d0,d1,..." (two or more ids, which may repeat:
// several contexts on one device, each with its own stream and work queues).  An
// empty or non-numeric entry is an error (empty result).
bool parse_uint(const std::string& s, unsigned& v) {
  if (s.empty() || s.size() > 9) return false;
  for (char ch : s)
    if (ch < '0' || ch > '9') return false;
  v = (unsigned)strtoul(s.c_str(), nullptr, 10);
  return true;
}
std::vector<int> parse_devices(const std::string& v, unsigned first) {
  std::vector<int> d;
  if (v.empty()) return {(int)first};
  unsigned x = 0;
  if (v.find(',') == std::string::npos) {
    if (!parse_uint(v, x) || x == 0) return {};
    for (unsigned k = 0; k < x; ++k) d.push_back((int)(first + k));
    return d;
  }
  size_t p = 0;
  while (p <= v.size()) {
    const size_t q = std::min(v.find(',', p), v.size());
    if (!parse_uint(v.substr(p, q - p), x)) return {};
    d.push_back((int)x);
    p = q + 1;
  }
  return d;
}

// Portable float map (little-endian RGB, rows bottom to top): the image as floats,
// for comparisons the RGBE .hdr cannot hold.
int write_pfm(const std::string& path, const float* rgba, unsigned w, unsigned h) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return 1;
  fprintf(f, "PF\n%u %u\n-1.0\n", w, h);
  std::vector<float> row((size_t)w * 3);
  for (unsigned y = h; y-- > 0;) {
    for (unsigned x = 0; x < w; ++x)
      for (int c = 0; c < 3; ++c) row[(size_t)x * 3 + c] = rgba[((size_t)y * w + x) * 4 + c];
    fwrite(row.data(), sizeof(float), row.size(), f);
  }
  return fclose(f) != 0;
}

int scene_type_id(const std::string& t) {
  if (t == "Auto") return CVR_SCENE_AUTO;
  if (t == "MitsubaXml") return CVR_SCENE_MITSUBA_XML;
  if (t == "Vdb") return CVR_SCENE_VDB;
  if (t == "VdbSparse") return CVR_SCENE_VDB_SPARSE;
  if (t == "Raw") return CVR_SCENE_RAW;
  if (t == "Mhd") return CVR_SCENE_MHD;
  return -1;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  int pr = parse(argc, argv, o);
  if (pr == 1) {
    usage();
    return 0;
  }
  if (pr) return pr;
  if (o.algorithm != "cudaVolPath") {
    fprintf(stderr, "[ConfigParser] algorithm %s not present in the list of algorithms\n", o.algorithm.c_str());
    return 2;
  }
  const int kernel = cvr_kernel_from_name(o.kernel.c_str());
  if (kernel == CVR_KERNEL_UNKNOWN) {  // RendererFactory.h:75-76 throws
    fprintf(stderr, "[RendererFactory] Error: kernel %s unknown\n", o.kernel.c_str());
    return 2;
  }
  cvr_scene* scene = nullptr;
  int r;
  if (!o.synthetic.empty()) {
    r = cvr_scene_synthetic(o.synthetic.c_str(), o.seed, nullptr, &scene);
  } else {
    if (o.scene_file.empty()) {
      fprintf(stderr, "Error: no scene file provided\n");
      return 2;
    }
    const int st = scene_type_id(o.scene_type);
    if (st < 0) {
      fprintf(stderr, "Error: scene type not correct\n");
      return 2;
    }
    cvr_load_options lo{};
    if (!o.default_albedo.empty()) {
      lo.flags = CVR_LOAD_DEFAULT_ALBEDO;
      for (int k = 0; k < 3; ++k) lo.default_albedo[k] = o.default_albedo[k];
    }
    r = cvr_scene_load_ex(o.scene_file.c_str(), st, &lo, &scene);
  }
  if (r != CVR_OK) {
    fprintf(stderr, "Error: could not load scene (%d): %s\n", r, cvr_last_error(nullptr));
    return 1;
  }
  printf("[ConfigParser] kernel set to %s.\n[ConfigParser] iterations set to %u.\n", o.kernel.c_str(), o.iterations);
  if (o.interactive) printf("[ConfigParser] interactive viewer not available in this build; rendering headless.\n");
  if (o.output.empty())  // Config::operator<< (Config.h:237-248)
    o.output = "algorithm_" + o.algorithm + "_kernel_" + o.kernel + "_iter_" + std::to_string(o.iterations);

  // Medium upload: dense textures as the reference; the 8^3-leaf upload for
  // sparse-only scenes, for --use-unified-memory true (the reference's
  // HostDeviceMedium choice for scenes too big for device memory,
  // Config.h:147-156), and when the dense grid is rejected as too large.
  cvr_medium_desc md;
  cvr_sparse_medium_desc sd;
  bool sparse = cvr_scene_is_sparse(scene) || o.unified;
  if (!sparse) cvr_scene_medium(scene, &md);
  if (sparse && (r = cvr_scene_sparse_medium(scene, &sd)) != CVR_OK) {
    fprintf(stderr, "Error: sparse view of the scene failed (%d)\n", r);
    return 1;
  }
  const unsigned W = o.resolution[0], H = o.resolution[1];
  float inv_view[12], r2v[2];
  cvr_scene_camera(scene, W, H, inv_view, r2v);  // default camera; XML scenes carry their fov
  const float full_res[2] = {(float)W, (float)H};
  std::vector<float> image((size_t)W * H * 4, 0.0f);
  std::vector<double> times;
  double mean = 0;
  if (o.rng_binding != "path" && o.rng_binding != "thread") {
    fprintf(stderr, "[ConfigParser] Error: --rng-binding must be path or thread\n");
    return 2;
  }
  if (o.world_to_aabb != "reference" && o.world_to_aabb != "fixed") {
    fprintf(stderr, "[ConfigParser] Error: --world-to-aabb must be reference or fixed\n");
    return 2;
  }
  if (o.mk_compaction != "fixed" && o.mk_compaction != "reference") {
    fprintf(stderr, "[ConfigParser] Error: --mk-compaction must be fixed or reference\n");
    return 2;
  }
  // One context: its options, the medium (its own upload, or `share`'s device copy when
  // another context on the same device already holds it), the camera.
  auto make_ctx = [&](int device, cvr_ctx* share) -> cvr_ctx* {
    cvr_ctx* ctx = nullptr;
    if (cvr_create(device, kernel, &ctx) != CVR_OK) {
      fprintf(stderr, "Error: %s\n", cvr_last_error(nullptr));
      return nullptr;
    }
    int rc = cvr_set_seed(ctx, o.seed);
    if (!rc && o.rng_binding == "thread") rc = cvr_set_option(ctx, CVR_OPT_RNG_BINDING, 1);
    if (!rc && o.world_to_aabb == "fixed") rc = cvr_set_option(ctx, CVR_OPT_WORLD_TO_AABB, 1);
    if (!rc && o.mk_compaction == "reference") rc = cvr_set_option(ctx, CVR_OPT_MK_COMPACTION, 1);
    if (!rc && share) {
      rc = cvr_share_medium(ctx, share);
    } else if (!rc) {
      if (!sparse && (rc = cvr_set_medium(ctx, &md)) == CVR_ERR_UNSUPPORTED) {
        printf("[Scene] dense grid rejected (%s); using the sparse leaf upload\n", cvr_last_error(ctx));
        if ((rc = cvr_scene_sparse_medium(scene, &sd)) == CVR_OK) sparse = true;
      }
      if (!rc && sparse) rc = cvr_set_medium_sparse(ctx, &sd);
    }
    if (!rc) rc = cvr_set_camera(ctx, inv_view, r2v, full_res);
    if (!rc) rc = cvr_init(ctx);
    if (rc) {
      fprintf(stderr, "Error: %s\n", cvr_last_error(ctx));
      cvr_destroy(ctx);
      return nullptr;
    }
    return ctx;
  };
  const std::vector<int> devs = parse_devices(o.devices, o.device);
  if (devs.empty()) {
    fprintf(stderr, "[ConfigParser] Error: --devices needs a count (N >= 1) or a list of two or more device ids "
                    "(d0,d1,...), digits only\n");
    return 2;
  }
  const unsigned ntiles = o.tiles[0] * o.tiles[1];
  size_t n_dev = devs.size();
  const bool tile_mode = ntiles > 1;
  if (n_dev > 1 && !tile_mode && (W % 8 || H % 8)) {
    printf("[Devices] one tile of %ux%u: block shards need sides that are multiples of 8; rendering on device %d\n", W,
           H, devs[0]);
    n_dev = 1;
  }
  if (n_dev > 1 && !tile_mode && o.rng_binding == "thread") {
    // the thread-bound RNG has no 8x8-block work order (cvr_render_share_to_host refuses it)
    printf("[Devices] --rng-binding thread renders paths in launch order, not in 8x8 blocks: no block shards; "
           "rendering on device %d\n", devs[0]);
    n_dev = 1;
  }
  if (n_dev > 1) {
    printf("[Devices] %zu contexts on devices", n_dev);
    for (int dv : devs) printf(" %d", dv);
    printf(": %s\n", tile_mode ? "tile k -> context k mod N" : "8x8-block shards of the image");
  }
  float* himg = nullptr;  // the shared pinned host image (multi-device)
  if (n_dev > 1 && cvr_host_alloc((size_t)W * H * 4 * sizeof(float), reinterpret_cast<void**>(&himg)) != CVR_OK) {
    fprintf(stderr, "Error: %s\n", cvr_last_error(nullptr));
    return 1;
  }
  cvr_render_desc d = {{W, H}, {o.tiles[0], o.tiles[1]}, o.iterations};
  for (unsigned t = 0; t < o.trials; ++t) {
    printf("---------------------------------------------------------------trial : %u \n", t);
    std::vector<cvr_ctx*> ctxs;
    for (size_t k = 0; k < n_dev; ++k) {
      cvr_ctx* share = nullptr;  // the first context on this device holds its medium
      for (size_t j = 0; j < k; ++j)
        if (devs[j] == devs[k]) {
          share = ctxs[j];
          break;
        }
      cvr_ctx* c = make_ctx(devs[k], share);
      if (!c) return 1;
      if (n_dev > 1 && !tile_mode && (r = cvr_set_block_shard(c, (uint32_t)k, (uint32_t)n_dev)) != CVR_OK) {
        fprintf(stderr, "Error: %s\n", cvr_last_error(c));
        return 1;
      }
      ctxs.push_back(c);
    }
    cvr_stats st{};
    const auto t0 = std::chrono::steady_clock::now();
    if (n_dev == 1) {
      r = cvr_render_image(ctxs[0], &d, nullptr, image.data(), &st);
      if (r != CVR_OK) {
        fprintf(stderr, "Error: %s\n", cvr_last_error(ctxs[0]));
        return 1;
      }
    } else {
      std::fill(himg, himg + (size_t)W * H * 4, 0.0f);  // pixels no tile covers stay 0 (Q1)
      std::vector<cvr_stats> sts(n_dev);
      std::vector<int> rcs(n_dev, CVR_OK);
      std::vector<std::string> errs(n_dev);
      std::vector<std::thread> th;
      for (size_t k = 0; k < n_dev; ++k)
        th.emplace_back([&, k] {
          rcs[k] = cvr_render_share_to_host(ctxs[k], &d, tile_mode ? (uint32_t)k : 0u, tile_mode ? (uint32_t)n_dev : 1u,
                                            himg, (size_t)W * H * 4, &sts[k]);
          if (rcs[k] != CVR_OK) errs[k] = cvr_last_error(ctxs[k]);
        });
      for (auto& x : th) x.join();
      for (size_t k = 0; k < n_dev; ++k) {
        if (rcs[k] != CVR_OK) {
          fprintf(stderr, "Error (context %zu, device %d): %s\n", k, devs[k], errs[k].c_str());
          return 1;
        }
        // every counter summed, as cvr_render_tiles sums its tiles'
        st.paths += sts[k].paths;
        st.segments += sts[k].segments;
        st.steps += sts[k].steps;
        st.density += sts[k].density;
        st.albedo += sts[k].albedo;
        st.escaped += sts[k].escaped;
        st.truncated += sts[k].truncated;
        st.fetches += sts[k].fetches;
        st.words += sts[k].words;
        st.iterations += sts[k].iterations;
        st.track_ms += sts[k].track_ms;
        st.events_ms += sts[k].events_ms;
        st.kernel_ms = std::max(st.kernel_ms, sts[k].kernel_ms);
      }
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (n_dev > 1) std::copy(himg, himg + (size_t)W * H * 4, image.begin());
    const double sec = std::chrono::duration<double>(t1 - t0).count();
    printf("rendering time      : %.2f sec \n", sec);
    printf("total traced rays %llu (woodcock steps %llu)\n", (unsigned long long)st.segments,
           (unsigned long long)st.steps);
    if (t > 0) {
      times.push_back(sec);
      mean += sec;
    }
    for (size_t k = n_dev; k-- > 0;) cvr_destroy(ctxs[k]);  // sharers before the medium's owner
    cvr_write_hdr((o.output + ".hdr").c_str(), image.data(), W, H);
    if (o.pfm && write_pfm(o.output + ".pfm", image.data(), W, H)) {
      fprintf(stderr, "Error: could not write %s.pfm\n", o.output.c_str());
      return 1;
    }
  }
  if (himg) cvr_host_free(himg);
  if (o.trials > 1) {
    mean /= (double)times.size();
    double var = 0;
    for (double x : times) var += (x - mean) * (x - mean);
    var /= (double)times.size();
    printf("execution mean time of %.2f sec on %zu iterations and std %.5f \n", mean, times.size(), std::sqrt(var));
    printf("paths per sec %lf \n", (double)W * H * o.iterations / mean);
  }
  cvr_scene_destroy(scene);
  return 0;
}
