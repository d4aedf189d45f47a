// launcher_order.cpp - drives libcvr through cvr::HipVolPTKernelLauncher
// (include/cvr_launcher.hpp) in exactly the order CudaVolPath<Launcher> calls
// its launcher (CudaVolPath.cpp:32-59, :88-115, :189-347), then renders the
// same image with cvr_render_image and compares the two.
//
//   launcher_order KERNEL W H NTX NTY ITERS [SCENE]
//
// Exit 0 when the images agree up to fp32 atomic summation order
// (|a - b| <= 2 (n - 1) 2^-24 max(|a|, |b|), n = ITERS contributions per
// pixel; NaN pixels must coincide), 1 on a mismatch, 2 on an error.  Host C++
// only: hipMalloc/hipMemcpy for the device output buffer as CudaVolPath's
// allocateDeviceMemory/getImage do with cudaMalloc/cudaMemcpy2DAsync.
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "cvr.h"
#include "cvr_launcher.hpp"

namespace {

struct U2 {
  unsigned x, y;
};
struct F2 {
  float x, y;
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// The renderer side of CudaVolPath<Launcher>, member for member, with the
// launcher calls in the reference's order.  Tile origins as initTileArray
// (CudaVolPath.cpp:13-29); the tile dimension as TilingConfig (Config.h:61-78,
// quirk Q1: floor division).
template <class Launcher>
class VolPathOrder {
 public:
  VolPathOrder(const cvr_medium_desc& medium, const float inv_view[12], F2 raster_to_view, U2 resolution, U2 n_tiles,
               unsigned iterations)
      : resolution_(resolution), n_tiles_(n_tiles), iterations_(iterations) {
    memcpy(inv_view_, inv_view, sizeof(inv_view_));
    tile_dim_ = U2{resolution.x / n_tiles.x, resolution.y / n_tiles.y};
    for (unsigned id = 0; id < n_tiles.x * n_tiles.y; ++id)
      tiles_.push_back(U2{tile_dim_.x * (id % n_tiles.x), tile_dim_.y * (unsigned)(int)((float)id / (float)n_tiles.x)});
    current_tile_ = 0;
    // constructor (CudaVolPath.cpp:41-58)
    launcher_.copyRasterToView(raster_to_view);
    struct {
      bool unified_memory = false;
    } cuda_config;
    launcher_.setCudaConfig(cuda_config);
    launcher_.setResolution(tile_dim_);
    launcher_.copyPixelIndexRange(F2{(float)resolution.x, (float)resolution.y});
    launcher_.init();
    // allocateDeviceMemory (:212-232)
    hip_check(hipMalloc(&d_output_, tile_px() * 4 * sizeof(float)), "hipMalloc(d_output_)");
    launcher_.setOutputPtr(reinterpret_cast<float4*>(d_output_));
    launcher_.allocateDeviceMemory();
    // initDeviceScene (:88-115), host volumes instead of textures
    typename Launcher::DeviceScene scene;
    for (int k = 0; k < 3; ++k) {
      scene.medium.density_volume.grid_resolution[k] = medium.res[k];
      scene.medium.albedo_volume.grid_resolution[k] = medium.res[k];
      scene.medium.density_AABB.box_min[k] = medium.box_min[k];
      scene.medium.density_AABB.box_max[k] = medium.box_max[k];
    }
    scene.medium.density_volume.host = medium.density;
    scene.medium.albedo_volume.host = medium.albedo;
    scene.medium.scale = medium.scale;
    scene.medium.max_density = medium.max_density;
    launcher_.setScene(scene);
  }
  ~VolPathOrder() {
    launcher_.releaseDeviceMemory();
    if (d_output_) (void)hipFree(d_output_);
  }

  // render (:339-347)
  void render(float* image_rgba) {
    launcher_.setNIterations(iterations_);  // setNIterations (:235-238)
    launcher_.copyInvViewMatrix(inv_view_, sizeof(float) * 12);  // initCamera (:67-85)
    current_iteration_ = 0;  // initRenderState (:203-209)
    hip_check(hipMemset(d_output_, 0, tile_px() * 4 * sizeof(float)), "hipMemset");
    while (current_tile_ != tiles_.size()) {
      run_iterations();
      get_image(image_rgba);
    }
  }

 private:
  size_t tile_px() const { return (size_t)tile_dim_.x * tile_dim_.y; }

  // runIterations (:249-280)
  void run_iterations() {
    if (current_tile_ == 0) current_iteration_ += launcher_.getNIterations();
    launcher_.copyOffset(tiles_[current_tile_]);
    launcher_.launchRender();
    ++current_tile_;
  }
  // getImage (:283-295): the tile, divided by current_iteration_
  // (UtilityFunctors::Scale), at its origin in the host image (the intended
  // semantics of HostImageBufferTansferDelegate::transfer, quirk Q10); then
  // prepareForNextIterations (:189-200).
  void get_image(float* image) {
    const U2 org = tiles_[current_tile_ - 1];
    std::vector<float> tile(tile_px() * 4);
    hip_check(hipStreamSynchronize(static_cast<hipStream_t>(launcher_.stream())), "sync");
    hip_check(hipMemcpy(tile.data(), d_output_, tile.size() * sizeof(float), hipMemcpyDeviceToHost), "D2H");
    const float scale = (float)current_iteration_;
    for (unsigned y = 0; y < tile_dim_.y; ++y)
      for (unsigned x = 0; x < tile_dim_.x; ++x)
        for (int c = 0; c < 4; ++c)
          image[(((size_t)(org.y + y) * resolution_.x) + org.x + x) * 4 + c] = tile[((size_t)y * tile_dim_.x + x) * 4 + c] / scale;
    launcher_.reset();
    if (tiles_.size() != 1) hip_check(hipMemset(d_output_, 0, tile_px() * 4 * sizeof(float)), "hipMemset");
  }

  Launcher launcher_{};
  U2 resolution_, n_tiles_, tile_dim_{};
  unsigned iterations_;
  float inv_view_[12];
  std::vector<U2> tiles_;
  size_t current_tile_;
  unsigned current_iteration_ = 0;
  void* d_output_ = nullptr;
};

template <int K>
void render_with(const cvr_medium_desc& m, const float* iv, F2 r2v, U2 res, U2 nt, unsigned it, float* img) {
  VolPathOrder<cvr::HipVolPTKernelLauncher<K>> vp(m, iv, r2v, res, nt, it);
  vp.render(img);
}

void render_order(int kernel, const cvr_medium_desc& m, const float* iv, F2 r2v, U2 res, U2 nt, unsigned it,
                  float* img) {
  switch (kernel) {
    case CVR_KERNEL_NAIVE_SK: return render_with<CVR_KERNEL_NAIVE_SK>(m, iv, r2v, res, nt, it, img);
    case CVR_KERNEL_NAIVE_MK: return render_with<CVR_KERNEL_NAIVE_MK>(m, iv, r2v, res, nt, it, img);
    case CVR_KERNEL_REGENERATION_SK: return render_with<CVR_KERNEL_REGENERATION_SK>(m, iv, r2v, res, nt, it, img);
    case CVR_KERNEL_STREAMING_MK: return render_with<CVR_KERNEL_STREAMING_MK>(m, iv, r2v, res, nt, it, img);
    case CVR_KERNEL_STREAMING_SK: return render_with<CVR_KERNEL_STREAMING_SK>(m, iv, r2v, res, nt, it, img);
    case CVR_KERNEL_SORTING_SK: return render_with<CVR_KERNEL_SORTING_SK>(m, iv, r2v, res, nt, it, img);
    default: throw std::runtime_error("unknown kernel");
  }
}

int fail(const char* what, int r) {
  fprintf(stderr, "launcher_order: %s failed (%d): %s\n", what, r, cvr_last_error(nullptr));
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s KERNEL W H NTX NTY ITERS [SCENE]\n", argv[0]);
    return 2;
  }
  const int kernel = cvr_kernel_from_name(argv[1]);
  const U2 res{(unsigned)atoi(argv[2]), (unsigned)atoi(argv[3])};
  const U2 nt{(unsigned)atoi(argv[4]), (unsigned)atoi(argv[5])};
  const unsigned iters = (unsigned)atoi(argv[6]);
  const char* scene_name = argc > 7 ? argv[7] : "bucky";
  if (kernel == CVR_KERNEL_UNKNOWN) {
    fprintf(stderr, "unknown kernel %s\n", argv[1]);
    return 2;
  }
  cvr_scene* scene = nullptr;
  int r = cvr_scene_synthetic(scene_name, 0, nullptr, &scene);
  if (r) return fail("cvr_scene_synthetic", r);
  cvr_medium_desc m{};
  if ((r = cvr_scene_medium(scene, &m))) return fail("cvr_scene_medium", r);
  float iv[12], r2v[2];
  if ((r = cvr_default_camera(res.x, res.y, iv, r2v))) return fail("cvr_default_camera", r);
  const size_t n = (size_t)res.x * res.y * 4;
  std::vector<float> a(n, 0.0f), b(n, 0.0f);
  try {
    render_order(kernel, m, iv, F2{r2v[0], r2v[1]}, res, nt, iters, a.data());
  } catch (const std::exception& e) {
    fprintf(stderr, "launcher_order: %s\n", e.what());
    return 2;
  }
  // the same render through the single-call tile loop
  cvr_ctx* ctx = nullptr;
  if ((r = cvr_create(0, kernel, &ctx))) return fail("cvr_create", r);
  const float full[2] = {(float)res.x, (float)res.y};
  cvr_render_desc rd{};
  rd.resolution[0] = res.x;
  rd.resolution[1] = res.y;
  rd.n_tiles[0] = nt.x;
  rd.n_tiles[1] = nt.y;
  rd.iterations = iters;
  cvr_stats st{};
  if ((r = cvr_set_medium(ctx, &m)) || (r = cvr_set_camera(ctx, iv, r2v, full)) || (r = cvr_init(ctx)) ||
      (r = cvr_render_image(ctx, &rd, nullptr, b.data(), &st)))
    return fail("cvr_render_image", r);
  cvr_destroy(ctx);
  cvr_scene_destroy(scene);
  size_t bad = 0, nan_a = 0, nonzero = 0;
  double worst = 0.0;
  for (size_t i = 0; i < n; ++i) {
    const bool na = std::isnan(a[i]), nb = std::isnan(b[i]);
    nan_a += na;
    if (na != nb) {
      ++bad;
      continue;
    }
    if (na) continue;
    nonzero += a[i] != 0.0f;
    const double d = std::fabs((double)a[i] - (double)b[i]);
    const double bound = 2.0 * (iters > 1 ? iters - 1 : 1) * std::ldexp(1.0, -24) *
                             std::fmax(std::fabs((double)a[i]), std::fabs((double)b[i])) + 1e-30;
    if (d > bound) ++bad;
    if (d > worst) worst = d;
  }
  printf("launcher_order %s %ux%u tiles %ux%u it %u scene %s: paths %llu, %zu nonzero, %zu NaN, worst diff %.3g, "
         "%zu out of tolerance\n",
         argv[1], res.x, res.y, nt.x, nt.y, iters, scene_name, (unsigned long long)st.paths, nonzero, nan_a, worst,
         bad);
  return bad == 0 && nonzero > 0 ? 0 : 1;
}
