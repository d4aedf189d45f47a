/*
 * cvr_launcher.hpp - the reference's kernel-launcher contract over libcvr's C ABI.
 *
 * CudaVolPath<VolPathKernelLauncher> (CudaVolPath.h:34-102, CudaVolPath.cpp)
 * is a class template over its launcher.  It holds the launcher by value
 * (`VolPathKernelLauncher kernel_launcher_{}`, CudaVolPath.h:67) and calls, by
 * name, the members of RenderKernelLauncher / VolPTKernelLauncher
 * (RenderKernelLauncher.h:20-73):
 *
 *   ctor      copyRasterToView, setCudaConfig, setResolution,
 *             copyPixelIndexRange, init                (CudaVolPath.cpp:41-55)
 *             setOutputPtr, allocateDeviceMemory       (:229-230)
 *             setScene(typename Launcher::DeviceScene) (:96-114)
 *   render    setNIterations, copyInvViewMatrix        (:235-244, :67-85)
 *   per tile  getNIterations, copyOffset, launchRender (:249-280)
 *             reset                                    (:189-200)
 *   dtor      releaseDeviceMemory                      (:298-331)
 *
 * HipVolPTKernelLauncher<K> provides exactly those names, so
 * CudaVolPath<cvr::HipVolPTKernelLauncher<CVR_KERNEL_REGENERATION_SK>>
 * compiles against it.  CudaVolPath names the concrete launcher type and
 * calls no member through a base pointer, so this class does not derive from
 * RenderKernelLauncher and pulls in no CUDA/HIP header: the vector arguments
 * (uint2, float2, float4*) are taken as templates that only need .x/.y.
 *
 * DeviceScene carries the HOST volumes instead of texture objects: libcvr
 * copies them into its own HBM layout (cells, brick bounds) at setScene.  The
 * reference's initDeviceScene (CudaVolPath.cpp:88-115) builds CUDA textures
 * first; a maintainer specialises it for this launcher,
 * which is the one reference-side change besides the RendererFactory entry.
 *
 * Errors: the reference's CHECK_CUDA_ERROR prints and exit()s (Debug.h:19-37);
 * here every failing C call throws cvr::LauncherError with cvr_last_error().
 */
#ifndef CVR_LAUNCHER_HPP_
#define CVR_LAUNCHER_HPP_

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "cvr.h"

namespace cvr {

class LauncherError : public std::runtime_error {
 public:
  LauncherError(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

/* Volume<T> / DeviceVolume<T> (Volume.h:31-73,125-160): grid resolution and,
 * here, the host voxel array (Volume::getVolumeData()), x fastest. */
template <class T>
struct HipVolume {
  const T* host = nullptr;
  uint32_t grid_resolution[3] = {0, 0, 0};
};

/* AABB (Geometry.h:26-52). */
struct HipAABB {
  float box_min[3] = {-0.5f, -0.5f, -0.5f};
  float box_max[3] = {0.5f, 0.5f, 0.5f};
};

/* HeterogeneousMedium (Medium.h:110-159): the fields initDeviceScene copies.
 * The albedo volume is float4 per voxel (r, g, b, 1) as the reference's. */
struct HipMedium {
  HipAABB density_AABB;
  float scale = 0.0f;
  float max_density = 0.0f;
  HipVolume<float> albedo_volume;  // 4 floats per voxel
  HipVolume<float> density_volume;
  float g = 0.0f;  // HG asymmetry: the reference never uploads one
};

/* GGX (Bsdf.h:17-30) with its default roughness and IOR ratio. */
struct HipGGX {
  float roughness[2] = {0.1f, 0.1f};
  float int_ior_over_ext_ior = 1.05f / 1.01f;
};

/* SimpleVolumeDeviceScene<Medium, GGX> (Medium.h:161-187). */
struct HipDeviceScene {
  HipMedium medium;
  HipGGX bsdf;
};

template <int Kernel>
class HipVolPTKernelLauncher {
 public:
  using DeviceScene = HipDeviceScene;
  using uint = unsigned int;

  HipVolPTKernelLauncher() = default;
  explicit HipVolPTKernelLauncher(int device) : device_(device) {}
  HipVolPTKernelLauncher(const HipVolPTKernelLauncher&) = delete;
  HipVolPTKernelLauncher& operator=(const HipVolPTKernelLauncher&) = delete;
  ~HipVolPTKernelLauncher() { releaseDeviceMemory(); }

  /* Device to create the context on (the reference uses the current CUDA
   * device); must precede the first other call. */
  void setDevice(int device) { device_ = device; }

  /* RenderKernelLauncher::setCudaConfig (RenderKernelLauncher.h:38).  The
   * reference's CudaConfig holds device properties and the unified-memory
   * switch (Config.h:35-40); libcvr sizes its launches itself (cvr_init). */
  template <class CudaConfigT>
  void setCudaConfig(const CudaConfigT&) {}

  /* setOutputPtr(float4*) (RenderKernelLauncher.h:31): a device buffer of
   * tile_w * tile_h float4. */
  template <class Float4>
  void setOutputPtr(Float4* d_output) {
    check(cvr_set_output(ctx(), static_cast<void*>(d_output)));
  }

  /* setResolution(uint2) -> copyResolution (RenderKernelLauncher.h:33-36). */
  template <class Uint2>
  void setResolution(Uint2 resolution) {
    check(cvr_set_resolution(ctx(), static_cast<uint32_t>(resolution.x), static_cast<uint32_t>(resolution.y)));
  }

  /* copyInvViewMatrix / copyRasterToView / copyPixelIndexRange
   * (RenderKernelLauncher.cu:86-101): libcvr takes the three camera constants
   * together; each call re-sends the current set. */
  void copyInvViewMatrix(const float* inv_view_mat, size_t size_of_mat) {
    const size_t n = size_of_mat / sizeof(float) < 12 ? size_of_mat / sizeof(float) : 12;
    for (size_t i = 0; i < n; ++i) inv_view_[i] = inv_view_mat[i];
    push_camera();
  }
  template <class Float2>
  void copyRasterToView(Float2 raster_to_view) {
    r2v_[0] = raster_to_view.x;
    r2v_[1] = raster_to_view.y;
    push_camera();
  }
  template <class Float2>
  void copyPixelIndexRange(Float2 pixel_index_range) {
    full_res_[0] = pixel_index_range.x;
    full_res_[1] = pixel_index_range.y;
    push_camera();
  }
  /* copyOffset(uint2) (RenderKernelLauncher.cu:103-105). */
  template <class Uint2>
  void copyOffset(Uint2 offset) {
    check(cvr_set_offset(ctx(), static_cast<uint32_t>(offset.x), static_cast<uint32_t>(offset.y)));
  }

  /* VolPTKernelLauncher::setScene (RenderKernelLauncher.h:67-69): uploads
   * the host volumes into HBM. */
  void setScene(const DeviceScene& scene) {
    const HipMedium& m = scene.medium;
    cvr_medium_desc d{};
    for (int k = 0; k < 3; ++k) {
      d.res[k] = m.density_volume.grid_resolution[k];
      if (m.albedo_volume.grid_resolution[k] != d.res[k])
        throw LauncherError(CVR_ERR_INVALID, "albedo and density grids differ in resolution");
      d.box_min[k] = m.density_AABB.box_min[k];
      d.box_max[k] = m.density_AABB.box_max[k];
    }
    d.density = m.density_volume.host;
    d.albedo = m.albedo_volume.host;
    d.scale = m.scale;
    d.max_density = m.max_density;
    d.g = m.g;
    d.roughness[0] = scene.bsdf.roughness[0];
    d.roughness[1] = scene.bsdf.roughness[1];
    d.eta = scene.bsdf.int_ior_over_ext_ior;
    check(cvr_set_medium(ctx(), &d));
    scene_ = scene;
  }
  DeviceScene& getScene() { return scene_; }

  /* VolPTKernelLauncher::setNIterations (RenderKernelLauncher.cu:122-127). */
  void setNIterations(uint n_iterations) {
    check(cvr_set_iterations(ctx(), n_iterations));
    n_iterations_ = n_iterations;
  }
  uint getNIterations() const { return n_iterations_; }

  /* init(): occupancy sizing (Occupancy.cuh:24-70 -> cvr_init). */
  void init() { check(cvr_init(ctx())); }
  void allocateDeviceMemory() {}
  /* launchRender(): asynchronous, accumulates into the output buffer. */
  void launchRender() { check(cvr_launch_render(ctx())); }
  /* reset(): synchronise, then the kernel's per-tile seed advance
   * (RenderKernelLauncher.cu:353-361, :480, :573, :664). */
  void reset() { check(cvr_reset(ctx())); }
  void releaseDeviceMemory() {
    if (ctx_) cvr_destroy(ctx_);
    ctx_ = nullptr;
  }

  /* Not in the reference interface: counters and device time of the last
   * launch, the stream launches run on (a hipStream_t), the C handle. */
  cvr_stats stats() {
    cvr_stats s{};
    check(cvr_get_stats(ctx(), &s));
    return s;
  }
  void* stream() { return cvr_own_stream(ctx()); }
  cvr_ctx* handle() { return ctx(); }

 private:
  cvr_ctx* ctx() {
    if (!ctx_) check(cvr_create(device_, Kernel, &ctx_));
    return ctx_;
  }
  void push_camera() { check(cvr_set_camera(ctx(), inv_view_, r2v_, full_res_)); }
  void check(int r) const {
    if (r != CVR_OK) throw LauncherError(r, cvr_last_error(ctx_));
  }

  int device_ = 0;
  cvr_ctx* ctx_ = nullptr;
  float inv_view_[12] = {1, 0, 0, 0, 0, -1, 0, 0, 0, 0, -1, 100};
  float r2v_[2] = {0, 0};
  float full_res_[2] = {0, 0};
  uint n_iterations_ = 1;
  DeviceScene scene_{};
};

/* Config::Kernel -> launcher (RendererFactory.h:37-115). */
using HipNaiveVolPTsk = HipVolPTKernelLauncher<CVR_KERNEL_NAIVE_SK>;
using HipNaiveVolPTmk = HipVolPTKernelLauncher<CVR_KERNEL_NAIVE_MK>;
using HipRegenerationVolPTsk = HipVolPTKernelLauncher<CVR_KERNEL_REGENERATION_SK>;
using HipStreamingVolPTmk = HipVolPTKernelLauncher<CVR_KERNEL_STREAMING_MK>;
using HipStreamingVolPTsk = HipVolPTKernelLauncher<CVR_KERNEL_STREAMING_SK>;
using HipSortingVolPTsk = HipVolPTKernelLauncher<CVR_KERNEL_SORTING_SK>;

}  // namespace cvr

#endif /* CVR_LAUNCHER_HPP_ */
