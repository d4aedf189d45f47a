"""The reference-side launcher binding (include/cvr_launcher.hpp).

build/launcher_order (tests/cpp/launcher_order.cpp, built by `make`) drives
libcvr through cvr::HipVolPTKernelLauncher<K> in CudaVolPath's call order
(CudaVolPath.cpp:32-59 constructor, :88-115 initDeviceScene, :235-347 render:
setResolution -> copyRasterToView / copyPixelIndexRange -> init ->
setOutputPtr -> setScene -> setNIterations -> copyInvViewMatrix, then per tile
copyOffset / launchRender / transfer / reset) and compares its image with
cvr_render_image's: equal up to fp32 atomic summation order.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "launcher_order")
HDR = os.path.join(ROOT, "include", "cvr_launcher.hpp")


def test_adapter_compiles_against_a_cudavolpath_shaped_template(tmp_path):
    """A class template that uses its launcher exactly as CudaVolPath does
    (by-value member, typename Launcher::DeviceScene, the member names of
    RenderKernelLauncher.h:20-73 with CUDA-like vector types) compiles for
    every kernel id.  Host-only g++, no GPU."""
    src = tmp_path / "shape.cpp"
    src.write_text(r"""
#include "cvr_launcher.hpp"
struct uint2 { unsigned x, y; };
struct float2 { float x, y; };
struct float4 { float x, y, z, w; };
struct CudaConfig { bool unified_memory = false; };
template <class VolPathKernelLauncher>
struct CudaVolPathShape {
  VolPathKernelLauncher kernel_launcher_{};
  void construct(float4* out) {
    kernel_launcher_.copyRasterToView(float2{0.1f, 0.1f});
    kernel_launcher_.setCudaConfig(CudaConfig{});
    kernel_launcher_.setResolution(uint2{64, 64});
    kernel_launcher_.copyPixelIndexRange(float2{64.f, 64.f});
    kernel_launcher_.init();
    kernel_launcher_.setOutputPtr(out);
    kernel_launcher_.allocateDeviceMemory();
    typename VolPathKernelLauncher::DeviceScene device_scene;
    auto& device_medium = device_scene.medium;
    device_medium.max_density = 1.f;
    device_medium.scale = 100.f;
    kernel_launcher_.setScene(device_scene);
  }
  void render() {
    kernel_launcher_.setNIterations(4);
    float m[12] = {};
    kernel_launcher_.copyInvViewMatrix(m, sizeof(float4) * 3);
    unsigned it = kernel_launcher_.getNIterations();
    (void)it;
    kernel_launcher_.copyOffset(uint2{0, 0});
    kernel_launcher_.launchRender();
    kernel_launcher_.reset();
  }
  ~CudaVolPathShape() { kernel_launcher_.releaseDeviceMemory(); }
};
template struct CudaVolPathShape<cvr::HipNaiveVolPTsk>;
template struct CudaVolPathShape<cvr::HipNaiveVolPTmk>;
template struct CudaVolPathShape<cvr::HipRegenerationVolPTsk>;
template struct CudaVolPathShape<cvr::HipStreamingVolPTmk>;
template struct CudaVolPathShape<cvr::HipStreamingVolPTsk>;
template struct CudaVolPathShape<cvr::HipSortingVolPTsk>;
int main() { return 0; }
""")
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_launcher_order_binary_is_built_and_reports_missing_gpu():
    """The compiled driver links libcvr and fails cleanly (exit 2, a message,
    no crash) where there is no GPU; on the GPU box see the -m gpu tests."""
    assert os.path.exists(BIN), "build/launcher_order missing: run make"
    r = subprocess.run([BIN, "regenerationSK", "32", "32", "1", "1", "1"], capture_output=True, text=True, timeout=120)
    if r.returncode == 2 and "no HIP device" in r.stderr:
        return
    assert r.returncode == 0, r.stdout + r.stderr  # a GPU is visible: then it must pass


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,W,H,ntx,nty,iters,scene", [
    ("regenerationSK", 96, 96, 1, 1, 4, "bucky"),
    ("regenerationSK", 128, 96, 4, 2, 3, "hetvol"),
    ("naiveSK", 96, 96, 3, 3, 4, "bucky"),
    ("streamingSK", 128, 128, 2, 2, 3, "hetvol"),
    ("sortingSK", 96, 64, 2, 1, 2, "bucky"),
    ("streamingMK", 64, 64, 2, 2, 2, "bucky"),
    ("naiveMK", 64, 64, 1, 2, 2, "bucky"),
])
def test_launcher_order_matches_render_image(kernel, W, H, ntx, nty, iters, scene):
    r = subprocess.run([BIN, kernel, str(W), str(H), str(ntx), str(nty), str(iters), scene], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 out of tolerance" in r.stdout
