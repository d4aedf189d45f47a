// cvr_scene.h - host-side scene representation behind the opaque cvr_scene.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

struct cvr_scene {
  std::string name;
  uint32_t dims[3] = {0, 0, 0};
  std::vector<float> density;  // x fastest
  std::vector<float> albedo;   // rgba per voxel
  float box_min[3] = {-0.5f, -0.5f, -0.5f};
  float box_max[3] = {0.5f, 0.5f, 0.5f};
  float scale = 1.0f;
  float max_density = 1.0f;
  float fov_x = 0.7f;        // camera horizontal fov in degrees (Camera.h:25; XML sensors set it)
  std::vector<uint8_t> raw;  // raw loader input bytes (for fixtures)
  // Sparse storage (cvr_sparse_medium_desc): 8^3 leaves.  Filled by the
  // sparse-only generators (sparse_only, density/albedo empty) or on demand
  // from the dense grid by cvr_scene_sparse_medium.
  bool sparse_only = false;
  bool have_leaves = false;
  uint32_t leaf_dims[3] = {0, 0, 0};
  std::vector<uint32_t> leaf_table;
  std::vector<float> leaf_density;  // 512 per leaf
  std::vector<float> leaf_albedo;   // 512 * 4 per leaf, empty: albedo_bg everywhere
  float albedo_bg[4] = {0.0f, 0.0f, 0.0f, 1.0f};
};

namespace cvr {
int scene_from_raw_bytes(const std::vector<uint8_t>& raw, const std::string& name, cvr_scene* s);
void finish_vdb_like(cvr_scene* s);
int load_vdb_scene(const std::string& path, cvr_scene* s, bool sparse, const float* default_albedo);
int load_mhd_scene(const std::string& path, cvr_scene* s);
int load_xml_scene(const std::string& path, cvr_scene* s);
void camera_for_fov(float fov_x, uint32_t w, uint32_t h, float inv_view[12], float r2v[2]);
const char* vdb_last_error();
void set_last_error(const std::string& msg);  // cvr_last_error(NULL) text
}  // namespace cvr
