// cvr_vdb.cpp - OpenVDB / MHD readers.
#include "cvr.h"
#include "cvr_scene.h"

namespace cvr {
int load_vdb_scene(const std::string&, cvr_scene*) { return CVR_ERR_UNSUPPORTED; }
int load_mhd_scene(const std::string&, cvr_scene*) { return CVR_ERR_UNSUPPORTED; }
}  // namespace cvr
