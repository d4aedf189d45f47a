// cvr_mhd.cpp - MetaImage (.mhd) scene type.
//
// The reference has no direct MHD reader: MHD volumes reach it through
// scripts/convert-mhd/mhd_to_vdb.py and the VDB loader.  Loading an .mhd
// here produces what that pipeline produces:
//   1. itk reads the image as float32 (mhd_to_vdb.py:39-44), numpy layout
//      (z, y, x);
//   2. normalized = (image - min) / (max - min) in float32 (:47-51);
//   3. density = smoothstep(0.2, 0.6, normalized) in float32 (:7-10, :52-53);
//   4. pyopenvdb copyFromArray stores array[i][j][k] at VDB (x=i, y=j, z=k)
//      (:56-58), i.e. VDB x = image z and VDB z = image x; values equal to the
//      background 0 are inactive;
//   5. albedo = (d, 0, 0) on the same voxels (:62-71);
//   6. the VDB loader densifies over the active bounding box (VDBAdapter.cpp)
//      and sets scale 100, max_density = max (VDBSceneBuilder.h:54-77).
// Header keys: NDims, DimSize, ElementType (MET_[U]CHAR/[U]SHORT/[U]INT/
// FLOAT/DOUBLE), ElementDataFile (path or LOCAL), CompressedData (zlib),
// BinaryDataByteOrderMSB, HeaderSize, ElementNumberOfChannels (1).
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "cvr.h"
#include "cvr_scene.h"

namespace cvr {

namespace {

std::string trim(const std::string& s) {
  const size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  const size_t b = s.find_last_not_of(" \t\r\n");
  return s.substr(a, b - a + 1);
}

bool read_file(const std::string& path, std::vector<uint8_t>& out) {
  FILE* fp = fopen(path.c_str(), "rb");
  if (!fp) return false;
  uint8_t chunk[1 << 16];
  size_t got;
  while ((got = fread(chunk, 1, sizeof(chunk), fp)) > 0) out.insert(out.end(), chunk, chunk + got);
  fclose(fp);
  return true;
}

template <typename T>
void to_float(const uint8_t* p, size_t n, bool msb, std::vector<float>& out) {
  out.resize(n);
  for (size_t i = 0; i < n; ++i) {
    uint8_t b[sizeof(T)];
    memcpy(b, p + i * sizeof(T), sizeof(T));
    if (msb)
      for (size_t k = 0; k < sizeof(T) / 2; ++k) std::swap(b[k], b[sizeof(T) - 1 - k]);
    T v;
    memcpy(&v, b, sizeof(T));
    out[i] = (float)v;
  }
}

// mhd_to_vdb.py:7-10 in float32: t = clip((x - 0.2) / (0.6 - 0.2), 0, 1);
// t * t * (3 - 2 t).  The edges are Python floats, taken as float32 by numpy.
float smooth_step_f32(float x) {
  const float e0 = 0.2f, span = (float)(0.6 - 0.2);
  float t = (x - e0) / span;
  t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
  const float tt = t * t;
  const float two_t = 2.0f * t;
  return tt * (3.0f - two_t);
}

}  // namespace

int load_mhd_scene(const std::string& path, cvr_scene* sc) {
  std::vector<uint8_t> file;
  if (!read_file(path, file)) return CVR_ERR_IO;
  // header: "Key = Value" lines up to and including ElementDataFile
  size_t pos = 0, header_end = 0;
  int ndims = 0, channels = 1;
  long header_size = 0;
  uint32_t dims[3] = {0, 0, 0};
  std::string etype, datafile;
  bool compressed = false, msb = false;
  while (pos < file.size()) {
    size_t eol = pos;
    while (eol < file.size() && file[eol] != '\n') ++eol;
    const std::string line(reinterpret_cast<const char*>(file.data() + pos), eol - pos);
    pos = eol + 1;
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    const std::string key = trim(line.substr(0, eq)), val = trim(line.substr(eq + 1));
    std::istringstream vs(val);
    if (key == "NDims") vs >> ndims;
    else if (key == "DimSize") vs >> dims[0] >> dims[1] >> dims[2];
    else if (key == "ElementType") etype = val;
    else if (key == "CompressedData") compressed = (val == "True" || val == "true");
    else if (key == "BinaryDataByteOrderMSB" || key == "ElementByteOrderMSB") msb = (val == "True" || val == "true");
    else if (key == "HeaderSize") vs >> header_size;
    else if (key == "ElementNumberOfChannels") vs >> channels;
    else if (key == "ElementDataFile") {
      datafile = val;
      header_end = pos;
      break;  // the data file key ends the header
    }
  }
  if (ndims != 3 || !dims[0] || !dims[1] || !dims[2] || channels != 1 || datafile.empty()) return CVR_ERR_IO;
  std::vector<uint8_t> payload;
  if (datafile == "LOCAL") {
    payload.assign(file.begin() + (long)header_end, file.end());
  } else {
    const size_t slash = path.find_last_of('/');
    const std::string dir = slash == std::string::npos ? "" : path.substr(0, slash + 1);
    if (!read_file(datafile[0] == '/' ? datafile : dir + datafile, payload)) return CVR_ERR_IO;
  }
  if (header_size > 0) {
    if ((size_t)header_size > payload.size()) return CVR_ERR_IO;
    payload.erase(payload.begin(), payload.begin() + header_size);
  }
  size_t esize = 0;
  if (etype == "MET_UCHAR" || etype == "MET_CHAR") esize = 1;
  else if (etype == "MET_SHORT" || etype == "MET_USHORT") esize = 2;
  else if (etype == "MET_INT" || etype == "MET_UINT" || etype == "MET_FLOAT") esize = 4;
  else if (etype == "MET_DOUBLE") esize = 8;
  else return CVR_ERR_UNSUPPORTED;
  const size_t n = (size_t)dims[0] * dims[1] * dims[2];
  std::vector<uint8_t> raw;
  if (compressed) {
    raw.resize(n * esize);
    uLongf len = (uLongf)raw.size();
    if (uncompress(raw.data(), &len, payload.data(), (uLong)payload.size()) != Z_OK || len != raw.size())
      return CVR_ERR_IO;
  } else {
    if (payload.size() < n * esize) return CVR_ERR_IO;
    raw.assign(payload.begin(), payload.begin() + (long)(n * esize));
  }
  std::vector<float> img;  // image x fastest (MetaImage order) == numpy (z, y, x)
  if (etype == "MET_UCHAR") to_float<uint8_t>(raw.data(), n, msb, img);
  else if (etype == "MET_CHAR") to_float<int8_t>(raw.data(), n, msb, img);
  else if (etype == "MET_SHORT") to_float<int16_t>(raw.data(), n, msb, img);
  else if (etype == "MET_USHORT") to_float<uint16_t>(raw.data(), n, msb, img);
  else if (etype == "MET_INT") to_float<int32_t>(raw.data(), n, msb, img);
  else if (etype == "MET_UINT") to_float<uint32_t>(raw.data(), n, msb, img);
  else if (etype == "MET_FLOAT") to_float<float>(raw.data(), n, msb, img);
  else to_float<double>(raw.data(), n, msb, img);
  float mn = img[0], mx = img[0];
  for (float v : img) {
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
  const float range = mx - mn;
  // density in VDB coordinates: X = image z, Y = image y, Z = image x
  const uint32_t dx = dims[2], dy = dims[1];
  std::vector<float> d(n);
  int64_t lo[3] = {INT64_MAX, INT64_MAX, INT64_MAX}, hi[3] = {-1, -1, -1};
  for (uint32_t iz = 0; iz < dims[2]; ++iz)
    for (uint32_t iy = 0; iy < dims[1]; ++iy)
      for (uint32_t ix = 0; ix < dims[0]; ++ix) {
        const float v = img[((size_t)iz * dims[1] + iy) * dims[0] + ix];
        const float nv = (v - mn) / range;
        const float dv = smooth_step_f32(nv);
        const uint32_t X = iz, Y = iy, Z = ix;
        d[((size_t)Z * dy + Y) * dx + X] = dv;
        if (dv != 0.0f) {  // copyFromArray, tolerance 0: background 0 is inactive
          const int64_t c[3] = {X, Y, Z};
          for (int k = 0; k < 3; ++k) {
            lo[k] = c[k] < lo[k] ? c[k] : lo[k];
            hi[k] = c[k] > hi[k] ? c[k] : hi[k];
          }
        }
      }
  if (hi[0] < 0) return CVR_ERR_IO;  // no active voxel
  uint32_t od[3];
  for (int k = 0; k < 3; ++k) od[k] = (uint32_t)(hi[k] - lo[k] + 1);
  sc->name = path;
  for (int k = 0; k < 3; ++k) sc->dims[k] = od[k];
  const size_t m = (size_t)od[0] * od[1] * od[2];
  sc->density.assign(m, 0.0f);
  sc->albedo.assign(m * 4, 0.0f);
  for (uint32_t z = 0; z < od[2]; ++z)
    for (uint32_t y = 0; y < od[1]; ++y)
      for (uint32_t x = 0; x < od[0]; ++x) {
        const size_t o = ((size_t)z * od[1] + y) * od[0] + x;
        const float v = d[((size_t)(z + lo[2]) * dy + (y + lo[1])) * dx + (x + lo[0])];
        sc->density[o] = v;
        sc->albedo[4 * o] = v;  // albedo (d, 0, 0), w = 1
        sc->albedo[4 * o + 3] = 1.0f;
      }
  finish_vdb_like(sc);
  return CVR_OK;
}

}  // namespace cvr
