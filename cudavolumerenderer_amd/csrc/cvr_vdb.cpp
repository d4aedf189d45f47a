// cvr_vdb.cpp - OpenVDB reader for the VDB scene type.
//
// Reads the two grids the reference's VDBAdapter loads (VDBAdapter.cpp:15-43):
// "density" (Tree_float_5_4_3) and "albedo" (Tree_vec3s_5_4_3), and densifies
// them over each grid's active-voxel bounding box, x fastest
// (VDBAdapter.cpp:47-131).  VDBSceneBuilder.h:40-80 then sets max_density =
// max voxel, scale 100, AABB [-0.5,0.5]^3.
//
// The file format is OpenVDB's (file versions 222-224, library 6-11): header,
// file metadata, grid descriptors; per grid: compression flags, metadata,
// transform, tree topology (root tiles/children, 32^3 and 16^3 internal
// nodes with child/value masks and mask-compressed tile values, 8^3 leaf
// value masks), then leaf buffers (mask-compressed values; zlib or blosc
// streams).  Blosc frames are decoded here (LZ4 codec, byte shuffle, split
// blocks); zlib through libz.  Half-float grids and point grids are not
// supported (CVR_ERR_UNSUPPORTED).
#include <zlib.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "cvr.h"
#include "cvr_scene.h"

namespace cvr {

namespace {

// ----------------------------------------------------------------- LZ4 ----
// LZ4 block format: sequences of [token | literal length ext | literals |
// offset (u16 LE) | match length ext]; the last sequence has literals only.
bool lz4_block_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_n) {
  size_t ip = 0, op = 0;
  while (ip < n) {
    const uint8_t token = src[ip++];
    size_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= n) return false;
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > n || op + lit > cap) return false;
    memcpy(dst + op, src + ip, lit);
    ip += lit;
    op += lit;
    if (ip >= n) break;  // last sequence: literals only
    if (ip + 2 > n) return false;
    const size_t off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return false;
    size_t ml = (size_t)(token & 15) + 4;
    if ((token & 15) == 15) {
      uint8_t b;
      do {
        if (ip >= n) return false;
        b = src[ip++];
        ml += b;
      } while (b == 255);
    }
    if (op + ml > cap) return false;
    for (size_t k = 0; k < ml; ++k, ++op) dst[op] = dst[op - off];  // may overlap
  }
  *out_n = op;
  return true;
}

uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }

// --------------------------------------------------------------- blosc ----
// Blosc1 frame: 16-byte header {version, versionlz, flags, typesize, nbytes,
// blocksize, ctbytes}, then one int32 start offset per block; each block is
// `typesize` split streams (or one), each {int32 cbytes, payload}, a payload
// of cbytes == stream size being stored raw.  flags: 0x01 byte shuffle, 0x02
// whole buffer stored raw, 0x04 bit shuffle, 0x10 blocks not split, bits 5-7
// codec (1 = LZ4).
bool blosc_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_n) {
  if (n < 16) return false;
  const uint8_t flags = src[2];
  const uint32_t typesize = src[3];
  const uint32_t nbytes = rd32(src + 4), blocksize = rd32(src + 8), ctbytes = rd32(src + 12);
  if (nbytes != dst_n || ctbytes > n) return false;
  if (flags & 0x02) {
    if (16 + (size_t)nbytes > n) return false;
    memcpy(dst, src + 16, nbytes);
    return true;
  }
  if (flags & 0x04) return false;  // bit shuffle: not produced by OpenVDB's writer
  const uint32_t codec = flags >> 5;
  if (codec != 1 && codec != 3) return false;  // LZ4 or zlib
  if (blocksize == 0 || typesize == 0) return false;
  const uint32_t nblocks = nbytes / blocksize + ((nbytes % blocksize) ? 1u : 0u);
  if (16 + 4 * (size_t)nblocks > n) return false;
  const bool shuffle = (flags & 0x01) && typesize > 1;
  std::vector<uint8_t> tmp(blocksize);
  for (uint32_t j = 0; j < nblocks; ++j) {
    const bool leftover = (j == nblocks - 1) && (nbytes % blocksize) != 0;
    const uint32_t bsize = leftover ? nbytes % blocksize : blocksize;
    const bool split = !(flags & 0x10) && !leftover && typesize <= 16 && bsize / typesize >= 128;
    const uint32_t nsplits = split ? typesize : 1u;
    const uint32_t neblock = bsize / nsplits;
    size_t sp = rd32(src + 16 + 4 * (size_t)j);
    uint8_t* out = shuffle ? tmp.data() : dst + (size_t)j * blocksize;
    size_t done = 0;
    for (uint32_t k = 0; k < nsplits; ++k) {
      if (sp + 4 > n) return false;
      const int32_t cbytes = (int32_t)rd32(src + sp);
      sp += 4;
      if (cbytes < 0 || sp + (size_t)cbytes > n) return false;
      size_t got = 0;
      if ((uint32_t)cbytes == neblock) {
        memcpy(out + done, src + sp, neblock);
        got = neblock;
      } else if (codec == 1) {
        if (!lz4_block_decode(src + sp, (size_t)cbytes, out + done, neblock, &got)) return false;
      } else {
        uLongf len = neblock;
        if (uncompress(out + done, &len, src + sp, (uLong)cbytes) != Z_OK) return false;
        got = len;
      }
      if (got != neblock) return false;
      sp += (size_t)cbytes;
      done += neblock;
    }
    if (done != bsize) return false;
    if (shuffle) {  // byte unshuffle: byte b of element e sits at b*elems + e
      uint8_t* d = dst + (size_t)j * blocksize;
      const uint32_t elems = bsize / typesize;
      for (uint32_t e = 0; e < elems; ++e)
        for (uint32_t b = 0; b < typesize; ++b) d[(size_t)e * typesize + b] = tmp[(size_t)b * elems + e];
      memcpy(d + (size_t)elems * typesize, tmp.data() + (size_t)elems * typesize, bsize - elems * typesize);
    }
  }
  return true;
}

// -------------------------------------------------------------- stream ----
struct Stream {
  const std::vector<uint8_t>& buf;
  size_t pos = 0;
  bool ok = true;
  explicit Stream(const std::vector<uint8_t>& b) : buf(b) {}
  bool read(void* dst, size_t n) {
    if (!ok || pos + n > buf.size()) return ok = false;
    memcpy(dst, buf.data() + pos, n);
    pos += n;
    return true;
  }
  template <typename T>
  T get() {
    T v{};
    read(&v, sizeof(T));
    return v;
  }
  bool skip(size_t n) {
    if (!ok || pos + n > buf.size()) return ok = false;
    pos += n;
    return true;
  }
  std::string str() {  // openvdb::io::readString: u32 length + bytes
    const uint32_t n = get<uint32_t>();
    if (!ok || pos + n > buf.size()) {
      ok = false;
      return {};
    }
    std::string s(reinterpret_cast<const char*>(buf.data() + pos), n);
    pos += n;
    return s;
  }
};

enum : uint32_t { COMPRESS_ZIP = 0x1, COMPRESS_ACTIVE_MASK = 0x2, COMPRESS_BLOSC = 0x4 };

// Bit i of a node mask: u64 words, least significant bit first.
struct Mask {
  std::vector<uint64_t> w;
  explicit Mask(size_t bits = 0) : w((bits + 63) / 64, 0) {}
  bool on(size_t i) const { return (w[i >> 6] >> (i & 63)) & 1u; }
  size_t count() const {
    size_t c = 0;
    for (uint64_t x : w) c += (size_t)__builtin_popcountll(x);
    return c;
  }
  bool load(Stream& s) { return s.read(w.data(), w.size() * 8); }
};

// readData (io/Compression.h): zlib / blosc / raw, each compressed stream
// prefixed by an int64 size (<= 0: -size bytes stored raw).
bool read_data(Stream& s, uint32_t compression, uint8_t* dst, size_t nbytes) {
  if (compression & (COMPRESS_BLOSC | COMPRESS_ZIP)) {
    const int64_t sz = s.get<int64_t>();
    if (!s.ok) return false;
    if (sz <= 0) {
      if ((size_t)(-sz) != nbytes) return false;
      return s.read(dst, nbytes);
    }
    if (s.pos + (size_t)sz > s.buf.size()) return false;
    const uint8_t* src = s.buf.data() + s.pos;
    s.pos += (size_t)sz;
    if (compression & COMPRESS_BLOSC) return blosc_decode(src, (size_t)sz, dst, nbytes);
    uLongf len = nbytes;
    return uncompress(dst, &len, src, (uLong)sz) == Z_OK && len == nbytes;
  }
  return s.read(dst, nbytes);
}

// readCompressedValues (io/Compression.h): per-node metadata byte selecting
// how inactive values were dropped, then the (active) values.
template <int VS>
bool read_compressed_values(Stream& s, uint32_t compression, uint8_t* dst, size_t count, const Mask& value_mask,
                            size_t mask_log2_bits, const uint8_t* background) {
  using Val = std::array<uint8_t, VS>;
  enum : int8_t {
    NO_MASK_OR_INACTIVE_VALS, NO_MASK_AND_MINUS_BG, NO_MASK_AND_ONE_INACTIVE_VAL, MASK_AND_NO_INACTIVE_VALS,
    MASK_AND_ONE_INACTIVE_VAL, MASK_AND_TWO_INACTIVE_VALS, NO_MASK_AND_ALL_VALS
  };
  const int8_t meta = s.get<int8_t>();
  Val inactive0, inactive1;
  memcpy(inactive0.data(), background, VS);
  memcpy(inactive1.data(), background, VS);
  if (meta == NO_MASK_AND_MINUS_BG) {  // -background, component-wise on floats
    for (int k = 0; k < VS; k += 4) {
      float f;
      memcpy(&f, background + k, 4);
      f = -f;
      memcpy(inactive0.data() + k, &f, 4);
    }
  } else if (meta == MASK_AND_ONE_INACTIVE_VAL || meta == MASK_AND_TWO_INACTIVE_VALS ||
             meta == NO_MASK_AND_ONE_INACTIVE_VAL) {
    s.read(inactive0.data(), VS);
    if (meta == MASK_AND_TWO_INACTIVE_VALS) s.read(inactive1.data(), VS);
  }
  Mask selection((size_t)1 << mask_log2_bits);
  if (meta == MASK_AND_NO_INACTIVE_VALS || meta == MASK_AND_ONE_INACTIVE_VAL || meta == MASK_AND_TWO_INACTIVE_VALS)
    selection.load(s);
  if (!s.ok) return false;
  const bool mask_compressed = (compression & COMPRESS_ACTIVE_MASK) && meta != NO_MASK_AND_ALL_VALS;
  const size_t n_read = mask_compressed ? value_mask.count() : count;
  if (!mask_compressed || n_read == count) return read_data(s, compression, dst, count * VS);
  std::vector<uint8_t> tmp(n_read * VS);
  if (!read_data(s, compression, tmp.data(), tmp.size())) return false;
  for (size_t i = 0, t = 0; i < count; ++i) {
    if (value_mask.on(i)) memcpy(dst + i * VS, tmp.data() + (t++) * VS, VS);
    else memcpy(dst + i * VS, (selection.on(i) ? inactive1 : inactive0).data(), VS);
  }
  return true;
}

// ---------------------------------------------------------------- tree ----
template <int VS>
struct Tree {
  struct Leaf {
    int32_t origin[3];
    Mask mask{512};
    std::vector<uint8_t> values;  // 512 * VS, x-major: index (x<<6)|(y<<3)|z
  };
  struct Tile {
    int32_t origin[3];
    int32_t extent;
    std::array<uint8_t, VS> value;
  };
  std::array<uint8_t, VS> background{};
  std::vector<Leaf> leaves;  // in file (buffer) order
  std::vector<Tile> active_tiles;

  // InternalNode::readTopology for LOG2DIM = log2dim, child total log2 = child_total.
  bool read_internal(Stream& s, uint32_t compression, const int32_t origin[3], int log2dim, int child_total) {
    const size_t nvals = (size_t)1 << (3 * log2dim);
    Mask child(nvals), value(nvals);
    if (!child.load(s) || !value.load(s)) return false;
    std::vector<uint8_t> vals(nvals * VS);
    if (!read_compressed_values<VS>(s, compression, vals.data(), nvals, value, 3 * log2dim, background.data()))
      return false;
    const int32_t dim = 1 << log2dim;
    for (size_t i = 0; i < nvals; ++i) {
      const int32_t x = (int32_t)(i >> (2 * log2dim)), y = (int32_t)((i >> log2dim) & (dim - 1)),
                    z = (int32_t)(i & (dim - 1));
      const int32_t o[3] = {origin[0] + (x << child_total), origin[1] + (y << child_total),
                            origin[2] + (z << child_total)};
      if (child.on(i)) {
        if (child_total == 3) {  // leaf: value mask now, values in the buffer pass
          Leaf lf;
          memcpy(lf.origin, o, sizeof(o));
          if (!lf.mask.load(s)) return false;
          leaves.push_back(std::move(lf));
        } else if (!read_internal(s, compression, o, 4, 3)) {
          return false;
        }
      } else if (value.on(i)) {
        Tile t;
        memcpy(t.origin, o, sizeof(o));
        t.extent = 1 << child_total;
        memcpy(t.value.data(), vals.data() + i * VS, VS);
        active_tiles.push_back(t);
      }
    }
    return true;
  }

  bool read(Stream& s, uint32_t compression) {
    if (s.get<int32_t>() != 1) return false;  // buffer count
    s.read(background.data(), VS);
    const uint32_t n_tiles = s.get<uint32_t>(), n_children = s.get<uint32_t>();
    for (uint32_t k = 0; k < n_tiles && s.ok; ++k) {
      Tile t;
      s.read(t.origin, 12);
      s.read(t.value.data(), VS);
      const uint8_t active = s.get<uint8_t>();
      t.extent = 1 << 12;  // a root tile covers a whole 4096^3 internal node
      if (active) active_tiles.push_back(t);
    }
    for (uint32_t k = 0; k < n_children && s.ok; ++k) {
      int32_t o[3];
      s.read(o, 12);
      if (!read_internal(s, compression, o, 5, 7)) return false;
    }
    // buffers: every leaf in topology order (LeafNode::readBuffers)
    for (auto& lf : leaves) {
      Mask m(512);
      if (!m.load(s)) return false;
      lf.mask = m;
      lf.values.resize(512 * VS);
      if (!read_compressed_values<VS>(s, compression, lf.values.data(), 512, lf.mask, 9, background.data()))
        return false;
    }
    return s.ok;
  }

  // evalActiveVoxelBoundingBox: active leaf voxels and the full extent of active tiles.
  bool bbox(int32_t lo[3], int32_t hi[3]) const {
    bool any = false;
    auto add = [&](int32_t x, int32_t y, int32_t z, int32_t ext) {
      const int32_t a[3] = {x, y, z};
      for (int k = 0; k < 3; ++k) {
        lo[k] = any ? std::min(lo[k], a[k]) : a[k];
        hi[k] = any ? std::max(hi[k], a[k] + ext - 1) : a[k] + ext - 1;
      }
      any = true;
    };
    for (const auto& lf : leaves)
      for (int i = 0; i < 512; ++i)
        if (lf.mask.on((size_t)i)) add(lf.origin[0] + (i >> 6), lf.origin[1] + ((i >> 3) & 7), lf.origin[2] + (i & 7), 1);
    for (const auto& t : active_tiles) add(t.origin[0], t.origin[1], t.origin[2], t.extent);
    return any;
  }

  // The ValueOn iterator of VDBAdapter::get*DataAsLinearArray: every active
  // leaf voxel and each active tile once, at the tile's origin (so a tile
  // fills one voxel, not its extent: reference behaviour).
  template <class F>
  void for_each_on(F&& put) const {
    for (const auto& lf : leaves)
      for (int i = 0; i < 512; ++i)
        if (lf.mask.on((size_t)i))
          put(lf.origin[0] + (i >> 6), lf.origin[1] + ((i >> 3) & 7), lf.origin[2] + (i & 7), lf.values.data() + (size_t)i * VS);
    for (const auto& t : active_tiles) put(t.origin[0], t.origin[1], t.origin[2], t.value.data());
  }
  void densify(const int32_t lo[3], const uint32_t dim[3], float* out, int channels) const {
    for_each_on([&](int32_t x, int32_t y, int32_t z, const uint8_t* v) {
      const size_t idx = (size_t)(x - lo[0]) + (size_t)dim[0] * ((size_t)(y - lo[1]) + (size_t)dim[1] * (size_t)(z - lo[2]));
      memcpy(out + idx * (size_t)channels, v, VS);
    });
  }
};

struct GridDesc {
  std::string name, type;
  int64_t grid_pos = 0, block_pos = 0, end_pos = 0;
};

// Skips the grid's transform (math/Transform.cc, Maps.h read()).
bool skip_transform(Stream& s) {
  const std::string type = s.str();
  if (type == "AffineMap" || type == "UnitaryMap") return s.skip(16 * 8);
  if (type == "UniformScaleMap" || type == "ScaleMap") return s.skip(5 * 24);
  if (type == "UniformScaleTranslateMap" || type == "ScaleTranslateMap") return s.skip(6 * 24);
  if (type == "TranslationMap") return s.skip(24);
  return false;  // NonlinearFrustumMap etc.: not used by volume files
}

bool skip_metamap(Stream& s) {
  const int32_t n = s.get<int32_t>();
  for (int32_t k = 0; k < n && s.ok; ++k) {
    s.str();
    s.str();
    const uint32_t sz = s.get<uint32_t>();
    s.skip(sz);
  }
  return s.ok;
}

std::string g_vdb_error;

int fail(const std::string& msg) {
  g_vdb_error = msg;
  return CVR_ERR_IO;
}

template <int VS>
int read_grid(const std::vector<uint8_t>& file, const GridDesc& gd, Tree<VS>& tree) {
  Stream s(file);
  if (gd.grid_pos < 0 || (size_t)gd.grid_pos >= file.size()) return fail("grid offset out of range");
  s.pos = (size_t)gd.grid_pos;
  const uint32_t compression = s.get<uint32_t>();
  if (!skip_metamap(s)) return fail("grid metadata");
  if (!skip_transform(s)) return fail("unsupported transform");
  if (!tree.read(s, compression)) return fail("tree of grid '" + gd.name + "'");
  return CVR_OK;
}

}  // namespace

// Sparse read: the active values go straight into 8^3 leaves of the
// density bounding box (the grid the dense path would build), without the
// dense arrays.  Stored leaves are those holding a non-zero density or a
// non-zero albedo; the rest read as density 0, albedo (0,0,0,1), which is
// what densification leaves there.  The albedo must share the density box
// (converter-made files do), so the reference's reinterpretation of the
// albedo array with the density's dimensions is the identity.
// Without an albedo tree (a density-only file read with a default albedo,
// quirk Q17's flag) the leaves carry no albedo and the background is
// `default_albedo` everywhere.
template <int VD, int VA>
int vdb_to_leaves(const Tree<VD>& dt, const Tree<VA>* at, const int32_t lo[3], const uint32_t dim[3],
                  const float* default_albedo, cvr_scene* sc) {
  const uint32_t lnx = (dim[0] + 7) / 8, lny = (dim[1] + 7) / 8, lnz = (dim[2] + 7) / 8;
  const size_t nleaf = (size_t)lnx * lny * lnz;
  if (nleaf > (1ull << 30)) return fail("density bounding box too large for the leaf table");
  sc->leaf_dims[0] = lnx;
  sc->leaf_dims[1] = lny;
  sc->leaf_dims[2] = lnz;
  sc->leaf_table.assign(nleaf, CVR_NO_LEAF);
  sc->leaf_density.clear();
  sc->leaf_albedo.clear();
  auto slot_of = [&](uint32_t x, uint32_t y, uint32_t z) -> size_t {
    uint32_t& e = sc->leaf_table[((size_t)(z >> 3) * lny + (y >> 3)) * lnx + (x >> 3)];
    if (e == CVR_NO_LEAF) {
      e = (uint32_t)(sc->leaf_density.size() / 512);
      sc->leaf_density.resize(sc->leaf_density.size() + 512, 0.0f);
      const size_t a = sc->leaf_albedo.size();
      sc->leaf_albedo.resize(a + 2048, 0.0f);
      for (size_t k = 3; k < 2048; k += 4) sc->leaf_albedo[a + k] = 1.0f;
    }
    return (size_t)e * 512 + (((z & 7) << 6) | ((y & 7) << 3) | (x & 7));
  };
  float mx = 0.0f;
  dt.for_each_on([&](int32_t x, int32_t y, int32_t z, const uint8_t* v) {
    float f;
    memcpy(&f, v, 4);
    mx = std::max(mx, f);
    if (f != 0.0f) sc->leaf_density[slot_of(x - lo[0], y - lo[1], z - lo[2])] = f;
  });
  bool albedo_set = false;
  if (at) at->for_each_on([&](int32_t x, int32_t y, int32_t z, const uint8_t* v) {
    float c[3];
    memcpy(c, v, 12);
    if (c[0] == 0.0f && c[1] == 0.0f && c[2] == 0.0f) return;
    const int32_t r[3] = {x - lo[0], y - lo[1], z - lo[2]};
    if (r[0] < 0 || r[1] < 0 || r[2] < 0 || r[0] >= (int32_t)dim[0] || r[1] >= (int32_t)dim[1] || r[2] >= (int32_t)dim[2])
      return;  // outside the density box: never read
    memcpy(&sc->leaf_albedo[4 * slot_of(r[0], r[1], r[2])], c, 12);
    albedo_set = true;
  });
  if (!albedo_set) std::vector<float>().swap(sc->leaf_albedo);
  float bg[4] = {0.0f, 0.0f, 0.0f, 1.0f};
  if (!at && default_albedo) memcpy(bg, default_albedo, 3 * sizeof(float));
  memcpy(sc->albedo_bg, bg, sizeof(bg));
  sc->sparse_only = true;
  sc->have_leaves = true;
  sc->max_density = mx;  // VDBSceneBuilder.h:54-77 (inactive voxels are 0)
  sc->scale = 100.0f;
  for (int k = 0; k < 3; ++k) {
    sc->box_min[k] = -0.5f;
    sc->box_max[k] = 0.5f;
  }
  return CVR_OK;
}

int load_vdb_scene(const std::string& path, cvr_scene* sc, bool sparse, const float* default_albedo) {
  FILE* fp = fopen(path.c_str(), "rb");
  if (!fp) return fail("cannot open " + path);
  std::vector<uint8_t> file;
  {
    uint8_t chunk[1 << 16];
    size_t got;
    while ((got = fread(chunk, 1, sizeof(chunk), fp)) > 0) file.insert(file.end(), chunk, chunk + got);
    fclose(fp);
  }
  Stream s(file);
  // header (io/Archive.cc readHeader)
  if (s.get<int64_t>() != 0x56444220LL) return fail("not a VDB file (magic)");
  const uint32_t version = s.get<uint32_t>();
  if (version < 222 || version > 224) return fail("unsupported VDB file version " + std::to_string(version));
  s.get<uint32_t>();  // library major
  s.get<uint32_t>();  // library minor
  s.get<uint8_t>();   // has grid offsets
  s.skip(36);         // uuid, ASCII
  if (!skip_metamap(s)) return fail("file metadata");
  const int32_t n_grids = s.get<int32_t>();
  std::map<std::string, GridDesc> grids;
  for (int32_t k = 0; k < n_grids && s.ok; ++k) {
    GridDesc gd;
    gd.name = s.str();
    const size_t sep = gd.name.find('\x1e');  // unique-name suffix
    if (sep != std::string::npos) gd.name.resize(sep);
    gd.type = s.str();
    s.str();  // instance parent
    gd.grid_pos = s.get<int64_t>();
    gd.block_pos = s.get<int64_t>();
    gd.end_pos = s.get<int64_t>();
    if (!s.ok || gd.end_pos < 0 || (size_t)gd.end_pos > file.size()) return fail("grid descriptor");
    s.pos = (size_t)gd.end_pos;
    if (!grids.count(gd.name)) grids[gd.name] = gd;
  }
  if (!s.ok) return fail("grid descriptors");
  // VDBAdapter::loadVDBFile (VDBAdapter.cpp:32-37): both grids are required
  // (quirk Q17), unless the caller gives a default albedo for files without one
  if (!grids.count("density")) return fail("VDB file does not contain a density grid");
  const bool has_albedo = grids.count("albedo") != 0;
  if (!has_albedo && !default_albedo)
    return fail("VDB file does not contain an albedo grid (give a default albedo: --default-albedo r g b)");
  const GridDesc& gd = grids["density"];
  if (gd.type != "Tree_float_5_4_3") return fail("density grid type " + gd.type + " is not supported");
  Tree<4> dt;
  Tree<12> at;
  int r = read_grid(file, gd, dt);
  if (r) return r;
  if (has_albedo) {
    const GridDesc& ga = grids["albedo"];
    if (ga.type != "Tree_vec3s_5_4_3") return fail("albedo grid type " + ga.type + " is not supported");
    if ((r = read_grid(file, ga, at))) return r;
  }
  int32_t lo[3], hi[3], alo[3], ahi[3];
  if (!dt.bbox(lo, hi)) return fail("density grid has no active voxels");
  uint32_t dim[3], adim[3] = {0, 0, 0};
  for (int k = 0; k < 3; ++k) dim[k] = (uint32_t)(hi[k] - lo[k] + 1);
  const size_t n = (size_t)dim[0] * dim[1] * dim[2];
  sc->name = path;
  for (int k = 0; k < 3; ++k) sc->dims[k] = dim[k];
  // more than 2^30 voxels (20 GB of dense host arrays): read sparse
  if (sparse || n > (1ull << 30)) {
    if (has_albedo && at.bbox(alo, ahi))
      for (int k = 0; k < 3; ++k)
        if (alo[k] != lo[k] || ahi[k] != hi[k])
          return fail("sparse VDB read needs the albedo grid on the density grid's bounding box");
    return vdb_to_leaves(dt, has_albedo ? &at : nullptr, lo, dim, default_albedo, sc);
  }
  sc->density.assign(n, 0.0f);  // inactive value 0
  dt.densify(lo, dim, sc->density.data(), 1);
  if (!has_albedo) {  // Q17 flag: the default albedo everywhere
    sc->albedo.resize(n * 4);
    for (size_t i = 0; i < n; ++i) {
      memcpy(&sc->albedo[4 * i], default_albedo, 3 * sizeof(float));
      sc->albedo[4 * i + 3] = 1.0f;
    }
    finish_vdb_like(sc);
    return CVR_OK;
  }
  // Albedo: densified over the albedo grid's own bounding box, then read as
  // if it had the density grid's dimensions (VDBSceneBuilder.h:57-66 indexes
  // it with volume_size_); identical boxes in every converter-made file.
  std::vector<float> albedo3;
  if (at.bbox(alo, ahi)) {
    for (int k = 0; k < 3; ++k) adim[k] = (uint32_t)(ahi[k] - alo[k] + 1);
    albedo3.assign((size_t)adim[0] * adim[1] * adim[2] * 3, 0.0f);
    at.densify(alo, adim, albedo3.data(), 3);
  }
  sc->albedo.assign(n * 4, 0.0f);
  for (size_t i = 0; i < n; ++i) {
    if (3 * i + 2 < albedo3.size()) memcpy(&sc->albedo[4 * i], &albedo3[3 * i], 3 * sizeof(float));
    sc->albedo[4 * i + 3] = 1.0f;
  }
  finish_vdb_like(sc);
  return CVR_OK;
}

const char* vdb_last_error() { return g_vdb_error.c_str(); }

}  // namespace cvr
