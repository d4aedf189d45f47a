// cvr_xml.cpp - Mitsuba XML scene type with .vol grid volumes.
//
// XmlSceneBuilder.h:39-266 semantics:
//   * <scene> / <medium type="heterogeneous"> (a direct child of <scene>) with
//     <volume name="density" type="gridvolume"> and <volume name="albedo"
//     type="gridvolume">, each naming a file by its <string value>, and
//     <float name="scale">; every one is required;
//   * .vol (Mitsuba grid volume, version 3): "VOL", u8 version, i32 type,
//     i32 xres, yres, zres, i32 channels, 6 floats bbox, then floats with
//     index ((z*yres + y)*xres + x)*channels + c;
//   * max_density = max(min(1, v)) over the density (Q15: the majorant is
//     capped at 1), the AABB is the bbox of the LAST file read, the albedo
//     (Q15), albedo w = 1;
//   * the camera: <sensor type="perspective"> <float name="fov"> (default 45)
//     with the reference's fixed eye/orientation (Camera.h:25-45).
// Only float32 .vol data (type 1) is accepted (the reference reads any type
// as floats).  The XML reader is a minimal tokenizer for this subset:
// elements, attributes, comments, declarations.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "cvr.h"
#include "cvr_scene.h"

namespace cvr {

namespace {

struct XmlNode {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<XmlNode>> kids;
  const char* attr(const char* k) const {
    for (const auto& a : attrs)
      if (a.first == k) return a.second.c_str();
    return nullptr;
  }
  // pugi::xml_node::find_child_by_attribute(name, attr, value)
  const XmlNode* child(const char* tag_name, const char* key, const char* value) const {
    for (const auto& k : kids) {
      const char* v = k->attr(key);
      if (k->tag == tag_name && v && strcmp(v, value) == 0) return k.get();
    }
    return nullptr;
  }
  const XmlNode* first(const char* tag_name) const {
    for (const auto& k : kids)
      if (k->tag == tag_name) return k.get();
    return nullptr;
  }
};

class XmlParser {
 public:
  explicit XmlParser(const std::string& s) : s_(s) {}
  std::unique_ptr<XmlNode> parse() {
    auto root = std::make_unique<XmlNode>();
    root->tag = "#document";
    std::vector<XmlNode*> stack{root.get()};
    while (pos_ < s_.size()) {
      const size_t lt = s_.find('<', pos_);
      if (lt == std::string::npos) break;
      pos_ = lt + 1;
      if (s_.compare(pos_, 3, "!--") == 0) {  // comment
        const size_t e = s_.find("-->", pos_);
        if (e == std::string::npos) return nullptr;
        pos_ = e + 3;
        continue;
      }
      if (s_[pos_] == '?' || s_[pos_] == '!') {  // declaration / doctype
        const size_t e = s_.find('>', pos_);
        if (e == std::string::npos) return nullptr;
        pos_ = e + 1;
        continue;
      }
      if (s_[pos_] == '/') {  // closing tag
        const size_t e = s_.find('>', pos_);
        if (e == std::string::npos || stack.size() < 2) return nullptr;
        if (s_.substr(pos_ + 1, e - pos_ - 1).find(stack.back()->tag) == std::string::npos) return nullptr;
        stack.pop_back();
        pos_ = e + 1;
        continue;
      }
      auto node = std::make_unique<XmlNode>();
      node->tag = name();
      bool self_close = false;
      for (;;) {
        skip_ws();
        if (pos_ >= s_.size()) return nullptr;
        if (s_[pos_] == '/') {
          self_close = true;
          ++pos_;
          continue;
        }
        if (s_[pos_] == '>') {
          ++pos_;
          break;
        }
        std::string k = name();
        skip_ws();
        if (k.empty() || pos_ >= s_.size() || s_[pos_] != '=') return nullptr;
        ++pos_;
        skip_ws();
        const char q = s_[pos_];
        if (q != '"' && q != '\'') return nullptr;
        const size_t e = s_.find(q, pos_ + 1);
        if (e == std::string::npos) return nullptr;
        node->attrs.emplace_back(k, s_.substr(pos_ + 1, e - pos_ - 1));
        pos_ = e + 1;
      }
      XmlNode* raw = node.get();
      stack.back()->kids.push_back(std::move(node));
      if (!self_close) stack.push_back(raw);
    }
    if (stack.size() != 1) return nullptr;
    return root;
  }

 private:
  void skip_ws() {
    while (pos_ < s_.size() && isspace((unsigned char)s_[pos_])) ++pos_;
  }
  std::string name() {
    const size_t b = pos_;
    while (pos_ < s_.size() && (isalnum((unsigned char)s_[pos_]) || strchr("_-:.", s_[pos_]))) ++pos_;
    return s_.substr(b, pos_ - b);
  }
  const std::string& s_;
  size_t pos_ = 0;
};

bool read_text(const std::string& path, std::string& out) {
  FILE* fp = fopen(path.c_str(), "rb");
  if (!fp) return false;
  char buf[1 << 16];
  size_t got;
  while ((got = fread(buf, 1, sizeof(buf), fp)) > 0) out.append(buf, got);
  fclose(fp);
  return true;
}

struct Vol {
  uint32_t res[3] = {0, 0, 0};
  int32_t channels = 0;
  float bbox[6] = {0, 0, 0, 0, 0, 0};
  std::vector<float> data;
};

bool read_vol(const std::string& path, Vol& v) {
  std::string f;
  if (!read_text(path, f) || f.size() < 48) return false;
  if (f[0] != 'V' || f[1] != 'O' || f[2] != 'L' || (uint8_t)f[3] != 3) return false;
  int32_t hdr[5];
  memcpy(hdr, f.data() + 4, sizeof(hdr));
  if (hdr[0] != 1) return false;  // float32 data only
  for (int k = 0; k < 3; ++k) {
    if (hdr[1 + k] <= 0) return false;
    v.res[k] = (uint32_t)hdr[1 + k];
  }
  v.channels = hdr[4];
  memcpy(v.bbox, f.data() + 24, sizeof(v.bbox));
  const size_t n = (size_t)v.res[0] * v.res[1] * v.res[2] * (size_t)(v.channels > 0 ? v.channels : 0);
  if (v.channels <= 0 || f.size() < 48 + n * 4) return false;
  v.data.resize(n);
  memcpy(v.data.data(), f.data() + 48, n * 4);
  return true;
}

}  // namespace

int load_xml_scene(const std::string& path, cvr_scene* sc) {
  std::string text;
  if (!read_text(path, text)) return CVR_ERR_IO;
  auto doc = XmlParser(text).parse();
  if (!doc) {
    set_last_error("XML: cannot parse " + path);
    return CVR_ERR_IO;
  }
  const XmlNode* scene = doc->first("scene");
  const XmlNode* medium = scene ? scene->child("medium", "type", "heterogeneous") : nullptr;
  const XmlNode* albedo = medium ? medium->child("volume", "name", "albedo") : nullptr;
  const XmlNode* density = medium ? medium->child("volume", "name", "density") : nullptr;
  const XmlNode* scale = medium ? medium->child("float", "name", "scale") : nullptr;
  auto gridfile = [](const XmlNode* vol) -> const char* {
    if (!vol || !vol->attr("type") || strcmp(vol->attr("type"), "gridvolume") != 0) return nullptr;
    const XmlNode* s = vol->first("string");
    return s ? s->attr("value") : nullptr;
  };
  const char* afile = gridfile(albedo);
  const char* dfile = gridfile(density);
  if (!afile || !dfile || !scale || !scale->attr("value")) {
    set_last_error("XML: " + path + " lacks the heterogeneous medium's density/albedo gridvolume or scale");
    return CVR_ERR_IO;
  }
  const size_t slash = path.find_last_of('/');
  const std::string base = slash == std::string::npos ? "" : path.substr(0, slash + 1);
  Vol dv, av;
  if (!read_vol(base + dfile, dv) || dv.channels != 1) {
    set_last_error(std::string("XML: cannot read density volume ") + base + dfile);
    return CVR_ERR_IO;
  }
  if (!read_vol(base + afile, av) || av.channels != 3) {
    set_last_error(std::string("XML: cannot read albedo volume ") + base + afile);
    return CVR_ERR_IO;
  }
  if (memcmp(dv.res, av.res, sizeof(dv.res)) != 0) {
    set_last_error("XML: density and albedo grids differ in resolution");
    return CVR_ERR_UNSUPPORTED;
  }
  sc->name = path;
  for (int k = 0; k < 3; ++k) sc->dims[k] = dv.res[k];
  const size_t n = dv.data.size();
  sc->density = dv.data;
  float mx = 0.0f;  // vol2Rawf: max(min(1, v)), Q15
  for (float v : sc->density) mx = std::max(std::min(1.0f, v), mx);
  sc->max_density = mx;
  sc->albedo.resize(n * 4);
  for (size_t i = 0; i < n; ++i) {
    sc->albedo[4 * i] = av.data[3 * i];
    sc->albedo[4 * i + 1] = av.data[3 * i + 1];
    sc->albedo[4 * i + 2] = av.data[3 * i + 2];
    sc->albedo[4 * i + 3] = 1.0f;
  }
  for (int k = 0; k < 3; ++k) {  // the last file read (albedo) sets the AABB, Q15
    sc->box_min[k] = av.bbox[k];
    sc->box_max[k] = av.bbox[3 + k];
  }
  sc->scale = (float)atof(scale->attr("value"));
  // setupCamera (XmlSceneBuilder.h:120-150): perspective sensor fov, default 45
  sc->fov_x = 45.0f;
  if (const XmlNode* sensor = scene->child("sensor", "type", "perspective"))
    if (const XmlNode* fov = sensor->child("float", "name", "fov"))
      if (fov->attr("value")) sc->fov_x = (float)atof(fov->attr("value"));
  return CVR_OK;
}

}  // namespace cvr
