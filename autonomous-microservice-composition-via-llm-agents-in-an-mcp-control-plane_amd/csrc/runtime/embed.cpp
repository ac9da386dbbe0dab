// Native feature-hashing embedder of the schema store (retrieval/store.py
// hash_embed): signed feature hashing of the words and "#word#" character
// trigrams of lower-cased ASCII text into `dim` buckets, word weight 1 and
// trigram weight 0.5, CRC-32 (IEEE, zlib.crc32) as the hash.  Accumulated in
// float32 in the same order as the Python loop, so the unnormalised sums are
// bit-identical (tests/test_retrieval_cpu.py); the row normalisation stays in
// numpy.  A 10k-service registry embeds in milliseconds instead of a
// per-feature Python loop.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <array>
#include <cstdint>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

const std::array<uint32_t, 256>& crc_table() {
  static const std::array<uint32_t, 256> t = [] {
    std::array<uint32_t, 256> a{};
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      a[i] = c;
    }
    return a;
  }();
  return t;
}

uint32_t crc32(const char* p, size_t n) {
  const auto& t = crc_table();
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = t[(c ^ (uint8_t)p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

inline bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); }

void add_feature(float* row, int dim, const char* p, size_t n, float w) {
  const uint32_t h = crc32(p, n);
  row[h % (uint32_t)dim] += (h >> 31) & 1 ? w : -w;
}

// texts must be ASCII (the caller routes others to the Python path)
py::array_t<float> hash_embed_sums(const std::vector<std::string>& texts, int dim) {
  if (dim <= 0) throw std::invalid_argument("hash_embed: dim must be positive");
  py::array_t<float> out({(py::ssize_t)texts.size(), (py::ssize_t)dim});
  float* o = out.mutable_data();
  std::fill(o, o + texts.size() * (size_t)dim, 0.f);
  std::vector<std::string> words;
  std::string gram(3, ' ');
  for (size_t r = 0; r < texts.size(); ++r) {
    float* row = o + r * (size_t)dim;
    words.clear();
    std::string cur;
    for (char c : texts[r]) {
      if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
      if (c == '_' || c == '-') c = ' ';
      if (alnum(c)) {
        cur.push_back(c);
      } else if (!cur.empty()) {
        words.push_back(cur);
        cur.clear();
      }
    }
    if (!cur.empty()) words.push_back(cur);
    for (const auto& w : words) add_feature(row, dim, w.data(), w.size(), 1.0f);
    for (const auto& w : words) {
      const std::string ww = "#" + w + "#";
      for (size_t i = 0; i + 3 <= ww.size(); ++i) add_feature(row, dim, ww.data() + i, 3, 0.5f);
    }
  }
  return out;
}

}  // namespace

void register_embed(py::module_& m) {
  m.def("hash_embed_sums", &hash_embed_sums, py::arg("texts"), py::arg("dim"),
        "unnormalised signed feature-hashing sums [len(texts), dim] float32 (ASCII texts)");
}
