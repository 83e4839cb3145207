#include "bincsr.h"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "parser.h"

namespace fm {

namespace {

constexpr char kMagic[8] = {'F', 'M', 'C', 'S', 'R', '\0', 'v', '1'};

int64_t align8(int64_t x) { return (x + 7) & ~int64_t(7); }

struct Layout {
  int64_t labels, weights, offsets, ids, vals, end;
};

Layout layout(int64_t n, int64_t nnz, uint32_t flags) {
  Layout L{};
  L.labels = sizeof(BinHeader);
  int64_t p = align8(L.labels + 4 * n);
  L.weights = (flags & kBinFlagWeights) ? p : -1;
  if (flags & kBinFlagWeights) p = align8(p + 4 * n);
  L.offsets = p;
  L.ids = p + 8 * (n + 1);
  p = align8(L.ids + 4 * nnz);
  L.vals = (flags & kBinFlagVals) ? p : -1;
  L.end = (flags & kBinFlagVals) ? p + 4 * nnz : L.ids + 4 * nnz;
  return L;
}

void pwrite_all(int fd, const void* p, size_t n, int64_t off, const std::string& path) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    const ssize_t w = ::pwrite(fd, c, n, off);
    if (w <= 0) throw std::runtime_error("write failed: " + path + ": " + std::strerror(errno));
    c += w;
    n -= static_cast<size_t>(w);
    off += w;
  }
}

struct Fd {
  int fd;
  Fd(const std::string& path, int flags) : fd(::open(path.c_str(), flags, 0644)) {
    if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
  }
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

struct LineSpans {
  std::vector<const char*> p;
  std::vector<size_t> len;
};

// Lines of a mapped file split at '\n' ('\r' dropped), like the text loader's split_lines.
void split(const MappedFile& f, LineSpans& out) {
  size_t s = 0;
  while (s < f.size) {
    const void* nl = std::memchr(f.data + s, '\n', f.size - s);
    const size_t e = nl ? static_cast<size_t>(static_cast<const char*>(nl) - f.data) : f.size;
    size_t len = e - s;
    if (len > 0 && f.data[s + len - 1] == '\r') --len;
    out.p.push_back(f.data + s);
    out.len.push_back(len);
    s = e + 1;
  }
}

ConvertStats convert_impl(const std::string& text_path, const std::string& weight_path, const std::string& tmp,
                          const std::string& vtmp, int64_t vocab_size, bool hash_feature_id, int threads,
                          int64_t chunk_lines) {
  MappedFile text(text_path);
  LineSpans all, wall;
  split(text, all);
  std::unique_ptr<MappedFile> wmap;
  const bool weighted = !weight_path.empty();
  if (weighted) {
    wmap = std::make_unique<MappedFile>(weight_path);
    split(*wmap, wall);
    if (wall.p.size() != all.p.size())
      throw std::runtime_error(weight_path + ": " + std::to_string(wall.p.size()) + " lines but " + text_path +
                               " has " + std::to_string(all.p.size()));
  }
  LineSpans lines, wlines;  // non-empty lines (and their weights)
  for (size_t i = 0; i < all.p.size(); ++i) {
    if (all.len[i] == 0) continue;
    lines.p.push_back(all.p[i]);
    lines.len.push_back(all.len[i]);
    if (weighted) {
      wlines.p.push_back(wall.p[i]);
      wlines.len.push_back(wall.len[i]);
    }
  }
  const int64_t n = static_cast<int64_t>(lines.p.size());
  uint32_t flags = (weighted ? kBinFlagWeights : 0) | (hash_feature_id ? kBinFlagHashed : 0);
  const Layout L0 = layout(n, 0, flags);  // sections up to the ids do not depend on nnz

  ConvertStats st;
  Fd out(tmp, O_WRONLY | O_CREAT | O_TRUNC);
  Fd vout(vtmp, O_RDWR | O_CREAT | O_TRUNC);
  CsrBatch csr;
  ParseWorkspace ws;
  std::vector<int32_t> ids32;
  std::vector<int64_t> offs;
  std::vector<float> w;
  int64_t nnz = 0;
  const int64_t zero = 0;
  pwrite_all(out.fd, &zero, 8, L0.offsets, tmp);
  for (int64_t i0 = 0; i0 < n; i0 += chunk_lines) {
    const int64_t m = std::min(chunk_lines, n - i0);
    csr = CsrBatch();
    parse_lines(lines.p.data() + i0, lines.len.data() + i0, static_cast<size_t>(m), vocab_size, hash_feature_id,
                threads, csr, &ws);
    const int64_t c = static_cast<int64_t>(csr.ids.size());
    ids32.resize(c);
    for (int64_t j = 0; j < c; ++j) ids32[j] = static_cast<int32_t>(csr.ids[j]);
    offs.resize(m);
    int64_t o = nnz;
    for (int64_t j = 0; j < m; ++j) {
      o += csr.sizes[j];
      offs[j] = o;
      st.max_feats = std::max(st.max_feats, csr.sizes[j]);
    }
    for (int64_t j = 0; j < c && !st.has_vals; ++j) st.has_vals = csr.vals[j] != 1.f;
    pwrite_all(out.fd, csr.labels.data(), 4 * m, L0.labels + 4 * i0, tmp);
    pwrite_all(out.fd, offs.data(), 8 * m, L0.offsets + 8 * (i0 + 1), tmp);
    pwrite_all(out.fd, ids32.data(), 4 * c, L0.ids + 4 * nnz, tmp);
    pwrite_all(vout.fd, csr.vals.data(), 4 * c, 4 * nnz, vtmp);
    if (weighted) {
      w.resize(m);
      parse_floats(wlines.p.data() + i0, wlines.len.data() + i0, static_cast<size_t>(m), w.data());
      pwrite_all(out.fd, w.data(), 4 * m, L0.weights + 4 * i0, tmp);
    }
    nnz += c;
  }
  if (st.has_vals) flags |= kBinFlagVals;
  const Layout L = layout(n, nnz, flags);
  if (st.has_vals) {  // move the values behind the ids
    std::vector<char> buf(8 << 20);
    for (int64_t off = 0; off < 4 * nnz;) {
      const size_t want = static_cast<size_t>(std::min<int64_t>(static_cast<int64_t>(buf.size()), 4 * nnz - off));
      const ssize_t r = ::pread(vout.fd, buf.data(), want, off);
      if (r <= 0) throw std::runtime_error("read failed: " + vtmp);
      pwrite_all(out.fd, buf.data(), static_cast<size_t>(r), L.vals + off, tmp);
      off += r;
    }
  }
  if (::ftruncate(out.fd, L.end) != 0) throw std::runtime_error("truncate failed: " + tmp);
  BinHeader h{};
  std::memcpy(h.magic, kMagic, 8);
  h.version = 1;
  h.flags = flags;
  h.n = n;
  h.nnz = nnz;
  h.vocab_size = vocab_size;
  h.max_feats = st.max_feats;
  pwrite_all(out.fd, &h, sizeof(h), 0, tmp);
  st.n = n;
  st.nnz = nnz;
  return st;
}

}  // namespace

bool is_bin_file(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  char m[8] = {};
  const bool ok = ::pread(fd, m, 8, 0) == 8 && std::memcmp(m, kMagic, 8) == 0;
  ::close(fd);
  return ok;
}

BinFile::BinFile(const std::string& path) : map(std::make_unique<MappedFile>(path, MADV_NORMAL)) {
  const MappedFile& f = *map;
  if (f.size < sizeof(BinHeader) || std::memcmp(f.data, kMagic, 8) != 0)
    throw std::runtime_error(path + ": not a binary CSR (.fmb) file");
  std::memcpy(&h, f.data, sizeof(h));
  if (h.version != 1) throw std::runtime_error(path + ": unsupported .fmb version " + std::to_string(h.version));
  if (h.n < 0 || h.nnz < 0 || h.max_feats < 0) throw std::runtime_error(path + ": corrupt header");
  const Layout L = layout(h.n, h.nnz, h.flags);
  if (static_cast<int64_t>(f.size) < L.end)
    throw std::runtime_error(path + ": truncated (" + std::to_string(f.size) + " bytes, header says " +
                             std::to_string(L.end) + ")");
  labels = reinterpret_cast<const float*>(f.data + L.labels);
  weights = L.weights >= 0 ? reinterpret_cast<const float*>(f.data + L.weights) : nullptr;
  offsets = reinterpret_cast<const int64_t*>(f.data + L.offsets);
  ids = reinterpret_cast<const int32_t*>(f.data + L.ids);
  vals = L.vals >= 0 ? reinterpret_cast<const float*>(f.data + L.vals) : nullptr;
  if (offsets[0] != 0 || offsets[h.n] != h.nnz) throw std::runtime_error(path + ": corrupt offsets");
  for (int64_t i = 0; i < h.n; ++i)
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > h.max_feats)
      throw std::runtime_error(path + ": corrupt offsets at example " + std::to_string(i));
}

ConvertStats convert_text_to_bin(const std::string& text_path, const std::string& weight_path,
                                 const std::string& out_path, int64_t vocab_size, bool hash_feature_id, int threads,
                                 int64_t chunk_lines) {
  if (vocab_size < 1 || vocab_size > (int64_t(1) << 31))
    throw std::invalid_argument("vocabulary_size must be in [1, 2^31] for int32 ids");
  if (chunk_lines < 1) chunk_lines = 1;
  const std::string tmp = out_path + ".tmp", vtmp = out_path + ".vals.tmp";
  ConvertStats st;
  try {
    st = convert_impl(text_path, weight_path, tmp, vtmp, vocab_size, hash_feature_id, threads, chunk_lines);
  } catch (...) {
    std::remove(tmp.c_str());
    std::remove(vtmp.c_str());
    throw;
  }
  std::remove(vtmp.c_str());
  if (std::rename(tmp.c_str(), out_path.c_str()) != 0) throw std::runtime_error("cannot rename " + tmp);
  return st;
}

}  // namespace fm
