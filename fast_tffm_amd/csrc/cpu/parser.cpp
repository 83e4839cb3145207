#include "parser.h"

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../hash64.h"

namespace fm {

namespace {

inline bool is_delim(char c) { return c == ' ' || c == ':' || c == '\0'; }

// Fast path for plain unsigned decimal integers ("12345") followed by a
// delimiter; falls back to strtoll for anything else (sign, leading blanks,
// overflow) so that the accepted language is exactly strtoll's.
inline bool fast_parse_id(const char* p, const char** end, long long* out) {
  const char* q = p;
  unsigned long long v = 0;
  int digits = 0;
  while (*q >= '0' && *q <= '9' && digits < 18) {
    v = v * 10 + static_cast<unsigned>(*q - '0');
    ++q;
    ++digits;
  }
  if (digits == 0 || (*q >= '0' && *q <= '9')) return false;
  *end = q;
  *out = static_cast<long long>(v);
  return true;
}

// Fast path for small plain integers used as values ("1", "12"); exact in
// float for up to 7 digits. Anything else goes through strtof.
inline bool fast_parse_small_int(const char* p, const char** end, float* out) {
  const char* q = p;
  int v = 0, digits = 0;
  while (*q >= '0' && *q <= '9' && digits < 7) {
    v = v * 10 + (*q - '0');
    ++q;
    ++digits;
  }
  if (digits == 0) return false;
  // must end on a token delimiter, not '.', 'e', another digit, ...
  if (!(*q == ' ' || *q == '\0')) return false;
  *end = q;
  *out = static_cast<float>(v);
  return true;
}

}  // namespace

void parse_line(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id, CsrBatch& out,
                std::string& scratch) {
  scratch.assign(s, len);  // NUL-terminated private copy: strto* never read past the line
  const char* line = scratch.c_str();
  const char* p = line;
  char* nextptr = nullptr;
  float fv = strtof(p, &nextptr);
  if (p == nextptr) throw ParseError(std::string("Label could not be read in example: ") + line);
  out.labels.push_back(fv);
  p = nextptr;
  int32_t cnt = 0;
  for (; *p != '\0'; ++cnt) {
    if (*p != ' ') throw ParseError(std::string("Invalid format in example: ") + line);
    ++p;
    if (*p == '\0') break;
    int64_t ori_id;
    const char* endp = nullptr;
    if (hash_feature_id) {
      const char* q = p;
      while (!is_delim(*q)) ++q;
      ori_id = static_cast<int64_t>(hash64(p, static_cast<size_t>(q - p)) % static_cast<uint64_t>(vocab_size));
      endp = q;
    } else {
      long long v;
      if (!fast_parse_id(p, &endp, &v)) {
        v = strtoll(p, &nextptr, 10);
        if (p == nextptr) throw ParseError(std::string("Invalid format in example: ") + line);
        endp = nextptr;
      }
      if (!(v >= 0 && v < vocab_size))
        throw ParseError(std::string("Invalid feature id. Should be in range [0, vocabulary_size).") + line);
      ori_id = v;
    }
    p = endp;
    if (*p == ':') {
      p += 1;
      const char* e2 = nullptr;
      if (!fast_parse_small_int(p, &e2, &fv)) {
        fv = strtof(p, &nextptr);
        if (p == nextptr) throw ParseError(std::string("Invalid feature value. ") + line);
        e2 = nextptr;
      }
      p = e2;
    } else {
      fv = 1.f;
    }
    out.ids.push_back(ori_id);
    out.vals.push_back(fv);
  }
  out.sizes.push_back(cnt);
}

void parse_lines(const char* const* ptrs, const size_t* lens, size_t n, int64_t vocab_size,
                 bool hash_feature_id, int threads, CsrBatch& out, ParseWorkspace* ws) {
  out.labels.clear(); out.sizes.clear(); out.ids.clear(); out.vals.clear();
  if (n == 0) return;
  if (threads < 1) threads = 1;
  const size_t min_per_thread = 2048;
  size_t nt = std::min<size_t>(threads, (n + min_per_thread - 1) / min_per_thread);
  if (nt <= 1) {
    std::string scratch;
    out.labels.reserve(n); out.sizes.reserve(n);
    for (size_t i = 0; i < n; ++i) parse_line(ptrs[i], lens[i], vocab_size, hash_feature_id, out, scratch);
    return;
  }
  ParseWorkspace local;
  if (!ws) ws = &local;
  if (ws->parts.size() < nt) ws->parts.resize(nt);
  std::vector<CsrBatch>& parts = ws->parts;
  std::vector<std::string> errors(nt);
  std::vector<size_t> err_line(nt, SIZE_MAX);
  const size_t per = (n + nt - 1) / nt;
  // phase 1: every thread parses its contiguous line range into private vectors
  {
    std::vector<std::thread> pool;
    for (size_t t = 0; t < nt; ++t) {
      pool.emplace_back([&, t]() {
        const size_t b = t * per, e = std::min(n, b + per);
        std::string scratch;
        CsrBatch& o = parts[t];
        o.labels.clear(); o.sizes.clear(); o.ids.clear(); o.vals.clear();
        o.labels.reserve(e - b); o.sizes.reserve(e - b);
        size_t bytes = 0;
        for (size_t i = b; i < e; ++i) bytes += lens[i];
        o.ids.reserve(bytes / 6 + 16); o.vals.reserve(bytes / 6 + 16);  // ~one token per 6+ bytes
        for (size_t i = b; i < e; ++i) {
          try {
            parse_line(ptrs[i], lens[i], vocab_size, hash_feature_id, o, scratch);
          } catch (const ParseError& ex) {
            errors[t] = ex.what();
            err_line[t] = i;
            return;
          }
        }
      });
    }
    for (auto& th : pool) th.join();
  }
  // report the first failing line in input order (same as a sequential parse)
  for (size_t t = 0; t < nt; ++t)
    if (err_line[t] != SIZE_MAX) throw ParseError(errors[t]);
  // phase 2: size the outputs once, every thread copies its piece into place
  std::vector<size_t> nz_off(nt + 1, 0), ln_off(nt + 1, 0);
  for (size_t t = 0; t < nt; ++t) {
    nz_off[t + 1] = nz_off[t] + parts[t].ids.size();
    ln_off[t + 1] = ln_off[t] + parts[t].labels.size();
  }
  out.labels.resize(ln_off[nt]); out.sizes.resize(ln_off[nt]);
  out.ids.resize(nz_off[nt]); out.vals.resize(nz_off[nt]);
  {
    std::vector<std::thread> pool;
    for (size_t t = 0; t < nt; ++t) {
      pool.emplace_back([&, t]() {
        CsrBatch& pt = parts[t];
        std::copy(pt.labels.begin(), pt.labels.end(), out.labels.begin() + ln_off[t]);
        std::copy(pt.sizes.begin(), pt.sizes.end(), out.sizes.begin() + ln_off[t]);
        std::copy(pt.ids.begin(), pt.ids.end(), out.ids.begin() + nz_off[t]);
        std::copy(pt.vals.begin(), pt.vals.end(), out.vals.begin() + nz_off[t]);
      });
    }
    for (auto& th : pool) th.join();
  }
}

void parse_floats(const char* const* ptrs, const size_t* lens, size_t n, float* out) {
  std::string scratch;
  for (size_t i = 0; i < n; ++i) {
    scratch.assign(ptrs[i], lens[i]);
    const char* p = scratch.c_str();
    char* e = nullptr;
    errno = 0;
    const float v = strtof(p, &e);
    if (e == p) throw ParseError("StringToNumberOp could not correctly convert string: " + scratch);
    while (*e == ' ' || *e == '\t' || *e == '\r' || *e == '\n') ++e;
    if (*e != '\0') throw ParseError("StringToNumberOp could not correctly convert string: " + scratch);
    out[i] = v;
  }
}

}  // namespace fm
