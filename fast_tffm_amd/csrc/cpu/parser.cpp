#include "parser.h"

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <omp.h>
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

// Fast path for plain decimals ("0.25", "-3", "7.", ".5", "2") read from [p, lim) (a char at
// or past lim reads as '\0'): the digits form an integer m < 2^24 with at most 10 of them after
// the point, so m and 10^f are exact floats and ONE IEEE division gives the correctly rounded
// value -- bit-identical to strtof.  The number must be followed by a character strtof cannot
// continue with (' ', ':', '\0', '\t', '\r', '\n'); anything else -- exponents, longer mantissas,
// hex, inf / nan, leading blanks -- returns false and the caller uses strtof.
constexpr float kPow10f[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};

inline bool fast_parse_decimal(const char* p, const char* lim, const char** end, float* out) {
  auto at = [&](const char* q) -> char { return q < lim ? *q : '\0'; };
  const char* q = p;
  bool neg = false;
  if (at(q) == '-' || at(q) == '+') {
    neg = at(q) == '-';
    ++q;
  }
  uint32_t m = 0;
  int digits = 0, frac = -1;
  for (;; ++q) {
    const char c = at(q);
    if (c >= '0' && c <= '9') {
      m = m * 10 + static_cast<uint32_t>(c - '0');
      if (m >= (1u << 24)) return false;
      ++digits;
      if (frac >= 0 && ++frac > 10) return false;
    } else if (c == '.' && frac < 0) {
      frac = 0;
    } else {
      break;
    }
  }
  if (digits == 0) return false;
  const char c = at(q);
  if (!(c == ' ' || c == ':' || c == '\0' || c == '\t' || c == '\r' || c == '\n')) return false;
  float v = static_cast<float>(m);
  if (frac > 0) v = v / kPow10f[frac];
  *out = neg ? -v : v;
  *end = q;
  return true;
}

// One line into (labels, sizes, ids, vals); IdVec holds int64 (CsrBatch) or int32 (Csr32) ids.
template <class IdVec>
void parse_line_into(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id, std::vector<float>& labels,
                     std::vector<int32_t>& sizes, IdVec& ids, std::vector<float>& vals, std::string& scratch);

// The common case without a private copy of the line: plain decimal label / values, plain
// digit ids (or hashed tokens), single spaces, no NUL byte.  Anything else -- including every
// malformed line -- returns false with the outputs untouched, and the caller parses the line
// with parse_line_general, whose results and error messages are the reference's.
template <class IdVec>
bool parse_line_fast(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id, std::vector<float>& labels,
                     std::vector<int32_t>& sizes, IdVec& ids, std::vector<float>& vals) {
  if (len == 0 || std::memchr(s, 0, len) != nullptr) return false;
  const char* const lim = s + len;
  const char* p = s;
  const char* e = nullptr;
  float label;
  if (!fast_parse_decimal(p, lim, &e, &label)) return false;
  p = e;
  const size_t mark = ids.size(), vmark = vals.size();  // (vals may be a line's own buffer)
  int32_t cnt = 0;
  while (p < lim) {
    if (*p != ' ') goto general;
    ++p;
    if (p == lim) break;  // one trailing space
    {
      int64_t id;
      const char* q = p;
      if (hash_feature_id) {
        while (q < lim && *q != ' ' && *q != ':') ++q;
        id = static_cast<int64_t>(hash64(p, static_cast<size_t>(q - p)) % static_cast<uint64_t>(vocab_size));
      } else {
        uint64_t v = 0;
        int digits = 0;
        if (lim - q >= 8) {  // up to 8 leading digits at once (SWAR), then the scalar loop
          uint64_t w;
          std::memcpy(&w, q, 8);
          const uint64_t x = w - 0x3030303030303030ull;
          // high bit of a byte: below '0' (borrow) or above '9' (+0x46 carries into it); a borrow
          // only disturbs the bytes after the first non-digit, whose position is all that is used
          const uint64_t nd = ((w + 0x4646464646464646ull) | x) & 0x8080808080808080ull;
          const int lead = nd ? __builtin_ctzll(nd) >> 3 : 8;
          if (lead > 0) {
            uint64_t d = (x & 0x0F0F0F0F0F0F0F0Full) << (8 * (8 - lead));
            d = (d * 2561) >> 8;
            d = ((d & 0x00FF00FF00FF00FFull) * 6553601) >> 16;
            d = ((d & 0x0000FFFF0000FFFFull) * 42949672960001ull) >> 32;
            v = d;
            digits = lead;
            q += lead;
          }
        }
        while (q < lim && *q >= '0' && *q <= '9' && digits < 18) {
          v = v * 10 + static_cast<unsigned>(*q - '0');
          ++q;
          ++digits;
        }
        if (digits == 0 || (q < lim && *q >= '0' && *q <= '9') || v >= static_cast<uint64_t>(vocab_size))
          goto general;
        id = static_cast<int64_t>(v);
      }
      p = q;
      float fv = 1.f;
      if (p < lim && *p == ':') {
        ++p;
        if (!fast_parse_decimal(p, lim, &e, &fv)) goto general;
        p = e;
      }
      ids.push_back(static_cast<typename IdVec::value_type>(id));
      vals.push_back(fv);
      ++cnt;
    }
  }
  labels.push_back(label);
  sizes.push_back(cnt);
  return true;
general:
  ids.resize(mark);
  vals.resize(vmark);
  return false;
}

template <class IdVec>
void parse_line_general(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id,
                        std::vector<float>& labels, std::vector<int32_t>& sizes, IdVec& ids, std::vector<float>& vals,
                        std::string& scratch);

template <class IdVec>
void parse_line_into(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id, std::vector<float>& labels,
                     std::vector<int32_t>& sizes, IdVec& ids, std::vector<float>& vals, std::string& scratch) {
  if (!parse_line_fast(s, len, vocab_size, hash_feature_id, labels, sizes, ids, vals))
    parse_line_general(s, len, vocab_size, hash_feature_id, labels, sizes, ids, vals, scratch);
}

}  // namespace

void parse_line(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id, CsrBatch& out,
                std::string& scratch) {
  parse_line_into(s, len, vocab_size, hash_feature_id, out.labels, out.sizes, out.ids, out.vals, scratch);
}

void parse_line_general_only(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id, CsrBatch& out,
                             std::string& scratch) {
  parse_line_general(s, len, vocab_size, hash_feature_id, out.labels, out.sizes, out.ids, out.vals, scratch);
}

namespace {

template <class IdVec>
void parse_line_general(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id,
                        std::vector<float>& labels, std::vector<int32_t>& sizes, IdVec& ids, std::vector<float>& vals,
                        std::string& scratch) {
  scratch.assign(s, len);  // NUL-terminated private copy: strto* never read past the line
  const char* line = scratch.c_str();
  const char* const lim = line + len;
  const char* p = line;
  char* nextptr = nullptr;
  float fv;
  const char* lend = nullptr;
  if (fast_parse_decimal(p, lim, &lend, &fv)) {
    p = lend;
  } else {
    fv = strtof(p, &nextptr);
    if (p == nextptr) throw ParseError(std::string("Label could not be read in example: ") + line);
    p = nextptr;
  }
  labels.push_back(fv);
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
      if (!fast_parse_small_int(p, &e2, &fv) && !fast_parse_decimal(p, lim, &e2, &fv)) {
        fv = strtof(p, &nextptr);
        if (p == nextptr) throw ParseError(std::string("Invalid feature value. ") + line);
        e2 = nextptr;
      }
      p = e2;
    } else {
      fv = 1.f;
    }
    ids.push_back(static_cast<typename IdVec::value_type>(ori_id));
    vals.push_back(fv);
  }
  sizes.push_back(cnt);
}

}  // namespace

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

void parse_lines32(const char* const* ptrs, const size_t* lens, size_t n, int64_t vocab_size, bool hash_feature_id,
                   int threads, Csr32& out, Csr32Workspace* ws) {
  out.ids.clear();
  out.vals.clear();
  out.max_feats = 0;
  out.has_vals = false;
  out.in_ext = false;
  if (n == 0) {
    out.labels.clear();
    out.offsets.assign(1, 0);
    return;
  }
  float* L = nullptr;    // destinations: the external buffer or the vectors (chosen once nnz is known)
  int32_t* O = nullptr;
  int32_t* I = nullptr;
  float* Vd = nullptr;
  Csr32Workspace local;
  if (!ws) ws = &local;
  const int T = static_cast<int>(std::max<size_t>(1, std::min<size_t>(std::max(threads, 1), n / 512)));
  if (ws->parts.size() < static_cast<size_t>(T)) ws->parts.resize(T);
  std::vector<std::string> errors(T);
  std::vector<size_t> err_line(T, SIZE_MAX);
  std::vector<size_t> nz_off(T + 1, 0);
  std::vector<int> mf(T, 0);
  bool any_vals = false;  // some value is not 1 (set once all parts are parsed)
  int nt_used = T;
  // phase 1: each thread parses a contiguous line range into its own part; phase 2 (after the
  // barrier and a serial prefix over the parts): each copies its part into place, building the
  // offsets as it goes -- int32 ids straight from the parser, no pass over the batch on one thread
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
#pragma omp single
    nt_used = nt;
    const size_t b = n * t / nt, e = n * (t + 1) / nt;
    Csr32Workspace::Part& o = ws->parts[t];
    o.labels.clear(); o.sizes.clear(); o.ids.clear(); o.vals.clear();
    o.unit = true;
    o.labels.reserve(e - b); o.sizes.reserve(e - b);
    size_t bytes = 0;
    for (size_t i = b; i < e; ++i) bytes += lens[i];
    o.ids.reserve(bytes / 4 + 16);
    std::string scratch;
    for (size_t i = b; i < e; ++i) {
      if (i + 6 < e) {  // lines are scattered over the mapped files: fetch a few ahead
        const char* q = ptrs[i + 6];
        for (size_t k = 0; k < lens[i + 6]; k += 64) __builtin_prefetch(q + k);
      }
      try {
        // the line's values into a small buffer: the part keeps no values while all of them are 1
        // (binary features), so the common batch writes and copies no value array at all
        const size_t mark = o.ids.size();
        o.line_vals.clear();
        parse_line_into(ptrs[i], lens[i], vocab_size, hash_feature_id, o.labels, o.sizes, o.ids, o.line_vals,
                        scratch);
        if (o.unit) {
          bool all1 = true;
          for (float v : o.line_vals) all1 &= v == 1.f;
          if (!all1) {
            o.vals.assign(mark, 1.f);
            o.unit = false;
          }
        }
        if (!o.unit) o.vals.insert(o.vals.end(), o.line_vals.begin(), o.line_vals.end());
      } catch (const ParseError& ex) {
        errors[t] = ex.what();
        err_line[t] = i;
        break;
      }
    }
    nz_off[t + 1] = o.ids.size();
#pragma omp barrier
#pragma omp single
    {
      for (int k = 0; k < nt; ++k) nz_off[k + 1] += nz_off[k];
      bool failed = false;
      for (int k = 0; k < nt; ++k) failed |= err_line[k] != SIZE_MAX;
      for (int k = 0; k < nt; ++k) any_vals |= !ws->parts[k].unit;
      if (!failed) {
        if (out.ext && out.ext(n, nz_off[nt], &L, &O, &I, &Vd)) {
          out.in_ext = true;
        } else {
          out.labels.resize(n);
          out.offsets.resize(n + 1);
          out.ids.resize(nz_off[nt]);
          if (any_vals) out.vals.resize(nz_off[nt]);
          L = out.labels.data();
          O = out.offsets.data();
          I = out.ids.data();
          Vd = out.vals.data();
        }
        O[0] = 0;
      }
    }
    if (O != nullptr && err_line[t] == SIZE_MAX) {
      std::copy(o.labels.begin(), o.labels.end(), L + b);
      std::copy(o.ids.begin(), o.ids.end(), I + nz_off[t]);
      if (any_vals) {  // (some value is not 1: every part's values, the unit parts' as 1s)
        if (o.unit)
          std::fill(Vd + nz_off[t], Vd + nz_off[t + 1], 1.f);
        else
          std::copy(o.vals.begin(), o.vals.end(), Vd + nz_off[t]);
      }
      int32_t off = static_cast<int32_t>(nz_off[t]), m = 0;
      for (size_t i = b; i < e; ++i) {
        const int32_t c = o.sizes[i - b];
        off += c;
        O[i + 1] = off;
        m = std::max(m, c);
      }
      mf[t] = m;
    }
  }
  // the first failing line in input order (same as a sequential parse)
  for (int t = 0; t < nt_used; ++t)
    if (err_line[t] != SIZE_MAX) throw ParseError(errors[t]);
  for (int t = 0; t < nt_used; ++t) out.max_feats = std::max(out.max_feats, mf[t]);
  out.has_vals = any_vals;
  if (!out.has_vals) out.vals.clear();
}

namespace {

bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }

}  // namespace

// tf.string_to_number on one weight line: the fast decimal path when the whole line is a plain
// decimal (+ trailing blanks), else strtof on a NUL-terminated copy.
float parse_float_line(const char* p, size_t len, std::string& scratch) {
  const char* const lim = p + len;
  const char* e = nullptr;
  float v;
  if (fast_parse_decimal(p, lim, &e, &v)) {
    while (e < lim && is_ws(*e)) ++e;
    if (e == lim) return v;
  }
  scratch.assign(p, len);
  const char* q = scratch.c_str();
  char* qe = nullptr;
  errno = 0;
  v = strtof(q, &qe);
  if (qe == q) throw ParseError("StringToNumberOp could not correctly convert string: " + scratch);
  while (is_ws(*qe)) ++qe;
  if (*qe != '\0') throw ParseError("StringToNumberOp could not correctly convert string: " + scratch);
  return v;
}

void parse_floats(const char* const* ptrs, const size_t* lens, size_t n, float* out, int threads) {
  const int T = static_cast<int>(std::max<size_t>(1, std::min<size_t>(std::max(threads, 1), n / 4096)));
  std::vector<size_t> err_line(T, SIZE_MAX);
  std::vector<std::string> errors(T);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const size_t b = n * t / nt, e = n * (t + 1) / nt;
    std::string scratch;
    for (size_t i = b; i < e; ++i) {
      try {
        out[i] = parse_float_line(ptrs[i], lens[i], scratch);
      } catch (const ParseError& ex) {
        errors[t] = ex.what();
        err_line[t] = i;
        break;
      }
    }
  }
  for (int t = 0; t < T; ++t)
    if (err_line[t] != SIZE_MAX) throw ParseError(errors[t]);
}

}  // namespace fm
