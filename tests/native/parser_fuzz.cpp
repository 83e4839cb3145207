// Sanitizer driver for the host libsvm parser (optional
// -fsanitize=address,undefined build of the C++ parser).  Built and run by
// tests/test_native_sanitizers.py with g++ -fsanitize=address,undefined.
//
// Feeds the parser the reference's grammar cases (cc/fm_parser_op.cc:58-109),
// edge cases (empty lines, trailing spaces, huge ids, overlong numbers, NULs,
// missing values) and deterministic random byte mutations of valid lines, on
// 1 and 4 threads; every parse must either succeed with consistent CSR sizes
// or throw fm::ParseError.  Exit code 0 = no crash / no sanitizer report.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "cpu/parser.h"

// the fast line path (parse_line) must equal the general parser, results and error messages
static int check_fast_vs_general(const std::string& l, long long vocab, bool hash) {
  fm::CsrBatch a, b;
  std::string sa, sb, ea, eb;
  try {
    fm::parse_line(l.data(), l.size(), vocab, hash, a, sa);
  } catch (const fm::ParseError& e) {
    ea = e.what();
  }
  try {
    fm::parse_line_general_only(l.data(), l.size(), vocab, hash, b, sb);
  } catch (const fm::ParseError& e) {
    eb = e.what();
  }
  bool same = ea == eb && a.ids == b.ids && a.sizes == b.sizes && a.labels.size() == b.labels.size() &&
              a.vals.size() == b.vals.size();
  for (size_t i = 0; same && i < a.labels.size(); ++i) same = std::memcmp(&a.labels[i], &b.labels[i], 4) == 0;
  for (size_t i = 0; same && i < a.vals.size(); ++i) same = std::memcmp(&a.vals[i], &b.vals[i], 4) == 0;
  if (!same) {
    std::fprintf(stderr, "fast path differs on '%s': '%s' vs '%s'\n", l.c_str(), ea.c_str(), eb.c_str());
    return 1;
  }
  return 0;
}

static int check(const std::vector<std::string>& lines, long long vocab, bool hash, int threads) {
  int bad = 0;
  for (const auto& l : lines) bad += check_fast_vs_general(l, vocab, hash);
  if (bad) return bad;
  std::vector<const char*> ptrs;
  std::vector<size_t> lens;
  for (const auto& l : lines) {
    ptrs.push_back(l.data());
    lens.push_back(l.size());
  }
  fm::CsrBatch out;
  fm::Csr32 o32;
  std::string e64, e32;
  try {
    fm::parse_lines(ptrs.data(), lens.data(), lines.size(), vocab, hash, threads, out);
  } catch (const fm::ParseError& e) {
    e64 = e.what();
  }
  try {  // the int32 loader parser: same acceptance, same first error, same CSR
    fm::parse_lines32(ptrs.data(), lens.data(), lines.size(), vocab, hash, threads, o32);
  } catch (const fm::ParseError& e) {
    e32 = e.what();
  }
  if (e64 != e32) {
    std::fprintf(stderr, "parse_lines32 error differs: '%s' vs '%s'\n", e64.c_str(), e32.c_str());
    return 1;
  }
  if (!e64.empty()) return 0;  // rejected input: fine
  if (o32.labels.size() != out.labels.size() || o32.ids.size() != out.ids.size() ||
      o32.offsets.size() != lines.size() + 1) {
    std::fprintf(stderr, "parse_lines32 sizes differ\n");
    return 1;
  }
  for (size_t i = 0; i < out.ids.size(); ++i)
    if (o32.ids[i] != out.ids[i] || (o32.has_vals ? o32.vals[i] : 1.f) != out.vals[i]) {
      std::fprintf(stderr, "parse_lines32 ids / values differ at %zu\n", i);
      return 1;
    }
  for (size_t i = 0; i < out.labels.size(); ++i)
    if (std::memcmp(&o32.labels[i], &out.labels[i], 4) != 0 || o32.offsets[i + 1] - o32.offsets[i] != out.sizes[i]) {
      std::fprintf(stderr, "parse_lines32 labels / offsets differ at %zu\n", i);
      return 1;
    }
  size_t nnz = 0;
  for (int s : out.sizes) nnz += (size_t)s;
  if (out.labels.size() != lines.size() || out.sizes.size() != lines.size() || out.ids.size() != nnz ||
      out.vals.size() != nnz) {
    std::fprintf(stderr, "inconsistent CSR output\n");
    return 1;
  }
  for (long long id : out.ids)
    if (id < 0 || id >= vocab) {
      std::fprintf(stderr, "id out of range: %lld\n", id);
      return 1;
    }
  return 0;
}

// tf.string_to_number semantics with strtof only (the pre-fast-path implementation)
static bool ref_float(const std::string& l, float* v) {
  const char* p = l.c_str();
  char* e = nullptr;
  *v = std::strtof(p, &e);
  if (e == p) return false;
  while (*e == ' ' || *e == '\t' || *e == '\r' || *e == '\n') ++e;
  return *e == '\0';
}

// parse_floats (decimal fast path + strtof fallback) must equal strtof bit for bit, errors included
static int check_float(const std::string& l, int threads) {
  const char* p = l.data();
  size_t len = l.size();
  float ref = 0.f, got = 0.f;
  const bool ok = ref_float(l, &ref) && l.find('\0') == std::string::npos;
  bool got_ok = true;
  try {
    fm::parse_floats(&p, &len, 1, &got, threads);
  } catch (const fm::ParseError&) {
    got_ok = false;
  }
  if (ok != got_ok || (ok && std::memcmp(&ref, &got, 4) != 0)) {
    std::fprintf(stderr, "parse_floats('%s') = %d %.9g, strtof %d %.9g\n", l.c_str(), got_ok, got, ok, ref);
    return 1;
  }
  return 0;
}

int main() {
  const std::vector<std::string> base = {
      "1 2 3", "0 1:0.5 7:2", "1 10:1 11:1 12:1 ", "-1.5 3:1e3", "1", "0 4294967296", "1 abc:1", "1 5:",
      "1 5:x", "1  5", " 1 5", "x 1", "", "1 999999999999999999999999 1", "1 -3", "1 3:1:2", "1 3 :2",
      "0.25 " + std::string(5000, '7'), "1 " + std::string(300, ' '), std::string("1 2\0 3", 6)};
  int bad = 0;
  for (bool hash : {false, true})
    for (int th : {1, 4}) {
      bad += check({base[0], base[1], base[2]}, 100, hash, th);
      for (const auto& l : base) bad += check({l}, 1000, hash, th);
    }
  std::mt19937 rng(12345);
  // ids of 1..20 digits around the 8-digit SWAR boundary, values and labels of every plain form
  for (int it = 0; it < 50000; ++it) {
    std::string l = (rng() % 2) ? "1" : "0.5";
    const int nt = rng() % 6;
    for (int t = 0; t < nt; ++t) {
      l += ' ';
      const int nd = 1 + rng() % 20;
      for (int k = 0; k < nd; ++k) l += char('0' + rng() % 10);
      if (rng() % 3 == 0) l += ":" + std::to_string(rng() % 1000) + ((rng() % 2) ? ".25" : "");
    }
    if (rng() % 7 == 0) l += ' ';
    bad += check({l}, 1 + (long long)(rng() % 2000000000ll), false, 1);
    if (bad > 20) break;
  }
  const std::string alphabet = "0123456789 :.-+eE\tab\n";
  for (int it = 0; it < 20000; ++it) {
    std::string l = base[rng() % 4];
    const int muts = 1 + rng() % 4;
    for (int m = 0; m < muts; ++m) {
      const size_t pos = l.empty() ? 0 : rng() % (l.size() + 1);
      switch (rng() % 3) {
        case 0: l.insert(l.begin() + pos, alphabet[rng() % alphabet.size()]); break;
        case 1: if (!l.empty() && pos < l.size()) l.erase(l.begin() + pos); break;
        default: if (!l.empty() && pos < l.size()) l[pos] = alphabet[rng() % alphabet.size()]; break;
      }
    }
    std::vector<std::string> batch = {l, base[1], l};
    bad += check(batch, 1 + rng() % 100000, rng() % 2, 1 + rng() % 4);
  }
  // decimal fast path vs strtof: random plain decimals (up to 9 digits, up to 12 after the point,
  // signs, leading / trailing points) and mutations of them
  const std::string falpha = "0123456789.-+eE \tx";
  for (int it = 0; it < 200000; ++it) {
    std::string l;
    if (rng() % 4 == 0) l += (rng() % 2) ? '-' : '+';
    const int id = rng() % 10, fd = rng() % 13;
    for (int k = 0; k < id; ++k) l += char('0' + rng() % 10);
    if (fd > 0 || rng() % 3 == 0) l += '.';
    for (int k = 0; k < fd; ++k) l += char('0' + rng() % 10);
    if (rng() % 5 == 0) l += (rng() % 2) ? " " : "\r";
    if (rng() % 8 == 0 && !l.empty()) l[rng() % l.size()] = falpha[rng() % falpha.size()];
    bad += check_float(l, 1);
    if (bad > 20) break;
  }
  for (const char* l : {"1", "2", "0.1", "1e5", " 1", "1 ", "nan", "inf", "0x10", "-0", "16777216", "16777215.5",
                        "0.3333333", "1234567.8", ".5", "5.", ".", "-", "1.0000000001", "3.40282347e38"})
    bad += check_float(l, 1);
  std::printf("parser_fuzz: %s\n", bad ? "FAILED" : "ok");
  return bad ? 1 : 0;
}
