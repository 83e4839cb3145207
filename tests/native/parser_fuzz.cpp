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

static int check(const std::vector<std::string>& lines, long long vocab, bool hash, int threads) {
  std::vector<const char*> ptrs;
  std::vector<size_t> lens;
  for (const auto& l : lines) {
    ptrs.push_back(l.data());
    lens.push_back(l.size());
  }
  fm::CsrBatch out;
  try {
    fm::parse_lines(ptrs.data(), lens.data(), lines.size(), vocab, hash, threads, out);
  } catch (const fm::ParseError&) {
    return 0;  // rejected input: fine
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
  std::printf("parser_fuzz: %s\n", bad ? "FAILED" : "ok");
  return bad ? 1 : 0;
}
