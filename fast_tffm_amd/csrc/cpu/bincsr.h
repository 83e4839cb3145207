// Binary CSR cache: libsvm text parsed once, trained on many times.
//
// SURVEY.md §7.3 ("Input throughput"): text parsing (the reference's FmParser,
// cc/fm_parser_op.cc:58-109, at ~1-2 M lines/s per core) cannot feed a GPU that
// steps 10^8 examples/s.  A `.fmb` file holds one text file's examples already
// parsed -- ids reduced modulo the vocabulary (hashed with Hash64 first when
// hash_feature_id), values, labels and the paired weight file's weights -- laid out
// as flat little-endian arrays that the loader (loader.h, binary mode) maps and
// copies batch rows out of, with the same epoch / shuffle-window / rank-sharding /
// resume semantics as the text path (the same seed draws the same examples).
//
// Layout (every section starts 8-byte aligned):
//   header (64 B): magic "FMCSR\0v1", u32 version = 1, u32 flags (1 = has vals,
//                  2 = has weights, 4 = hashed ids), i64 n, i64 nnz, i64 vocab_size,
//                  i32 max_feats, zero padding
//   labels  f32[n]      weights f32[n] (flag 2)     offsets i64[n + 1]
//   ids     i32[nnz]    vals    f32[nnz] (flag 1; absent when every value is 1)
// Empty text lines are dropped (the text loader skips them too).
#pragma once
#include <cstdint>
#include <memory>
#include <string>

#include "mapped_file.h"

namespace fm {

constexpr uint32_t kBinFlagVals = 1, kBinFlagWeights = 2, kBinFlagHashed = 4;

struct BinHeader {
  char magic[8];
  uint32_t version;
  uint32_t flags;
  int64_t n;
  int64_t nnz;
  int64_t vocab_size;
  int32_t max_feats;
  int32_t pad[5];
};
static_assert(sizeof(BinHeader) == 64, "header is 64 bytes");

// A mapped, validated .fmb file.
struct BinFile {
  explicit BinFile(const std::string& path);
  std::unique_ptr<MappedFile> map;
  BinHeader h{};
  const float* labels = nullptr;
  const float* weights = nullptr;  // null without flag 2
  const int64_t* offsets = nullptr;
  const int32_t* ids = nullptr;
  const float* vals = nullptr;     // null without flag 1
};

bool is_bin_file(const std::string& path);

struct ConvertStats {
  int64_t n = 0, nnz = 0;
  int32_t max_feats = 0;
  bool has_vals = false;
};

// Parse `text_path` (+ its weight file, or "") with `threads` parser threads in chunks of
// `chunk_lines` lines and write `out_path` (via out_path + ".tmp", renamed when complete).
ConvertStats convert_text_to_bin(const std::string& text_path, const std::string& weight_path,
                                 const std::string& out_path, int64_t vocab_size, bool hash_feature_id, int threads,
                                 int64_t chunk_lines = 1 << 20);

}  // namespace fm
