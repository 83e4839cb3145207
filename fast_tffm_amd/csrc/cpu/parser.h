// libsvm -> CSR parser (host C++), the replacement for the reference's
// FmParser TF op (cc/fm_parser_op.cc:8-123).
//
// Grammar, exactly as the reference's ParseLine (cc/fm_parser_op.cc:58-109):
//   <label> <fid>[:<fval>] <fid>[:<fval>] ...
//   * label via strtof; failure -> "Label could not be read in example: <line>"
//   * every token is preceded by exactly one ' ' (else "Invalid format in
//     example: <line>"); a single trailing ' ' is accepted;
//   * non-hash ids: strtoll base 10, must be in [0, vocab_size) (else
//     "Invalid format in example: ..." / "Invalid feature id. Should be in
//     range [0, vocabulary_size).<line>");
//   * hash ids: the token up to ' ', ':' or end is hashed with TF Hash64 and
//     taken modulo vocab_size (cc/fm_parser_op.cc:82-84);
//   * optional ":<fval>" via strtof (else "Invalid feature value. <line>"),
//     default value 1.
// Unlike the reference (one line at a time on one thread) a batch is split
// over worker threads; the per-thread CSR pieces are concatenated in line
// order, so the output is identical to a sequential parse.
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <functional>
#include <vector>

namespace fm {

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct CsrBatch {
  std::vector<float> labels;
  std::vector<int32_t> sizes;
  std::vector<int64_t> ids;
  std::vector<float> vals;
};

// Parse one line (not NUL-terminated: [s, s+len)) and append to `out`.
void parse_line(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id, CsrBatch& out,
                std::string& scratch);

// The general (strto*-based) line parser alone, without the fast path: the fast path's
// differential-test reference (tests/native/parser_fuzz.cpp).
void parse_line_general_only(const char* s, size_t len, int64_t vocab_size, bool hash_feature_id, CsrBatch& out,
                             std::string& scratch);

// Per-thread scratch of parse_lines, reusable across calls (a long-lived caller,
// e.g. the loader, keeps it so the pieces' memory stays mapped: no page faults).
struct ParseWorkspace {
  std::vector<CsrBatch> parts;
};

// Parse `n` lines given as (pointer, length) spans with up to `threads` threads.
void parse_lines(const char* const* ptrs, const size_t* lens, size_t n, int64_t vocab_size,
                 bool hash_feature_id, int threads, CsrBatch& out, ParseWorkspace* ws = nullptr);

// Allocator whose resize() leaves new elements default-initialised (uninitialised for scalars): a
// batch's CSR arrays are sized once and then written in parallel, and value-initialising them --
// a serial zero-fill that also took every first-touch page fault of a fresh 13 MB batch -- was a
// large share of the loader's per-batch host time (profiles/r4/e2e.txt).
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind { using other = NoInitAlloc<U>; };
  NoInitAlloc() noexcept = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
template <class T>
using uvector = std::vector<T, NoInitAlloc<T>>;

// int32 CSR of a batch (the loader's and the device's layout): labels [n], offsets [n + 1],
// ids / vals [nnz] (vals empty when every value is 1), max features per line.
struct Csr32 {
  uvector<float> labels;
  uvector<int32_t> offsets;
  uvector<int32_t> ids;
  uvector<float> vals;
  int max_feats = 0;
  bool has_vals = false;
  // External destination (optional): called once the batch's nnz is known; when it returns true
  // the arrays are written to *labels [n], *offsets [n + 1], *ids / *vals [nnz] instead of the
  // vectors above (which stay empty), e.g. a consumer's page-locked buffer (loader_api.h).
  std::function<bool(size_t n, size_t nnz, float** labels, int32_t** offsets, int32_t** ids, float** vals)> ext;
  bool in_ext = false;  // out: the arrays went to the external destination
};

struct Csr32Workspace {
  struct Part {
    std::vector<float> labels;
    std::vector<int32_t> sizes;
    std::vector<int32_t> ids;
    std::vector<float> vals;   // empty while every value so far is 1 (unit)
    std::vector<float> line_vals;
    bool unit = true;
  };
  std::vector<Part> parts;
};

// parse_lines into int32 CSR with an OpenMP team of up to `threads` (ids < vocab_size < 2^31):
// the per-thread pieces are copied into place and the offsets built in parallel, so no pass over
// the batch runs on one thread.  Same grammar, results and first-error message as parse_lines.
void parse_lines32(const char* const* ptrs, const size_t* lens, size_t n, int64_t vocab_size, bool hash_feature_id,
                   int threads, Csr32& out, Csr32Workspace* ws = nullptr);

// Parse one float per line (weight files; tf.string_to_number semantics:
// the whole line must be a number, surrounding whitespace allowed), with up to `threads`
// threads; the first failing line (in order) is reported.
void parse_floats(const char* const* ptrs, const size_t* lens, size_t n, float* out, int threads = 1);
// One weight line ([p, p + len), not NUL-terminated) with parse_floats' semantics and message.
float parse_float_line(const char* p, size_t len, std::string& scratch);

}  // namespace fm
