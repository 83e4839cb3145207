// C ABI between the host loader (module _fm_cpu, csrc/cpu/loader.h) and the GPU feeder
// (module _fm_hip, csrc/hip/feeder.hip).
//
// The two extension modules are built by different compilers and keep their C++ symbols
// hidden, so no C++ object crosses between them: the loader hands out a table of plain C
// function pointers plus an opaque handle (TextLoader::c_api(), exposed to Python as an
// integer address), and the feeder's thread calls through it without ever touching Python.
// The table lives inside the TextLoader and is valid until that loader is destroyed; the
// Python side keeps the loader alive for as long as a feeder uses it.
#pragma once
#include <cstddef>
#include <cstdint>

extern "C" {

// One batch as the loader produced it, valid until handed back with FmLoaderApi::done:
//  * kind 0 (raw mode, GPU tokenizer): '\n'-terminated lines, in page-locked memory when it came
//    from one of the caller's slots (`slot` >= 0), else in a heap buffer owned by the loader;
//  * kind 1 (parse mode / binary caches): the CPU parser's or the cache's int32 CSR -- in a
//    page-locked buffer of the consumer's pinned pool when one is set (`pinned` >= 0: the
//    consumer copies it to the device directly and gives the buffer back to its pool once the
//    copy is done), else in loader-owned pageable memory (`pinned` = -1).
struct FmRawView {
  int32_t kind;
  int32_t slot;                 // host slot index, -1 for a heap batch
  int32_t epoch;
  int32_t max_feats;            // kind 1
  int64_t count;                // batches of `epoch` consumed once this one is
  const uint8_t* bytes;         // kind 0
  const int64_t* line_start;    // kind 0: [nlines + 1]
  const float* weights;         // [nlines] or null (no weight files)
  int64_t nbytes, nlines;
  const float* labels;          // kind 1: [nlines]
  const int32_t* offsets;       // kind 1: [nlines + 1]
  const int32_t* ids;           // kind 1: [nnz]
  const float* vals;            // kind 1: [nnz] or null (every value 1)
  int64_t nnz;                  // kind 1
  int32_t pinned;               // kind 1: tag of the consumer's pinned buffer holding the arrays, or -1
  void* owner;                  // loader-private (the batch)
};

// Page-locked output buffers a consumer offers for kind-1 batches (set_pinned_pool): the loader
// assembles a batch's CSR arrays straight into one, so the consumer's host-to-device copy needs
// no staging copy.  acquire blocks until a buffer of >= bytes is free and returns it with its
// tag; null (consumer closing, or no buffer that large): the loader uses its own memory.  release
// hands a tag back unused (a batch that failed after its buffer was acquired); a delivered batch's
// buffer is freed by its consumer.
struct FmPinnedPool {
  void* ctx;
  void* (*acquire)(void* ctx, size_t bytes, int32_t* tag);
  void (*release)(void* ctx, int32_t tag);
};

// Host CSR written by FmLoaderApi::parse into caller-owned arrays.
struct FmParsedOut {
  float* labels;                // [nlines]
  int32_t* offsets;             // [nlines + 1]
  int32_t* ids;                 // [cap]
  float* vals;                  // [cap]
  int64_t cap;
  int64_t nnz;                  // out
  int32_t max_feats;            // out
  int32_t has_vals;             // out: some value != 1
};

struct FmLoaderApi {
  int32_t version;              // kFmLoaderApiVersion
  void* handle;
  // 1: a batch in *v; 0: no more batches; -1: parse error, -2: other failure (message in err)
  int (*next)(void* handle, FmRawView* v, char* err, int errlen);
  // the consumer is done with v's host memory (its slot goes back to the loader)
  void (*done)(void* handle, FmRawView* v);
  // the CPU parser (the reference grammar and error strings) over a raw view, with the loader's
  // thread count: 0 ok, -1 parse error (message in err), -3 output capacity too small
  int (*parse)(void* handle, const FmRawView* v, FmParsedOut* out, char* err, int errlen);
  // stop the loader (a consumer blocked in next() returns 0): lets the consumer's own shutdown
  // join a thread that is waiting for the next batch
  void (*stop)(void* handle);
  // offer (pool != null) or withdraw (null) pinned output buffers for kind-1 batches; the pool
  // must outlive the loader's use of it (withdraw before destroying it)
  void (*set_pinned_pool)(void* handle, const FmPinnedPool* pool);
};

}  // extern "C"

constexpr int32_t kFmLoaderApiVersion = 4;
