// Native training-data loader: files -> shuffled lines -> parsed CSR batches.
//
// Replaces the reference's TF input pipeline (tffm/fm_model.py:34-126):
// string_input_producer(train_files, num_epochs, shuffle=True) ->
// TextLineReader.read_up_to -> shuffle_batch(capacity = 4.5 B,
// min_after_dequeue = 3 B, allow_smaller_final_batch) -> FmParser, run by
// `shuffle_threads` QueueRunner threads into a FIFOQueue(queue_size).
//
// Here one producer thread owns the whole host pipeline:
//  * files are mmap'ed (no copy, no per-line objects); weight files are paired
//    with data files by index and checked line-for-line;
//  * per epoch the file order is shuffled with a (seed, epoch)-seeded RNG; with
//    world > 1 rank r takes files r, r+W, ... (or every W-th line when there are
//    fewer files than ranks);
//  * lines enter a shuffle window of 4.5 B spans; once it is full a batch of B
//    random spans is drawn (partial Fisher-Yates, O(B)); the epoch's tail is
//    drained in batches of <= B (allow_smaller_final_batch);
//  * each batch is parsed by the multi-threaded libsvm parser (parser.h) into
//    CSR with int32 ids / offsets and queued (bounded by queue_size);
//  * the consumer (Python, GIL released while waiting) takes batches in order.
//  * raw mode (GPU tokenizer, hip/parse.hip): instead of parsing, the chosen
//    lines are gathered into one '\n'-separated buffer + line offsets that the
//    consumer copies to the device and tokenizes there.
//  * binary mode (bincsr.h): the files are pre-parsed .fmb caches; the window
//    holds examples instead of lines (same RNG draws) and a batch is assembled
//    by copying the chosen examples' ids / values with `threads` threads; with
//    `rows` set only the chosen examples' global row numbers (file rows
//    concatenated in `files` order) and the batch's CSR offsets are emitted, and
//    the device gathers the data from an HBM-resident copy (hip/batch_gather.hip).
// A (start_epoch, skip_batches) position resumes exactly where a checkpoint
// was taken: the RNGs are re-seeded per epoch, skipped batches are not parsed.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../loader_api.h"
#include "parser.h"

namespace fm {

// Caller-owned output buffers of raw mode (e.g. page-locked host memory the GPU copies from):
// a batch is assembled straight into a free slot, so it needs no staging copy before its
// host-to-device transfer.  The consumer returns a slot with release() once the copy is done.
struct RawSlot {
  uint8_t* bytes = nullptr;
  size_t bytes_cap = 0;
  int64_t* line_start = nullptr;
  size_t ls_cap = 0;          // entries (lines + 1)
  float* weights = nullptr;   // optional: the batch's weights are parsed straight into it
  size_t w_cap = 0;
};

struct LoaderOptions {
  std::vector<std::string> files;
  std::vector<std::string> weight_files;  // empty, or one per data file
  int64_t batch_size = 1;
  int64_t vocab_size = 1;
  bool hash_feature_id = false;
  bool shuffle = true;
  int num_epochs = 1;
  uint64_t seed = 0;
  int threads = 4;            // parser threads per batch
  int rank = 0, world = 1;
  int queue_size = 4;         // parsed batches buffered ahead of the consumer
  int start_epoch = 0;
  int64_t skip_batches = 0;   // batches of start_epoch already consumed
  double capacity_factor = 4.5;
  bool raw = false;           // emit the batch's line bytes (GPU tokenizer) instead of parsed CSR
  bool binary = false;        // files are .fmb binary CSR caches (weights inside; weight_files empty)
  bool rows = false;          // binary: emit row numbers + offsets instead of the data
  std::vector<RawSlot> raw_slots;  // raw mode: assemble into these (a batch too large for a slot: heap)
};

struct LoadedBatch {
  uvector<float> labels;
  uvector<int32_t> offsets;       // [B+1]
  uvector<int32_t> ids;           // [nnz]
  uvector<float> vals;            // [nnz], empty when every value is 1
  uvector<float> weights;         // [B], empty without weight files
  // raw mode: the batch's lines, each '\n'-terminated, and their start offsets [B+1]
  std::vector<uint8_t> bytes;
  std::vector<int64_t> line_start;
  // rows mode: global example rows [B] (offsets, max_feats filled; has_vals = some row has values)
  std::vector<int64_t> rows;
  bool has_vals = false;
  int max_feats = 0;
  // raw mode into a RawSlot: its index, bytes and lines (bytes / line_start above stay empty;
  // weights too when the slot has a weights buffer: weights_in_slot)
  int slot = -1;
  bool weights_in_slot = false;
  size_t nbytes = 0, nlines = 0;
  int epoch = 0;
  int64_t count = 0;              // batches of this epoch consumed after this one
  // kind-1 batch in a consumer's page-locked buffer (FmPinnedPool, loader_api.h): its tag and the
  // arrays' places there; labels / offsets / ids / vals / weights above stay empty
  int pinned = -1;
  float* x_labels = nullptr;
  int32_t* x_offsets = nullptr;
  int32_t* x_ids = nullptr;
  float* x_vals = nullptr;         // null: every value is 1
  float* x_weights = nullptr;
  int64_t x_n = 0, x_nnz = 0;
};

class TextLoader {
 public:
  explicit TextLoader(LoaderOptions o);
  ~TextLoader();
  TextLoader(const TextLoader&) = delete;
  TextLoader& operator=(const TextLoader&) = delete;

  // Next batch in order; false once every epoch is exhausted.  Rethrows a
  // producer failure (ParseError for malformed input, runtime_error for I/O).
  bool next(LoadedBatch& out);
  size_t queued();
  // Shuffle-window fill (items in the window / window capacity) at the latest draw: the
  // reference's -m "shuffle_queue" figure (run_tffm.py:52-63, shuffle_batch queue size).
  float window_fill() const { return fill_.load(std::memory_order_relaxed); }
  void close();
  // Raw slots: hand slot `s` (of a batch returned by next()) back to the producer.
  void release(int slot);
  // C function table over this loader (loader_api.h) for a native consumer in another module
  // (the GPU feeder, hip/feeder.hip); valid while the loader lives.
  const FmLoaderApi* c_api() { return &api_; }
  const LoaderOptions& options() const { return o_; }

  // Batch buffers handed back by a native consumer (the feeder's api_done): the next batches
  // reuse them, so their pages are already resident (a fresh 13 MB batch took ~3k first-touch
  // page faults on the assembling threads).
  void recycle(LoadedBatch& b);
  template <class T>
  void reuse(uvector<T>& v);

 private:
  static int api_parse(void* h, const FmRawView* v, FmParsedOut* out, char* err, int errlen);
  static void api_set_pinned_pool(void* h, const FmPinnedPool* pool) {
    static_cast<TextLoader*>(h)->pinned_pool_.store(pool, std::memory_order_release);
  }
  // A pinned output buffer of >= bytes from the consumer's pool (its tag in *tag), or null.
  void* acquire_pinned(size_t bytes, int32_t* tag) {
    const FmPinnedPool* p = pinned_pool_.load(std::memory_order_acquire);
    return p ? p->acquire(p->ctx, bytes, tag) : nullptr;
  }
  // Give an acquired, undelivered pinned buffer back (the batch being built failed).
  void release_pinned(int32_t tag) {
    const FmPinnedPool* p = pinned_pool_.load(std::memory_order_acquire);
    if (p && p->release && tag >= 0) p->release(p->ctx, tag);
  }
  static void api_stop(void* h) { static_cast<TextLoader*>(h)->close(); }

  void run();
  bool push(LoadedBatch&& b);
  int acquire_slot();         // a free raw slot (blocks), -1 once stopped

  std::deque<int> free_slots_;
  std::condition_variable cv_slot_;

  LoaderOptions o_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_put_, cv_get_;
  std::deque<LoadedBatch> q_;
  bool done_ = false, stop_ = false;
  bool failed_ = false, parse_error_ = false;
  std::string error_;
  std::atomic<float> fill_{0.f};
  FmLoaderApi api_{};
  std::atomic<const FmPinnedPool*> pinned_pool_{nullptr};
  Csr32Workspace api_ws_;     // CPU parses requested through api_ (one consumer thread)
  std::mutex pool_mu_;
  std::vector<uvector<int32_t>> pool_i32_;
  std::vector<uvector<float>> pool_f32_;
};

}  // namespace fm
