// Device feeder: the host loader's batches -> CSR batches on the device, driven by a native
// thread (no Python, no GIL between file bytes and a ready device batch).  Raw batches go
// through the GPU tokenizer; batches the loader parsed itself (CPU parser) are copied over.
//
// The reference's input path is a set of TF queue runners feeding the step (tffm/fm_model.py:
// 34-126, run_tffm.py:79-81: examples/s is measured file-fed).  Here the host side is the C++
// loader (csrc/cpu/loader.h: mmap'ed files, shuffle window, lines gathered into page-locked
// slots by a thread pool) and this feeder owns everything between that and the training step:
//   * a ring of device slots (input bytes / line starts / weights, tokenizer outputs), allocated
//     by the caller (torch tensors, so the batches it returns are views of them);
//   * its own non-blocking HIP stream: per batch, wait for the slot's release event, copy the
//     raw lines (page-locked -> HBM), launch the tokenizer (parse.hip), copy its 5-int status
//     back, wait, hand the host slot back to the loader and queue the batch as ready;
//   * a batch the GPU subset declines (syntax outside it, any malformed line) is parsed by the
//     loader's CPU parser (the reference grammar and error strings) and uploaded instead;
//   * release(d, stream) from the consumer records an event on the consumer's stream: the slot
//     is overwritten only after the work queued there (the step that read the batch) has run;
//   * a batch with more features than its slot's ids / vals hold (slot sizes are estimated from
//     the heads of the files) is not an error: the thread asks the consumer for larger buffers
//     (next() -> -4, resize_ids) and waits, holding the batch, until they arrive.
// The loader crosses into this module only as a table of C function pointers (loader_api.h).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../loader_api.h"

namespace fm {

struct FeederSlot {
  uint8_t* bytes = nullptr;
  size_t bytes_cap = 0;
  int64_t* ls = nullptr;
  size_t ls_cap = 0;            // entries: lines + 1
  float* weights = nullptr;     // [ls_cap - 1]
  float* labels = nullptr;      // [ls_cap - 1]
  int* offsets = nullptr;       // [ls_cap]
  int* counts = nullptr;        // [ls_cap]
  int* ids = nullptr;           // [ids_cap]
  size_t ids_cap = 0;
  float* vals = nullptr;        // [ids_cap]
  int* status = nullptr;        // [>= 5]
  void* ws = nullptr;
  size_t ws_bytes = 0;
  hipEvent_t ready = nullptr;   // the slot's batch is complete
  hipEvent_t freed = nullptr;   // recorded by release() on the consumer's stream
  int* info_h = nullptr;        // page-locked [8]: fallback, max_feats, non-unit, -, nnz
};

struct FeederBatch {
  int d = -1;
  int64_t n = 0, nnz = 0;
  int max_feats = 0;
  bool has_vals = false, weighted = false;
  int epoch = 0;
  int64_t count = 0;
};

// A few persistent host threads for the staging copies (a std::thread per part per batch cost
// ~50 us of creation each on the feeder's critical path)
class CopyPool {
 public:
  explicit CopyPool(int n) : nth_(n < 1 ? 1 : n) {
    for (int i = 1; i < nth_; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return nth_; }
  // f(t) for t in [0, size()): t = 0 on the caller, the rest on the pool; returns when all are done
  void run(const std::function<void(int)>& f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      ++gen_;
      pending_ = nth_ - 1;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
      }
      (*f)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  int nth_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

class GpuTextFeeder {
 public:
  GpuTextFeeder(const FmLoaderApi* api, int device, long long vocab, bool hash)
      : api_(api), device_(device), vocab_(vocab), hash_(hash) {
    if (!api_ || api_->version != kFmLoaderApiVersion) throw std::invalid_argument("loader C API version mismatch");
  }
  ~GpuTextFeeder() { close(); }
  GpuTextFeeder(const GpuTextFeeder&) = delete;
  GpuTextFeeder& operator=(const GpuTextFeeder&) = delete;

  void add_slot(FeederSlot s) {
    if (!s.bytes || !s.ls || !s.labels || !s.offsets || !s.counts || !s.ids || !s.vals || !s.status || s.ls_cap < 2)
      throw std::invalid_argument("feeder slot: null buffer");
    hip_ok(hipSetDevice(device_), "hipSetDevice");
    hip_ok(hipEventCreateWithFlags(&s.ready, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventCreateWithFlags(&s.freed, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipHostMalloc(reinterpret_cast<void**>(&s.info_h), 8 * sizeof(int), hipHostMallocDefault), "hipHostMalloc");
    std::lock_guard<std::mutex> lk(mu_);
    slots_.push_back(s);
    free_.push_back(static_cast<int>(slots_.size()) - 1);
    cv_slot_.notify_one();
  }

  void start() {
    std::lock_guard<std::mutex> lk(mu_);
    if (th_.joinable() || closed_) return;
    // host-parsed / binary-cache batches are assembled straight into this feeder's page-locked
    // buffers (no staging copy on the feeder thread)
    pool_api_.ctx = this;
    pool_api_.acquire = &GpuTextFeeder::pin_acquire_cb;
    pool_api_.release = &GpuTextFeeder::pin_release_cb;
    api_->set_pinned_pool(api_->handle, &pool_api_);
    th_ = std::thread([this] { run(); });
  }

  // 1: *out is the next batch; 0: no more batches; -1: timed out while the producer waits for a
  // free slot (every slot is held by the consumer); -2: timed out; -3: failed (*err, *parse_err);
  // -4: slot out->d needs ids / vals of out->nnz entries (answer with resize_ids)
  int next(FeederBatch* out, int timeout_ms, std::string* err, bool* parse_err) {
    std::unique_lock<std::mutex> lk(mu_);
    const auto pred = [&] { return !ready_.empty() || done_ || resize_ask_; };
    if (timeout_ms < 0) {
      cv_ready_.wait(lk, pred);
    } else if (!cv_ready_.wait_for(lk, std::chrono::milliseconds(timeout_ms), pred)) {
      return starving_ ? -1 : -2;
    }
    if (resize_ask_) {
      resize_ask_ = false;
      out->d = resize_d_;
      out->nnz = resize_need_;
      return -4;
    }
    if (!ready_.empty()) {
      *out = ready_.front();
      ready_.pop_front();
      return 1;
    }
    if (failed_) {
      *err = error_;
      *parse_err = parse_error_;
      return -3;
    }
    return 0;
  }

  void release(int d, hipStream_t consumer) {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_ || d < 0 || d >= static_cast<int>(slots_.size())) return;
    for (int s : free_)
      if (s == d) throw std::logic_error("feeder slot released twice");
    hip_ok(hipSetDevice(device_), "hipSetDevice");
    hip_ok(hipEventRecord(slots_[d].freed, consumer), "hipEventRecord");
    free_.push_back(d);
    cv_slot_.notify_one();
  }

  // New ids / vals buffers (>= the requested entries) for the slot a -4 from next() named
  void resize_ids(int d, int* ids, float* vals, size_t cap) {
    std::lock_guard<std::mutex> lk(mu_);
    if (d != resize_d_ || !ids || !vals || static_cast<int64_t>(cap) < resize_need_)
      throw std::invalid_argument("feeder resize_ids: not the requested slot / size");
    slots_[d].ids = ids;
    slots_[d].vals = vals;
    slots_[d].ids_cap = cap;
    resize_d_ = -1;
    cv_slot_.notify_all();
  }

  size_t queued() {
    std::lock_guard<std::mutex> lk(mu_);
    return ready_.size();
  }
  long long fallbacks() const { return fallbacks_.load(); }
  long long resizes() const { return resizes_.load(); }
  long long batches() const { return batches_.load(); }

  void close() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (closed_) return;
      closed_ = stop_ = true;
    }
    cv_slot_.notify_all();
    cv_ready_.notify_all();
    {  // a loader thread waiting for a pinned buffer gets none (it falls back to its own memory)
      std::lock_guard<std::mutex> lk(pmu_);
      pclosed_ = true;
    }
    pcv_.notify_all();
    api_->set_pinned_pool(api_->handle, nullptr);
    // the thread may be blocked in the loader's next(): stop the loader first (joins its thread:
    // nothing writes the pinned buffers after this)
    api_->stop(api_->handle);
    if (th_.joinable()) th_.join();
    if (st_) {
      (void)hipStreamSynchronize(st_);
      (void)hipStreamDestroy(st_);
      st_ = nullptr;
    }
    for (int i = 0; i < 2; ++i) {
      if (pin_[i]) (void)hipHostFree(pin_[i]);
      if (pin_ev_[i]) (void)hipEventDestroy(pin_ev_[i]);
      pin_[i] = nullptr;
      pin_ev_[i] = nullptr;
      pin_cap_[i] = 0;
    }
    for (PinBuf& pb : pbufs_)
      if (pb.p) (void)hipHostFree(pb.p);
    pbufs_.clear();
    for (FeederSlot& s : slots_) {
      if (s.ready) (void)hipEventDestroy(s.ready);
      if (s.freed) (void)hipEventDestroy(s.freed);
      if (s.info_h) (void)hipHostFree(s.info_h);
      s.ready = s.freed = nullptr;
      s.info_h = nullptr;
    }
  }

 private:
  static void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
  }

  int acquire() {
    std::unique_lock<std::mutex> lk(mu_);
    starving_ = free_.empty();
    cv_slot_.wait(lk, [&] { return stop_ || !free_.empty(); });
    starving_ = false;
    if (stop_) return -1;
    const int d = free_.front();
    free_.pop_front();
    return d;
  }

  void give_back(int d) {
    std::lock_guard<std::mutex> lk(mu_);
    free_.push_front(d);
  }

  void publish(const FeederBatch& b) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      ready_.push_back(b);
    }
    batches_.fetch_add(1);
    cv_ready_.notify_one();
  }

  // Slot d (the thread's copy s) holds nnz features, asking the consumer for larger buffers
  // first; false when the feeder is stopped meanwhile
  bool fit_ids(int d, FeederSlot& s, int64_t nnz) {
    if (static_cast<size_t>(nnz) <= s.ids_cap) return true;
    std::unique_lock<std::mutex> lk(mu_);
    resize_d_ = d;
    resize_need_ = nnz;
    resize_ask_ = true;
    cv_ready_.notify_all();
    cv_slot_.wait(lk, [&] { return stop_ || resize_d_ < 0; });
    resize_ask_ = false;
    if (stop_) return false;
    s = slots_[d];
    resizes_.fetch_add(1);
    return static_cast<size_t>(nnz) <= s.ids_cap;
  }

  // Page-locked staging buffer i (of 2) of at least `bytes` (grown on demand; the thread's own).
  uint8_t* staging(int i, size_t bytes) {
    if (!pin_ev_[i]) hip_ok(hipEventCreateWithFlags(&pin_ev_[i], hipEventDisableTiming), "hipEventCreate");
    if (bytes > pin_cap_[i]) {
      if (pin_[i]) (void)hipHostFree(pin_[i]);
      pin_[i] = nullptr;
      pin_cap_[i] = 0;
      const size_t cap = bytes + bytes / 4;
      hip_ok(hipHostMalloc(reinterpret_cast<void**>(&pin_[i]), cap, hipHostMallocDefault), "hipHostMalloc");
      pin_cap_[i] = cap;
    }
    return pin_[i];
  }

  // The staged batch whose copies are queued: wait for them, then hand it to the consumer.
  void flush_pending() {
    if (!pend_on_) return;
    pend_on_ = false;
    hip_ok(hipEventSynchronize(pin_ev_[pend_buf_]), "hipEventSynchronize");
    if (pin_tag_[pend_buf_] >= 0) {  // its arrays were copied from a pool buffer: free it for the loader
      pin_release(pin_tag_[pend_buf_]);
      pin_tag_[pend_buf_] = -1;
    }
    publish(pend_b_);
  }

  // --- pinned output pool offered to the loader (loader_api.h FmPinnedPool) ---
  struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool busy = false;
  };
  static constexpr int kPinPoolMax = 16;  // (>= the loader's queue + the batch being built + 2 in flight)
  static void* pin_acquire_cb(void* ctx, size_t bytes, int32_t* tag) {
    return static_cast<GpuTextFeeder*>(ctx)->pin_acquire(bytes, tag);
  }
  static void pin_release_cb(void* ctx, int32_t tag) { static_cast<GpuTextFeeder*>(ctx)->pin_release(tag); }
  // Smallest idle buffer of >= bytes; else a NEW buffer while the pool has room (an idle smaller one
  // -- an epoch's short last batch -- is kept for later small batches), else an idle smaller one grown.
  // The page-locked allocation runs outside pmu_ (hipHostMalloc / hipHostFree can wait for device
  // work): the slot is reserved busy first.
  void* pin_acquire(size_t bytes, int32_t* tag) {
    std::unique_lock<std::mutex> lk(pmu_);
    for (;;) {
      if (pclosed_) return nullptr;
      int fit = -1, small = -1;
      for (size_t i = 0; i < pbufs_.size(); ++i) {
        if (pbufs_[i].busy) continue;
        if (pbufs_[i].cap >= bytes) {
          if (fit < 0 || pbufs_[i].cap < pbufs_[fit].cap) fit = static_cast<int>(i);
        } else if (small < 0) {
          small = static_cast<int>(i);
        }
      }
      if (fit >= 0) {
        pbufs_[fit].busy = true;
        *tag = fit;
        return pbufs_[fit].p;
      }
      int slot = -1;
      if (static_cast<int>(pbufs_.size()) < kPinPoolMax) {
        pbufs_.emplace_back();
        slot = static_cast<int>(pbufs_.size()) - 1;
      } else if (small >= 0) {
        slot = small;
      }
      if (slot < 0) {
        pcv_.wait_for(lk, std::chrono::milliseconds(100));
        continue;
      }
      pbufs_[slot].busy = true;  // (reserved: no other acquire takes it while it is reallocated)
      void* old = pbufs_[slot].p;
      pbufs_[slot].p = nullptr;
      pbufs_[slot].cap = 0;
      lk.unlock();
      (void)hipSetDevice(device_);
      if (old) (void)hipHostFree(old);
      const size_t cap = bytes + bytes / 8 + 4096;  // (room for a somewhat denser batch)
      void* p = nullptr;
      const bool ok = hipHostMalloc(&p, cap, hipHostMallocDefault) == hipSuccess;
      lk.lock();
      if (!ok) {
        pbufs_[slot].busy = false;  // (an empty idle slot: a later acquire allocates it again)
        pcv_.notify_one();
        return nullptr;  // (no page-locked memory: the loader uses its own)
      }
      pbufs_[slot].p = p;
      pbufs_[slot].cap = cap;
      *tag = slot;
      return p;
    }
  }
  void pin_release(int tag) {
    {
      std::lock_guard<std::mutex> lk(pmu_);
      if (tag >= 0 && tag < static_cast<int>(pbufs_.size())) pbufs_[tag].busy = false;
    }
    pcv_.notify_one();
  }

  // dst + offs[k] <- srcs[k] (bytes[k]) for the k with bytes: large arrays split over the copy pool
  void parallel_copy(uint8_t* dst, const size_t* offs, const void* const* srcs, const size_t* bytes, int n) {
    constexpr size_t kChunk = 1 << 20;
    constexpr int kThreads = 8;
    struct Piece { uint8_t* d; const uint8_t* s; size_t b; };
    std::vector<Piece> pieces;
    for (int k = 0; k < n; ++k)
      for (size_t o = 0; o < bytes[k]; o += kChunk)
        pieces.push_back({dst + offs[k] + o, static_cast<const uint8_t*>(srcs[k]) + o, std::min(kChunk, bytes[k] - o)});
    if (pieces.size() <= 1) {
      for (const Piece& p : pieces) std::memcpy(p.d, p.s, p.b);
      return;
    }
    if (!copy_pool_) copy_pool_ = std::make_unique<CopyPool>(kThreads);
    const int T = copy_pool_->size();
    copy_pool_->run([&](int t) {
      for (size_t i = t; i < pieces.size(); i += T) std::memcpy(pieces[i].d, pieces[i].s, pieces[i].b);
    });
  }

  void fail(const std::string& msg, bool parse) {
    std::lock_guard<std::mutex> lk(mu_);
    failed_ = true;
    parse_error_ = parse;
    error_ = msg;
  }

  // CPU parse of a raw batch (declined by the tokenizer, or larger than the slot) into slot d
  bool cpu_parse(int d, FeederSlot& s, const FmRawView& v, FeederBatch& b) {
    const int64_t n = v.nlines;
    if (static_cast<size_t>(n) + 1 > s.ls_cap) {
      fail("batch of " + std::to_string(n) + " lines exceeds the feeder's slots", false);
      return false;
    }
    const int64_t cap = static_cast<int64_t>(v.nbytes) / 2 + n + 1;
    h_labels_.resize(n);
    h_offsets_.resize(n + 1);
    h_ids_.resize(cap);
    h_vals_.resize(cap);
    FmParsedOut o{h_labels_.data(), h_offsets_.data(), h_ids_.data(), h_vals_.data(), cap, 0, 0, 0};
    char err[4096];
    err[0] = 0;
    const int r = api_->parse(api_->handle, &v, &o, err, sizeof(err));
    if (r != 0) {
      fail(r == -1 ? std::string(err) : std::string("CPU parse of a raw batch failed: ") + err, r == -1);
      return false;
    }
    if (!fit_ids(d, s, o.nnz)) {
      if (!stop_) fail("batch of " + std::to_string(o.nnz) + " features exceeds the feeder's slots", false);
      return false;
    }
    hip_ok(hipStreamWaitEvent(st_, s.freed, 0), "hipStreamWaitEvent");
    hip_ok(hipMemcpyAsync(s.labels, o.labels, 4 * n, hipMemcpyHostToDevice, st_), "H2D");
    hip_ok(hipMemcpyAsync(s.offsets, o.offsets, 4 * (n + 1), hipMemcpyHostToDevice, st_), "H2D");
    if (o.nnz > 0) hip_ok(hipMemcpyAsync(s.ids, o.ids, 4 * o.nnz, hipMemcpyHostToDevice, st_), "H2D");
    if (o.has_vals && o.nnz > 0) hip_ok(hipMemcpyAsync(s.vals, o.vals, 4 * o.nnz, hipMemcpyHostToDevice, st_), "H2D");
    if (v.weights && s.weights) hip_ok(hipMemcpyAsync(s.weights, v.weights, 4 * n, hipMemcpyHostToDevice, st_), "H2D");
    hip_ok(hipStreamSynchronize(st_), "hipStreamSynchronize");
    b.nnz = o.nnz;
    b.max_feats = o.max_feats;
    b.has_vals = o.has_vals != 0;
    fallbacks_.fetch_add(1);
    return true;
  }

  void run() {
    try {
      hip_ok(hipSetDevice(device_), "hipSetDevice");
      hip_ok(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
      char err[4096];
      while (true) {
        {  // a pending batch is published before the thread can block waiting for a free slot
          bool none;
          {
            std::lock_guard<std::mutex> lk(mu_);
            none = free_.empty();
          }
          if (none) flush_pending();
        }
        const int d = acquire();
        if (d < 0) break;
        FmRawView v{};
        err[0] = 0;
        const int r = api_->next(api_->handle, &v, err, sizeof(err));
        if (r <= 0) {
          give_back(d);
          if (r < 0) fail(err, r == -1);
          break;
        }
        FeederSlot s;
        {
          std::lock_guard<std::mutex> lk(mu_);
          s = slots_[d];
        }
        FeederBatch b;
        b.d = d;
        b.n = v.nlines;
        b.weighted = v.weights != nullptr;
        b.epoch = v.epoch;
        b.count = v.count;
        const int64_t n = v.nlines;
        const bool fits = static_cast<size_t>(v.nbytes) <= s.bytes_cap && static_cast<size_t>(n) + 1 <= s.ls_cap &&
                          n < (int64_t(1) << 31);
        bool ok = true, deferred = false;
        if (v.kind != 1) flush_pending();  // (keeps the batch order)
        if (v.kind == 1) {  // parsed on the host (CPU parser / binary cache): copy the CSR over
          if (static_cast<size_t>(n) + 1 > s.ls_cap) {
            fail("batch of " + std::to_string(n) + " lines exceeds the feeder's slots", false);
            ok = false;
          } else if (!fit_ids(d, s, v.nnz)) {
            if (!stop_) fail("batch of " + std::to_string(v.nnz) + " features exceeds the feeder's slots", false);
            ok = false;
          } else {
            // the loader's CSR is in pageable memory: gather it into the feeder's page-locked staging
            // buffer (parallel memcpy) and copy that with one DMA per array at full PCIe / xGMI rate
            // (pageable H2D copies ran the .fmb path at 1.3e7 ex/s, profiles/r4/e2e.txt)
            const int64_t nnz = v.nnz;
            const size_t parts[5] = {size_t(4 * n), size_t(4 * (n + 1)), size_t(4 * nnz),
                                     v.vals ? size_t(4 * nnz) : 0, (v.weights && s.weights) ? size_t(4 * n) : 0};
            const void* srcs[5] = {v.labels, v.offsets, v.ids, v.vals, v.weights};
            void* dsts[5] = {s.labels, s.offsets, s.ids, s.vals, s.weights};
            size_t offs[5], total = 0;
            for (int k = 0; k < 5; ++k) {
              offs[k] = total;
              total += (parts[k] + 255) / 256 * 256;
            }
            // two staging buffers: batch k's gather overlaps batch k-1's DMA, which is waited for (and
            // k-1 published) only after k's copies are queued
            if (!pin_ev_[pin_cur_])
              hip_ok(hipEventCreateWithFlags(&pin_ev_[pin_cur_], hipEventDisableTiming), "hipEventCreate");
            if (v.pinned >= 0) {  // assembled in one of this feeder's page-locked buffers: copy it directly
              hip_ok(hipStreamWaitEvent(st_, s.freed, 0), "hipStreamWaitEvent");
              for (int k = 0; k < 5; ++k)
                if (parts[k]) hip_ok(hipMemcpyAsync(dsts[k], srcs[k], parts[k], hipMemcpyHostToDevice, st_), "H2D");
              pin_tag_[pin_cur_] = v.pinned;  // (back to the pool once this copy has been waited for)
            } else {
              uint8_t* pin = staging(pin_cur_, total);  // (its previous DMA completed: flushed a batch ago)
              parallel_copy(pin, offs, srcs, parts, 5);
              hip_ok(hipStreamWaitEvent(st_, s.freed, 0), "hipStreamWaitEvent");
              for (int k = 0; k < 5; ++k)
                if (parts[k]) hip_ok(hipMemcpyAsync(dsts[k], pin + offs[k], parts[k], hipMemcpyHostToDevice, st_), "H2D");
            }
            hip_ok(hipEventRecord(pin_ev_[pin_cur_], st_), "hipEventRecord");
            deferred = true;
            b.nnz = v.nnz;
            b.max_feats = v.max_feats;
            b.has_vals = v.vals != nullptr;
          }
        } else if (n == 0) {
          b.nnz = 0;
          hip_ok(hipStreamWaitEvent(st_, s.freed, 0), "hipStreamWaitEvent");
          hip_ok(hipMemsetAsync(s.offsets, 0, sizeof(int), st_), "hipMemsetAsync");
          hip_ok(hipStreamSynchronize(st_), "hipStreamSynchronize");
        } else if (!fits) {
          ok = cpu_parse(d, s, v, b);
        } else {
          hip_ok(hipStreamWaitEvent(st_, s.freed, 0), "hipStreamWaitEvent");
          hip_ok(hipMemcpyAsync(s.bytes, v.bytes, v.nbytes, hipMemcpyHostToDevice, st_), "H2D");
          hip_ok(hipMemcpyAsync(s.ls, v.line_start, 8 * (n + 1), hipMemcpyHostToDevice, st_), "H2D");
          if (v.weights && s.weights)
            hip_ok(hipMemcpyAsync(s.weights, v.weights, 4 * n, hipMemcpyHostToDevice, st_), "H2D");
          ParseArgs a{};
          a.buf = reinterpret_cast<const char*>(s.bytes);
          a.line_start = reinterpret_cast<const long long*>(s.ls);
          a.n = static_cast<int>(n);
          a.vocab = vocab_;
          a.hash = hash_ ? 1 : 0;
          a.require_vals = 0;
          a.counts = s.counts;
          a.labels = s.labels;
          a.ids = s.ids;
          a.vals = s.vals;
          a.status = s.status;
          const int pr = launch_parse(a, s.ws, s.ws_bytes, s.offsets, st_);
          if (pr != 0) throw std::runtime_error("GPU tokenizer launch failed: " + std::to_string(pr));
          hip_ok(hipMemcpyAsync(s.info_h, s.status, 4 * sizeof(int), hipMemcpyDeviceToHost, st_), "D2H");
          hip_ok(hipMemcpyAsync(s.info_h + 4, s.offsets + n, sizeof(int), hipMemcpyDeviceToHost, st_), "D2H");
          hip_ok(hipEventRecord(s.ready, st_), "hipEventRecord");
          hip_ok(hipEventSynchronize(s.ready), "hipEventSynchronize");
          if (s.info_h[0]) {
            ok = cpu_parse(d, s, v, b);  // syntax outside the GPU subset, or an error to report exactly
          } else {
            b.nnz = s.info_h[4];
            b.max_feats = s.info_h[1];
            b.has_vals = s.info_h[2] != 0;
          }
        }
        api_->done(api_->handle, &v);  // the host bytes are on the device / staged (or parsed): back to the loader
        if (!ok) {
          flush_pending();
          give_back(d);
          break;
        }
        if (deferred) {  // publish the previous staged batch (its DMA ran before this one's), keep this one
          flush_pending();
          pend_b_ = b;
          pend_buf_ = pin_cur_;
          pend_on_ = true;
          pin_cur_ ^= 1;
        } else {
          publish(b);
        }
      }
      flush_pending();
    } catch (const std::exception& e) {
      fail(e.what(), false);
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      done_ = true;
    }
    cv_ready_.notify_all();
  }

  const FmLoaderApi* api_;
  int device_;
  long long vocab_;
  bool hash_;
  hipStream_t st_ = nullptr;
  std::deque<FeederSlot> slots_;  // (guarded by mu_; the thread works on copies)
  std::deque<int> free_;
  std::deque<FeederBatch> ready_;
  std::mutex mu_;
  std::condition_variable cv_slot_, cv_ready_;
  std::thread th_;
  std::unique_ptr<CopyPool> copy_pool_;  // (the feeder thread's staging copies)
  bool stop_ = false, closed_ = false, done_ = false, starving_ = false;
  bool failed_ = false, parse_error_ = false;
  std::string error_;
  int resize_d_ = -1;             // slot waiting for larger ids / vals (guarded by mu_)
  int64_t resize_need_ = 0;
  bool resize_ask_ = false;        // the request is not yet returned by next()
  std::atomic<long long> fallbacks_{0}, batches_{0}, resizes_{0};
  // page-locked staging of host-parsed batches (the thread's; double-buffered) and the batch whose
  // copies are queued but not yet waited for
  uint8_t* pin_[2] = {nullptr, nullptr};
  size_t pin_cap_[2] = {0, 0};
  hipEvent_t pin_ev_[2] = {nullptr, nullptr};
  int pin_cur_ = 0;
  int pin_tag_[2] = {-1, -1};     // pool buffer whose copies pin_ev_[i] marks (-1: staging)
  std::vector<PinBuf> pbufs_;     // (guarded by pmu_)
  std::mutex pmu_;
  std::condition_variable pcv_;
  bool pclosed_ = false;
  FmPinnedPool pool_api_{};
  bool pend_on_ = false;
  int pend_buf_ = 0;
  FeederBatch pend_b_;
  std::vector<float> h_labels_, h_vals_;
  std::vector<int32_t> h_offsets_, h_ids_;
};

}  // namespace fm
