#include "loader.h"

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <memory>
#include <omp.h>
#include <random>
#include <stdexcept>

#include "bincsr.h"

#include <functional>
#include "mapped_file.h"

namespace fm {

namespace {

struct Span {
  const char* p;
  uint32_t len;
};

// Lines of a buffer split at '\n' (a trailing '\r' is dropped, like the
// reference's TextLineReader); a final line without '\n' counts.
void split_lines(const MappedFile& f, std::vector<Span>& out) {
  out.clear();
  size_t s = 0;
  while (s < f.size) {
    const void* nl = std::memchr(f.data + s, '\n', f.size - s);
    const size_t e = nl ? static_cast<size_t>(static_cast<const char*>(nl) - f.data) : f.size;
    size_t len = e - s;
    if (len > 0 && f.data[s + len - 1] == '\r') --len;
    out.push_back({f.data + s, static_cast<uint32_t>(len)});
    s = e + 1;
  }
}

// A window entry of the text path (8 bytes: the window is shuffled in place, B random swaps per
// batch over 4.5 B entries, so it pays to keep it cache-sized): the line's file visit (index
// into the epoch's span tables) and its line number there; the spans are looked up only for the
// chosen lines, by the assembling threads.
struct Item {
  uint32_t f, l;
};

// A window entry of the binary path (16 bytes: the window is shuffled in place, so it
// pays to keep it small): global row (file rows concatenated in option order), its
// feature count and file index; the data is looked up only for the chosen rows.
struct BinItem {
  int64_t row;
  uint32_t len;
  uint32_t file;
};

// Uniform integer in [0, range) from one 64-bit draw (multiply-high, no division: the partial
// Fisher-Yates below takes one per drawn line, B per batch on the loader's single thread).
template <class R>
inline uint64_t bounded(R& rng, uint64_t range) {
  return static_cast<uint64_t>((static_cast<unsigned __int128>(rng()) * range) >> 64);
}

// Take n entries from the window into `out`: a uniform sample moved to the back by a
// partial Fisher-Yates when shuffling, else the FIFO head.
template <class T, class R>
void draw(std::vector<T>& win, size_t& head, size_t n, bool shuffle, R& rng, std::vector<T>& out) {
  if (shuffle) {
    // the swap partners first (the RNG stream does not depend on the data), then the swaps with
    // the random partner prefetched 16 swaps ahead: the window is larger than L2, and a swap
    // waiting on its cache miss was ~30 ns of the loader thread's serial time per drawn line
    const size_t w = win.size();
    thread_local std::vector<size_t> js;
    js.resize(n);
    for (size_t i = 0; i < n; ++i) js[i] = w - 1 - (i + static_cast<size_t>(bounded(rng, w - i)));
    constexpr size_t kAhead = 16;
    for (size_t i = 0; i < n; ++i) {
      if (i + kAhead < n) __builtin_prefetch(&win[js[i + kAhead]], 1);
      std::swap(win[w - 1 - i], win[js[i]]);
    }
    out.assign(win.end() - static_cast<std::ptrdiff_t>(n), win.end());
    win.resize(w - n);
  } else {
    out.assign(win.begin() + static_cast<std::ptrdiff_t>(head), win.begin() + static_cast<std::ptrdiff_t>(head + n));
    head += n;
    if (head > (1u << 20) && head * 2 > win.size()) {
      win.erase(win.begin(), win.begin() + static_cast<std::ptrdiff_t>(head));
      head = 0;
    }
  }
}

struct BinSet {
  std::vector<std::unique_ptr<BinFile>> files;
  std::vector<int64_t> base;  // first global row of each file
};

// rows mode: the batch's CSR offsets + global rows, the data stays where it is
void emit_rows(const std::vector<BinItem>& its, const BinSet& bs, LoadedBatch& b) {
  const size_t n = its.size();
  b.offsets.resize(n + 1);
  b.rows.resize(n);
  b.offsets[0] = 0;
  int mf = 0;
  bool vals = false;
  for (size_t i = 0; i < n; ++i) {
    const int c = static_cast<int>(its[i].len);
    b.offsets[i + 1] = b.offsets[i] + c;
    mf = std::max(mf, c);
    b.rows[i] = its[i].row;
    vals |= bs.files[its[i].file]->vals != nullptr;
  }
  b.max_feats = mf;
  b.has_vals = vals;
}

// Places of a kind-1 batch's arrays in one consumer-pinned buffer (256-byte aligned sections).
struct PinLayout {
  size_t labels, offsets, ids, vals, weights, total;
};
PinLayout pin_layout(size_t n, size_t nnz, bool vals, bool weights) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  PinLayout L{};
  size_t o = 0;
  L.labels = o; o += al(4 * n);
  L.offsets = o; o += al(4 * (n + 1));
  L.ids = o; o += al(4 * nnz);
  L.vals = o; o += vals ? al(4 * nnz) : 0;
  L.weights = o; o += weights ? al(4 * n) : 0;
  L.total = o;
  return L;
}

using PinAcquire = std::function<void*(size_t bytes, int32_t* tag)>;

// Point a batch's x_* arrays into a pinned buffer laid out by pin_layout.
void pin_batch(LoadedBatch& b, void* buf, int32_t tag, const PinLayout& L, size_t n, size_t nnz, bool vals,
               bool weights) {
  uint8_t* p = static_cast<uint8_t*>(buf);
  b.pinned = tag;
  b.x_labels = reinterpret_cast<float*>(p + L.labels);
  b.x_offsets = reinterpret_cast<int32_t*>(p + L.offsets);
  b.x_ids = reinterpret_cast<int32_t*>(p + L.ids);
  b.x_vals = vals ? reinterpret_cast<float*>(p + L.vals) : nullptr;
  b.x_weights = weights ? reinterpret_cast<float*>(p + L.weights) : nullptr;
  b.x_n = static_cast<int64_t>(n);
  b.x_nnz = static_cast<int64_t>(nnz);
}

// Copy n chosen binary examples into a CSR batch (offsets, ids, values, labels, weights)
// with up to `threads` threads -- into a consumer's pinned buffer when `pin` yields one (the
// host-to-device copy then needs no staging copy), else into the batch's vectors; ids are
// range-checked on the way (a corrupt cache must not reach the device kernels as an
// out-of-bounds row).
void assemble_binary(const std::vector<BinItem>& its, const BinSet& bs, bool weighted, int64_t vocab, int threads,
                     LoadedBatch& b, const PinAcquire& pin) {
  const size_t n = its.size();
  b.offsets.resize(n + 1);
  b.offsets[0] = 0;
  bool any_vals = false;
  int mf = 0;
  for (size_t i = 0; i < n; ++i) {
    const int c = static_cast<int>(its[i].len);
    b.offsets[i + 1] = b.offsets[i] + c;
    mf = std::max(mf, c);
    any_vals |= bs.files[its[i].file]->vals != nullptr;
  }
  b.max_feats = mf;
  const size_t nnz = static_cast<size_t>(b.offsets[n]);
  int32_t* ids_out;
  float *vals_out, *lab_out, *w_out;
  const int32_t* offs;
  const PinLayout PL = pin_layout(n, nnz, any_vals, weighted);
  int32_t tag = -1;
  void* buf = pin ? pin(PL.total, &tag) : nullptr;
  if (buf) {
    pin_batch(b, buf, tag, PL, n, nnz, any_vals, weighted);
    std::memcpy(b.x_offsets, b.offsets.data(), 4 * (n + 1));
    b.offsets.clear();
    ids_out = b.x_ids;
    vals_out = b.x_vals;
    lab_out = b.x_labels;
    w_out = b.x_weights;
    offs = b.x_offsets;
  } else {
    b.labels.resize(n);
    if (weighted) b.weights.resize(n);
    b.ids.resize(nnz);
    if (any_vals) b.vals.resize(nnz);
    ids_out = b.ids.data();
    vals_out = any_vals ? b.vals.data() : nullptr;
    lab_out = b.labels.data();
    w_out = weighted ? b.weights.data() : nullptr;
    offs = b.offsets.data();
  }
  // >= 64k ids per thread; pointers hoisted so the copies are plain memcpy (no aliasing
  // through `b`), the range check runs over the thread's contiguous output afterwards
  const int T = std::max(1, std::min<int>(threads, static_cast<int>(nnz >> 16)));
  std::vector<char> bad(static_cast<size_t>(T), 0);
  const BinItem* const items = its.data();
  const BinFile* const* const files = reinterpret_cast<const BinFile* const*>(bs.files.data());
  const int64_t* const base = bs.base.data();
  const uint32_t V = static_cast<uint32_t>(vocab);
  auto work = [=, &bad](int t) {
    const size_t i0 = n * t / T, i1 = n * (t + 1) / T;
    for (size_t i = i0; i < i1; ++i) {
      const BinItem& it = items[i];
      const BinFile& f = *files[it.file];
      const int64_t r = it.row - base[it.file];
      const int64_t o = f.offsets[r];
      std::memcpy(ids_out + offs[i], f.ids + o, 4 * static_cast<size_t>(it.len));
      lab_out[i] = f.labels[r];
      if (w_out) w_out[i] = f.weights ? f.weights[r] : 1.f;
      if (vals_out) {
        float* v = vals_out + offs[i];
        if (f.vals)
          std::memcpy(v, f.vals + o, 4 * static_cast<size_t>(it.len));
        else
          std::fill(v, v + it.len, 1.f);
      }
    }
    uint32_t any = 0;
    for (int32_t j = offs[i0]; j < offs[i1]; ++j) any |= static_cast<uint32_t>(ids_out[j]) >= V;
    bad[t] = any != 0;
  };
  // (the OpenMP team persists across batches: a std::thread per part per batch cost ~30 us each)
#pragma omp parallel for num_threads(T) schedule(static) if (T > 1)
  for (int t = 0; t < T; ++t) work(t);
  for (char x : bad)
    if (x) throw std::runtime_error("binary CSR cache holds a feature id outside [0, vocabulary_size)");
}

void copy_err(const char* msg, char* err, int errlen) {
  if (!err || errlen <= 0) return;
  std::strncpy(err, msg, static_cast<size_t>(errlen) - 1);
  err[errlen - 1] = 0;
}

// ---- C API (loader_api.h) ----
int api_next(void* h, FmRawView* v, char* err, int errlen) {
  TextLoader* L = static_cast<TextLoader*>(h);
  try {
    auto b = std::make_unique<LoadedBatch>();
    if (!L->next(*b)) return 0;
    v->kind = 0;
    v->slot = b->slot;
    v->epoch = b->epoch;
    v->count = b->count;
    v->max_feats = b->max_feats;
    v->labels = nullptr;
    v->offsets = nullptr;
    v->ids = nullptr;
    v->vals = nullptr;
    v->nnz = 0;
    v->pinned = b->pinned;
    if (b->slot >= 0) {
      const RawSlot& rs = L->options().raw_slots[static_cast<size_t>(b->slot)];
      v->bytes = rs.bytes;
      v->line_start = rs.line_start;
      v->nbytes = static_cast<int64_t>(b->nbytes);
      v->nlines = static_cast<int64_t>(b->nlines);
      v->weights = b->weights_in_slot ? rs.weights : (b->weights.empty() ? nullptr : b->weights.data());
    } else if (!b->line_start.empty()) {
      v->bytes = b->bytes.data();
      v->line_start = b->line_start.data();
      v->nbytes = static_cast<int64_t>(b->bytes.size());
      v->nlines = static_cast<int64_t>(b->line_start.size()) - 1;
      v->weights = b->weights.empty() ? nullptr : b->weights.data();
    } else if (b->pinned >= 0) {  // parsed / binary CSR in the consumer's pinned buffer
      v->kind = 1;
      v->bytes = nullptr;
      v->line_start = nullptr;
      v->nbytes = 0;
      v->nlines = b->x_n;
      v->labels = b->x_labels;
      v->offsets = b->x_offsets;
      v->ids = b->x_ids;
      v->vals = b->x_vals;
      v->nnz = b->x_nnz;
      v->weights = b->x_weights;
    } else if (b->rows.empty() && !b->offsets.empty()) {  // parsed / binary CSR
      v->kind = 1;
      v->bytes = nullptr;
      v->line_start = nullptr;
      v->nbytes = 0;
      v->nlines = static_cast<int64_t>(b->labels.size());
      v->labels = b->labels.data();
      v->offsets = b->offsets.data();
      v->ids = b->ids.data();
      v->vals = b->vals.empty() ? nullptr : b->vals.data();
      v->nnz = static_cast<int64_t>(b->ids.size());
      v->weights = b->weights.empty() ? nullptr : b->weights.data();
    } else {
      copy_err("row-number batches (device-resident caches) have no host data for the feeder", err, errlen);
      return -2;
    }
    v->owner = b.release();
    return 1;
  } catch (const ParseError& e) {
    copy_err(e.what(), err, errlen);
    return -1;
  } catch (const std::exception& e) {
    copy_err(e.what(), err, errlen);
    return -2;
  }
}

void api_done(void* h, FmRawView* v) {
  TextLoader* L = static_cast<TextLoader*>(h);
  LoadedBatch* b = static_cast<LoadedBatch*>(v->owner);
  if (!b) return;
  if (b->slot >= 0) {
    try {
      L->release(b->slot);
    } catch (const std::exception&) {
    }
  }
  L->recycle(*b);
  delete b;
  v->owner = nullptr;
}

}  // namespace

namespace {
constexpr size_t kPoolMax = 24;  // buffers of each element type kept for reuse
}

void TextLoader::recycle(LoadedBatch& b) {
  std::lock_guard<std::mutex> lk(pool_mu_);
  for (uvector<int32_t>* v : {&b.offsets, &b.ids})
    if (v->capacity() && pool_i32_.size() < kPoolMax) pool_i32_.push_back(std::move(*v));
  for (uvector<float>* v : {&b.labels, &b.vals, &b.weights})
    if (v->capacity() && pool_f32_.size() < kPoolMax) pool_f32_.push_back(std::move(*v));
}

template <class T>
void TextLoader::reuse(uvector<T>& v) {
  std::lock_guard<std::mutex> lk(pool_mu_);
  auto& pool = [this]() -> std::vector<uvector<T>>& {
    if constexpr (std::is_same<T, int32_t>::value) return pool_i32_;
    else return pool_f32_;
  }();
  if (pool.empty()) return;
  size_t best = 0;  // the largest buffer: batches are about the same size
  for (size_t i = 1; i < pool.size(); ++i)
    if (pool[i].capacity() > pool[best].capacity()) best = i;
  if (pool[best].capacity() <= v.capacity()) return;
  v.swap(pool[best]);
  v.clear();
  pool[best] = std::move(pool.back());
  pool.pop_back();
}
template void TextLoader::reuse<int32_t>(uvector<int32_t>&);
template void TextLoader::reuse<float>(uvector<float>&);

int TextLoader::api_parse(void* h, const FmRawView* v, FmParsedOut* out, char* err, int errlen) {
  TextLoader* L = static_cast<TextLoader*>(h);
  try {
    const int64_t n = v->nlines;
    std::vector<const char*> ptrs(static_cast<size_t>(n));
    std::vector<size_t> lens(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) {  // lines are '\n'-terminated in the raw buffer
      const int64_t s = v->line_start[i], e = v->line_start[i + 1];
      ptrs[i] = reinterpret_cast<const char*>(v->bytes) + s;
      lens[i] = static_cast<size_t>(e > s && v->bytes[e - 1] == '\n' ? e - s - 1 : e - s);
    }
    Csr32 c;
    parse_lines32(ptrs.data(), lens.data(), static_cast<size_t>(n), L->o_.vocab_size, L->o_.hash_feature_id,
                  L->o_.threads, c, &L->api_ws_);
    if (static_cast<int64_t>(c.ids.size()) > out->cap) return -3;
    std::memcpy(out->labels, c.labels.data(), 4 * c.labels.size());
    std::memcpy(out->offsets, c.offsets.data(), 4 * c.offsets.size());
    if (!c.ids.empty()) std::memcpy(out->ids, c.ids.data(), 4 * c.ids.size());
    if (c.has_vals && !c.vals.empty()) std::memcpy(out->vals, c.vals.data(), 4 * c.vals.size());
    out->nnz = static_cast<int64_t>(c.ids.size());
    out->max_feats = c.max_feats;
    out->has_vals = c.has_vals ? 1 : 0;
    return 0;
  } catch (const ParseError& e) {
    copy_err(e.what(), err, errlen);
    return -1;
  } catch (const std::exception& e) {
    copy_err(e.what(), err, errlen);
    return -2;
  }
}

TextLoader::TextLoader(LoaderOptions o) : o_(std::move(o)) {
  api_.version = kFmLoaderApiVersion;
  api_.handle = this;
  api_.next = &api_next;
  api_.done = &api_done;
  api_.parse = &TextLoader::api_parse;
  api_.stop = &TextLoader::api_stop;
  api_.set_pinned_pool = &TextLoader::api_set_pinned_pool;
  if (o_.batch_size < 1) throw std::invalid_argument("batch_size must be >= 1");
  if (!o_.weight_files.empty() && o_.weight_files.size() != o_.files.size())
    throw std::invalid_argument("The numbers of train files and weight files do not match.");
  if (o_.binary && !o_.weight_files.empty())
    throw std::invalid_argument("binary CSR caches carry their weights; pass no weight files");
  if (o_.binary && o_.raw) throw std::invalid_argument("raw (GPU tokenizer) mode needs text files");
  if (o_.rows && !o_.binary) throw std::invalid_argument("rows mode needs binary CSR caches");
  if (o_.queue_size < 1) o_.queue_size = 1;
  if (!o_.raw_slots.empty() && !o_.raw) throw std::invalid_argument("raw slots need raw mode");
  for (size_t s = 0; s < o_.raw_slots.size(); ++s) free_slots_.push_back(static_cast<int>(s));
  th_ = std::thread([this] { run(); });
}

int TextLoader::acquire_slot() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_slot_.wait(lk, [&] { return stop_ || !free_slots_.empty(); });
  if (stop_) return -1;
  const int s = free_slots_.front();
  free_slots_.pop_front();
  return s;
}

void TextLoader::release(int slot) {
  if (slot < 0 || slot >= static_cast<int>(o_.raw_slots.size())) throw std::out_of_range("raw slot");
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int s : free_slots_)
      if (s == slot) throw std::logic_error("raw slot released twice");
    free_slots_.push_back(slot);
  }
  cv_slot_.notify_one();
}

TextLoader::~TextLoader() { close(); }

void TextLoader::close() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_put_.notify_all();
  cv_get_.notify_all();
  cv_slot_.notify_all();
  if (th_.joinable()) th_.join();
}

size_t TextLoader::queued() {
  std::lock_guard<std::mutex> lk(mu_);
  return q_.size();
}

bool TextLoader::push(LoadedBatch&& b) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_put_.wait(lk, [&] { return stop_ || (int)q_.size() < o_.queue_size; });
  if (stop_) return false;
  q_.push_back(std::move(b));
  cv_get_.notify_one();
  return true;
}

bool TextLoader::next(LoadedBatch& out) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_get_.wait(lk, [&] { return !q_.empty() || done_ || stop_; });
  if (!q_.empty()) {
    out = std::move(q_.front());
    q_.pop_front();
    cv_put_.notify_one();
    return true;
  }
  if (failed_) {
    if (parse_error_) throw ParseError(error_);
    throw std::runtime_error(error_);
  }
  return false;
}

void TextLoader::run() {
  try {
    const int64_t B = o_.batch_size;
    const size_t cap = std::max<size_t>(static_cast<size_t>(o_.capacity_factor * static_cast<double>(B)), B);
    const size_t nf = o_.files.size();
    bool weighted = !o_.weight_files.empty();
    BinSet bs;  // binary: every cache mapped and validated once, for all epochs
    if (o_.binary && nf > 0) {  // every cache must match the model's id space and agree on weights
      bs.base.assign(nf + 1, 0);
      for (size_t i = 0; i < nf; ++i) {
        bs.files.push_back(std::make_unique<BinFile>(o_.files[i]));
        const BinFile& f = *bs.files.back();
        bs.base[i + 1] = bs.base[i] + f.h.n;
        if (f.h.vocab_size != o_.vocab_size || ((f.h.flags & kBinFlagHashed) != 0) != o_.hash_feature_id)
          throw std::runtime_error(o_.files[i] + ": converted with vocabulary_size " + std::to_string(f.h.vocab_size) +
                                   ", hash_feature_id " + ((f.h.flags & kBinFlagHashed) ? "True" : "False") +
                                   "; the model uses " + std::to_string(o_.vocab_size) + ", " +
                                   (o_.hash_feature_id ? "True" : "False"));
        const bool w = (f.h.flags & kBinFlagWeights) != 0;
        if (i == 0) weighted = w;
        if (w != weighted) throw std::runtime_error("binary CSR caches disagree on weights: " + o_.files[i]);
      }
    }
    std::vector<Item> window, chosen;
    std::vector<BinItem> bwindow, bchosen;
    std::vector<const char*> ptrs, wptrs;
    std::vector<size_t> lens, wlens;
    std::vector<Span> rline, rweight;
    Csr32 csr;
    Csr32Workspace pws;  // per-thread parse pieces, reused batch after batch
    // Text files stay mapped and their line index is kept across epochs (up to kMaxCachedLines
    // lines in all): re-mapping and re-splitting every file each epoch (page-table faults +
    // a memchr pass over every byte) was most of the loader's per-batch host time.
    constexpr size_t kMaxCachedLines = size_t(64) << 20;
    size_t cached_lines = 0;
    std::vector<std::unique_ptr<MappedFile>> cmap(2 * nf);
    std::vector<std::vector<Span>> clines(2 * nf);
    // (a file beyond the cache is mapped and split once per epoch; its spans live in `elines`
    // until the epoch's batches are built)
    auto file_lines = [&](size_t fi, bool weight, std::vector<std::unique_ptr<MappedFile>>& maps,
                          std::vector<std::vector<Span>>& elines) -> const std::vector<Span>& {
      const size_t slot = 2 * fi + (weight ? 1 : 0);
      if (cmap[slot]) return clines[slot];
      auto m = std::make_unique<MappedFile>(weight ? o_.weight_files[fi] : o_.files[fi]);
      std::vector<Span> sp;
      split_lines(*m, sp);
      if (cached_lines + sp.size() <= kMaxCachedLines) {
        cached_lines += sp.size();
        clines[slot] = std::move(sp);
        cmap[slot] = std::move(m);
        return clines[slot];
      }
      maps.push_back(std::move(m));
      elines.push_back(std::move(sp));
      return elines.back();
    };

    for (int epoch = o_.start_epoch; epoch < o_.num_epochs; ++epoch) {
      const int64_t skip = epoch == o_.start_epoch ? o_.skip_batches : 0;
      std::vector<size_t> order(nf);
      for (size_t i = 0; i < nf; ++i) order[i] = i;
      if (o_.shuffle) {
        std::mt19937_64 frng(o_.seed * 1000003ull + static_cast<uint64_t>(epoch));
        for (size_t i = nf; i > 1; --i) std::swap(order[i - 1], order[frng() % i]);
      }
      const bool line_shard = o_.world > 1 && nf < static_cast<size_t>(o_.world);
      if (o_.world > 1 && !line_shard) {
        std::vector<size_t> mine;
        for (size_t i = o_.rank; i < nf; i += o_.world) mine.push_back(order[i]);
        order.swap(mine);
      }
      std::mt19937_64 rng(o_.seed + 7919ull * static_cast<uint64_t>(o_.rank) +
                          0x9E3779B97F4A7C15ull * static_cast<uint64_t>(epoch + 1));
      int64_t count = 0;
      window.clear();
      bwindow.clear();
      size_t head = 0;  // FIFO start (no-shuffle mode)
      std::vector<std::unique_ptr<MappedFile>> maps;  // alive until the epoch's batches are parsed
      std::vector<std::vector<Span>> elines;          // spans of the files outside the cache
      elines.reserve(2 * nf);                         // (no reallocation: references stay valid)
      std::vector<const Span*> ftab, wtab;            // per file visit: its line / weight spans

      const PinAcquire pin_acquire = [this](size_t bytes, int32_t* tag) { return acquire_pinned(bytes, tag); };
      // Draw n items from the window (random when shuffling, FIFO otherwise) and build the
      // batch unless it is skipped (resume).
      auto emit = [&](size_t n) -> bool {
        ++count;
        const size_t in_win = (o_.binary ? bwindow.size() : window.size()) - (o_.shuffle ? 0 : head);
        fill_.store(std::min(1.f, static_cast<float>(in_win) / static_cast<float>(cap)), std::memory_order_relaxed);
        if (o_.binary) {
          draw(bwindow, head, n, o_.shuffle, rng, bchosen);
          if (count <= skip) return true;
          LoadedBatch b;
          if (o_.rows) {
            emit_rows(bchosen, bs, b);
          } else {
            reuse(b.offsets);
            if (!pinned_pool_.load(std::memory_order_acquire)) {
              reuse(b.labels); reuse(b.ids); reuse(b.vals);
              if (weighted) reuse(b.weights);
            }
            try {
              assemble_binary(bchosen, bs, weighted, o_.vocab_size, o_.threads, b, pin_acquire);
            } catch (...) {  // (an out-of-range id: the pinned buffer goes back before the error does)
              release_pinned(b.pinned);
              throw;
            }
          }
          b.epoch = epoch;
          b.count = count;
          return push(std::move(b));
        }
        draw(window, head, n, o_.shuffle, rng, chosen);
        if (count <= skip) return true;
        LoadedBatch b;
        // the chosen lines' spans, resolved by the thread team (random reads of the span tables)
        rline.resize(n);
        if (weighted) rweight.resize(n);
        {
          const Item* const ch = chosen.data();
          const Span* const* const ft = ftab.data();
          const Span* const* const wt = wtab.data();
          Span* const rl = rline.data();
          Span* const rw = weighted ? rweight.data() : nullptr;
#pragma omp parallel for num_threads(std::max(1, o_.threads)) schedule(static) if (n >= 8192)
          for (long long i = 0; i < (long long)n; ++i) {
            if (i + 16 < (long long)n) __builtin_prefetch(&ft[ch[i + 16].f][ch[i + 16].l]);
            rl[i] = ft[ch[i].f][ch[i].l];
            if (rw) rw[i] = wt[ch[i].f][ch[i].l];
          }
        }
        const Span* const rl = rline.data();
        const Span* const rw = weighted ? rweight.data() : nullptr;
        if (o_.raw) {
          // into a caller's (page-locked) slot when one is configured and the batch fits; the
          // line offsets, the copies and the weights are all built by the thread team (a serial
          // pass over 50k lines + strtof per weight line capped this path near 2e7 ex/s)
          size_t total = 0;
          for (size_t i = 0; i < n; ++i) total += rl[i].len + 1;
          int64_t* ls = nullptr;
          uint8_t* dst = nullptr;
          float* wdst = nullptr;
          if (!o_.raw_slots.empty()) {
            const int s = acquire_slot();
            if (s < 0) return false;  // stopped
            const RawSlot& rs = o_.raw_slots[static_cast<size_t>(s)];
            if (total <= rs.bytes_cap && n + 1 <= rs.ls_cap) {
              b.slot = s;
              ls = rs.line_start;
              dst = rs.bytes;
              if (weighted && rs.weights && n <= rs.w_cap) {
                wdst = rs.weights;
                b.weights_in_slot = true;
              }
            } else {
              release(s);
            }
          }
          if (b.slot < 0) {
            b.line_start.resize(n + 1);
            b.bytes.resize(total);
            ls = b.line_start.data();
            dst = b.bytes.data();
          }
          if (weighted && !wdst) {
            b.weights.resize(n);
            wdst = b.weights.data();
          }
          const int T = static_cast<int>(std::max<size_t>(1, std::min<size_t>(std::max(o_.threads, 1), n / 2048)));
          std::vector<size_t> part(static_cast<size_t>(T) + 1, 0);
          std::vector<size_t> werr(static_cast<size_t>(T), SIZE_MAX);
#pragma omp parallel num_threads(T)
          {
            const int t = omp_get_thread_num(), nt = omp_get_num_threads();
            const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
            size_t sum = 0;
            for (size_t i = i0; i < i1; ++i) sum += rl[i].len + 1;
            part[t + 1] = sum;
#pragma omp barrier
#pragma omp single
            for (int k = 0; k < nt; ++k) part[k + 1] += part[k];
            size_t off = part[t];
            for (size_t i = i0; i < i1; ++i) {
              if (i + 8 < i1) __builtin_prefetch(rl[i + 8].p);
              const uint32_t len = rl[i].len;
              ls[i] = static_cast<int64_t>(off);
              std::memcpy(dst + off, rl[i].p, len);
              dst[off + len] = '\n';
              off += len + 1;
            }
            if (wdst) {
              std::string scratch;
              for (size_t i = i0; i < i1; ++i) {
                try {
                  if (i + 8 < i1) __builtin_prefetch(rw[i + 8].p);
                  wdst[i] = parse_float_line(rw[i].p, rw[i].len, scratch);
                } catch (const ParseError&) {
                  werr[t] = i;
                  break;
                }
              }
            }
          }
          ls[n] = static_cast<int64_t>(total);
          for (size_t t = 0; t < werr.size(); ++t)
            if (werr[t] != SIZE_MAX) {  // the first bad weight line, with parse_floats' message
              std::string scratch;
              if (b.slot >= 0) release(b.slot);
              parse_float_line(rw[werr[t]].p, rw[werr[t]].len, scratch);
            }
          b.nbytes = total;
          b.nlines = n;
          b.epoch = epoch;
          b.count = count;
          return push(std::move(b));
        }
        ptrs.resize(n); lens.resize(n);
        for (size_t i = 0; i < n; ++i) {
          ptrs[i] = rl[i].p;
          lens[i] = rl[i].len;
        }
        const bool pool = pinned_pool_.load(std::memory_order_acquire) != nullptr;
        if (!pool) {
          reuse(csr.labels); reuse(csr.offsets); reuse(csr.ids); reuse(csr.vals);
        }
        // with a consumer pool the parser's pieces go straight into a pinned buffer (values and
        // weights sections reserved; the values are dropped from the view when all are 1)
        void* pbuf = nullptr;
        int32_t ptag = -1;
        PinLayout PL{};
        if (pool) {
          csr.ext = [&](size_t nn, size_t nz, float** l, int32_t** o, int32_t** ii, float** vv) {
            PL = pin_layout(nn, nz, true, weighted);
            pbuf = pin_acquire(PL.total, &ptag);
            if (!pbuf) return false;
            uint8_t* q = static_cast<uint8_t*>(pbuf);
            *l = reinterpret_cast<float*>(q + PL.labels);
            *o = reinterpret_cast<int32_t*>(q + PL.offsets);
            *ii = reinterpret_cast<int32_t*>(q + PL.ids);
            *vv = reinterpret_cast<float*>(q + PL.vals);
            return true;
          };
        }
        // (a parse / weight error after the pinned buffer was acquired gives it back before the error
        // propagates: the consumer's pool must not shrink by a failed batch)
        struct PinGuard {
          TextLoader* ld;
          const int32_t* tag;
          bool armed = true;
          ~PinGuard() {
            if (armed) ld->release_pinned(*tag);
          }
        } pin_guard{this, &ptag};
        parse_lines32(ptrs.data(), lens.data(), n, o_.vocab_size, o_.hash_feature_id, o_.threads, csr, &pws);
        float* wdst = nullptr;
        if (csr.in_ext) {
          const size_t nz = static_cast<size_t>(reinterpret_cast<int32_t*>(static_cast<uint8_t*>(pbuf) + PL.offsets)[n]);
          pin_batch(b, pbuf, ptag, PL, n, nz, csr.has_vals, weighted);
          wdst = b.x_weights;
        } else {
          b.labels = std::move(csr.labels);
          b.offsets = std::move(csr.offsets);
          b.ids = std::move(csr.ids);
          if (csr.has_vals) b.vals = std::move(csr.vals);
        }
        b.max_feats = csr.max_feats;
        if (weighted) {
          wptrs.resize(n); wlens.resize(n);
          for (size_t i = 0; i < n; ++i) {
            wptrs[i] = rw[i].p;
            wlens[i] = rw[i].len;
          }
          if (!wdst) {
            reuse(b.weights);
            b.weights.resize(n);
            wdst = b.weights.data();
          }
          parse_floats(wptrs.data(), wlens.data(), n, wdst, o_.threads);
        }
        b.epoch = epoch;
        b.count = count;
        csr = Csr32();
        pin_guard.armed = false;  // (the batch owns the buffer now: its consumer frees it)
        return push(std::move(b));
      };

      for (size_t fi : order) {
        if (o_.binary) {
          const BinFile& f = *bs.files[fi];
          const size_t step = line_shard ? static_cast<size_t>(o_.world) : 1;
          for (size_t i = line_shard ? static_cast<size_t>(o_.rank) : 0; i < static_cast<size_t>(f.h.n); i += step) {
            bwindow.push_back({bs.base[fi] + static_cast<int64_t>(i), static_cast<uint32_t>(f.offsets[i + 1] - f.offsets[i]),
                               static_cast<uint32_t>(fi)});
            if (bwindow.size() - head >= cap) {
              if (!emit(static_cast<size_t>(B))) return;
            }
          }
          std::lock_guard<std::mutex> lk(mu_);
          if (stop_) return;
          continue;
        }
        const std::vector<Span>& fl = file_lines(fi, false, maps, elines);
        const std::vector<Span>* wl = weighted ? &file_lines(fi, true, maps, elines) : nullptr;
        if (wl && wl->size() != fl.size())
          throw std::runtime_error(o_.weight_files[fi] + ": " + std::to_string(wl->size()) + " lines but " +
                                   o_.files[fi] + " has " + std::to_string(fl.size()));
        if (fl.size() >= (size_t(1) << 32)) throw std::runtime_error(o_.files[fi] + ": more than 2^32 lines");
        const uint32_t fid = static_cast<uint32_t>(ftab.size());
        ftab.push_back(fl.data());
        wtab.push_back(wl ? wl->data() : nullptr);
        const size_t step = line_shard ? static_cast<size_t>(o_.world) : 1;
        for (size_t i = line_shard ? static_cast<size_t>(o_.rank) : 0; i < fl.size(); i += step) {
          if (fl[i].len == 0) continue;
          window.push_back({fid, static_cast<uint32_t>(i)});
          if (window.size() - head >= cap) {
            if (!emit(static_cast<size_t>(B))) return;
          }
        }
        {
          std::lock_guard<std::mutex> lk(mu_);
          if (stop_) return;
        }
      }
      const auto left = [&] { return (o_.binary ? bwindow.size() : window.size()) - head; };
      while (left() > 0) {
        if (!emit(std::min<size_t>(static_cast<size_t>(B), left()))) return;
      }
    }
  } catch (const ParseError& e) {
    std::lock_guard<std::mutex> lk(mu_);
    failed_ = parse_error_ = true;
    error_ = e.what();
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> lk(mu_);
    failed_ = true;
    error_ = e.what();
  }
  std::lock_guard<std::mutex> lk(mu_);
  done_ = true;
  cv_get_.notify_all();
}

}  // namespace fm
