#include "loader.h"

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <memory>
#include <random>
#include <stdexcept>

#include "bincsr.h"
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

// A window entry of the text path: a line (+ its weight line).
struct Item {
  Span line, weight;
};

// A window entry of the binary path (16 bytes: the window is shuffled in place, so it
// pays to keep it small): global row (file rows concatenated in option order), its
// feature count and file index; the data is looked up only for the chosen rows.
struct BinItem {
  int64_t row;
  uint32_t len;
  uint32_t file;
};

// Take n entries from the window into `out`: a uniform sample moved to the back by a
// partial Fisher-Yates when shuffling, else the FIFO head.
template <class T, class R>
void draw(std::vector<T>& win, size_t& head, size_t n, bool shuffle, R& rng, std::vector<T>& out) {
  if (shuffle) {
    const size_t w = win.size();
    for (size_t i = 0; i < n; ++i) {
      const size_t j = i + static_cast<size_t>(rng() % (w - i));
      std::swap(win[w - 1 - i], win[w - 1 - j]);
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

// Copy n chosen binary examples into a CSR batch (offsets, ids, values, labels, weights)
// with up to `threads` threads; ids are range-checked on the way (a corrupt cache must
// not reach the device kernels as an out-of-bounds row).
void assemble_binary(const std::vector<BinItem>& its, const BinSet& bs, bool weighted, int64_t vocab, int threads,
                     LoadedBatch& b) {
  const size_t n = its.size();
  b.labels.resize(n);
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
  if (weighted) b.weights.resize(n);
  b.max_feats = mf;
  const size_t nnz = static_cast<size_t>(b.offsets[n]);
  b.ids.resize(nnz);
  if (any_vals) b.vals.resize(nnz);
  // >= 256k ids per thread; pointers hoisted so the copies are plain memcpy (no aliasing
  // through `b`), the range check runs over the thread's contiguous output afterwards
  const int T = std::max(1, std::min<int>(threads, static_cast<int>(nnz >> 18)));
  std::vector<char> bad(static_cast<size_t>(T), 0);
  int32_t* const ids_out = b.ids.data();
  float* const vals_out = any_vals ? b.vals.data() : nullptr;
  float* const lab_out = b.labels.data();
  float* const w_out = weighted ? b.weights.data() : nullptr;
  const int32_t* const offs = b.offsets.data();
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
  if (T == 1) {
    work(0);
  } else {
    std::vector<std::thread> ths;
    for (int t = 1; t < T; ++t) ths.emplace_back(work, t);
    work(0);
    for (auto& th : ths) th.join();
  }
  for (char x : bad)
    if (x) throw std::runtime_error("binary CSR cache holds a feature id outside [0, vocabulary_size)");
}

}  // namespace

TextLoader::TextLoader(LoaderOptions o) : o_(std::move(o)) {
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
    std::vector<Span> lines, wlines;
    CsrBatch csr;
    ParseWorkspace pws;  // per-thread parse pieces, reused batch after batch
    // Text files stay mapped and their line index is kept across epochs (up to kMaxCachedLines
    // lines in all): re-mapping and re-splitting every file each epoch (page-table faults +
    // a memchr pass over every byte) was most of the loader's per-batch host time.
    constexpr size_t kMaxCachedLines = size_t(64) << 20;
    size_t cached_lines = 0;
    std::vector<std::unique_ptr<MappedFile>> cmap(2 * nf);
    std::vector<std::vector<Span>> clines(2 * nf);
    auto file_lines = [&](size_t fi, bool weight, std::vector<std::unique_ptr<MappedFile>>& maps,
                          std::vector<Span>& scratch) -> const std::vector<Span>& {
      const size_t slot = 2 * fi + (weight ? 1 : 0);
      if (cmap[slot]) return clines[slot];
      auto m = std::make_unique<MappedFile>(weight ? o_.weight_files[fi] : o_.files[fi]);
      split_lines(*m, scratch);
      if (cached_lines + scratch.size() <= kMaxCachedLines) {
        cached_lines += scratch.size();
        clines[slot] = std::move(scratch);
        scratch = std::vector<Span>();
        cmap[slot] = std::move(m);
        return clines[slot];
      }
      maps.push_back(std::move(m));  // (alive until the epoch's batches are parsed)
      return scratch;
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
          if (o_.rows)
            emit_rows(bchosen, bs, b);
          else
            assemble_binary(bchosen, bs, weighted, o_.vocab_size, o_.threads, b);
          b.epoch = epoch;
          b.count = count;
          return push(std::move(b));
        }
        draw(window, head, n, o_.shuffle, rng, chosen);
        if (count <= skip) return true;
        ptrs.clear(); lens.clear(); wptrs.clear(); wlens.clear();
        for (const Item& it : chosen) {
          ptrs.push_back(it.line.p); lens.push_back(it.line.len);
          wptrs.push_back(it.weight.p); wlens.push_back(it.weight.len);
        }
        LoadedBatch b;
        if (o_.raw) {
          // offsets first, then the line copies in parallel (one thread copying ~15 MB of
          // 300-byte lines per 50k-line batch capped the GPU-tokenizer path near 1e7 ex/s);
          // into a caller's (pinned) slot when one is configured and the batch fits
          size_t total = 0;
          for (size_t i = 0; i < n; ++i) total += lens[i] + 1;
          int64_t* ls = nullptr;
          uint8_t* dst = nullptr;
          if (!o_.raw_slots.empty()) {
            const int s = acquire_slot();
            if (s < 0) return false;  // stopped
            const RawSlot& rs = o_.raw_slots[static_cast<size_t>(s)];
            if (total <= rs.bytes_cap && n + 1 <= rs.ls_cap) {
              b.slot = s;
              ls = rs.line_start;
              dst = rs.bytes;
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
          size_t off = 0;
          for (size_t i = 0; i < n; ++i) {
            ls[i] = static_cast<int64_t>(off);
            off += lens[i] + 1;
          }
          ls[n] = static_cast<int64_t>(off);
          b.nbytes = off;
          b.nlines = n;
#pragma omp parallel for num_threads(std::max(1, o_.threads)) schedule(static, 1024) if (n >= 4096)
          for (long long i = 0; i < (long long)n; ++i) {
            std::memcpy(dst + ls[i], ptrs[i], lens[i]);
            dst[ls[i] + lens[i]] = '\n';
          }
          if (weighted) {
            b.weights.resize(n);
            parse_floats(wptrs.data(), wlens.data(), n, b.weights.data());
          }
          b.epoch = epoch;
          b.count = count;
          return push(std::move(b));
        }
        parse_lines(ptrs.data(), lens.data(), ptrs.size(), o_.vocab_size, o_.hash_feature_id, o_.threads, csr,
                    &pws);
        const size_t nb = csr.labels.size(), nnz = csr.ids.size();
        b.labels = std::move(csr.labels);
        b.offsets.resize(nb + 1);
        b.offsets[0] = 0;
        int mf = 0;
        for (size_t i = 0; i < nb; ++i) {
          b.offsets[i + 1] = b.offsets[i] + csr.sizes[i];
          mf = std::max(mf, csr.sizes[i]);
        }
        b.max_feats = mf;
        b.ids.resize(nnz);
        for (size_t i = 0; i < nnz; ++i) b.ids[i] = static_cast<int32_t>(csr.ids[i]);  // ids < vocab < 2^31
        bool unit = true;
        for (size_t i = 0; i < nnz && unit; ++i) unit = csr.vals[i] == 1.f;
        if (!unit) b.vals = std::move(csr.vals);
        if (weighted) {
          b.weights.resize(nb);
          parse_floats(wptrs.data(), wlens.data(), nb, b.weights.data());
        }
        b.epoch = epoch;
        b.count = count;
        csr = CsrBatch();
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
        const std::vector<Span>& fl = file_lines(fi, false, maps, lines);
        const std::vector<Span>* wl = weighted ? &file_lines(fi, true, maps, wlines) : nullptr;
        if (wl && wl->size() != fl.size())
          throw std::runtime_error(o_.weight_files[fi] + ": " + std::to_string(wl->size()) + " lines but " +
                                   o_.files[fi] + " has " + std::to_string(fl.size()));
        const size_t step = line_shard ? static_cast<size_t>(o_.world) : 1;
        for (size_t i = line_shard ? static_cast<size_t>(o_.rank) : 0; i < fl.size(); i += step) {
          if (fl[i].len == 0) continue;
          window.push_back({fl[i], wl ? (*wl)[i] : Span{nullptr, 0}});
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
