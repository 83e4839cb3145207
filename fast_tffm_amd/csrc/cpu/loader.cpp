#include "loader.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <memory>
#include <random>
#include <stdexcept>

namespace fm {

namespace {

// Read-only mapping of a whole file (empty files map to nothing).
struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  explicit MappedFile(const std::string& path) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    struct stat st {};
    if (::fstat(fd, &st) != 0) {
      ::close(fd);
      throw std::runtime_error("cannot stat " + path);
    }
    size = static_cast<size_t>(st.st_size);
    if (size > 0) {
      void* p = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) {
        ::close(fd);
        throw std::runtime_error("cannot map " + path);
      }
      ::madvise(p, size, MADV_SEQUENTIAL);
      data = static_cast<const char*>(p);
    }
    ::close(fd);
  }
  ~MappedFile() {
    if (data) ::munmap(const_cast<char*>(data), size);
  }
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
};

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

struct Item {
  Span line, weight;
};

}  // namespace

TextLoader::TextLoader(LoaderOptions o) : o_(std::move(o)) {
  if (o_.batch_size < 1) throw std::invalid_argument("batch_size must be >= 1");
  if (!o_.weight_files.empty() && o_.weight_files.size() != o_.files.size())
    throw std::invalid_argument("The numbers of train files and weight files do not match.");
  if (o_.queue_size < 1) o_.queue_size = 1;
  th_ = std::thread([this] { run(); });
}

TextLoader::~TextLoader() { close(); }

void TextLoader::close() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_put_.notify_all();
  cv_get_.notify_all();
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
    const bool weighted = !o_.weight_files.empty();
    std::vector<Item> window;
    std::vector<const char*> ptrs, wptrs;
    std::vector<size_t> lens, wlens;
    std::vector<Span> lines, wlines;
    CsrBatch csr;
    ParseWorkspace pws;  // per-thread parse pieces, reused batch after batch

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
      size_t head = 0;  // FIFO start (no-shuffle mode)
      std::vector<std::unique_ptr<MappedFile>> maps;  // alive until the epoch's batches are parsed

      // Draw n items from the window into ptrs/lens (random when shuffling, FIFO otherwise)
      // and parse them unless the batch is skipped (resume).
      auto emit = [&](size_t n) -> bool {
        ++count;
        ptrs.clear(); lens.clear(); wptrs.clear(); wlens.clear();
        if (o_.shuffle) {
          const size_t w = window.size();
          for (size_t i = 0; i < n; ++i) {  // partial Fisher-Yates: a uniform sample moved to the back
            const size_t j = i + static_cast<size_t>(rng() % (w - i));
            std::swap(window[w - 1 - i], window[w - 1 - j]);
          }
          for (size_t i = 0; i < n; ++i) {
            const Item& it = window[w - n + i];
            ptrs.push_back(it.line.p); lens.push_back(it.line.len);
            wptrs.push_back(it.weight.p); wlens.push_back(it.weight.len);
          }
          window.resize(w - n);
        } else {
          for (size_t i = 0; i < n; ++i) {
            const Item& it = window[head + i];
            ptrs.push_back(it.line.p); lens.push_back(it.line.len);
            wptrs.push_back(it.weight.p); wlens.push_back(it.weight.len);
          }
          head += n;
          if (head > (1u << 20) && head * 2 > window.size()) {
            window.erase(window.begin(), window.begin() + static_cast<std::ptrdiff_t>(head));
            head = 0;
          }
        }
        if (count <= skip) return true;
        LoadedBatch b;
        if (o_.raw) {
          size_t total = 0;
          for (size_t i = 0; i < n; ++i) total += lens[i] + 1;
          b.bytes.resize(total);
          b.line_start.resize(n + 1);
          size_t off = 0;
          for (size_t i = 0; i < n; ++i) {
            b.line_start[i] = static_cast<int64_t>(off);
            std::memcpy(b.bytes.data() + off, ptrs[i], lens[i]);
            off += lens[i];
            b.bytes[off++] = '\n';
          }
          b.line_start[n] = static_cast<int64_t>(off);
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
        maps.push_back(std::make_unique<MappedFile>(o_.files[fi]));
        split_lines(*maps.back(), lines);
        if (weighted) {
          maps.push_back(std::make_unique<MappedFile>(o_.weight_files[fi]));
          split_lines(*maps.back(), wlines);
          if (wlines.size() != lines.size())
            throw std::runtime_error(o_.weight_files[fi] + ": " + std::to_string(wlines.size()) + " lines but " +
                                     o_.files[fi] + " has " + std::to_string(lines.size()));
        }
        const size_t step = line_shard ? static_cast<size_t>(o_.world) : 1;
        for (size_t i = line_shard ? static_cast<size_t>(o_.rank) : 0; i < lines.size(); i += step) {
          if (lines[i].len == 0) continue;
          window.push_back({lines[i], weighted ? wlines[i] : Span{nullptr, 0}});
          if (window.size() - head >= cap) {
            if (!emit(static_cast<size_t>(B))) return;
          }
        }
        {
          std::lock_guard<std::mutex> lk(mu_);
          if (stop_) return;
        }
      }
      while (window.size() > head) {
        if (!emit(std::min<size_t>(static_cast<size_t>(B), window.size() - head))) return;
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
