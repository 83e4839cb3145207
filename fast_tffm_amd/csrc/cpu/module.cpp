// Python binding of the host-side native components
// (module fast_tffm_amd._native._fm_cpu): libsvm parser, TF-compatible
// Hash64, and the CPU step kernels.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <string>
#include <vector>

#include "../hash64.h"
#include "bincsr.h"
#include "kernels.h"
#include "loader.h"
#include "parser.h"

namespace py = pybind11;
using u64 = std::uintptr_t;

namespace {

template <typename T> T* P(u64 p) { return reinterpret_cast<T*>(p); }

template <typename T>
py::array_t<T> to_numpy(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete static_cast<std::vector<T>*>(p); });
  return py::array_t<T>({static_cast<py::ssize_t>(heap->size())}, {sizeof(T)}, heap->data(), owner);
}
template <class T>
py::array_t<T> to_numpy(fm::uvector<T>&& v) {
  auto* heap = new fm::uvector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete static_cast<fm::uvector<T>*>(p); });
  return py::array_t<T>({static_cast<py::ssize_t>(heap->size())}, {sizeof(T)}, heap->data(), owner);
}

// Collect (ptr, len) spans from a list of str/bytes, stripping one trailing
// "\n" (and a preceding "\r") like TF's TextLineReader.
void collect_spans(const py::sequence& lines, std::vector<const char*>& ptrs, std::vector<size_t>& lens) {
  const size_t n = py::len(lines);
  ptrs.resize(n);
  lens.resize(n);
  for (size_t i = 0; i < n; ++i) {
    PyObject* o = PyList_Check(lines.ptr()) ? PyList_GET_ITEM(lines.ptr(), i) : lines[i].ptr();
    const char* p = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_Check(o)) {
      char* q = nullptr;
      PyBytes_AsStringAndSize(o, &q, &len);
      p = q;
    } else if (PyUnicode_Check(o)) {
      p = PyUnicode_AsUTF8AndSize(o, &len);
      if (!p) throw py::error_already_set();
    } else {
      throw py::type_error("lines must be str or bytes");
    }
    if (len > 0 && p[len - 1] == '\n') --len;
    if (len > 0 && p[len - 1] == '\r') --len;
    ptrs[i] = p;
    lens[i] = static_cast<size_t>(len);
  }
}

py::tuple csr_to_py(fm::CsrBatch&& b) {
  return py::make_tuple(to_numpy(std::move(b.labels)), to_numpy(std::move(b.sizes)), to_numpy(std::move(b.ids)),
                        to_numpy(std::move(b.vals)));
}

fm::cpu::OptParams opt_params(int type, float lr, float l1, float l2, float beta) {
  return fm::cpu::OptParams{type, lr, l1, l2, beta};
}

}  // namespace

namespace {

// CRC-32C (Castagnoli), hardware crc32 instructions (SSE4.2) with a portable
// table fallback: checksums of TF tensor bundles and TensorBoard event records.
uint32_t crc32c_table(uint32_t crc, const uint8_t* p, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc32c_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}
#endif

uint32_t crc32c(const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (__builtin_cpu_supports("sse4.2")) return ~crc32c_hw(~0u, p, n);
#endif
  return ~crc32c_table(~0u, p, n);
}

}  // namespace

// Content hash of the sources / flags this module was built from (build_native.py); the
// marker string lets the loader check a shipped binary without importing it.
#ifndef FM_BUILD_HASH
#define FM_BUILD_HASH "unhashed"
#endif
extern "C" __attribute__((used, visibility("default"))) const char fm_build_hash_marker[] = "FMBUILDHASH:" FM_BUILD_HASH;

PYBIND11_MODULE(_fm_cpu, m) {
  m.attr("BUILD_HASH") = FM_BUILD_HASH;
  m.def(
      "crc32c",
      [](py::buffer b) {
        py::buffer_info info = b.request();
        const size_t n = (size_t)info.size * (size_t)info.itemsize;
        py::gil_scoped_release nogil;
        return crc32c(static_cast<const uint8_t*>(info.ptr), n);
      },
      py::arg("data"), "CRC-32C of a contiguous buffer");
  m.doc() = "host native components of fast_tffm_amd (parser, hash64, CPU step kernels)";
  py::register_exception<fm::ParseError>(m, "ParseError", PyExc_ValueError);

  m.def(
      "hash64",
      [](py::bytes s) {
        std::string v = s;
        return fm::hash64(v.data(), v.size());
      },
      py::arg("data"));

  m.def(
      "hash_bucket",
      [](const py::sequence& items, long long num_buckets) {
        std::vector<const char*> ptrs;
        std::vector<size_t> lens;
        collect_spans(items, ptrs, lens);
        std::vector<int64_t> out(ptrs.size());
        for (size_t i = 0; i < ptrs.size(); ++i)
          out[i] = static_cast<int64_t>(fm::hash64(ptrs[i], lens[i]) % static_cast<uint64_t>(num_buckets));
        return to_numpy(std::move(out));
      },
      py::arg("items"), py::arg("num_buckets"));

  m.def(
      "parse_lines",
      [](const py::sequence& lines, long long vocab_size, bool hash_feature_id, int threads) {
        std::vector<const char*> ptrs;
        std::vector<size_t> lens;
        collect_spans(lines, ptrs, lens);
        fm::CsrBatch b;
        {
          py::gil_scoped_release nogil;
          fm::parse_lines(ptrs.data(), lens.data(), ptrs.size(), vocab_size, hash_feature_id, threads, b);
        }
        return csr_to_py(std::move(b));
      },
      py::arg("lines"), py::arg("vocab_size"), py::arg("hash_feature_id") = false, py::arg("threads") = 1);

  // Parse every '\n'-terminated line of a byte buffer (a chunk of a file).
  m.def(
      "parse_buffer",
      [](py::buffer buf, long long vocab_size, bool hash_feature_id, int threads) {
        py::buffer_info info = buf.request();
        const char* data = static_cast<const char*>(info.ptr);
        const size_t size = static_cast<size_t>(info.size * info.itemsize);
        fm::CsrBatch b;
        {
          py::gil_scoped_release nogil;
          std::vector<const char*> ptrs;
          std::vector<size_t> lens;
          size_t s = 0;
          while (s < size) {
            const void* nl = std::memchr(data + s, '\n', size - s);
            size_t e = nl ? static_cast<size_t>(static_cast<const char*>(nl) - data) : size;
            size_t len = e - s;
            if (len > 0 && data[s + len - 1] == '\r') --len;
            ptrs.push_back(data + s);
            lens.push_back(len);
            s = e + 1;
          }
          fm::parse_lines(ptrs.data(), lens.data(), ptrs.size(), vocab_size, hash_feature_id, threads, b);
        }
        return csr_to_py(std::move(b));
      },
      py::arg("buffer"), py::arg("vocab_size"), py::arg("hash_feature_id") = false, py::arg("threads") = 1);

  // Native training-data loader (loader.h): mmap'ed files -> shuffle window -> parsed CSR batches.
  py::class_<fm::TextLoader>(m, "TextLoader")
      .def(py::init([](std::vector<std::string> files, std::vector<std::string> weight_files, long long batch_size,
                       long long vocab_size, bool hash_feature_id, bool shuffle, int num_epochs,
                       unsigned long long seed, int threads, int rank, int world, int queue_size, int start_epoch,
                       long long skip_batches, bool raw, bool binary, bool rows,
                       std::vector<std::vector<unsigned long long>> raw_slots) {
             fm::LoaderOptions o;
             o.files = std::move(files); o.weight_files = std::move(weight_files); o.batch_size = batch_size;
             o.vocab_size = vocab_size; o.hash_feature_id = hash_feature_id; o.shuffle = shuffle;
             o.num_epochs = num_epochs; o.seed = seed; o.threads = threads; o.rank = rank; o.world = world;
             o.queue_size = queue_size; o.start_epoch = start_epoch; o.skip_batches = skip_batches; o.raw = raw;
             o.binary = binary; o.rows = rows;
             for (const auto& s : raw_slots) {
               // [bytes ptr, bytes cap, line_start ptr, line_start entries (, weights ptr, weights cap)]
               if ((s.size() != 4 && s.size() != 6) || !s[0] || !s[2])
                 throw std::invalid_argument("raw slot: [bytes, cap, ls, cap(, weights, cap)]");
               fm::RawSlot r;
               r.bytes = reinterpret_cast<uint8_t*>(s[0]); r.bytes_cap = s[1];
               r.line_start = reinterpret_cast<int64_t*>(s[2]); r.ls_cap = s[3];
               if (s.size() == 6) {
                 r.weights = reinterpret_cast<float*>(s[4]); r.w_cap = s[5];
               }
               o.raw_slots.push_back(r);
             }
             return new fm::TextLoader(std::move(o));
           }),
           py::arg("files"), py::arg("weight_files"), py::arg("batch_size"), py::arg("vocab_size"),
           py::arg("hash_feature_id") = false, py::arg("shuffle") = true, py::arg("num_epochs") = 1,
           py::arg("seed") = 0, py::arg("threads") = 4, py::arg("rank") = 0, py::arg("world") = 1,
           py::arg("queue_size") = 4, py::arg("start_epoch") = 0, py::arg("skip_batches") = 0,
           py::arg("raw") = false, py::arg("binary") = false, py::arg("rows") = false,
           py::arg("raw_slots") = std::vector<std::vector<unsigned long long>>{})
      // -> (labels, offsets, ids, vals | None, weights | None, max_feats, epoch, count) or None at the end
      .def("next",
           [](fm::TextLoader& L) -> py::object {
             fm::LoadedBatch b;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = L.next(b);
             }
             if (!ok) return py::none();
             if (b.pinned >= 0)  // (a native consumer's pinned pool is set: that consumer reads the batches)
               throw std::runtime_error("TextLoader.next: the loader feeds a native consumer's pinned buffers");
             if (!b.rows.empty()) {  // rows mode: (rows, offsets, has_vals, max_feats, epoch, count)
               return py::make_tuple(to_numpy(std::move(b.rows)), to_numpy(std::move(b.offsets)), b.has_vals,
                                     b.max_feats, b.epoch, b.count);
             }
             if (b.slot >= 0) {  // raw mode into a slot: (slot, nbytes, nlines, weights | None, epoch, count)
               if (b.weights_in_slot) {
                 const float* sw = L.options().raw_slots[static_cast<size_t>(b.slot)].weights;
                 b.weights.assign(sw, sw + b.nlines);
               }
               py::object w = b.weights.empty() ? py::object(py::none()) : py::object(to_numpy(std::move(b.weights)));
               return py::make_tuple(b.slot, b.nbytes, b.nlines, w, b.epoch, b.count);
             }
             if (!b.line_start.empty()) {  // raw mode: (bytes, line_start, weights | None, epoch, count)
               py::object w = b.weights.empty() ? py::object(py::none()) : py::object(to_numpy(std::move(b.weights)));
               return py::make_tuple(to_numpy(std::move(b.bytes)), to_numpy(std::move(b.line_start)), w, b.epoch,
                                     b.count);
             }
             py::object vals = b.vals.empty() ? py::object(py::none()) : py::object(to_numpy(std::move(b.vals)));
             py::object w = b.weights.empty() ? py::object(py::none()) : py::object(to_numpy(std::move(b.weights)));
             return py::make_tuple(to_numpy(std::move(b.labels)), to_numpy(std::move(b.offsets)),
                                   to_numpy(std::move(b.ids)), vals, w, b.max_feats, b.epoch, b.count);
           })
      // address of the loader's C function table (loader_api.h) for the GPU feeder (_fm_hip)
      .def("c_api", [](fm::TextLoader& L) { return reinterpret_cast<std::uintptr_t>(L.c_api()); })
      .def("queued", &fm::TextLoader::queued)
      .def("release", &fm::TextLoader::release, py::arg("slot"))
      .def("window_fill", &fm::TextLoader::window_fill)
      .def("close", [](fm::TextLoader& L) {
        py::gil_scoped_release nogil;
        L.close();
      });

  // Binary CSR cache (bincsr.h): text (+ weight) file -> .fmb, and a magic check.
  m.def(
      "convert_to_bin",
      [](const std::string& text, const std::string& weights, const std::string& out, long long vocab_size,
         bool hash_feature_id, int threads, long long chunk_lines) {
        fm::ConvertStats st;
        {
          py::gil_scoped_release nogil;
          st = fm::convert_text_to_bin(text, weights, out, vocab_size, hash_feature_id, threads, chunk_lines);
        }
        py::dict d;
        d["examples"] = st.n;
        d["nnz"] = st.nnz;
        d["max_feats"] = st.max_feats;
        d["has_vals"] = st.has_vals;
        return d;
      },
      py::arg("text"), py::arg("weights"), py::arg("out"), py::arg("vocab_size"), py::arg("hash_feature_id") = false,
      py::arg("threads") = 4, py::arg("chunk_lines") = 1 << 20);
  m.def("is_bin_file", &fm::is_bin_file, py::arg("path"));

  m.def(
      "parse_floats",
      [](const py::sequence& lines) {
        std::vector<const char*> ptrs;
        std::vector<size_t> lens;
        collect_spans(lines, ptrs, lens);
        std::vector<float> out(ptrs.size());
        fm::parse_floats(ptrs.data(), lens.data(), ptrs.size(), out.data());
        return to_numpy(std::move(out));
      },
      py::arg("lines"));

  // ---- step kernels (raw host pointers) -----------------------------------
  m.def(
      "fwd",
      [](int B, u64 offsets, u64 rows, u64 vals, u64 v, long long v_stride, u64 w, long long w_stride, int Kp,
         int dtype, u64 labels, u64 weights, int loss_type, float grad_scale, u64 pred, u64 r1, u64 dpred,
         int threads, u64 bias) {
        fm::cpu::FwdResult r;
        {
          py::gil_scoped_release nogil;
          r = fm::cpu::fwd(B, P<const int>(offsets), P<const int>(rows), P<const float>(vals), P<const void>(v),
                           v_stride, P<const float>(w), w_stride, Kp, dtype, P<const float>(labels),
                           P<const float>(weights), loss_type, grad_scale, P<float>(pred), P<float>(r1),
                           P<float>(dpred), threads, P<const float>(bias));
        }
        return py::make_tuple(r.loss_sum, r.regv_sum, r.regw_sum);
      },
      py::arg("B"), py::arg("offsets"), py::arg("rows"), py::arg("vals"), py::arg("v"), py::arg("v_stride"),
      py::arg("w"), py::arg("w_stride"), py::arg("Kp"), py::arg("dtype"), py::arg("labels"), py::arg("weights"),
      py::arg("loss_type"), py::arg("grad_scale"), py::arg("pred"), py::arg("r1"), py::arg("dpred"),
      py::arg("threads"), py::arg("bias") = 0);

  m.def(
      "dedup",
      [](int n, u64 keys, u64 skeys, u64 perm, u64 uniq, u64 seg_start, u64 inv, u64 ex_of_occ, u64 sorted_ex,
         u64 vals, u64 sorted_x) {
        py::gil_scoped_release nogil;
        return fm::cpu::dedup(n, P<const uint32_t>(keys), P<uint32_t>(skeys), P<int>(perm), P<uint32_t>(uniq),
                              P<int>(seg_start), P<int>(inv), P<const int>(ex_of_occ), P<int>(sorted_ex),
                              P<const float>(vals), P<float>(sorted_x));
      },
      py::arg("n"), py::arg("keys"), py::arg("skeys"), py::arg("perm"), py::arg("uniq"), py::arg("seg_start"),
      py::arg("inv"), py::arg("ex_of_occ"), py::arg("sorted_ex"), py::arg("vals"), py::arg("sorted_x"));

  m.def(
      "bwd",
      [](int mode, int U, u64 seg_start, u64 uniq, u64 sorted_ex, u64 sorted_x, u64 dpred, u64 r1, int Kp, u64 v,
         long long v_stride, u64 w, long long w_stride, u64 s0v, u64 s1v, long long s_stride, u64 s0w, u64 s1w,
         float reg_v, float reg_w, int opt_type, float lr, float l1, float l2, float beta, u64 grad_out,
         long long g_stride, int dtype, int threads) {
        py::gil_scoped_release nogil;
        fm::cpu::bwd(mode, U, P<const int>(seg_start), P<const int>(uniq), P<const int>(sorted_ex),
                     P<const float>(sorted_x), P<const float>(dpred), P<const float>(r1), Kp, P<void>(v), v_stride,
                     P<float>(w), w_stride, P<float>(s0v), P<float>(s1v), s_stride, P<float>(s0w), P<float>(s1w),
                     reg_v, reg_w, opt_params(opt_type, lr, l1, l2, beta), P<float>(grad_out), g_stride, dtype,
                     threads);
      },
      py::arg("mode"), py::arg("U"), py::arg("seg_start"), py::arg("uniq"), py::arg("sorted_ex"),
      py::arg("sorted_x"), py::arg("dpred"), py::arg("r1"), py::arg("Kp"), py::arg("v"), py::arg("v_stride"),
      py::arg("w"), py::arg("w_stride"), py::arg("s0v"), py::arg("s1v"), py::arg("s_stride"), py::arg("s0w"),
      py::arg("s1w"), py::arg("reg_v"), py::arg("reg_w"), py::arg("opt_type"), py::arg("lr"), py::arg("l1"),
      py::arg("l2"), py::arg("beta"), py::arg("grad_out"), py::arg("g_stride"), py::arg("dtype"),
      py::arg("threads") = 0);

  m.def(
      "gather_rows",
      [](int R, u64 req, u64 v, long long v_stride, u64 w, long long w_stride, int Kp, int dtype, u64 out,
         long long o_stride, int threads) {
        py::gil_scoped_release nogil;
        fm::cpu::gather_rows(R, P<const int>(req), P<const void>(v), v_stride, P<const float>(w), w_stride, Kp,
                             dtype, P<float>(out), o_stride, threads);
      },
      py::arg("R"), py::arg("req"), py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"),
      py::arg("Kp"), py::arg("dtype"), py::arg("out"), py::arg("o_stride"), py::arg("threads") = 0);

  m.def(
      "apply_rows",
      [](int U, u64 seg_start, u64 uniq, u64 perm, u64 grad_in, long long g_stride, int Kp, u64 v,
         long long v_stride, u64 w, long long w_stride, u64 s0v, u64 s1v, long long s_stride, u64 s0w, u64 s1w,
         int opt_type, float lr, float l1, float l2, float beta, int dtype, int threads) {
        py::gil_scoped_release nogil;
        fm::cpu::apply_rows(U, P<const int>(seg_start), P<const int>(uniq), P<const int>(perm),
                            P<const float>(grad_in), g_stride, Kp, P<void>(v), v_stride, P<float>(w), w_stride,
                            P<float>(s0v), P<float>(s1v), s_stride, P<float>(s0w), P<float>(s1w),
                            opt_params(opt_type, lr, l1, l2, beta), dtype, threads);
      },
      py::arg("U"), py::arg("seg_start"), py::arg("uniq"), py::arg("perm"), py::arg("grad_in"), py::arg("g_stride"),
      py::arg("Kp"), py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"), py::arg("s0v"),
      py::arg("s1v"), py::arg("s_stride"), py::arg("s0w"), py::arg("s1w"), py::arg("opt_type"), py::arg("lr"),
      py::arg("l1"), py::arg("l2"), py::arg("beta"), py::arg("dtype"), py::arg("threads") = 0);

  m.def(
      "init_rows",
      [](u64 v, long long v_stride, u64 w, long long w_stride, long long rows, int K, int Kp, int dtype,
         long long gid_mul, long long gid_add, unsigned long long seed, float range, int threads) {
        py::gil_scoped_release nogil;
        fm::cpu::init_rows(P<void>(v), v_stride, P<float>(w), w_stride, rows, K, Kp, dtype, gid_mul, gid_add, seed,
                           range, threads);
      },
      py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"), py::arg("rows"), py::arg("K"),
      py::arg("Kp"), py::arg("dtype"), py::arg("gid_mul"), py::arg("gid_add"), py::arg("seed"), py::arg("range"),
      py::arg("threads") = 0);

  m.def(
      "csr_rows",
      [](int B, u64 offsets, u64 ex_of_occ) { fm::cpu::csr_rows(B, P<const int>(offsets), P<int>(ex_of_occ)); },
      py::arg("B"), py::arg("offsets"), py::arg("ex_of_occ"));
}
