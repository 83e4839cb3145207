// Python binding of the gfx950 kernels (module fast_tffm_amd._native._fm_hip).
//
// The binding is deliberately thin: every entry point takes raw device
// pointers (Python ints from torch.Tensor.data_ptr()) and the HIP stream handle
// (torch.cuda.current_stream().cuda_stream), launches asynchronously and
// returns. Shape/dtype validation lives in fast_tffm_amd/ops/kernels.py; no
// libtorch headers are needed here, which keeps the gfx950 build small and
// lets the same kernels be called from torch streams, hipGraph captures and
// the C++ step executor alike.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdexcept>
#include <string>
#include "fm_common.h"

namespace py = pybind11;

#ifndef FM_HIP_MODULE
#define FM_HIP_MODULE _fm_hip
#endif
using u64 = std::uintptr_t;

// Unity build: all kernel sources are compiled in this translation unit.
#include "fm_bwd.hip"
#include "fm_fwd.hip"
#include "dedup.hip"
#include "shard.hip"
#include "init.hip"
#include "parse.hip"
#include "batch_gather.hip"
#include "feeder.hip"

namespace {

template <typename T> T* P(u64 p) { return reinterpret_cast<T*>(p); }
hipStream_t S(u64 s) { return reinterpret_cast<hipStream_t>(s); }

void check(int code, const char* what) {
  if (code != 0) {
    std::string msg = std::string(what) + " failed: ";
    msg += code > 0 ? hipGetErrorString(static_cast<hipError_t>(code)) : ("code " + std::to_string(code));
    throw std::runtime_error(msg);
  }
}

// Self rows (fm::SelfRows) arrive packed in one int64 list -- [u0, u1, base, keys, excl, v,
// v_stride, w, w_stride] -- or empty (off); the kernel entry points already take ~60
// arguments, past what pybind11's keyword dispatch handles comfortably.
fm::SelfRows self_rows(const std::vector<long long>& f) {
  fm::SelfRows r{};
  if (f.empty()) return r;
  if (f.size() != 9) throw std::invalid_argument("self_rows: [u0, u1, base, keys, excl, v, v_stride, w, w_stride]");
  if (f[1] > f[0] && (!f[3] || !f[5] || !f[7])) throw std::runtime_error("self rows need keys and the table");
  r.u0 = (int)f[0]; r.u1 = (int)(f[1] > f[0] ? f[1] : f[0]); r.base = f[2];
  r.keys = P<const int>((u64)f[3]); r.excl = P<const int>((u64)f[4]);
  r.v = P<const void>((u64)f[5]); r.v_stride = f[6]; r.w = P<float>((u64)f[7]); r.w_stride = f[8];
  return r;
}

fm::OptParams opt_params(int type, float lr, float l1, float l2, float beta) {
  fm::OptParams o;
  o.type = type; o.lr = lr; o.l1 = l1; o.l2 = l2; o.beta = beta;
  return o;
}

}  // namespace

// Content hash of the sources / flags this module was built from (build_native.py); the
// marker string lets the loader check a shipped binary without importing it.
#ifndef FM_BUILD_HASH
#define FM_BUILD_HASH "unhashed"
#endif
extern "C" __attribute__((used, visibility("default"))) const char fm_build_hash_marker[] = "FMBUILDHASH:" FM_BUILD_HASH;

PYBIND11_MODULE(FM_HIP_MODULE, m) {
  m.doc() = "gfx950 HIP kernels for fast_tffm_amd (FM forward/backward/optimizer, dedup, sharding)";
  m.attr("ARCH") = "gfx950";
  m.attr("BUILD_HASH") = FM_BUILD_HASH;
  m.attr("MAX_CH") = fm::kMaxCH;

  m.def("fwd_grid", &fm::fwd_grid, py::arg("B"));
  m.def("fwd_mfma_enabled", &fm::fwd_mfma_enabled);
  m.def("set_fwd_mfma", &fm::set_fwd_mfma, py::arg("on"));
#if FM_MF_PROF
  m.def("mf_prof", [] {  // (build variant "mfprof") phase clocks of the MFMA forward, then cleared
    unsigned long long h[8] = {};
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(h, HIP_SYMBOL(fm::g_mf_prof), sizeof(h));
    const unsigned long long z[8] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(fm::g_mf_prof), z, sizeof(z));
    return std::vector<unsigned long long>(h, h + 8);
  });
#endif
  m.def("lanes_per_row", &fm::lanes_per_row, py::arg("Kp"), py::arg("dtype"));

  m.def(
      "fwd",
      [](int B, u64 offsets, u64 rows, u64 vals, u64 v, long long v_stride, u64 w, long long w_stride, int Kp,
         int dtype, u64 labels, u64 weights, int loss_type, float grad_scale, u64 pred, u64 r1, u64 dpred,
         u64 loss_partial, u64 reg_partial, int grid, u64 stream, u64 bias, const std::vector<long long>& self,
         u64 seg_idx, u64 seg_keys, int seg_shift, int max_feats) {
        fm::FwdArgs a{};
        a.max_feats = max_feats;
        a.seg_idx = P<const int>(seg_idx); a.seg_keys = P<const int>(seg_keys); a.seg_shift = seg_shift;
        if (a.seg_idx && (!a.seg_keys || seg_shift < 0 || seg_shift > 31))
          throw std::invalid_argument("fm_fwd: segment lookup needs the sorted keys and a shift in [0, 31]");
        a.self = self_rows(self);
        a.B = B; a.offsets = P<const int>(offsets); a.rows = P<const int>(rows);
        a.vals = P<const float>(vals); a.v = P<const void>(v); a.v_stride = v_stride;
        a.w = P<const float>(w); a.w_stride = w_stride; a.Kp = Kp;
        a.labels = P<const float>(labels); a.weights = P<const float>(weights);
        a.loss_type = loss_type; a.grad_scale = grad_scale; a.pred = P<float>(pred);
        a.r1 = P<void>(r1); a.dpred = P<float>(dpred); a.loss_partial = P<float>(loss_partial);
        a.reg_partial = P<float>(reg_partial); a.bias = P<const float>(bias);
        check(fm::launch_fwd(a, dtype, grid, S(stream)), "fm_fwd");
      },
      py::arg("B"), py::arg("offsets"), py::arg("rows"), py::arg("vals"), py::arg("v"), py::arg("v_stride"),
      py::arg("w"), py::arg("w_stride"), py::arg("Kp"), py::arg("dtype"), py::arg("labels"), py::arg("weights"),
      py::arg("loss_type"), py::arg("grad_scale"), py::arg("pred"), py::arg("r1"), py::arg("dpred"),
      py::arg("loss_partial"), py::arg("reg_partial"), py::arg("grid"), py::arg("stream"), py::arg("bias") = 0,
      py::arg("self_rows") = std::vector<long long>{}, py::arg("seg_idx") = 0, py::arg("seg_keys") = 0,
      py::arg("seg_shift") = 0, py::arg("max_feats") = -1);

  m.def(
      "seg_index",
      [](int n_max, u64 uniq, u64 counts, int shift, int nb, u64 idx, u64 stream) {
        check(fm::launch_seg_index(n_max, P<const uint32_t>(uniq), P<const int>(counts), shift, nb, P<int>(idx),
                                   S(stream)),
              "seg_index");
      },
      py::arg("n_max"), py::arg("uniq"), py::arg("counts"), py::arg("shift"), py::arg("nb"), py::arg("idx"),
      py::arg("stream"));

  m.def(
      "bwd",
      [](int mode, u64 counts, u64 chunk_start, u64 chunk_seg, u64 chunk_key, u64 seg_start, u64 seg_chunk, u64 uniq,
         u64 sorted_ex, int ex_shift, u64 sorted_x, u64 dpred, u64 r1, int Kp, u64 v, long long v_stride, u64 w,
         long long w_stride, u64 s0v, u64 s1v, long long s_stride, u64 s0w, u64 s1w, float reg_v, float reg_w,
         int opt_type, float lr, float l1, float l2, float beta, u64 grad_out, long long g_stride, u64 partial,
         u64 big_list, u64 big_count, u64 multi, int nex, int dtype,
         long long max_chunks, long long max_unique, u64 stream, int g_wcol, int g_bf16, u64 sr_counter,
         int counters_ready, u64 seg_bounds, int piece, int n_owners,
         const std::vector<long long>& self) {
        fm::BwdArgs a{};
        a.self = self_rows(self);
        if (a.self.u1 > a.self.u0 && a.self.keys != P<const int>(uniq))
          throw std::runtime_error("fm_bwd: self-row keys must be the dedup's unique keys");
        if (a.self.u1 > a.self.u0 && (mode != 1 || !s0v || !s0w))
          throw std::runtime_error("fm_bwd: self rows are an EMIT-mode path and need the table's optimizer state");
        a.counters_ready = counters_ready;
        a.seg_bounds = P<const int>(seg_bounds); a.piece = piece; a.n_owners = n_owners;
        a.sr_counter = P<const int>(sr_counter);
        a.mode = mode; a.counts = P<const int>(counts); a.chunk_start = P<const int>(chunk_start);
        a.chunk_seg = P<const int>(chunk_seg); a.chunk_key = P<const int>(chunk_key);
        a.seg_start = P<const int>(seg_start);
        a.seg_chunk = P<const int>(seg_chunk); a.uniq = P<const int>(uniq);
        a.sorted_ex = P<const int>(sorted_ex); a.ex_shift = ex_shift; a.sorted_x = P<const float>(sorted_x);
        a.dpred = P<const float>(dpred); a.r1 = P<const void>(r1); a.Kp = Kp;
        a.v = P<void>(v); a.v_stride = v_stride; a.w = P<float>(w); a.w_stride = w_stride;
        a.s0v = P<void>(s0v); a.s1v = P<void>(s1v); a.s_stride = s_stride; a.s0w = P<float>(s0w);
        a.s1w = P<float>(s1w); a.reg_v = reg_v; a.reg_w = reg_w;
        a.opt = opt_params(opt_type, lr, l1, l2, beta);
        a.grad_out = P<float>(grad_out); a.g_stride = g_stride; a.g_wcol = g_wcol < 0 ? Kp : g_wcol;
        a.g_bf16 = g_bf16; a.partial = P<float>(partial);
        a.big_list = P<int>(big_list); a.big_count = P<int>(big_count); a.multi = P<int>(multi);
        a.counts_rw = P<int>(counts);
        a.nex = nex;
        check(fm::launch_bwd(a, dtype, max_chunks, max_unique, S(stream)), "fm_bwd");
      },
      py::arg("mode"), py::arg("counts"), py::arg("chunk_start"), py::arg("chunk_seg"), py::arg("chunk_key"),
      py::arg("seg_start"),
      py::arg("seg_chunk"), py::arg("uniq"), py::arg("sorted_ex"), py::arg("ex_shift"), py::arg("sorted_x"), py::arg("dpred"),
      py::arg("r1"), py::arg("Kp"), py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"),
      py::arg("s0v"), py::arg("s1v"), py::arg("s_stride"), py::arg("s0w"), py::arg("s1w"), py::arg("reg_v"),
      py::arg("reg_w"), py::arg("opt_type"), py::arg("lr"), py::arg("l1"), py::arg("l2"), py::arg("beta"),
      py::arg("grad_out"), py::arg("g_stride"), py::arg("partial"), py::arg("big_list"), py::arg("big_count"),
      py::arg("multi"), py::arg("nex"), py::arg("dtype"),
      py::arg("max_chunks"), py::arg("max_unique"), py::arg("stream"), py::arg("g_wcol") = -1,
      py::arg("g_bf16") = 0, py::arg("sr_counter") = 0, py::arg("counters_ready") = 0, py::arg("seg_bounds") = 0,
      py::arg("piece") = -1, py::arg("n_owners") = 0,
      py::arg("self_rows") = std::vector<long long>{});

  m.def("dedup_workspace_bytes", &fm::dedup_workspace_bytes, py::arg("n"));
  m.def("set_sort_algo", &fm::set_sort_algo, py::arg("in_tree"));  // 1: radix_sort.hip, 0: rocPRIM onesweep
  m.def("sort_algo", &fm::sort_algo);
  m.def(
      "radix_sort",  // stable (key, value) sort of the in-tree backend (tests / benchmarks; synchronous:
                     // the look-back error word is checked)
      [](u64 keys, u64 vals, u64 kout, u64 vout, int n, int end_bit, u64 ws, size_t ws_bytes, u64 stream) {
        check(fm::launch_radix_sort(P<const uint32_t>(keys), P<const int>(vals), P<uint32_t>(kout), P<int>(vout), n,
                                    end_bit, P<void>(ws), ws_bytes, S(stream)),
              "radix_sort");
        if (n <= 0) return;
        int err = 0;
        check((int)hipMemcpyAsync(&err, fm::radix_sort_error(P<void>(ws), n), sizeof(int), hipMemcpyDeviceToHost,
                                  S(stream)),
              "radix_sort error word");
        check((int)hipStreamSynchronize(S(stream)), "radix_sort sync");
        if (err) throw std::runtime_error("radix_sort: look-back spin bound hit");
      },
      py::arg("keys"), py::arg("vals"), py::arg("kout"), py::arg("vout"), py::arg("n"), py::arg("end_bit"),
      py::arg("ws"), py::arg("ws_bytes"), py::arg("stream"));
  m.def("radix_sort_ws_bytes", &fm::radix_sort_ws_bytes, py::arg("n"));
  m.def("bwd_wide_launches", &fm::bwd_wide_launches);  // launches of the wide fp8 chunk kernel so far
  m.def("set_sort_spin_cap", &fm::set_sort_spin_cap, py::arg("cap"));  // (< 0: injected look-back failure)
  m.def(
      "device_errors",  // the current device's sticky error word (synchronous), cleared when `clear`
      [](bool clear) {
        int v = 0;
        check((int)hipDeviceSynchronize(), "device_errors sync");
        check((int)hipMemcpyFromSymbol(&v, HIP_SYMBOL(fm::g_fm_dev_error), sizeof(int)), "device_errors read");
        if (clear && v) {
          const int z = 0;
          check((int)hipMemcpyToSymbol(HIP_SYMBOL(fm::g_fm_dev_error), &z, sizeof(int)), "device_errors clear");
        }
        return v;
      },
      py::arg("clear") = false);
  m.def(
      "dedup",
      [](int n, int end_bit, int CH, u64 keys, u64 payload, u64 skeys, u64 spay, u64 uniq, u64 seg_start,
         u64 seg_chunk, u64 chunk_start, u64 chunk_seg, u64 chunk_key, u64 counts, u64 inv, u64 ex_of_occ,
         u64 sorted_ex, u64 vals, u64 sorted_x, int payload_is_ex, int ex_shift, u64 offsets, u64 ws,
         size_t ws_bytes, u64 stream, u64 ids, int kW, int kRps, int gen_codes, int B) {
        if (CH < 1 || CH > fm::kMaxCH) throw std::invalid_argument("CH must be in [1, MAX_CH]");
        fm::DedupArgs a;
        a.n = n; a.end_bit = end_bit; a.CH = CH; a.keys = P<const uint32_t>(keys);
        a.payload = P<const int>(payload); a.skeys = P<uint32_t>(skeys); a.spay = P<int>(spay);
        a.uniq = P<uint32_t>(uniq); a.seg_start = P<int>(seg_start); a.seg_chunk = P<int>(seg_chunk);
        a.chunk_start = P<int>(chunk_start); a.chunk_seg = P<int>(chunk_seg); a.counts = P<int>(counts);
        a.chunk_key = P<int>(chunk_key);
        a.inv = P<int>(inv); a.ex_of_occ = P<const int>(ex_of_occ); a.sorted_ex = P<int>(sorted_ex);
        a.vals = P<const float>(vals); a.sorted_x = P<float>(sorted_x); a.ws = P<void>(ws);
        a.payload_is_ex = payload_is_ex; a.ex_shift = ex_shift; a.offsets = P<const int>(offsets);
        a.ws_bytes = ws_bytes;
        a.ids = P<const int>(ids); a.kW = kW; a.kRps = kRps; a.gen_codes = gen_codes; a.B = B;
        check(fm::launch_dedup(a, S(stream)), "dedup");
      },
      py::arg("n"), py::arg("end_bit"), py::arg("CH"), py::arg("keys"), py::arg("payload"), py::arg("skeys"),
      py::arg("spay"), py::arg("uniq"), py::arg("seg_start"), py::arg("seg_chunk"), py::arg("chunk_start"),
      py::arg("chunk_seg"), py::arg("chunk_key"), py::arg("counts"), py::arg("inv"), py::arg("ex_of_occ"),
      py::arg("sorted_ex"),
      py::arg("vals"), py::arg("sorted_x"), py::arg("payload_is_ex"), py::arg("ex_shift"), py::arg("offsets"),
      py::arg("ws"), py::arg("ws_bytes"), py::arg("stream"), py::arg("ids") = 0, py::arg("kW") = 1,
      py::arg("kRps") = 0, py::arg("gen_codes") = 0, py::arg("B") = 0);

  m.def(
      "gather_rows",
      [](int R, u64 req, u64 v, long long v_stride, u64 w, long long w_stride, int Kp, int dtype, u64 out,
         long long o_stride, u64 stream, int skip0, int skip1) {
        fm::GatherArgs a;
        a.skip0 = skip0; a.skip1 = skip1;
        a.R = R; a.req = P<const int>(req); a.v = P<const void>(v); a.v_stride = v_stride;
        a.w = P<const float>(w); a.w_stride = w_stride; a.Kp = Kp; a.out = P<float>(out); a.o_stride = o_stride;
        check(fm::launch_gather_rows(a, dtype, S(stream)), "gather_rows");
      },
      py::arg("R"), py::arg("req"), py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"),
      py::arg("Kp"), py::arg("dtype"), py::arg("out"), py::arg("o_stride"), py::arg("stream"), py::arg("skip0") = 0,
      py::arg("skip1") = 0);

  m.def(
      "gather_wire",
      [](int R, u64 req, u64 v, long long v_bytes_stride, u64 w, long long w_stride, int vbytes, int scaled,
         int to_bf16, u64 out, long long rb, int vb, u64 stream, u64 idx, u64 run_off, int W, int skip0, int skip1) {
        fm::GatherWireArgs a{};
        a.skip0 = skip0; a.skip1 = skip1;
        a.idx = P<const int>(idx); a.run_off = P<const int>(run_off); a.W = W;
        a.R = R; a.req = P<const int>(req); a.v = P<const void>(v); a.v_bytes_stride = v_bytes_stride;
        a.w = P<const float>(w); a.w_stride = w_stride; a.vbytes = vbytes; a.scaled = scaled; a.to_bf16 = to_bf16;
        a.out = P<unsigned char>(out); a.rb = rb; a.vb = vb;
        check(fm::launch_gather_wire(a, S(stream)), "gather_wire");
      },
      py::arg("R"), py::arg("req"), py::arg("v"), py::arg("v_bytes_stride"), py::arg("w"), py::arg("w_stride"),
      py::arg("vbytes"), py::arg("scaled"), py::arg("to_bf16"), py::arg("out"), py::arg("rb"), py::arg("vb"),
      py::arg("stream"), py::arg("idx") = 0, py::arg("run_off") = 0, py::arg("W") = 1, py::arg("skip0") = 0,
      py::arg("skip1") = 0);

  m.def(
      "apply_rows",
      [](u64 num_unique, u64 seg_start, u64 uniq, u64 perm, u64 grad_in, long long g_stride, int Kp, u64 v,
         long long v_stride, u64 w, long long w_stride, u64 s0v, u64 s1v, long long s_stride, u64 s0w, u64 s1w,
         int opt_type, float lr, float l1, float l2, float beta, int dtype, long long max_unique, u64 stream,
         int g_wcol, int g_bf16, u64 sr_counter) {
        fm::ApplyArgs a{};
        a.sr_counter = P<const int>(sr_counter);
        a.g_wcol = g_wcol < 0 ? Kp : g_wcol; a.g_bf16 = g_bf16;
        a.num_unique = P<const int>(num_unique); a.seg_start = P<const int>(seg_start);
        a.uniq = P<const int>(uniq); a.perm = P<const int>(perm); a.grad_in = P<const float>(grad_in);
        a.g_stride = g_stride; a.Kp = Kp; a.v = P<void>(v); a.v_stride = v_stride; a.w = P<float>(w);
        a.w_stride = w_stride; a.s0v = P<void>(s0v); a.s1v = P<void>(s1v); a.s_stride = s_stride;
        a.s0w = P<float>(s0w); a.s1w = P<float>(s1w); a.opt = opt_params(opt_type, lr, l1, l2, beta);
        check(fm::launch_apply_rows(a, dtype, max_unique, S(stream)), "apply_rows");
      },
      py::arg("num_unique"), py::arg("seg_start"), py::arg("uniq"), py::arg("perm"), py::arg("grad_in"),
      py::arg("g_stride"), py::arg("Kp"), py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"),
      py::arg("s0v"), py::arg("s1v"), py::arg("s_stride"), py::arg("s0w"), py::arg("s1w"), py::arg("opt_type"),
      py::arg("lr"), py::arg("l1"), py::arg("l2"), py::arg("beta"), py::arg("dtype"), py::arg("max_unique"),
      py::arg("stream"), py::arg("g_wcol") = -1, py::arg("g_bf16") = 0, py::arg("sr_counter") = 0);

  m.def(
      "apply_runs",
      [](int R, int W, u64 run_off, u64 req, u64 match, u64 grad_in, long long g_stride, int Kp, u64 v,
         long long v_stride, u64 w, long long w_stride, u64 s0v, u64 s1v, long long s_stride, u64 s0w, u64 s1w,
         int opt_type, float lr, float l1, float l2, float beta, int dtype, u64 stream, int g_wcol, int g_bf16,
         u64 sr_counter, int self_run, u64 self_excl) {
        fm::ApplyArgs a{};
        a.self_run = self_run; a.self_excl = P<const int>(self_excl);
        a.sr_counter = P<const int>(sr_counter);
        a.g_wcol = g_wcol < 0 ? Kp : g_wcol; a.g_bf16 = g_bf16;
        a.R = R; a.W = W; a.run_off = P<const int>(run_off); a.req = P<const int>(req);
        a.match = P<const int>(match); a.grad_in = P<const float>(grad_in);
        a.g_stride = g_stride; a.Kp = Kp; a.v = P<void>(v); a.v_stride = v_stride; a.w = P<float>(w);
        a.w_stride = w_stride; a.s0v = P<void>(s0v); a.s1v = P<void>(s1v); a.s_stride = s_stride;
        a.s0w = P<float>(s0w); a.s1w = P<float>(s1w); a.opt = opt_params(opt_type, lr, l1, l2, beta);
        check(fm::launch_apply_runs(a, P<int>(match), dtype, S(stream)), "apply_runs");
      },
      py::arg("R"), py::arg("W"), py::arg("run_off"), py::arg("req"), py::arg("match"), py::arg("grad_in"),
      py::arg("g_stride"), py::arg("Kp"), py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"),
      py::arg("s0v"), py::arg("s1v"), py::arg("s_stride"), py::arg("s0w"), py::arg("s1w"), py::arg("opt_type"),
      py::arg("lr"), py::arg("l1"), py::arg("l2"), py::arg("beta"), py::arg("dtype"), py::arg("stream"),
      py::arg("g_wcol") = -1, py::arg("g_bf16") = 0, py::arg("sr_counter") = 0, py::arg("self_run") = -1,
      py::arg("self_excl") = 0);

  m.def(
      "dense_apply",
      [](long long R, long long row0, u64 grad, long long g_stride, int touch_col, int zero, int Kp, u64 v,
         long long v_stride, u64 w, long long w_stride, u64 s0v, u64 s1v, long long s_stride, u64 s0w, u64 s1w,
         int opt_type, float lr, float l1, float l2, float beta, int dtype, u64 stream, u64 sr_counter) {
        fm::ApplyArgs a{};
        a.sr_counter = P<const int>(sr_counter);
        a.g_wcol = Kp; a.g_bf16 = 0;
        a.R = (int)R; a.row0 = row0; a.touch_col = touch_col;
        a.grad_in = P<const float>(grad); a.grad_zero = zero ? P<float>(grad) : nullptr;
        a.g_stride = g_stride; a.Kp = Kp; a.v = P<void>(v); a.v_stride = v_stride; a.w = P<float>(w);
        a.w_stride = w_stride; a.s0v = P<void>(s0v); a.s1v = P<void>(s1v); a.s_stride = s_stride;
        a.s0w = P<float>(s0w); a.s1w = P<float>(s1w); a.opt = opt_params(opt_type, lr, l1, l2, beta);
        check(fm::launch_dense_apply(a, dtype, S(stream)), "dense_apply");
      },
      py::arg("R"), py::arg("row0"), py::arg("grad"), py::arg("g_stride"), py::arg("touch_col"), py::arg("zero"),
      py::arg("Kp"), py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"), py::arg("s0v"),
      py::arg("s1v"), py::arg("s_stride"), py::arg("s0w"), py::arg("s1w"), py::arg("opt_type"), py::arg("lr"),
      py::arg("l1"), py::arg("l2"), py::arg("beta"), py::arg("dtype"), py::arg("stream"), py::arg("sr_counter") = 0);

  m.def(
      "init_rows",
      [](u64 v, long long v_stride, u64 w, long long w_stride, long long rows, int K, int Kp, int dtype,
         long long gid_mul, long long gid_add, unsigned long long seed, float range, u64 stream) {
        fm::InitArgs a;
        a.v = P<void>(v); a.v_stride = v_stride; a.w = P<float>(w); a.w_stride = w_stride; a.rows = rows;
        a.K = K; a.Kp = Kp; a.dtype = dtype; a.gid_mul = gid_mul; a.gid_add = gid_add; a.seed = seed;
        a.range = range;
        check(fm::launch_init_rows(a, S(stream)), "init_rows");
      },
      py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"), py::arg("rows"), py::arg("K"),
      py::arg("Kp"), py::arg("dtype"), py::arg("gid_mul"), py::arg("gid_add"), py::arg("seed"), py::arg("range"),
      py::arg("stream"));
  m.def(
      "fp8_row_norms",
      [](u64 v, long long v_stride, u64 w, long long w_stride, long long rows, int Kp, u64 stream, u64 idx) {
        check(fm::launch_fp8_norms(P<const uint8_t>(v), v_stride, P<float>(w), w_stride, rows, Kp, S(stream),
                                   P<const long long>(idx)),
              "fp8_row_norms");
      },
      py::arg("v"), py::arg("v_stride"), py::arg("w"), py::arg("w_stride"), py::arg("rows"), py::arg("Kp"),
      py::arg("stream"), py::arg("idx") = 0);
  m.attr("FP8_NORM_COL") = fm::kFp8Norm;

  m.def(
      "owner_counts",
      [](u64 uniq, u64 num_unique, long long Rps, int W, u64 out, u64 stream, long long stride, u64 out2) {
        check(fm::launch_owner_counts(P<const uint32_t>(uniq), P<const int>(num_unique), Rps, W, P<long long>(out),
                                      S(stream), stride, P<long long>(out2)),
              "owner_counts");
      },
      py::arg("uniq"), py::arg("num_unique"), py::arg("Rps"), py::arg("W"), py::arg("out"), py::arg("stream"),
      py::arg("stride") = 1, py::arg("out2") = 0);

  m.def(
      "zero_listed_rows",
      [](u64 buf, long long row_words, u64 list, u64 count, int max_n, u64 stream) {
        check(fm::launch_zero_listed_rows(P<float>(buf), row_words, P<const int>(list), P<const int>(count), max_n,
                                          S(stream)),
              "zero_listed_rows");
      },
      py::arg("buf"), py::arg("row_words"), py::arg("list"), py::arg("count"), py::arg("max_n"), py::arg("stream"));

  m.def(
      "shard_keys",
      [](int n, u64 ids, int W, int Rps, u64 keys, u64 stream) {
        check(fm::launch_shard_keys(n, P<const int>(ids), W, Rps, P<int>(keys), S(stream)), "shard_keys");
      },
      py::arg("n"), py::arg("ids"), py::arg("W"), py::arg("Rps"), py::arg("keys"), py::arg("stream"));

  m.def(
      "run_member",
      [](int R, u64 req, int W, u64 run_off, u64 prev, u64 flag, u64 stream) {
        check(fm::launch_run_member(R, P<const int>(req), W, P<const int>(run_off), P<const int>(prev), P<int>(flag),
                                    S(stream)),
              "run_member");
      },
      py::arg("R"), py::arg("req"), py::arg("W"), py::arg("run_off"), py::arg("prev"), py::arg("flag"),
      py::arg("stream"));
  m.def(
      "dirty_scan",
      [](int R, u64 req, int W, u64 run_off, int Wp, u64 prev_off, u64 prev, u64 flag, u64 dcount, u64 stream,
         int skip0, int skip1) {
        check(fm::launch_dirty_scan(R, P<const int>(req), W, P<const int>(run_off), Wp, P<const int>(prev_off),
                                    P<const int>(prev), P<int>(flag), P<int>(dcount), skip0, skip1, S(stream)),
              "dirty_scan");
      },
      py::arg("R"), py::arg("req"), py::arg("W"), py::arg("run_off"), py::arg("Wp"), py::arg("prev_off"),
      py::arg("prev"), py::arg("flag"), py::arg("dcount"), py::arg("stream"), py::arg("skip0") = 0,
      py::arg("skip1") = 0);
  m.def(
      "self_excl",
      [](u64 req, int W, u64 run_off, int me, int n, u64 excl, u64 stream) {
        check(fm::launch_self_excl(P<const int>(req), W, P<const int>(run_off), me, n, P<int>(excl), S(stream)),
              "self_excl");
      },
      py::arg("req"), py::arg("W"), py::arg("run_off"), py::arg("me"), py::arg("n"), py::arg("excl"),
      py::arg("stream"));
  m.def("select_workspace_bytes", &fm::select_workspace_bytes, py::arg("n"));
  m.def(
      "select_flagged",
      [](int n, u64 flag, u64 out, u64 count, u64 ws, long long ws_bytes, u64 stream) {
        check(fm::launch_select_flagged(n, P<const int>(flag), P<int>(out), P<int>(count), P<void>(ws),
                                        (size_t)ws_bytes, S(stream)),
              "select_flagged");
      },
      py::arg("n"), py::arg("flag"), py::arg("out"), py::arg("count"), py::arg("ws"), py::arg("ws_bytes"),
      py::arg("stream"));
  m.def(
      "patch_scatter",
      [](int D, u64 recv, long long rb, int W, u64 recv_off, u64 sc_start, u64 gathered, u64 stream) {
        check(fm::launch_patch_scatter(D, P<const unsigned char>(recv), rb, W, P<const int>(recv_off),
                                       P<const int>(sc_start), P<unsigned char>(gathered), S(stream)),
              "patch_scatter");
      },
      py::arg("D"), py::arg("recv"), py::arg("rb"), py::arg("W"), py::arg("recv_off"), py::arg("sc_start"),
      py::arg("gathered"), py::arg("stream"));
  m.def("parse_workspace_bytes", &fm::parse_workspace_bytes, py::arg("n"));
  m.def(
      "parse",
      [](u64 buf, u64 line_start, int n, long long vocab, int hash, u64 counts, u64 offsets, u64 labels, u64 ids,
         u64 vals, u64 status, u64 ws, long long ws_bytes, u64 stream, int require_vals) {
        fm::ParseArgs a{};
        a.require_vals = require_vals;
        a.buf = P<const char>(buf); a.line_start = P<const long long>(line_start); a.n = n; a.vocab = vocab;
        a.hash = hash; a.counts = P<int>(counts); a.labels = P<float>(labels); a.ids = P<int>(ids);
        a.vals = P<float>(vals); a.status = P<int>(status);
        check(fm::launch_parse(a, P<void>(ws), (size_t)ws_bytes, P<int>(offsets), S(stream)), "parse");
      },
      py::arg("buf"), py::arg("line_start"), py::arg("n"), py::arg("vocab"), py::arg("hash"), py::arg("counts"),
      py::arg("offsets"), py::arg("labels"), py::arg("ids"), py::arg("vals"), py::arg("status"), py::arg("ws"),
      py::arg("ws_bytes"), py::arg("stream"), py::arg("require_vals") = 0);

  // GPU-tokenizer feeder (feeder.hip): a native thread from the loader's raw batches to device CSR
  // (module_local: a build variant of this module can be loaded beside it in one process)
  py::class_<fm::GpuTextFeeder>(m, "GpuTextFeeder", py::module_local())
      .def(py::init([](u64 api, int device, long long vocab, bool hash) {
             return new fm::GpuTextFeeder(P<const FmLoaderApi>(api), device, vocab, hash);
           }),
           py::arg("api"), py::arg("device"), py::arg("vocab"), py::arg("hash"))
      // [bytes, bytes cap, ls, ls entries, weights, labels, offsets, counts, ids, ids cap, vals, status, ws, ws bytes]
      .def("add_slot",
           [](fm::GpuTextFeeder& F, std::vector<u64> p) {
             if (p.size() != 14) throw std::invalid_argument("feeder slot: 14 entries");
             fm::FeederSlot s;
             s.bytes = P<uint8_t>(p[0]); s.bytes_cap = p[1]; s.ls = P<int64_t>(p[2]); s.ls_cap = p[3];
             s.weights = P<float>(p[4]); s.labels = P<float>(p[5]); s.offsets = P<int>(p[6]); s.counts = P<int>(p[7]);
             s.ids = P<int>(p[8]); s.ids_cap = p[9]; s.vals = P<float>(p[10]); s.status = P<int>(p[11]);
             s.ws = P<void>(p[12]); s.ws_bytes = p[13];
             F.add_slot(s);
           })
      .def("start", &fm::GpuTextFeeder::start)
      // -> (slot, n, nnz, max_feats, has_vals, weighted, epoch, count) | None at the end | -1 (timed out,
      //    the feeder waits for a free slot) | -2 (timed out) | ("error", is_parse_error, message) |
      //    ("resize", slot, entries): answer with resize_ids
      .def("next",
           [](fm::GpuTextFeeder& F, int timeout_ms) -> py::object {
             fm::FeederBatch b;
             std::string err;
             bool perr = false;
             int r;
             {
               py::gil_scoped_release nogil;
               r = F.next(&b, timeout_ms, &err, &perr);
             }
             if (r == 1)
               return py::make_tuple(b.d, b.n, b.nnz, b.max_feats, b.has_vals, b.weighted, b.epoch, b.count);
             if (r == 0) return py::none();
             if (r == -3) return py::make_tuple(std::string("error"), perr, err);
             if (r == -4) return py::make_tuple(std::string("resize"), b.d, b.nnz);
             return py::int_(r);
           },
           py::arg("timeout_ms") = -1)
      .def("resize_ids",
           [](fm::GpuTextFeeder& F, int d, u64 ids, u64 vals, long long cap) {
             F.resize_ids(d, P<int>(ids), P<float>(vals), static_cast<size_t>(cap));
           },
           py::arg("slot"), py::arg("ids"), py::arg("vals"), py::arg("cap"))
      .def("resizes", &fm::GpuTextFeeder::resizes)
      .def("release", [](fm::GpuTextFeeder& F, int d, u64 stream) { F.release(d, S(stream)); }, py::arg("slot"),
           py::arg("stream"))
      .def("queued", &fm::GpuTextFeeder::queued)
      .def("fallbacks", &fm::GpuTextFeeder::fallbacks)
      .def("batches", &fm::GpuTextFeeder::batches)
      .def("close", [](fm::GpuTextFeeder& F) {
        py::gil_scoped_release nogil;
        F.close();
      });

  m.def(
      "batch_gather",
      [](u64 rows, u64 boff, int B, long long N, u64 src_off, u64 src_ids, u64 src_vals, u64 src_labels,
         u64 src_weights, u64 ids, u64 vals, u64 labels, u64 weights, u64 stream) {
        fm::BatchGatherArgs a{};
        a.rows = P<const long long>(rows); a.boff = P<const int>(boff); a.B = B; a.N = N;
        a.src_off = P<const long long>(src_off); a.src_ids = P<const int>(src_ids);
        a.src_vals = P<const float>(src_vals); a.src_labels = P<const float>(src_labels);
        a.src_weights = P<const float>(src_weights); a.ids = P<int>(ids); a.vals = P<float>(vals);
        a.labels = P<float>(labels); a.weights = P<float>(weights);
        check(fm::launch_batch_gather(a, S(stream)), "batch_gather");
      },
      py::arg("rows"), py::arg("boff"), py::arg("B"), py::arg("N"), py::arg("src_off"), py::arg("src_ids"),
      py::arg("src_vals"), py::arg("src_labels"), py::arg("src_weights"), py::arg("ids"), py::arg("vals"),
      py::arg("labels"), py::arg("weights"), py::arg("stream"));

  m.def(
      "csr_rows",
      [](int B, u64 offsets, u64 ex_of_occ, int slot_bits, u64 stream) {
        check(fm::launch_csr_rows(B, P<const int>(offsets), P<int>(ex_of_occ), slot_bits, S(stream)), "csr_rows");
      },
      py::arg("B"), py::arg("offsets"), py::arg("ex_of_occ"), py::arg("slot_bits"), py::arg("stream"));
}
