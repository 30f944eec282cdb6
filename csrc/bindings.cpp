// Python bindings for the gfx950 kernels, the native GGUF loader and the step executor.
// Deliberately torch-header-free: device pointers and HIP streams cross the boundary as integers
// (tensor.data_ptr(), torch.cuda.current_stream().cuda_stream), which keeps the build to seconds
// and lets the executor's launches be captured by torch.cuda.CUDAGraph (hipGraph) unchanged.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <stdexcept>

#include "gguf/gguf.h"
#include "kernels/ops.h"
#include "runtime/executor.h"

namespace py = pybind11;
using namespace omx;

static inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
template <class T>
static inline T* Pp(uintptr_t p) { return reinterpret_cast<T*>(p); }

static QMat qmat(py::object o) {
  QMat m{};
  if (o.is_none()) return m;
  auto t = o.cast<py::tuple>();
  if (t.size() < 7 || t.size() > 9)
    throw std::runtime_error("qmat tuple must be (s0, s1, s2, s3, N, K, qtype[, s4[, mt]])");
  m.s0 = Pp<const uint8_t>(t[0].cast<uintptr_t>());
  m.s1 = Pp<const uint8_t>(t[1].cast<uintptr_t>());
  m.s2 = Pp<const uint8_t>(t[2].cast<uintptr_t>());
  m.s3 = Pp<const uint8_t>(t[3].cast<uintptr_t>());
  m.N = t[4].cast<int>();
  m.K = t[5].cast<int>();
  m.qtype = t[6].cast<int>();
  m.s4 = t.size() >= 8 ? Pp<const uint8_t>(t[7].cast<uintptr_t>()) : nullptr;
  m.mt = t.size() >= 9 ? Pp<const uint8_t>(t[8].cast<uintptr_t>()) : nullptr;
  if (m.s4 && m.qtype != QT_Q6_K) throw std::runtime_error("widened codes are for Q6_K only");
  if (m.qtype != QT_Q4_0 && m.qtype != QT_Q8_0 && m.qtype != QT_Q4_K && m.qtype != QT_Q5_K && m.qtype != QT_Q6_K &&
      m.qtype != QT_F16)
    throw std::runtime_error("unsupported device quant type " + std::to_string(m.qtype));
  const int blk = (m.qtype == QT_Q4_K || m.qtype == QT_Q5_K || m.qtype == QT_Q6_K) ? 256 : m.qtype == QT_F16 ? 1 : 32;
  if (m.K % blk || m.K <= 0 || m.N <= 0) throw std::runtime_error("bad qmat geometry");
  return m;
}

// D: the kernels' head dim = KV cache row stride; Dv: valid dims (a padded head: Orca Mini 100 in 112)
static void check_attn(int H, int n_kv, int D, int Dv = 0) {
  if (n_kv <= 0 || H % n_kv) throw std::runtime_error("H must be a multiple of n_kv");
  // any group size: decode blocks take a divisor of G in {1, 2, 4, 8} (attention.hip heads_per_block)
  if (D != 64 && D != 80 && D != 96 && D != 112 && D != 128 && D != 256) throw std::runtime_error("unsupported head dim");
  if (Dv && (Dv > D || Dv <= D - 16 || Dv % 4)) throw std::runtime_error("unsupported padded head dim");
}

static ARParams ar_params(py::dict d) {
  ARParams P{};
  auto data = d["data"].cast<std::vector<uintptr_t>>();
  auto flags = d["flags"].cast<std::vector<uintptr_t>>();
  P.rank = d["rank"].cast<int>();
  P.world = d["world"].cast<int>();
  if (P.world < 1 || P.world > AR_MAX_RANKS || (int)data.size() != P.world || (int)flags.size() != P.world ||
      P.rank < 0 || P.rank >= P.world)
    throw std::runtime_error("ar: bad rank / world / peer pointer lists");
  for (int r = 0; r < P.world; ++r) {
    if (!data[r] || !flags[r]) throw std::runtime_error("ar: null peer pointer");
    P.data[r] = Pp<float>(data[r]);
    P.flags[r] = Pp<unsigned>(flags[r]);
  }
  P.epoch = Pp<unsigned>(d["epoch"].cast<uintptr_t>());
  P.err = Pp<int>(d["err"].cast<uintptr_t>());
  P.err_host = Pp<int>(d.contains("err_host") ? d["err_host"].cast<uintptr_t>() : 0);
  P.slab_floats = d["slab_floats"].cast<long long>();
  P.timeout_ticks = d["timeout_ticks"].cast<unsigned long long>();
  if (!P.epoch || !P.err || P.slab_floats <= 0 || P.slab_floats % 4) throw std::runtime_error("ar: bad workspace");
  return P;
}

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static StepInputs step_inputs(py::dict d) {
  StepInputs in;
  auto ptr = [&](const char* k) -> uintptr_t { return d.contains(k) ? d[k].cast<uintptr_t>() : 0; };
  in.B = d.contains("B") ? d["B"].cast<int>() : 0;
  in.tokens = Pp<const int>(ptr("tokens"));
  in.pos = Pp<const int>(ptr("pos"));
  in.slot = Pp<const int>(ptr("slot"));
  in.q_len = Pp<const int>(ptr("q_len"));
  in.q_seq = Pp<const int>(ptr("q_seq"));
  in.block_table = Pp<const int>(ptr("block_table"));
  in.max_blocks = d["max_blocks"].cast<int>();
  in.bs = d["bs"].cast<int>();
  in.prefill = d.contains("prefill") ? d["prefill"].cast<int>() : 0;
  in.n_logits = d.contains("n_logits") ? d["n_logits"].cast<int>() : 0;
  in.logit_idx = Pp<const int>(ptr("logit_idx"));
  in.logits = Pp<float>(ptr("logits"));
  in.full_logits = Pp<float>(ptr("full_logits"));
  in.ld_full = d.contains("ld_full") ? d["ld_full"].cast<int>() : 0;
  return in;
}

enum { ST_FORWARD = 0, ST_EMBED = 1, ST_ATTN = 2, ST_FFN = 3, ST_HEAD = 4, ST_FORWARD_TP = 5 };

static void run_stage(Executor& e, int stage, int layer, const StepInputs& in, hipStream_t s) {
  if (in.B > e.ws.max_B) throw std::runtime_error("batch exceeds workspace max_B");
  if ((stage == ST_ATTN || stage == ST_FFN) && (layer < 0 || layer >= (int)e.layers.size()))
    throw std::runtime_error("layer index");
  switch (stage) {
    case ST_FORWARD: e.forward(in, s); break;
    case ST_EMBED: e.embed(in, s); break;
    case ST_ATTN: e.attn_block(layer, in, s); break;
    case ST_FFN: e.ffn_block(layer, in, s); break;
    case ST_HEAD: e.head(in, s); break;
    case ST_FORWARD_TP: e.forward_tp(in, s); break;
    default: throw std::runtime_error("unknown stage");
  }
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "ollama-operator-amd native core: gfx950 HIP kernels, GGUF loader, step executor";

  // ------------------------------------------------------------------ GGUF
  py::class_<GGUFMap>(m, "GGUFMap")
      .def(py::init<const std::string&>())
      .def_property_readonly("size", &GGUFMap::size)
      .def_property_readonly("version", &GGUFMap::version)
      .def("tensors", [](const GGUFMap& g) {
        py::list out;
        for (const auto& e : g.tensors()) {
          py::dict d;
          d["name"] = e.name;
          d["dims"] = e.dims;
          d["type"] = e.type;
          d["offset"] = e.offset;
          d["nbytes"] = e.nbytes;
          out.append(d);
        }
        return out;
      })
      .def("release", [](const GGUFMap& g, const std::string& name) { g.release(g.get(name)); })
      .def("data_ptr", [](const GGUFMap& g, const std::string& name) {
        return reinterpret_cast<uintptr_t>(g.data(g.get(name)));
      })
      .def("repack", [](const GGUFMap& g, const std::string& name, py::array_t<int64_t> rows,
                        py::array_t<int64_t> dst_rows, int64_t K_src, int64_t kb0, int64_t kb1,
                        std::vector<uintptr_t> dst, int n_threads, int64_t K_out) {
        const auto& e = g.get(name);
        uint8_t* d[4] = {nullptr, nullptr, nullptr, nullptr};
        for (size_t i = 0; i < dst.size() && i < 4; ++i) d[i] = Pp<uint8_t>(dst[i]);
        auto r = rows.unchecked<1>();
        const int64_t n_src_rows = e.n_elements / K_src;
        for (py::ssize_t i = 0; i < r.shape(0); ++i)
          if (r(i) < 0 || r(i) >= n_src_rows) throw std::runtime_error("repack: row out of range");
        if (dst_rows.shape(0) != rows.shape(0)) throw std::runtime_error("repack: rows/dst_rows length");
        py::gil_scoped_release nogil;
        repack_rows(g.data(e), e.type, K_src, rows.data(), dst_rows.data(), rows.shape(0), kb0, kb1, d, n_threads, K_out);
      }, py::arg("name"), py::arg("rows"), py::arg("dst_rows"), py::arg("K_src"), py::arg("kb0"), py::arg("kb1"),
         py::arg("dst"), py::arg("n_threads"), py::arg("K_out") = 0);
  m.def("repack_ptr", [](uintptr_t src, int qtype, int64_t K_src, py::array_t<int64_t> rows,
                         py::array_t<int64_t> dst_rows, int64_t kb0, int64_t kb1, std::vector<uintptr_t> dst,
                         int n_threads, int64_t K_out) {
    uint8_t* d[4] = {nullptr, nullptr, nullptr, nullptr};
    for (size_t i = 0; i < dst.size() && i < 4; ++i) d[i] = Pp<uint8_t>(dst[i]);
    if (dst_rows.shape(0) != rows.shape(0)) throw std::runtime_error("repack: rows/dst_rows length");
    py::gil_scoped_release nogil;
    repack_rows(Pp<const uint8_t>(src), qtype, K_src, rows.data(), dst_rows.data(), rows.shape(0), kb0, kb1, d,
                n_threads, K_out);
  }, py::arg("src"), py::arg("qtype"), py::arg("K_src"), py::arg("rows"), py::arg("dst_rows"), py::arg("kb0"),
     py::arg("kb1"), py::arg("dst"), py::arg("n_threads"), py::arg("K_out") = 0);

  // ------------------------------------------------------------------ single ops (tests, prefill)
  m.def("gemv", [](py::object w, int B, uintptr_t x, int ldx, int norm, uintptr_t norm_w, uintptr_t norm_b,
                   float eps, int epi, uintptr_t y, int ldy, uintptr_t bias, int row_offset, py::dict qkv,
                   uintptr_t stream) {
    GemvParams P{};
    P.w = qmat(w);
    P.B = B;
    P.x = Pp<const float>(x);
    P.ldx = ldx;
    P.norm = norm;
    P.norm_w = Pp<const float>(norm_w);
    P.norm_b = Pp<const float>(norm_b);
    P.eps = eps;
    P.epi = epi;
    P.y = Pp<float>(y);
    P.ldy = ldy;
    P.bias = Pp<const float>(bias);
    P.row_offset = row_offset;
    P.n_sel = 1;
    if (qkv.contains("xws")) P.xws = Pp<void>(qkv["xws"].cast<uintptr_t>());  // enables the GEMM path
    if (qkv.contains("xws_elems")) P.xws_elems = qkv["xws_elems"].cast<long long>();
    if (qkv.contains("dbg_ts")) P.dbg_ts = Pp<unsigned long long>(qkv["dbg_ts"].cast<uintptr_t>());
    if (qkv.contains("gws")) {  // split-K slabs for small-M GEMMs
      P.gws = Pp<float>(qkv["gws"].cast<uintptr_t>());
      P.gws_elems = qkv["gws_elems"].cast<long long>();
    }
    if (qkv.contains("w16ws")) {  // large-M library GEMM scratch (gemm.hip gemm_lib)
      P.w16ws = Pp<void>(qkv["w16ws"].cast<uintptr_t>());
      P.w16_elems = qkv["w16_elems"].cast<long long>();
      P.yws = Pp<float>(qkv["yws"].cast<uintptr_t>());
      P.yws_elems = qkv["yws_elems"].cast<long long>();
    }
    if (epi == EPI_QKV) {
      P.pos = Pp<const int>(qkv["pos"].cast<uintptr_t>());
      P.slot = Pp<const int>(qkv["slot"].cast<uintptr_t>());
      P.kc = Pp<void>(qkv["kc"].cast<uintptr_t>());
      P.vc = Pp<void>(qkv["vc"].cast<uintptr_t>());
      P.inv_freq = Pp<const float>(qkv["inv_freq"].cast<uintptr_t>());
      P.Eq = qkv["Eq"].cast<int>();
      P.Ekv = qkv["Ekv"].cast<int>();
      P.D = qkv["D"].cast<int>();
      P.n_rot = qkv["n_rot"].cast<int>();
      P.n_kv = qkv["n_kv"].cast<int>();
      P.bs = qkv["bs"].cast<int>();
    }
    // batched matrix-core decode chain (gemv_mfma.hip): fp16 activations in, RMS partials, emission
    auto ip = [&](const char* k) -> uintptr_t { return qkv.contains(k) ? qkv[k].cast<uintptr_t>() : 0; };
    auto ii = [&](const char* k) -> int { return qkv.contains(k) ? qkv[k].cast<int>() : 0; };
    P.x16 = Pp<const void>(ip("x16"));
    P.ld16 = ii("ld16");
    P.zrow16 = ii("zrow16");
    P.xstat = Pp<const float>(ip("xstat"));
    P.xstat_n = ii("xstat_n");
    P.emit16 = Pp<void>(ip("emit16"));
    P.ld_emit = ii("ld_emit");
    P.emit_nw = Pp<const float>(ip("emit_nw"));
    P.emit_stat = Pp<float>(ip("emit_stat"));
    P.emit_prev = Pp<const float>(ip("emit_prev"));
    P.emit_prev_n = ii("emit_prev_n");
    P.emit_scale = Pp<float>(ip("emit_scale"));
    P.xscale = Pp<const float>(ip("xscale"));
    P.rexp_out = Pp<float>(ip("rexp_out"));
    P.rexp_in = Pp<const float>(ip("rexp_in"));
    P.y16 = Pp<void>(ip("y16"));
    P.ld16y = ii("ld16y");
    if ((P.x16 || P.emit16 || P.y16) && !gemv_mb_supported(P))
      throw std::runtime_error("gemv: fp16 chain operands given for a shape the matrix-core GEMV does not take");
    // batch-1 int8 activation chain (gemv8.hip)
    P.x8 = Pp<const void>(ip("x8"));
    P.x8_stat = Pp<const float>(ip("x8_stat"));
    P.emit8 = Pp<void>(ip("emit8"));
    P.emit8_nw = Pp<const float>(ip("emit8_nw"));
    P.emit8_stat = Pp<float>(ip("emit8_stat"));
    P.dbg8 = ii("dbg8");
    P.kb_ws = Pp<float>(ip("kb_ws"));
    P.kb_cnt = Pp<int>(ip("kb_cnt"));
    if (qkv.contains("merge_S")) {
      P.merge_S = ii("merge_S");
      P.merge_ml = Pp<const float>(ip("merge_ml"));
      P.merge_D = ii("merge_D");
    }
    if ((P.x8 || P.emit8) && !gemv8_supported(P))
      throw std::runtime_error("gemv: int8 chain operands given for a shape gemv8 does not take");
    if (qkv.contains("expert_ids")) {
      P.expert_ids = Pp<const int>(qkv["expert_ids"].cast<uintptr_t>());
      P.expert_w = Pp<const float>(qkv.contains("expert_w") ? qkv["expert_w"].cast<uintptr_t>() : 0);
      P.n_sel = qkv["n_sel"].cast<int>();
      P.x_per_sel = qkv.contains("x_sel_stride") ? 1 : 0;
      P.x_sel_stride = qkv.contains("x_sel_stride") ? qkv["x_sel_stride"].cast<long long>() : 0;
      P.y_sel_stride = qkv.contains("y_sel_stride") ? qkv["y_sel_stride"].cast<long long>() : 0;
    }
    gemv(P, S(stream));
  });
  m.def("attention", [](uintptr_t q, int ldq, uintptr_t kc, uintptr_t vc, uintptr_t block_table, int max_blocks,
                        uintptr_t q_seq, uintptr_t q_len, int NQ, int H, int n_kv, int D, int bs, float scale,
                        int window, uintptr_t out, int ldo, uintptr_t ws, int n_splits, uintptr_t counters,
                        uintptr_t stream, int prefill, int Dv) {
    if (n_splits < 1 || n_splits > 64) throw std::runtime_error("n_splits must be in [1, 64]");
    if (n_splits > 1 && (!ws || !counters)) throw std::runtime_error("split attention needs ws and counters");
    check_attn(H, n_kv, D, Dv);
    AttnParams A{};
    A.q = Pp<const float>(q);
    A.ldq = ldq;
    A.kc = Pp<const void>(kc);
    A.vc = Pp<const void>(vc);
    A.block_table = Pp<const int>(block_table);
    A.max_blocks = max_blocks;
    A.q_seq = Pp<const int>(q_seq);
    A.q_len = Pp<const int>(q_len);
    A.NQ = NQ;
    A.H = H;
    A.n_kv = n_kv;
    A.D = D;
    A.bs = bs;
    A.scale = scale;
    A.window = window;
    A.out = Pp<float>(out);
    A.ldo = ldo;
    A.ws = Pp<float>(ws);
    A.n_splits = n_splits;
    A.counters = Pp<int>(counters);
    A.prefill = prefill;
    A.Dv = Dv;
    attention_decode(A, S(stream));
  }, py::arg("q"), py::arg("ldq"), py::arg("kc"), py::arg("vc"), py::arg("block_table"), py::arg("max_blocks"),
     py::arg("q_seq"), py::arg("q_len"), py::arg("NQ"), py::arg("H"), py::arg("n_kv"), py::arg("D"), py::arg("bs"),
     py::arg("scale"), py::arg("window"), py::arg("out"), py::arg("ldo"), py::arg("ws"), py::arg("n_splits"),
     py::arg("counters"), py::arg("stream"), py::arg("prefill") = 0, py::arg("Dv") = 0);
  m.def("attention_ws_floats", &attention_ws_floats);
  m.def("set_attn_tuning", &set_attn_tuning, py::arg("kps"), py::arg("hpb") = -1);
  m.def("gemv_merge_supported", &gemv_merge_supported);
  m.def("set_gemv_tuning", &set_gemv_tuning, py::arg("blocks_per_cu") = 0, py::arg("rows") = 0,
        py::arg("debug") = 0, py::arg("ks") = -1, py::arg("xfirst") = -1, py::arg("xbar") = -1,
        py::arg("stream") = -1, py::arg("stream_bpc") = -1, py::arg("pf") = -1, py::arg("ws") = -1);
  m.def("embed_rows", [](py::object w, uintptr_t rows, int n, uintptr_t out, int ldo, uintptr_t stream) {
    embed_rows(qmat(w), Pp<const int>(rows), n, Pp<float>(out), ldo, S(stream));
  });
  m.def("set_gemm_lib_min_m", &set_gemm_lib_min_m, "prefill rows from which the hipBLASLt path runs (0 = off)");
  m.def("gemm_lib_min_m", &gemm_lib_min_m);
  m.def("set_moe_lib_min_m", &set_moe_lib_min_m, "MoE prefill pairs from which experts run on hipBLASLt (0 = off)");
  m.def("moe_lib_min_m", &moe_lib_min_m);
  m.def("set_dq_gemm", &set_dq_gemm, "1: prefill GEMMs from 128 rows on the stream-order dequant kernel (gemm_dq.hip)");
  m.def("set_dq_tuning", &set_dq_tuning, "microbenchmarks: force the dq GEMM tile config (0..3, -1 auto) and split-K factor (0 auto)");
  m.def("dq_gemm_enabled", &dq_gemm_enabled);
  m.def("set_gemv8_geo", [](int nsb, int ks) { set_gemv8_geo(nsb, ks); });
  m.def("set_gemv8_kb", [](int mode) { set_gemv8_kb(mode); });
  m.def("gemv8_merge_supported", &gemv8_merge_supported);
  m.def("set_dq_ring", &set_dq_ring, "1: prefill dq GEMMs on the register-ring kernel, 0: the glds kernel");
  // launch counters (ops.h LC_*): tests assert which kernel family a call enqueued
  m.def("launch_counts", []() {
    static const char* names[LC_N] = {"dq_gemm", "gemm_tile", "gemm_lib", "gemv8_row1", "gemv8_rows", "gemv8_dual",
                                      "gemv_mb", "gemv_flight", "attn_decode", "attn_prefill", "gemv8_pair"};
    py::dict d;
    for (int i = 0; i < LC_N; ++i) d[names[i]] = launch_count(i);
    return d;
  });
  m.def("reset_launch_counts", &reset_launch_counts);
  m.def("gemm_lib_prepare", [](int N, int K, int min_M, int max_M, size_t ws_bytes) {
    blas_prepare(N, K, min_M, max_M, ws_bytes);
  });
  m.def("dequant_f16", [](py::object w, uintptr_t out, uintptr_t stream, int perm) {
    dequant_f16(qmat(w), Pp<void>(out), S(stream), perm);
  }, py::arg("w"), py::arg("out"), py::arg("stream"), py::arg("perm") = 0);
  m.def("argmax", [](uintptr_t logits, int B, int V, int ld, uintptr_t out, uintptr_t stream) {
    argmax(Pp<const float>(logits), B, V, ld, Pp<int>(out), S(stream));
  });
  m.def("moe_router", [](py::object wq, int B, uintptr_t x, int ldx, uintptr_t norm_w, float eps, int k, uintptr_t ids,
                         uintptr_t w, uintptr_t stream, uintptr_t dbg_ts) {
    GemvParams P{};
    P.dbg_ts = Pp<unsigned long long>(dbg_ts);  // [B][8] phase stamps (scripts/bench_router.py) or null
    P.w = qmat(wq);
    if (P.w.N > 64 || k < 1 || k > P.w.N) throw std::runtime_error("moe_router: X <= 64 experts, 1 <= k <= X");
    P.B = B;
    P.x = Pp<const float>(x);
    P.ldx = ldx;
    P.norm = norm_w ? NORM_RMS : NORM_NONE;
    P.norm_w = Pp<const float>(norm_w);
    P.eps = eps;
    if (!moe_router(P, k, Pp<int>(ids), Pp<float>(w), S(stream))) throw std::runtime_error("moe_router: shape not covered");
  }, py::arg("w"), py::arg("B"), py::arg("x"), py::arg("ldx"), py::arg("norm_w"), py::arg("eps"), py::arg("k"),
     py::arg("ids"), py::arg("wout"), py::arg("stream"), py::arg("dbg_ts") = 0);
  m.def("moe_route", [](uintptr_t logits, int B, int X, int k, uintptr_t ids, uintptr_t w, uintptr_t stream) {
    moe_route(Pp<const float>(logits), B, X, k, Pp<int>(ids), Pp<float>(w), S(stream));
  });
  m.def("add_inplace", [](uintptr_t y, uintptr_t x, long long n, uintptr_t stream) {
    add_inplace(Pp<float>(y), Pp<const float>(x), n, S(stream));
  });
  m.def("mfma_layout_bytes", &mfma_layout_bytes);
  m.def("x8_bytes", [](int K) { return x8_bytes(K); });
  m.def("x8_stat_ld", [](int K) { return x8_stat_ld(K); });
  m.def("x8_slots", [](int K) { return x8_slots(K); });
  m.def("repack_m", [](py::object w, uintptr_t out, uintptr_t stream) {
    QMat q = qmat(w);
    if (!out || !mfma_layout_bytes(q.qtype, q.N, q.K)) throw std::runtime_error("repack_m: no layout M for this matrix");
    repack_m(q, Pp<void>(out), S(stream));
  });
  m.def("set_mb_enable", &set_mb_enable);
  m.def("set_mb_tuning", &set_mb_tuning, py::arg("dbg") = -1, py::arg("bpc") = 0);
  m.def("widen_q6k", [](py::object w, uintptr_t out, uintptr_t stream) {
    QMat q = qmat(w);
    if (q.qtype != QT_Q6_K || !out) throw std::runtime_error("widen_q6k: Q6_K matrix and output required");
    widen_q6k(q, Pp<void>(out), S(stream));
  });
  // host-mapped pinned buffer: (host pointer, device pointer); kernels store tokens into it directly
  m.def("host_alloc_mapped", [](size_t bytes) {
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, bytes, hipHostMallocMapped) != hipSuccess || !h)
      throw std::runtime_error("hipHostMalloc(mapped) failed");
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
      (void)hipHostFree(h);
      throw std::runtime_error("hipHostGetDevicePointer failed");
    }
    std::memset(h, 0, bytes);
    return py::make_tuple((uintptr_t)h, (uintptr_t)d);
  });
  m.def("host_free_mapped", [](uintptr_t h) {
    if (h) (void)hipHostFree((void*)h);
  });
  m.def("sample", [](py::dict d, uintptr_t stream) {
    SampleParams P{};
    P.logits = Pp<const float>(d["logits"].cast<uintptr_t>());
    P.B = d["B"].cast<int>();
    P.V = d["V"].cast<int>();
    P.ld = d["ld"].cast<int>();
    P.temperature = Pp<const float>(d["temperature"].cast<uintptr_t>());
    P.top_k = Pp<const int>(d["top_k"].cast<uintptr_t>());
    P.top_p = Pp<const float>(d["top_p"].cast<uintptr_t>());
    P.min_p = Pp<const float>(d["min_p"].cast<uintptr_t>());
    P.repeat_penalty = Pp<const float>(d["repeat_penalty"].cast<uintptr_t>());
    P.presence_penalty = Pp<const float>(d["presence_penalty"].cast<uintptr_t>());
    P.frequency_penalty = Pp<const float>(d["frequency_penalty"].cast<uintptr_t>());
    P.history = Pp<int>(d["history"].cast<uintptr_t>());
    P.hist_count = Pp<int>(d["hist_count"].cast<uintptr_t>());
    P.hist_cap = d["hist_cap"].cast<int>();
    P.repeat_last_n = Pp<const int>(d["repeat_last_n"].cast<uintptr_t>());
    P.seed = Pp<const unsigned long long>(d["seed"].cast<uintptr_t>());
    P.step = Pp<int>(d["step"].cast<uintptr_t>());
    P.out = Pp<int>(d["out"].cast<uintptr_t>());
    P.out_logprob = Pp<float>(d.contains("out_logprob") ? d["out_logprob"].cast<uintptr_t>() : 0);
    P.ws = Pp<float>(d.contains("ws") ? d["ws"].cast<uintptr_t>() : 0);
    P.counters = Pp<int>(d.contains("counters") ? d["counters"].cast<uintptr_t>() : 0);
    P.err = Pp<int>(d.contains("err") ? d["err"].cast<uintptr_t>() : 0);
    if (d.contains("fb_step")) {
      P.fb_step = Pp<int>(d["fb_step"].cast<uintptr_t>());
      P.fb_ld = d["fb_ld"].cast<int>();
      P.fb_block_table = Pp<const int>(d["fb_block_table"].cast<uintptr_t>());
      P.fb_max_blocks = d["fb_max_blocks"].cast<int>();
      P.fb_bs = d["fb_bs"].cast<int>();
      P.fb_host_ring = Pp<int>(d.contains("fb_host_ring") ? d["fb_host_ring"].cast<uintptr_t>() : 0);
      P.fb_ring = d.contains("fb_ring") ? d["fb_ring"].cast<int>() : 0;
      P.fb_sysfence = d.contains("fb_sysfence") ? d["fb_sysfence"].cast<int>() : 1;
      if (P.B > P.fb_ld || P.fb_bs <= 0 || P.fb_max_blocks <= 0) throw std::runtime_error("sample: bad feedback args");
      if (P.fb_host_ring && P.fb_ring <= 0) throw std::runtime_error("sample: bad feedback ring");
    }
    sample(P, S(stream));
  });

  // ------------------------------------------------------------------ executor
  py::class_<Executor>(m, "Executor")
      .def(py::init<>())
      .def("configure", [](Executor& e, py::dict c) {
        ExecConfig& k = e.cfg;
        k.arch = c["arch"].cast<int>();
        k.E = c["E"].cast<int>();
        k.H = c["H"].cast<int>();
        k.Hkv = c["Hkv"].cast<int>();
        k.D = c["D"].cast<int>();
        k.n_rot = c["n_rot"].cast<int>();
        k.F = c["F"].cast<int>();
        k.F_valid = c.contains("F_valid") ? c["F_valid"].cast<int>() : 0;
        k.n_layer = c["n_layer"].cast<int>();
        k.V = c["V"].cast<int>();
        k.eps = c["eps"].cast<float>();
        k.n_expert = c["n_expert"].cast<int>();
        k.n_expert_used = c["n_expert_used"].cast<int>();
        k.window = c["window"].cast<int>();
        k.tp = c["tp"].cast<int>();
        k.embed_scale = c.contains("embed_scale") ? c["embed_scale"].cast<float>() : 1.f;
        k.glu_act = c.contains("glu_act") ? c["glu_act"].cast<int>() : 0;
        k.Dc = c.contains("Dc") ? c["Dc"].cast<int>() : k.D;
        k.kv8 = c.contains("kv8") ? c["kv8"].cast<int>() : 0;
        check_attn(k.H, k.Hkv, k.Dc, k.D);
        e.layers.assign(k.n_layer, LayerW{});
      })
      .def("set_globals", [](Executor& e, py::object tok_embd, uintptr_t out_norm, uintptr_t out_norm_b,
                             py::object lm_head, uintptr_t lm_bias, uintptr_t inv_freq) {
        e.tok_embd = qmat(tok_embd);
        e.out_norm = Pp<const float>(out_norm);
        e.out_norm_b = Pp<const float>(out_norm_b);
        e.lm_head = qmat(lm_head);
        e.lm_bias = Pp<const float>(lm_bias);
        e.inv_freq = Pp<const float>(inv_freq);
      })
      .def("set_layer", [](Executor& e, int i, py::dict d) {
        if (i < 0 || i >= (int)e.layers.size()) throw std::runtime_error("layer index");
        LayerW& L = e.layers[i];
        auto ptr = [&](const char* k) -> uintptr_t { return d.contains(k) ? d[k].cast<uintptr_t>() : 0; };
        auto qm = [&](const char* k) { return d.contains(k) ? qmat(d[k]) : QMat{}; };
        L.attn_norm = Pp<const float>(ptr("attn_norm"));
        L.attn_norm_b = Pp<const float>(ptr("attn_norm_b"));
        L.ffn_norm = Pp<const float>(ptr("ffn_norm"));
        L.wqk = qm("wqk");
        L.wv = qm("wv");
        L.qkv_fused = d.contains("wv") ? 0 : 1;
        L.qkv_bias = Pp<const float>(ptr("qkv_bias"));
        L.wo = qm("wo");
        L.bo = Pp<const float>(ptr("bo"));
        L.wgu = qm("wgu");
        L.bup = Pp<const float>(ptr("bup"));
        L.wdown = qm("wdown");
        L.bdown = Pp<const float>(ptr("bdown"));
        L.router = qm("router");
        L.gu_exps = qm("gu_exps");
        L.down_exps = qm("down_exps");
        L.kc = Pp<void>(ptr("kc"));
        L.vc = Pp<void>(ptr("vc"));
        L.c1_qkv = Pp<const float>(ptr("c1_qkv"));
        L.c2_qkv = Pp<const float>(ptr("c2_qkv"));
        L.c1_up = Pp<const float>(ptr("c1_up"));
        L.c2_up = Pp<const float>(ptr("c2_up"));
      })
      .def("set_head_ln", [](Executor& e, uintptr_t c1, uintptr_t c2) {
        e.lm_c1 = Pp<const float>(c1);
        e.lm_c2 = Pp<const float>(c2);
      })
      .def("set_workspace", [](Executor& e, py::dict d) {
        auto ptr = [&](const char* k) -> uintptr_t { return d.contains(k) ? d[k].cast<uintptr_t>() : 0; };
        Workspace& w = e.ws;
        w.resid = Pp<float>(ptr("resid"));
        w.qbuf = Pp<float>(ptr("qbuf"));
        w.abuf = Pp<float>(ptr("abuf"));
        w.hbuf = Pp<float>(ptr("hbuf"));
        w.ypart = Pp<float>(ptr("ypart"));
        w.lbuf = Pp<float>(ptr("lbuf"));
        w.rlogits = Pp<float>(ptr("rlogits"));
        w.eids = Pp<int>(ptr("eids"));
        w.ew = Pp<float>(ptr("ew"));
        w.attn_ws = Pp<float>(ptr("attn_ws"));
        w.attn_cnt = Pp<int>(ptr("attn_cnt"));
        w.x16 = Pp<void>(ptr("x16"));
        w.x16_elems = d.contains("x16_elems") ? d["x16_elems"].cast<long long>() : 0;
        w.gws = Pp<float>(ptr("gws"));
        w.gws_elems = d.contains("gws_elems") ? d["gws_elems"].cast<long long>() : 0;
        w.ext = Pp<const float>(ptr("ext"));
        w.w16 = Pp<void>(ptr("w16"));
        w.w16_elems = d.contains("w16_elems") ? d["w16_elems"].cast<long long>() : 0;
        w.yws = Pp<float>(ptr("yws"));
        w.yws_elems = d.contains("yws_elems") ? d["yws_elems"].cast<long long>() : 0;
        w.moe_rows = Pp<int>(ptr("moe_rows"));
        w.moe_tiles = Pp<int>(ptr("moe_tiles"));
        w.moe_ntiles = Pp<int>(ptr("moe_ntiles"));
        w.mb_ok = (d.contains("mb_ok") ? d["mb_ok"].cast<int>() : 0) && e.chain_capable() ? 1 : 0;
        w.xa16 = Pp<void>(ptr("xa16"));
        w.h16 = Pp<void>(ptr("h16"));
        w.a16 = Pp<void>(ptr("a16"));
        w.st[0] = Pp<float>(ptr("st0"));
        w.st[1] = Pp<float>(ptr("st1"));
        w.ld_e = d.contains("ld_e") ? d["ld_e"].cast<int>() : 0;
        w.ld_f = d.contains("ld_f") ? d["ld_f"].cast<int>() : 0;
        w.ld_q = d.contains("ld_q") ? d["ld_q"].cast<int>() : 0;
        w.max_B = d["max_B"].cast<int>();
        w.n_splits = d["n_splits"].cast<int>();
        w.x8e = Pp<void>(ptr("x8e"));
        w.x8f = Pp<void>(ptr("x8f"));
        w.x8st = Pp<float>(ptr("x8st"));
        w.x8sum = Pp<float>(ptr("x8sum"));
        w.kb_ws = Pp<float>(ptr("x8kb"));
        w.kb_cnt = Pp<int>(ptr("x8cnt"));
        w.x8_ok = (d.contains("x8_ok") ? d["x8_ok"].cast<int>() : 0) && e.x8_capable() ? 1 : 0;
        {  // continuous-batching rows on the chain: as many as asked for and every emitter covers
          const int want = d.contains("x8_bmax") ? d["x8_bmax"].cast<int>() : 1;
          w.x8_bmax = 1;
          if (w.x8_ok)
            for (int b = 2; b <= want && b <= 4 && e.x8_capable(b); ++b) w.x8_bmax = b;
        }
      })
      .def_property_readonly("x8_on", [](const Executor& e) { return e.ws.x8_ok; })
      .def_property_readonly("x8_bmax", [](const Executor& e) { return e.ws.x8_ok ? e.ws.x8_bmax : 0; })
      .def("set_segments", [](Executor& e, std::vector<std::pair<int, int>> segs) { e.segments = std::move(segs); })
      .def("set_splits", [](Executor& e, int n, int defer) {
        e.ws.n_splits = n;
        e.ws.defer = defer;
      }, py::arg("n"), py::arg("defer") = 0)
      .def("run", [](Executor& e, const std::string& what, int layer, py::dict d, uintptr_t stream) {
        static const std::pair<const char*, int> names[] = {{"forward", ST_FORWARD}, {"embed", ST_EMBED},
            {"attn", ST_ATTN}, {"ffn", ST_FFN}, {"head", ST_HEAD}, {"forward_tp", ST_FORWARD_TP}};
        for (const auto& nm : names)
          if (what == nm.first) return run_stage(e, nm.second, layer, step_inputs(d), S(stream));
        throw std::runtime_error("unknown stage " + what);
      })
      // pre-bound inputs: bind the step buffers once, then each stage call passes only integers
      .def("set_inputs", [](Executor& e, py::dict d) { e.bound = step_inputs(d); })
      .def("step", [](Executor& e, int stage, int layer, int B, int n_logits, bool use_idx, bool prefill,
                      uintptr_t stream) {
        StepInputs in = e.bound;
        in.B = B;
        in.n_logits = n_logits;
        if (!use_idx) in.logit_idx = nullptr;
        in.prefill = prefill ? 1 : 0;
        run_stage(e, stage, layer, in, S(stream));
      })
      .def("set_ar", [](Executor& e, py::dict d) {
        e.ws.ar = ar_params(d);
        e.ws.ar_on = 1;
      })
      .def("clear_ar", [](Executor& e) { e.ws.ar_on = 0; })
      .def("ar_fits", &Executor::ar_fits)
      .def_property_readonly("mb_chain", [](const Executor& e) { return e.ws.mb_ok != 0; });
  m.attr("ST_FORWARD") = (int)ST_FORWARD;
  m.attr("ST_EMBED") = (int)ST_EMBED;
  m.attr("ST_ATTN") = (int)ST_ATTN;
  m.attr("ST_FFN") = (int)ST_FFN;
  m.attr("ST_HEAD") = (int)ST_HEAD;
  m.attr("ST_FORWARD_TP") = (int)ST_FORWARD_TP;

  // ------------------------------------------------------------------ custom all-reduce (TP decode)
  m.attr("AR_MAX_RANKS") = AR_MAX_RANKS;
  m.attr("AR_SLABS") = AR_SLABS;
  // this rank's slab buffer + flags (uncached) + epoch / error words, with IPC handles of the two
  // peer-visible allocations (bytes) for the other ranks to open
  m.def("ar_alloc", [](long long slab_floats) {
    if (slab_floats <= 0 || slab_floats % 4) throw std::runtime_error("ar_alloc: slab_floats must be a positive multiple of 4");
    void *data = nullptr, *flags = nullptr, *local = nullptr;
    const size_t dbytes = sizeof(float) * (size_t)AR_SLABS * slab_floats;
    const size_t fbytes = sizeof(unsigned) * AR_MAX_BLOCKS * AR_MAX_RANKS;
    hip_check(hipMalloc(&data, dbytes), "ar_alloc data");
    hip_check(hipMemset(data, 0, dbytes), "ar_alloc memset");
    if (hipExtMallocWithFlags(&flags, fbytes, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      hip_check(hipMalloc(&flags, fbytes), "ar_alloc flags");
    }
    hip_check(hipMemset(flags, 0, fbytes), "ar_alloc memset");
    hip_check(hipMalloc(&local, sizeof(unsigned) * AR_MAX_BLOCKS + 64), "ar_alloc local");
    hip_check(hipMemset(local, 0, sizeof(unsigned) * AR_MAX_BLOCKS + 64), "ar_alloc memset");
    hip_check(hipDeviceSynchronize(), "ar_alloc sync");
    hipIpcMemHandle_t hd, hf;
    hip_check(hipIpcGetMemHandle(&hd, data), "hipIpcGetMemHandle(data)");
    hip_check(hipIpcGetMemHandle(&hf, flags), "hipIpcGetMemHandle(flags)");
    py::dict r;
    r["data"] = reinterpret_cast<uintptr_t>(data);
    r["flags"] = reinterpret_cast<uintptr_t>(flags);
    r["epoch"] = reinterpret_cast<uintptr_t>(local);
    r["err"] = reinterpret_cast<uintptr_t>(local) + sizeof(unsigned) * AR_MAX_BLOCKS;
    r["data_handle"] = py::bytes(reinterpret_cast<const char*>(&hd), sizeof(hd));
    r["flags_handle"] = py::bytes(reinterpret_cast<const char*>(&hf), sizeof(hf));
    return r;
  });
  m.def("ar_open", [](py::bytes h) {
    std::string s = h;
    hipIpcMemHandle_t hh;
    if (s.size() != sizeof(hh)) throw std::runtime_error("ar_open: bad handle size");
    memcpy(&hh, s.data(), sizeof(hh));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, hh, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    return reinterpret_cast<uintptr_t>(p);
  });
  m.def("ar_close", [](uintptr_t p) { hip_check(hipIpcCloseMemHandle(Pp<void>(p)), "hipIpcCloseMemHandle"); });
  m.def("ar_free", [](uintptr_t p) { hip_check(hipFree(Pp<void>(p)), "hipFree"); });
  m.def("ar_error", [](uintptr_t err) {  // host read of the error word (synchronous)
    int v = 0;
    hip_check(hipMemcpy(&v, Pp<void>(err), sizeof(int), hipMemcpyDeviceToHost), "ar_error");
    return v;
  });
  m.def("wall_clock_khz", []() {
    int dev = 0, khz = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    hip_check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev), "wall clock rate");
    return khz;
  });
  m.def("copy_d2d", [](uintptr_t dst, uintptr_t src, size_t bytes, uintptr_t stream) {
    hip_check(hipMemcpyAsync(Pp<void>(dst), Pp<const void>(src), bytes, hipMemcpyDeviceToDevice, S(stream)), "copy_d2d");
  });
  m.def("ar_allreduce_add", [](py::dict d, int slab, uintptr_t y, int n, uintptr_t stream) {
    ARParams P = ar_params(d);
    if (slab < 0 || slab >= AR_SLABS || n % 4 || n > P.slab_floats) throw std::runtime_error("ar_allreduce_add: bad slab / n");
    ar_allreduce_add(P, slab, Pp<float>(y), n, S(stream));
  });
  m.def("ar_allreduce_add_emit", [](py::dict d, int slab, uintptr_t y, int E, int B, uintptr_t img, uintptr_t nw,
                                     uintptr_t stat, uintptr_t stream) {
    ARParams P = ar_params(d);
    if (slab < 0 || slab >= AR_SLABS || (long long)E * B > P.slab_floats)
      throw std::runtime_error("ar_allreduce_add_emit: bad slab / shape");
    if (!ar_allreduce_add_emit(P, slab, Pp<float>(y), E, B, Pp<void>(img), Pp<const float>(nw), Pp<float>(stat), S(stream)))
      throw std::runtime_error("ar_allreduce_add_emit: shape not covered");
  });
  m.def("ar_allgather", [](py::dict d, int slab, uintptr_t out, int rows, int n_local, int ld_out, uintptr_t stream) {
    ARParams P = ar_params(d);
    if (slab < 0 || slab >= AR_SLABS || (long long)rows * n_local > P.slab_floats || ld_out < n_local * P.world)
      throw std::runtime_error("ar_allgather: bad slab / shape");
    ar_allgather(P, slab, Pp<float>(out), rows, n_local, ld_out, S(stream));
  });

  m.attr("NORM_NONE") = (int)NORM_NONE;
  m.attr("NORM_RMS") = (int)NORM_RMS;
  m.attr("NORM_LAYER") = (int)NORM_LAYER;
  m.attr("EPI_STORE") = (int)EPI_STORE;
  m.attr("EPI_ADD") = (int)EPI_ADD;
  m.attr("EPI_GLU") = (int)EPI_GLU;
  m.attr("EPI_GEGLU") = (int)EPI_GEGLU;
  m.attr("EPI_GELU") = (int)EPI_GELU;
  m.attr("EPI_QKV") = (int)EPI_QKV;
}
