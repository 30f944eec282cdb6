// pybind11 module `ollama_operator_amd._cpu`: the CPU serving backend (cpu_engine.h). Same call
// surface as the gfx950 executor binding (csrc/bindings.cpp `Executor`), so the runner's adapter
// (engine/runner.py NativeExec) drives either one. Built by build_native.py with the host compiler
// only -- no HIP runtime is needed on a CPU-only node (BASELINE config 1).
#include <omp.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>

#include "cpu_engine.h"

namespace py = pybind11;
using namespace omxcpu;

template <class T>
static T* Pp(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}

static QMat qmat(py::object o) {
  auto t = o.cast<py::tuple>();
  if (t.size() != 7 && t.size() != 8) throw std::runtime_error("qmat tuple must be (s0, s1, s2, s3, N, K, qtype[, s4])");
  QMat m;
  for (int i = 0; i < 4; ++i) m.s[i] = Pp<const uint8_t>(t[i].cast<uintptr_t>());
  m.N = t[4].cast<int>();
  m.K = t[5].cast<int>();
  m.qtype = t[6].cast<int>();
  if (m.qtype != QT_Q4_0 && m.qtype != QT_Q8_0 && m.qtype != QT_Q4_K && m.qtype != QT_Q5_K && m.qtype != QT_Q6_K)
    throw std::runtime_error("unsupported quant type " + std::to_string(m.qtype));
  if (m.N <= 0 || m.K <= 0 || !m.s[0] || !m.s[1]) throw std::runtime_error("bad qmat");
  return m;
}

enum { ST_FORWARD = 0, ST_EMBED = 1, ST_ATTN = 2, ST_FFN = 3, ST_HEAD = 4 };

PYBIND11_MODULE(_cpu, m) {
  m.doc() = "CPU serving backend: quantised int8-dot GEMM + transformer stages (AVX2, OpenMP)";
  m.def("isa", &isa);
  m.def("threads", &threads);
  m.def("set_threads", [](int n) {
    if (n > 0) omp_set_num_threads(n);
  });
  m.def("gemm", [](py::object w, long long row_base, int N, uintptr_t x, int ldx, int B, uintptr_t y, int ldy,
                   bool accumulate) {
    QMat q = qmat(w);
    if (N <= 0 || B <= 0 || ldx < q.K || ldy < N) throw std::runtime_error("gemm: bad shape");
    py::gil_scoped_release nogil;
    gemm(q, row_base, N, Pp<const float>(x), ldx, B, Pp<float>(y), ldy, accumulate);
  });
  m.def("dequant_row", [](py::object w, long long row, uintptr_t out) { dequant_row(qmat(w), row, Pp<float>(out)); });
  m.attr("ST_FORWARD") = (int)ST_FORWARD;
  m.attr("ST_EMBED") = (int)ST_EMBED;
  m.attr("ST_ATTN") = (int)ST_ATTN;
  m.attr("ST_FFN") = (int)ST_FFN;
  m.attr("ST_HEAD") = (int)ST_HEAD;
  m.attr("ST_FORWARD_TP") = -1;  // the one-shot all-reduce path is GPU-only

  py::class_<Engine>(m, "Executor")
      .def(py::init<>())
      .def("configure", [](Engine& e, py::dict c) {
        Config& k = e.cfg;
        k.arch = c["arch"].cast<int>();
        k.E = c["E"].cast<int>();
        k.H = c["H"].cast<int>();
        k.Hkv = c["Hkv"].cast<int>();
        k.D = c["D"].cast<int>();
        k.n_rot = c["n_rot"].cast<int>();
        k.F = c["F"].cast<int>();
        k.n_layer = c["n_layer"].cast<int>();
        k.V = c["V"].cast<int>();
        k.eps = c["eps"].cast<float>();
        k.n_expert = c["n_expert"].cast<int>();
        k.n_expert_used = c["n_expert_used"].cast<int>();
        k.window = c["window"].cast<int>();
        k.tp = c["tp"].cast<int>();
        k.embed_scale = c.contains("embed_scale") ? c["embed_scale"].cast<float>() : 1.f;
        k.glu_act = c.contains("glu_act") ? c["glu_act"].cast<int>() : 0;
        if (k.H <= 0 || k.Hkv <= 0 || k.H % k.Hkv || k.D <= 0 || k.n_rot > k.D) throw std::runtime_error("bad heads");
        e.layers.assign(k.n_layer, Layer{});
      })
      .def("set_globals", [](Engine& e, py::object tok, uintptr_t on, uintptr_t onb, py::object lm, uintptr_t lb,
                             uintptr_t inv) {
        e.tok_embd = qmat(tok);
        e.out_norm = Pp<const float>(on);
        e.out_norm_b = Pp<const float>(onb);
        e.lm_head = qmat(lm);
        e.lm_bias = Pp<const float>(lb);
        e.inv_freq = Pp<const float>(inv);
      })
      .def("set_layer", [](Engine& e, int i, py::dict d) {
        if (i < 0 || i >= (int)e.layers.size()) throw std::runtime_error("layer index");
        Layer& L = e.layers[i];
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
        L.kc = Pp<uint16_t>(ptr("kc"));
        L.vc = Pp<uint16_t>(ptr("vc"));
      })
      .def("set_workspace", [](Engine& e, py::dict d) {
        auto ptr = [&](const char* k) -> uintptr_t { return d.contains(k) ? d[k].cast<uintptr_t>() : 0; };
        Buffers& b = e.buf;
        b.resid = Pp<float>(ptr("resid"));
        b.qbuf = Pp<float>(ptr("qbuf"));
        b.abuf = Pp<float>(ptr("abuf"));
        b.hbuf = Pp<float>(ptr("hbuf"));
        b.ypart = Pp<float>(ptr("ypart"));
        b.ext = Pp<const float>(ptr("ext"));
        b.max_B = d["max_B"].cast<int>();
        b.ld_logits = d.contains("ld_logits") ? d["ld_logits"].cast<int>() : e.cfg.V;
      })
      .def("set_splits", [](Engine&, int, int, int) {}, py::arg("n"), py::arg("defer") = 0, py::arg("fuse") = 0)
      .def("set_inputs", [](Engine& e, py::dict d) {
        auto ptr = [&](const char* k) -> uintptr_t { return d.contains(k) ? d[k].cast<uintptr_t>() : 0; };
        Buffers& b = e.buf;
        b.tokens = Pp<const int>(ptr("tokens"));
        b.pos = Pp<const int>(ptr("pos"));
        b.slot = Pp<const int>(ptr("slot"));
        b.q_len = Pp<const int>(ptr("q_len"));
        b.q_seq = Pp<const int>(ptr("q_seq"));
        b.block_table = Pp<const int>(ptr("block_table"));
        b.max_blocks = d["max_blocks"].cast<int>();
        b.bs = d["bs"].cast<int>();
        b.logits = Pp<float>(ptr("logits"));
        b.logit_idx = Pp<const int>(ptr("logit_idx"));
      })
      .def("step", [](Engine& e, int stage, int layer, int B, int n_logits, bool use_idx, bool /*prefill*/,
                      uintptr_t /*stream*/) {
        if (B <= 0 || B > e.buf.max_B) throw std::runtime_error("batch exceeds workspace");
        if ((stage == ST_ATTN || stage == ST_FFN) && (layer < 0 || layer >= (int)e.layers.size()))
          throw std::runtime_error("layer index");
        py::gil_scoped_release nogil;
        switch (stage) {
          case ST_FORWARD: e.forward(B, n_logits, use_idx); break;
          case ST_EMBED: e.embed(B); break;
          case ST_ATTN: e.attn(layer, B); break;
          case ST_FFN: e.ffn(layer, B); break;
          case ST_HEAD: e.head(n_logits, use_idx); break;
          default: throw std::runtime_error("unknown stage");
        }
      })
      .def("ar_fits", [](Engine&, int) { return false; });
}
