// torch op registration for the gfx950 kernels (namespace `dcr`, loaded with
// torch.ops.load_library).  Only argument checking and stream plumbing lives here; every op
// launches hand-written HIP kernels from the *.hip files on the current HIP stream.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "kernels.h"
#include "debug_env.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_ALIGN16(t) \
  TORCH_CHECK((reinterpret_cast<uintptr_t>((t).data_ptr()) & 15) == 0, #t " must be 16-B aligned")

template <typename T>
T* ptr(const at::Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
using bf16 = dcr::bf16;

// ------------------------------------------------------------------------------------------
// optimizer
// ------------------------------------------------------------------------------------------
void global_norm(const at::Tensor& g, at::Tensor& partials, at::Tensor& norm_out) {
  CHECK_DEV(g); CHECK_CONTIG(g); CHECK_F32(g); CHECK_ALIGN16(g);
  CHECK_F32(partials); CHECK_F32(norm_out);
  TORCH_CHECK(partials.numel() >= dcr::opt_num_partials(g.numel()), "partials too small");
  dcr::launch_global_norm(ptr<float>(g), g.numel(), ptr<float>(partials), ptr<float>(norm_out),
                          cur_stream());
}

// out[0] = sum(x^2) with fp32 accumulation; x fp32 or bf16
void sumsq(const at::Tensor& x, at::Tensor& partials, at::Tensor& out,
           const c10::optional<at::Tensor>& ticket, const c10::optional<at::Tensor>& extra,
           const c10::optional<at::Tensor>& guard) {
  CHECK_DEV(x); CHECK_CONTIG(x); CHECK_ALIGN16(x);
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16,
              "sumsq: fp32 or bf16");
  CHECK_F32(partials); CHECK_F32(out);
  TORCH_CHECK(partials.numel() >= dcr::opt_num_partials(x.numel()), "partials too small");
  unsigned* tk = nullptr;  // one-launch form: a zeroed int32 ticket counter owned by the caller
  if (ticket.has_value() && ticket->defined()) {
    CHECK_DEV(*ticket); CHECK_I32(*ticket);
    TORCH_CHECK(ticket->numel() >= 1, "sumsq: ticket needs one int32");
    tk = reinterpret_cast<unsigned*>(ticket->data_ptr());
  }
  // extra (one fp32 element added to the sum) / guard (an int32 word copied as a float value
  // into out[1]): one-launch form only
  const bool hx = extra.has_value() && extra->defined();
  const bool hg = guard.has_value() && guard->defined();
  if (hx) {
    CHECK_DEV(*extra); CHECK_F32(*extra);
    TORCH_CHECK(tk && extra->numel() >= 1, "sumsq: extra needs the ticket form");
  }
  if (hg) {
    CHECK_DEV(*guard); CHECK_I32(*guard);
    TORCH_CHECK(tk && guard->numel() >= 1 && out.numel() >= 2, "sumsq: guard needs the ticket "
                "form and out[2]");
  }
  dcr::launch_sumsq(x.data_ptr(), x.scalar_type() == at::kBFloat16, x.numel(),
                    ptr<float>(partials), ptr<float>(out), tk, cur_stream(),
                    hx ? reinterpret_cast<const float*>(extra->data_ptr()) : nullptr,
                    hg ? reinterpret_cast<const int*>(guard->data_ptr()) : nullptr);
}

void adam_clip(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v,
               const c10::optional<at::Tensor>& pbf, at::Tensor& partials, at::Tensor& norm_out,
               double lr_t, double b1, double b2, double eps, double clip, double gscale,
               int64_t n_norm, const c10::optional<at::Tensor>& extra_sq,
               const c10::optional<at::Tensor>& skip_if,
               const c10::optional<at::Tensor>& lr_dev) {
  for (const at::Tensor* t : {(const at::Tensor*)&p, &g, (const at::Tensor*)&m, (const at::Tensor*)&v}) {
    CHECK_DEV(*t); CHECK_CONTIG(*t); CHECK_F32(*t); CHECK_ALIGN16(*t);
    TORCH_CHECK(t->numel() == p.numel(), "adam buffers must have equal numel");
  }
  bf16* pb = nullptr;
  if (pbf.has_value() && pbf->defined()) {
    CHECK_BF16(*pbf); CHECK_CONTIG(*pbf); CHECK_ALIGN16(*pbf);
    TORCH_CHECK(pbf->numel() == p.numel(), "bf16 mirror numel mismatch");
    pb = ptr<bf16>(*pbf);
  }
  TORCH_CHECK(partials.numel() >= dcr::opt_num_partials(p.numel()), "partials too small");
  if (n_norm < 0) n_norm = p.numel();
  TORCH_CHECK(n_norm <= p.numel(), "adam_clip: n_norm must be <= numel");
  const float* ex = nullptr;
  if (extra_sq.has_value() && extra_sq->defined()) {
    CHECK_DEV(*extra_sq); CHECK_F32(*extra_sq);
    TORCH_CHECK(extra_sq->numel() >= 1, "extra_sq: one element");
    ex = ptr<float>(*extra_sq);
  }
  if (skip_if.has_value() && skip_if->defined()) {
    CHECK_DEV(*skip_if);
    TORCH_CHECK(skip_if->element_size() == 4 && skip_if->numel() >= 1, "skip_if: one 32-bit word");
  }
  if (lr_dev.has_value() && lr_dev->defined()) {
    CHECK_DEV(*lr_dev); CHECK_F32(*lr_dev);
    TORCH_CHECK(lr_dev->numel() >= 1, "lr_dev: one fp32 element");
  }
  dcr::launch_adam_clip(ptr<float>(p), ptr<float>(g), ptr<float>(m), ptr<float>(v), pb,
                        p.numel(), ptr<float>(partials), ptr<float>(norm_out), (float)lr_t,
                        (float)b1, (float)b2, (float)eps, (float)clip, (float)gscale, n_norm, ex,
                        skip_if.has_value() && skip_if->defined()
                            ? reinterpret_cast<const unsigned*>(skip_if->data_ptr())
                            : nullptr,
                        lr_dev.has_value() && lr_dev->defined() ? ptr<float>(*lr_dev) : nullptr,
                        cur_stream());
}

// ------------------------------------------------------------------------------------------
// recurrent sequences: C++ time loop over the per-step kernels (rnn_step.hip)
// ------------------------------------------------------------------------------------------
template <typename T>
T* optr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}
bool has(const c10::optional<at::Tensor>& t) { return t.has_value() && t->defined(); }

void check_seq(const at::Tensor& t, at::ScalarType st, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == st, name, " has the wrong dtype");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name, " must be 16-B aligned");
}
void check_opt(const c10::optional<at::Tensor>& t, at::ScalarType st, const char* name) {
  if (has(t)) check_seq(*t, st, name);
}

void rnn_fwd_seq(int64_t cell, const at::Tensor& WT, const c10::optional<at::Tensor>& WT2,
                 const at::Tensor& zx, const c10::optional<at::Tensor>& ids, at::Tensor& hbuf,
                 const c10::optional<at::Tensor>& h32, const c10::optional<at::Tensor>& cbuf,
                 const c10::optional<at::Tensor>& gates, const c10::optional<at::Tensor>& pre,
                 const c10::optional<at::Tensor>& aux, const c10::optional<at::Tensor>& rh,
                 const c10::optional<at::Tensor>& hlast32, double forget_bias) {
  check_seq(WT, at::kBFloat16, "WT");
  check_seq(zx, at::kFloat, "zx");
  check_seq(hbuf, at::kBFloat16, "hbuf");
  check_opt(WT2, at::kBFloat16, "WT2");
  check_opt(ids, at::kInt, "ids");
  check_opt(h32, at::kFloat, "h32");
  check_opt(cbuf, at::kFloat, "cbuf");
  check_opt(gates, at::kBFloat16, "gates");
  check_opt(pre, at::kFloat, "pre");
  check_opt(aux, at::kFloat, "aux");
  check_opt(rh, at::kBFloat16, "rh");
  check_opt(hlast32, at::kFloat, "hlast32");
  TORCH_CHECK(hbuf.dim() == 3, "hbuf must be [T+1, B, H]");
  const int T = (int)hbuf.size(0) - 1, B = (int)hbuf.size(1), H = (int)hbuf.size(2);
  TORCH_CHECK(T >= 1 && B >= 1, "empty sequence");
  TORCH_CHECK(H % 32 == 0, "rnn_size must be a multiple of 32 on the GPU path");
  const int GW = (int)zx.size(-1);
  const bool gather = has(ids);
  if (gather) {
    TORCH_CHECK(ids->numel() == (int64_t)T * B, "ids must be [T, B]");
  } else {
    TORCH_CHECK(zx.numel() == (int64_t)T * B * GW, "zx must be [T, B, GW]");
  }
  TORCH_CHECK(GW % 4 == 0, "zx row must be a multiple of 4 floats");
  const size_t BH = (size_t)B * H;
  const int c = (int)cell;
  const int G = c == dcr::CELL_LSTM ? 4 : c == dcr::CELL_NAS ? 8 : c == dcr::CELL_GRU_A ? 3 : 1;
  TORCH_CHECK(WT.size(0) == (c == dcr::CELL_GRU_A ? 2 : G) * H && WT.size(1) == H, "WT shape");
  if (c == dcr::CELL_LSTM || c == dcr::CELL_NAS) TORCH_CHECK(has(cbuf), "cbuf required");
  if (c == dcr::CELL_GRU_A) TORCH_CHECK(has(h32) && has(rh) && has(gates) && has(WT2), "GRU buffers");
  if (c == dcr::CELL_NAS) TORCH_CHECK(has(pre) && has(aux), "NAS buffers");
  const int gld = has(gates) ? (int)gates->size(-1) : has(pre) ? (int)pre->size(-1) : 0;
  auto st = cur_stream();
  for (int t = 0; t < T; ++t) {
    dcr::FwdStepArgs a{};
    a.WT = ptr<bf16>(WT);
    a.ids = gather ? ptr<int>(*ids) + (size_t)t * B : nullptr;
    a.zx = gather ? ptr<float>(zx) : ptr<float>(zx) + (size_t)t * B * GW;
    a.zx_ld = GW;
    a.zx_off = 0;
    a.hop = ptr<bf16>(hbuf) + t * BH;
    a.hprev32 = has(h32) ? optr<float>(h32) + t * BH : nullptr;
    a.cprev = has(cbuf) ? optr<float>(cbuf) + t * BH : nullptr;
    a.hout = ptr<bf16>(hbuf) + (t + 1) * BH;
    a.hout32 = has(h32) ? optr<float>(h32) + (t + 1) * BH
                        : (t == T - 1 ? optr<float>(hlast32) : nullptr);
    a.cout = has(cbuf) ? optr<float>(cbuf) + (t + 1) * BH : nullptr;
    a.gates = has(gates) ? optr<bf16>(gates) + (size_t)t * B * gld : nullptr;
    a.pre = has(pre) ? optr<float>(pre) + (size_t)t * B * gld : nullptr;
    a.aux = has(aux) ? optr<float>(aux) + t * BH : nullptr;
    a.rh = has(rh) ? optr<bf16>(rh) + t * BH : nullptr;
    a.gates_ld = gld;
    a.B = B;
    a.H = H;
    a.forget_bias = (float)forget_bias;
    dcr::launch_fwd_step(c, a, st);
    if (c == dcr::CELL_GRU_A) {
      dcr::FwdStepArgs b2 = a;
      b2.WT = optr<bf16>(WT2);
      b2.zx_off = 2 * H;
      b2.hop = a.rh;
      dcr::launch_fwd_step(dcr::CELL_GRU_B, b2, st);
    }
  }
}

// One epilogue-only LSTM step (large-H library path, native_backend._lstm_seq_lib): the
// recurrent GEMM zrec = h_{t-1}·W_h ran as a library GEMM; this applies the cell forward
// (zx = input projection + bias rows, or the [V, 4H] table gathered by ids).
void lstm_step_ew_fwd(const at::Tensor& zrec, const at::Tensor& zx,
                      const c10::optional<at::Tensor>& ids, const at::Tensor& cprev,
                      at::Tensor& hout, const c10::optional<at::Tensor>& hout32, at::Tensor& cout,
                      at::Tensor& gates, double forget_bias,
                      const c10::optional<at::Tensor>& bias) {
  check_seq(zrec, at::kFloat, "zrec");
  check_seq(zx, at::kFloat, "zx");
  check_seq(cprev, at::kFloat, "cprev");
  check_seq(hout, at::kBFloat16, "hout");
  check_seq(cout, at::kFloat, "cout");
  check_seq(gates, at::kBFloat16, "gates");
  check_opt(ids, at::kInt, "ids");
  check_opt(hout32, at::kFloat, "hout32");
  const int B = (int)hout.size(0), H = (int)hout.size(1);
  TORCH_CHECK(H % 32 == 0 && zrec.numel() % ((int64_t)B * 4 * H) == 0 &&
                  gates.numel() == (int64_t)B * 4 * H, "lstm_step_ew_fwd: shapes");
  TORCH_CHECK(cprev.numel() == (int64_t)B * H && cout.numel() == cprev.numel(), "c shapes");
  TORCH_CHECK(zx.size(-1) == 4 * H, "zx row must be 4H");
  if (has(ids)) {
    TORCH_CHECK(ids->numel() == B, "ids must be [B]");
  } else {
    TORCH_CHECK(zx.numel() == (int64_t)B * 4 * H, "zx must be [B, 4H]");
  }
  dcr::LstmEwArgs a{};
  a.B = B;
  a.H = H;
  a.nsplit = (int)(zrec.numel() / ((int64_t)B * 4 * H));  // split-K slabs (step_gemm)
  a.forget_bias = (float)forget_bias;
  a.zrec = ptr<float>(zrec);
  a.zx = ptr<float>(zx);
  a.ids = has(ids) ? ptr<int>(*ids) : nullptr;
  if (has(bias)) {
    check_seq(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == 4 * H, "bias must be [4H]");
    a.bias = ptr<float>(*bias);
  }
  a.cprev = ptr<float>(cprev);
  a.hout = ptr<bf16>(hout);
  a.hout32 = optr<float>(hout32);
  a.cout = ptr<float>(cout);
  a.gates = ptr<bf16>(gates);
  dcr::launch_lstm_ew(false, a, cur_stream());
}

// One epilogue-only LSTM BPTT step: dh = dtop_t + dhrec (dhrec = dZ_{t+1}·W_hᵀ from a library
// GEMM, absent at the last step) -> dZ_t, dc.
void lstm_step_ew_bwd(const at::Tensor& dtop, const c10::optional<at::Tensor>& dhrec,
                      const at::Tensor& gates, const at::Tensor& c, const at::Tensor& cprev,
                      at::Tensor& dc, at::Tensor& dz_out) {
  check_seq(dtop, at::kFloat, "dtop");
  check_opt(dhrec, at::kFloat, "dhrec");
  if (has(dhrec)) {
    TORCH_CHECK(dhrec->numel() % dtop.numel() == 0, "dhrec must be [S, B, H]");
  }
  check_seq(gates, at::kBFloat16, "gates");
  check_seq(c, at::kFloat, "c");
  check_seq(cprev, at::kFloat, "cprev");
  check_seq(dc, at::kFloat, "dc");
  check_seq(dz_out, at::kBFloat16, "dz_out");
  const int B = (int)dtop.size(0), H = (int)dtop.size(1);
  TORCH_CHECK(H % 32 == 0 && gates.numel() == (int64_t)B * 4 * H &&
                  dz_out.numel() == gates.numel(), "lstm_step_ew_bwd: shapes");
  TORCH_CHECK(c.numel() == (int64_t)B * H && cprev.numel() == c.numel() && dc.numel() == c.numel(),
              "lstm_step_ew_bwd: state shapes");
  dcr::LstmEwArgs a{};
  a.B = B;
  a.H = H;
  a.nsplit = has(dhrec) ? (int)(dhrec->numel() / dtop.numel()) : 0;
  a.dtop = ptr<float>(dtop);
  a.dhrec = optr<float>(dhrec);
  a.gates_in = ptr<bf16>(gates);
  a.c = ptr<float>(c);
  a.cprev = ptr<float>(cprev);
  a.dc = ptr<float>(dc);
  a.dz_out = ptr<bf16>(dz_out);
  dcr::launch_lstm_ew(true, a, cur_stream());
}

int num_cus();

// Fused large-H LSTM steps (lstm_gemm_step.hip): the recurrent MFMA GEMM of one time step with
// the cell (or cell-backward) epilogue in the same launch.  ws / cnt: split-K slabs and arrival
// tickets (big_step_workspace; cnt zero-initialised once, the kernels leave it zero).
void check_big_ws(bool bwd, int B, int H, int64_t force_S, const at::Tensor& ws,
                  const at::Tensor& cnt) {
  TORCH_CHECK(dcr::big_step_supported(B, H), "big step: H must be a multiple of 128");
  int64_t wf = 0, nt = 0;
  dcr::big_step_workspace(bwd, B, H, num_cus(), (int)force_S, &wf, &nt);
  check_seq(ws, at::kFloat, "ws");
  TORCH_CHECK(ws.numel() >= wf, "big step: workspace too small (", ws.numel(), " < ", wf, ")");
  TORCH_CHECK(cnt.is_cuda() && cnt.element_size() == 4 && cnt.numel() >= nt,
              "big step: ticket buffer too small");
}

int64_t lstm_big_step_fwd(const at::Tensor& WhT, const at::Tensor& hprev, const at::Tensor& zx,
                          const c10::optional<at::Tensor>& ids, const at::Tensor& cprev,
                          at::Tensor& hout, const c10::optional<at::Tensor>& hout32,
                          at::Tensor& cout, at::Tensor& gates, at::Tensor& ws, at::Tensor& cnt,
                          double forget_bias, int64_t force_S,
                          const c10::optional<at::Tensor>& bias) {
  check_seq(WhT, at::kBFloat16, "WhT");
  check_seq(hprev, at::kBFloat16, "hprev");
  check_seq(zx, at::kFloat, "zx");
  check_seq(cprev, at::kFloat, "cprev");
  check_seq(hout, at::kBFloat16, "hout");
  check_seq(cout, at::kFloat, "cout");
  check_seq(gates, at::kBFloat16, "gates");
  check_opt(ids, at::kInt, "ids");
  check_opt(hout32, at::kFloat, "hout32");
  const int B = (int)hout.size(0), H = (int)hout.size(1);
  TORCH_CHECK(WhT.size(0) == 4 * H && WhT.size(1) == H, "WhT must be [4H, H]");
  TORCH_CHECK(hprev.numel() == (int64_t)B * H && cprev.numel() == hprev.numel() &&
                  cout.numel() == hprev.numel() && gates.numel() == (int64_t)B * 4 * H,
              "lstm_big_step_fwd: shapes");
  TORCH_CHECK(zx.size(-1) == 4 * H, "zx row must be 4H");
  if (has(ids)) {
    TORCH_CHECK(ids->numel() == B, "ids must be [B]");
  } else {
    TORCH_CHECK(zx.numel() == (int64_t)B * 4 * H, "zx must be [B, 4H]");
  }
  if (has(hout32)) TORCH_CHECK(hout32->numel() == (int64_t)B * H, "hout32 shape");
  check_big_ws(false, B, H, force_S, ws, cnt);
  dcr::BigStepArgs a{};
  a.B = B;
  a.H = H;
  a.A = ptr<bf16>(WhT);
  a.X = ptr<bf16>(hprev);
  a.ws = ptr<float>(ws);
  a.cnt = reinterpret_cast<unsigned*>(cnt.data_ptr());
  a.ew.B = B;
  a.ew.H = H;
  a.ew.forget_bias = (float)forget_bias;
  a.ew.zx = ptr<float>(zx);
  if (has(bias)) {
    check_seq(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == 4 * H, "bias must be [4H]");
    a.ew.bias = ptr<float>(*bias);
  }
  a.ew.ids = has(ids) ? ptr<int>(*ids) : nullptr;
  a.ew.cprev = ptr<float>(cprev);
  a.ew.hout = ptr<bf16>(hout);
  a.ew.hout32 = optr<float>(hout32);
  a.ew.cout = ptr<float>(cout);
  a.ew.gates = ptr<bf16>(gates);
  return dcr::launch_big_step(false, a, num_cus(), (int)force_S, cur_stream());
}

int64_t lstm_big_step_bwd(const at::Tensor& Wh, const at::Tensor& dznext, const at::Tensor& dtop,
                          const at::Tensor& gates, const at::Tensor& c, const at::Tensor& cprev,
                          at::Tensor& dc, at::Tensor& dz_out, at::Tensor& ws, at::Tensor& cnt,
                          int64_t force_S) {
  check_seq(Wh, at::kBFloat16, "Wh");
  check_seq(dznext, at::kBFloat16, "dznext");
  check_seq(dtop, at::kFloat, "dtop");
  check_seq(gates, at::kBFloat16, "gates");
  check_seq(c, at::kFloat, "c");
  check_seq(cprev, at::kFloat, "cprev");
  check_seq(dc, at::kFloat, "dc");
  check_seq(dz_out, at::kBFloat16, "dz_out");
  const int B = (int)dtop.size(0), H = (int)dtop.size(1);
  TORCH_CHECK(Wh.size(0) == H && Wh.size(1) == 4 * H, "Wh must be [H, 4H]");
  TORCH_CHECK(dznext.numel() == (int64_t)B * 4 * H && gates.numel() == dznext.numel() &&
                  dz_out.numel() == dznext.numel(), "lstm_big_step_bwd: shapes");
  TORCH_CHECK(c.numel() == (int64_t)B * H && cprev.numel() == c.numel() && dc.numel() == c.numel(),
              "lstm_big_step_bwd: state shapes");
  TORCH_CHECK(dznext.data_ptr() != dz_out.data_ptr(), "dznext and dz_out must differ");
  check_big_ws(true, B, H, force_S, ws, cnt);
  dcr::BigStepArgs a{};
  a.B = B;
  a.H = H;
  a.A = ptr<bf16>(Wh);
  a.X = ptr<bf16>(dznext);
  a.ws = ptr<float>(ws);
  a.cnt = reinterpret_cast<unsigned*>(cnt.data_ptr());
  a.ew.B = B;
  a.ew.H = H;
  a.ew.dtop = ptr<float>(dtop);
  a.ew.gates_in = ptr<bf16>(gates);
  a.ew.c = ptr<float>(c);
  a.ew.cprev = ptr<float>(cprev);
  a.ew.dc = ptr<float>(dc);
  a.ew.dz_out = ptr<bf16>(dz_out);
  return dcr::launch_big_step(true, a, num_cus(), (int)force_S, cur_stream());
}

// fp32-operand sequences (cell_f32.hip): the native --dtype fp32 recurrence
dcr::F32Seq f32_seq_common(int64_t cell, const at::Tensor& hs, const at::Tensor& gates_or_dz) {
  check_seq(hs, at::kFloat, "hs");
  TORCH_CHECK(hs.dim() == 3, "hs must be [T+1, B, H]");
  dcr::F32Seq q{};
  q.cell = (int)cell;
  q.T = (int)hs.size(0) - 1;
  q.B = (int)hs.size(1);
  q.H = (int)hs.size(2);
  q.GW = (int)gates_or_dz.size(-1);
  TORCH_CHECK(q.T >= 1 && q.B >= 1, "empty sequence");
  TORCH_CHECK(dcr::f32_seq_supported(q.cell, q.H), "f32 sequence: unsupported cell / rnn_size");
  const int G = q.cell == dcr::CELL_LSTM ? 4 : q.cell == dcr::CELL_GRU_A ? 3 : 1;
  TORCH_CHECK(q.GW == G * q.H, "row width must be G * H");
  return q;
}

void f32_fwd_seq(int64_t cell, const at::Tensor& WT, const c10::optional<at::Tensor>& WT2,
                 const at::Tensor& zx, at::Tensor& hs, const c10::optional<at::Tensor>& cs,
                 const c10::optional<at::Tensor>& gates, const c10::optional<at::Tensor>& rh,
                 double forget_bias) {
  dcr::F32Seq q = f32_seq_common(cell, hs, zx);
  check_seq(WT, at::kFloat, "WT");
  check_seq(zx, at::kFloat, "zx");
  check_opt(WT2, at::kFloat, "WT2");
  check_opt(cs, at::kFloat, "cs");
  check_opt(gates, at::kFloat, "gates");
  check_opt(rh, at::kFloat, "rh");
  const int64_t T = q.T, B = q.B, H = q.H;
  TORCH_CHECK(zx.numel() == T * B * q.GW, "zx must be [T, B, GW]");
  const bool gru = q.cell == dcr::CELL_GRU_A, lstm = q.cell == dcr::CELL_LSTM;
  TORCH_CHECK(WT.size(0) == (gru ? 2 : lstm ? 4 : 1) * H && WT.size(1) == H, "WT shape");
  if (lstm) TORCH_CHECK(has(cs) && cs->numel() == (T + 1) * B * H, "cs must be [T+1, B, H]");
  if (lstm || gru) TORCH_CHECK(has(gates) && gates->numel() == T * B * q.GW, "gates must be [T, B, GW]");
  if (gru) {
    TORCH_CHECK(has(WT2) && WT2->size(0) == H && WT2->size(1) == H, "WT2 must be [H, H]");
    TORCH_CHECK(has(rh) && rh->numel() == T * B * H, "rh must be [T, B, H]");
  }
  q.WT = ptr<float>(WT);
  q.WT2 = optr<float>(WT2);
  q.zx = ptr<float>(zx);
  q.hs = ptr<float>(hs);
  q.cs = optr<float>(cs);
  q.gates = optr<float>(gates);
  q.rh = optr<float>(rh);
  q.forget_bias = (float)forget_bias;
  dcr::launch_f32_fwd_seq(q, cur_stream());
}

void f32_bwd_seq(int64_t cell, const at::Tensor& W, const c10::optional<at::Tensor>& W2,
                 const c10::optional<at::Tensor>& dtop, const at::Tensor& hs,
                 const c10::optional<at::Tensor>& cs, const c10::optional<at::Tensor>& gates,
                 at::Tensor& dz, at::Tensor& work0, at::Tensor& work1) {
  dcr::F32Seq q = f32_seq_common(cell, hs, dz);
  check_seq(W, at::kFloat, "W");
  check_opt(W2, at::kFloat, "W2");
  check_opt(dtop, at::kFloat, "dtop");
  check_opt(cs, at::kFloat, "cs");
  check_opt(gates, at::kFloat, "gates");
  check_seq(dz, at::kFloat, "dz");
  check_seq(work0, at::kFloat, "work0");
  check_seq(work1, at::kFloat, "work1");
  const int64_t T = q.T, B = q.B, H = q.H;
  const bool gru = q.cell == dcr::CELL_GRU_A, lstm = q.cell == dcr::CELL_LSTM;
  TORCH_CHECK(dz.numel() == T * B * q.GW, "dz must be [T, B, GW]");
  TORCH_CHECK(work0.numel() >= B * H && work1.numel() >= B * H, "work buffers must hold [B, H]");
  if (has(dtop)) TORCH_CHECK(dtop->numel() == T * B * H, "dtop must be [T, B, H]");
  if (lstm) TORCH_CHECK(has(cs) && cs->numel() == (T + 1) * B * H, "cs must be [T+1, B, H]");
  if (lstm || gru) TORCH_CHECK(has(gates) && gates->numel() == T * B * q.GW, "gates must be [T, B, GW]");
  if (gru) {
    TORCH_CHECK(W.size(0) == H && W.size(1) == H, "W (Wc_h) must be [H, H]");
    TORCH_CHECK(has(W2) && W2->size(0) == H && W2->size(1) == 2 * H, "W2 (Wg_h) must be [H, 2H]");
  } else {
    TORCH_CHECK(W.size(0) == H && W.size(1) == q.GW, "W must be [H, GW]");
  }
  q.W = ptr<float>(W);
  q.W2 = optr<float>(W2);
  q.dtop = optr<float>(dtop);
  q.hs = const_cast<float*>(ptr<float>(hs));
  q.cs = const_cast<float*>(optr<float>(cs));
  q.gates = optr<float>(gates);
  q.dz = ptr<float>(dz);
  q.work0 = ptr<float>(work0);
  q.work1 = ptr<float>(work1);
  dcr::launch_f32_bwd_seq(q, cur_stream());
}

void rnn_bwd_seq(int64_t cell, const at::Tensor& W, const c10::optional<at::Tensor>& W2,
                 const at::Tensor& dtop, at::Tensor& dz, const c10::optional<at::Tensor>& dzx,
                 const c10::optional<at::Tensor>& gates, const c10::optional<at::Tensor>& pre,
                 const c10::optional<at::Tensor>& aux, const c10::optional<at::Tensor>& zx,
                 const c10::optional<at::Tensor>& cbuf, const c10::optional<at::Tensor>& h32,
                 const c10::optional<at::Tensor>& hbuf, at::Tensor& dc,
                 const c10::optional<at::Tensor>& partial) {
  check_seq(W, at::kBFloat16, "W");
  check_seq(dtop, at::kFloat, "dtop");
  check_seq(dz, at::kBFloat16, "dz");
  check_seq(dc, at::kFloat, "dc");
  check_opt(W2, at::kBFloat16, "W2");
  check_opt(dzx, at::kBFloat16, "dzx");
  check_opt(gates, at::kBFloat16, "gates");
  check_opt(pre, at::kFloat, "pre");
  check_opt(aux, at::kFloat, "aux");
  check_opt(zx, at::kFloat, "zx");
  check_opt(cbuf, at::kFloat, "cbuf");
  check_opt(h32, at::kFloat, "h32");
  check_opt(hbuf, at::kBFloat16, "hbuf");
  check_opt(partial, at::kFloat, "partial");
  TORCH_CHECK(dtop.dim() == 3, "dtop must be [T, B, H]");
  const int T = (int)dtop.size(0), B = (int)dtop.size(1), H = (int)dtop.size(2);
  TORCH_CHECK(H % 32 == 0, "rnn_size must be a multiple of 32 on the GPU path");
  const int GW = (int)dz.size(-1);
  TORCH_CHECK(dz.numel() == (int64_t)T * B * GW, "dz must be [T, B, GW]");
  TORCH_CHECK(dc.numel() == (int64_t)B * H, "dc must be [B, H]");
  const size_t BH = (size_t)B * H;
  const size_t BG = (size_t)B * GW;
  auto st = cur_stream();
  const int c = (int)cell;
  (void)hipMemsetAsync(dc.data_ptr(), 0, sizeof(float) * BH, st);
  if (c == dcr::CELL_GRU_A) {
    TORCH_CHECK(has(W2) && has(gates) && has(h32) && has(partial), "GRU buffers");
    TORCH_CHECK(GW == 3 * H, "GRU dz must be [T, B, 3H]");
    const int gld = (int)gates->size(-1);
    dcr::BwdStepArgs i{};
    i.dtop = ptr<float>(dtop) + (T - 1) * BH;
    i.gates = optr<bf16>(gates) + (size_t)(T - 1) * B * gld;
    i.dc = ptr<float>(dc);
    i.dz_out = ptr<bf16>(dz) + (T - 1) * BG + 2 * H;
    i.dz_out_ld = GW;
    i.gates_ld = gld;
    i.B = B;
    i.H = H;
    dcr::launch_bwd_step(dcr::CELL_GRU_B, i, st);
    for (int t = T - 1; t >= 0; --t) {
      dcr::BwdStepArgs a{};
      a.W = ptr<bf16>(W);
      a.K = H;
      a.dz_next = ptr<bf16>(dz) + t * BG + 2 * H;
      a.dz_ld = GW;
      a.gates = optr<bf16>(gates) + (size_t)t * B * gld;
      a.gates_ld = gld;
      a.hprev32 = optr<float>(h32) + t * BH;
      a.dc = ptr<float>(dc);
      a.partial = optr<float>(partial);
      a.dz_out = ptr<bf16>(dz) + t * BG;
      a.dz_out_ld = GW;
      a.B = B;
      a.H = H;
      dcr::launch_bwd_step(dcr::CELL_GRU_A, a, st);
      if (t > 0) {
        dcr::BwdStepArgs b{};
        b.W = optr<bf16>(W2);
        b.K = 2 * H;
        b.dz_next = ptr<bf16>(dz) + t * BG;
        b.dz_ld = GW;
        b.dtop = ptr<float>(dtop) + (t - 1) * BH;
        b.partial = optr<float>(partial);
        b.gates = optr<bf16>(gates) + (size_t)(t - 1) * B * gld;
        b.gates_ld = gld;
        b.dc = ptr<float>(dc);
        b.dz_out = ptr<bf16>(dz) + (t - 1) * BG + 2 * H;
        b.dz_out_ld = GW;
        b.B = B;
        b.H = H;
        dcr::launch_bwd_step(dcr::CELL_GRU_B, b, st);
      }
    }
    return;
  }
  const int K = GW;  // LSTM 4H, RNN H, NAS 8H
  TORCH_CHECK(W.size(0) == H && W.size(1) == K, "W must be [H, G*H]");
  if (c == dcr::CELL_LSTM) TORCH_CHECK(has(gates) && has(cbuf), "LSTM buffers");
  if (c == dcr::CELL_RNN) TORCH_CHECK(has(hbuf), "RNN buffers");
  if (c == dcr::CELL_NAS) TORCH_CHECK(has(pre) && has(aux) && has(zx) && has(cbuf) && has(dzx), "NAS buffers");
  const int gld = has(gates) ? (int)gates->size(-1) : has(pre) ? (int)pre->size(-1) : 0;
  for (int t = T - 1; t >= 0; --t) {
    dcr::BwdStepArgs a{};
    a.W = ptr<bf16>(W);
    a.K = K;
    a.dz_next = (t < T - 1) ? ptr<bf16>(dz) + (t + 1) * BG : nullptr;
    a.dz_ld = GW;
    a.dtop = ptr<float>(dtop) + t * BH;
    a.gates = has(gates) ? optr<bf16>(gates) + (size_t)t * B * gld : nullptr;
    a.pre = has(pre) ? optr<float>(pre) + (size_t)t * B * gld : nullptr;
    a.aux = has(aux) ? optr<float>(aux) + t * BH : nullptr;
    a.zx3 = has(zx) ? optr<float>(zx) + (size_t)t * B * GW + 3 * H : nullptr;
    a.zx3_ld = GW;
    a.c = has(cbuf) ? optr<float>(cbuf) + (t + 1) * BH : nullptr;
    a.cprev = has(cbuf) ? optr<float>(cbuf) + t * BH : nullptr;
    a.hcur = has(hbuf) ? optr<bf16>(hbuf) + (t + 1) * BH : nullptr;
    a.dc = ptr<float>(dc);
    a.dz_out = ptr<bf16>(dz) + t * BG;
    a.dzx_out = has(dzx) ? optr<bf16>(dzx) + t * BG : nullptr;
    a.dz_out_ld = GW;
    a.gates_ld = gld;
    a.B = B;
    a.H = H;
    dcr::launch_bwd_step(c, a, st);
  }
}

// ------------------------------------------------------------------------------------------
// loss + segment sums
// ------------------------------------------------------------------------------------------
void xent(const at::Tensor& logits, const at::Tensor& targets, double grad_scale,
          const c10::optional<at::Tensor>& row_loss, const c10::optional<at::Tensor>& dlogits,
          at::Tensor& partial, at::Tensor& loss_out) {
  check_seq(logits, at::kFloat, "logits");
  check_seq(targets, at::kInt, "targets");
  check_opt(row_loss, at::kFloat, "row_loss");
  check_opt(dlogits, at::kBFloat16, "dlogits");
  TORCH_CHECK(logits.dim() == 2, "logits must be [N, V]");
  const int N = (int)logits.size(0), V = (int)logits.size(1);
  TORCH_CHECK(targets.numel() == N, "targets must be [N]");
  TORCH_CHECK(partial.numel() >= dcr::xent_num_partials(N), "partial too small");
  dcr::launch_xent(ptr<float>(logits), ptr<int>(targets), N, V, (float)grad_scale,
                   optr<float>(row_loss), optr<bf16>(dlogits), ptr<float>(partial),
                   ptr<float>(loss_out), cur_stream());
}

// wide-vocabulary CE with fused d softmax_b (workspace: [xent_wide_waves(N), V] column partials)
void xent_wide(const at::Tensor& logits, const c10::optional<at::Tensor>& bias,
               const at::Tensor& targets, double grad_scale,
               const c10::optional<at::Tensor>& row_loss, const c10::optional<at::Tensor>& dlogits,
               const c10::optional<at::Tensor>& colpart, const c10::optional<at::Tensor>& db,
               at::Tensor& partial, at::Tensor& loss_out) {
  check_seq(logits, at::kFloat, "logits");
  check_seq(targets, at::kInt, "targets");
  check_opt(row_loss, at::kFloat, "row_loss");
  check_opt(dlogits, at::kBFloat16, "dlogits");
  check_opt(colpart, at::kFloat, "colpart");
  check_opt(db, at::kFloat, "db");
  TORCH_CHECK(logits.dim() == 2, "logits must be [N, V]");
  const int N = (int)logits.size(0), V = (int)logits.size(1);
  TORCH_CHECK(dcr::xent_wide_supported(V), "xent_wide needs V % 4 == 0 and V <= 16384");
  check_opt(bias, at::kFloat, "bias");
  if (has(bias)) TORCH_CHECK(bias->numel() == V, "bias must be [V]");
  TORCH_CHECK(targets.numel() == N, "targets must be [N]");
  if (has(dlogits)) TORCH_CHECK(dlogits->numel() == (int64_t)N * V, "dlogits must be [N, V]");
  if (has(db)) {
    TORCH_CHECK(has(colpart) && has(dlogits), "db needs dlogits and colpart");
    TORCH_CHECK(db->numel() == V, "db must be [V]");
  }
  if (has(colpart))
    TORCH_CHECK(colpart->numel() >= (int64_t)dcr::xent_wide_waves(N) * V, "colpart too small");
  TORCH_CHECK(partial.numel() >= dcr::xent_wide_blocks(N), "partial too small");
  dcr::launch_xent_wide(ptr<float>(logits), optr<float>(bias), ptr<int>(targets), N, V,
                        (float)grad_scale,
                        optr<float>(row_loss), optr<bf16>(dlogits), optr<float>(colpart),
                        optr<float>(db), ptr<float>(partial), ptr<float>(loss_out), cur_stream());
}

// fused wide-vocabulary head (head_wide.hip); colpart [head_wide_colpart_rows(N), V]; workspace ws
// [head_wide_workspace(N)] = loss partials + the two passes' softmax stats
void head_wide(const at::Tensor& O, const at::Tensor& WsT, const c10::optional<at::Tensor>& bias,
               const c10::optional<at::Tensor>& targets, double grad_scale,
               const c10::optional<at::Tensor>& row_loss, const c10::optional<at::Tensor>& dlogits,
               const c10::optional<at::Tensor>& logits, const c10::optional<at::Tensor>& colpart,
               const c10::optional<at::Tensor>& db, at::Tensor& ws, at::Tensor& loss_out) {
  TORCH_CHECK(O.is_cuda() && O.dim() == 2 && O.scalar_type() == at::kBFloat16 && O.stride(1) == 1,
              "O must be a row-major bf16 [N, H] GPU tensor");
  check_seq(WsT, at::kBFloat16, "WsT");
  const int N = (int)O.size(0), H = (int)O.size(1), V = (int)WsT.size(0);
  TORCH_CHECK(WsT.dim() == 2 && WsT.size(1) == H, "WsT must be [V, H]");
  TORCH_CHECK(dcr::head_wide_supported(V, H), "fused wide head: H = 512, V % 64 == 0");
  check_opt(bias, at::kFloat, "bias");
  check_opt(targets, at::kInt, "targets");
  check_opt(row_loss, at::kFloat, "row_loss");
  check_opt(dlogits, at::kBFloat16, "dlogits");
  check_opt(logits, at::kFloat, "logits");
  check_opt(colpart, at::kFloat, "colpart");
  check_opt(db, at::kFloat, "db");
  check_seq(ws, at::kFloat, "ws");
  if (has(bias)) TORCH_CHECK(bias->numel() == V, "bias must be [V]");
  if (has(targets)) TORCH_CHECK(targets->numel() == N, "targets must be [N]");
  if (has(row_loss)) TORCH_CHECK(row_loss->numel() == N, "row_loss must be [N]");
  if (has(dlogits)) TORCH_CHECK(dlogits->numel() == (int64_t)N * V, "dlogits must be [N, V]");
  if (has(logits)) TORCH_CHECK(logits->numel() == (int64_t)N * V, "logits must be [N, V]");
  const int nb = dcr::head_wide_blocks(N);
  if (has(colpart))
    TORCH_CHECK(colpart->numel() >= (int64_t)dcr::head_wide_colpart_rows(N) * V, "colpart too small");
  if (has(db)) TORCH_CHECK(has(colpart) && has(dlogits) && db->numel() == V, "db needs colpart, dlogits, [V]");
  const int64_t soff = (nb + 3) / 4 * 4;  // stats 16-B aligned behind the partials
  TORCH_CHECK(ws.numel() >= soff + (int64_t)dcr::head_wide_stats_floats(N), "ws too small");
  dcr::HeadWideArgs a{};
  a.O = ptr<bf16>(O); a.ldo = (int)O.stride(0);
  a.WsT = ptr<bf16>(WsT); a.bias = optr<float>(bias); a.targets = optr<int>(targets);
  a.N = N; a.V = V; a.H = H; a.grad_scale = (float)grad_scale;
  a.row_loss = optr<float>(row_loss); a.dlogits = optr<bf16>(dlogits);
  a.logits = optr<float>(logits); a.colpart = optr<float>(colpart);
  a.partial = ptr<float>(ws);
  a.stats = ptr<float>(ws) + soff;
  TORCH_CHECK(dcr::launch_head_wide(a, optr<float>(db), ptr<float>(loss_out), cur_stream()) == 0,
              "fused wide head not launched");
}

void segsum(const at::Tensor& X, const c10::optional<at::Tensor>& ids, int64_t V, at::Tensor& out,
            at::Tensor& workspace, bool accumulate, const c10::optional<at::Tensor>& perm) {
  TORCH_CHECK(X.is_cuda() && X.dim() == 2 && X.stride(1) == 1, "X must be a row-major 2-D GPU tensor");
  const int N = (int)X.size(0), W = (int)X.size(1), ldx = (int)X.stride(0);
  check_opt(ids, at::kInt, "ids");
  check_seq(out, at::kFloat, "out");
  TORCH_CHECK(out.numel() == V * W, "out must be [V, W]");
  TORCH_CHECK((size_t)workspace.numel() >= dcr::segsum_workspace_floats(N, W, (int)V), "workspace too small");
  if (has(ids)) {
    TORCH_CHECK(ids->numel() == N, "ids must be [N]");
  } else {
    TORCH_CHECK(V == 1, "without ids, V must be 1 (column sum)");
  }
  check_opt(perm, at::kInt, "perm");
  if (has(perm))
    TORCH_CHECK(has(ids) && perm->numel() == N, "perm needs (sorted) ids and must be [N]");
  if (X.scalar_type() == at::kBFloat16) {
    dcr::launch_segsum_bf16(ptr<bf16>(X), ldx, optr<int>(ids), N, W, (int)V, ptr<float>(out),
                            ptr<float>(workspace), accumulate ? 1 : 0, cur_stream(),
                            optr<int>(perm));
  } else {
    TORCH_CHECK(X.scalar_type() == at::kFloat, "X must be bf16 or fp32");
    dcr::launch_segsum_f32(ptr<float>(X), ldx, optr<int>(ids), N, W, (int)V, ptr<float>(out),
                           ptr<float>(workspace), accumulate ? 1 : 0, cur_stream(),
                           optr<int>(perm));
  }
}

// stable counting sort of ids (embed.hip): sid = sorted ids, perm = their source positions
// zero (optional): an fp32 buffer the first launch clears on the side (the atomic segment sum's
// output, so that it needs no fill launch); returns whether it did (alignment / size permitting)
bool id_sort(const at::Tensor& ids, int64_t V, at::Tensor& ws, at::Tensor& sid, at::Tensor& perm,
             const c10::optional<at::Tensor>& zero) {
  check_seq(ids, at::kInt, "ids");
  check_seq(ws, at::kInt, "ws");
  check_seq(sid, at::kInt, "sid");
  check_seq(perm, at::kInt, "perm");
  const int N = (int)ids.numel();
  TORCH_CHECK(sid.numel() == N && perm.numel() == N, "id_sort: sid and perm must be [N]");
  TORCH_CHECK(V > 0 && (size_t)ws.numel() >= dcr::id_sort_workspace(N, (int)V),
              "id_sort: workspace too small");
  float* zp = nullptr;
  size_t zn = 0;
  if (has(zero)) {
    TORCH_CHECK(zero->is_cuda() && zero->scalar_type() == at::kFloat && zero->is_contiguous(),
                "id_sort: zero must be a contiguous fp32 GPU tensor");
    if (zero->numel() % 4 == 0 && (reinterpret_cast<uintptr_t>(zero->data_ptr()) & 15) == 0) {
      zp = zero->data_ptr<float>();
      zn = (size_t)zero->numel();
    }
  }
  TORCH_CHECK(dcr::launch_id_sort(ptr<int>(ids), N, (int)V, ptr<int>(ws), ptr<int>(sid),
                                  ptr<int>(perm), cur_stream(), zp, zn) == 0,
              "id_sort: unsupported vocabulary size ", V);
  return zp != nullptr;
}

// ------------------------------------------------------------------------------------------
// persistent LSTM recurrence (lstm_persist.hip)
// ------------------------------------------------------------------------------------------
int num_cus() {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    cus = (hipGetDeviceProperties(&prop, dev) == hipSuccess) ? prop.multiProcessorCount : 0;
  }
  return cus;
}

int64_t lstm_persist_nt_tiles(int64_t H, int64_t B) {
  return dcr::lstm_persist_nt_tiles((int)H, (int)B, num_cus());
}

int64_t lstm_persist_supported(int64_t H, int64_t B) {
  return dcr::lstm_persist_supported((int)H, (int)B, num_cus());
}

void lstm_persist_fwd(const at::Tensor& WT, const at::Tensor& zx, const c10::optional<at::Tensor>& ids,
                      at::Tensor& hbuf, at::Tensor& cbuf, const c10::optional<at::Tensor>& gates,
                      at::Tensor& hlast32, at::Tensor& cnt, at::Tensor& err, double forget_bias,
                      int64_t spin_limit, at::Tensor& hring,
                      const c10::optional<at::Tensor>& diag, const c10::optional<at::Tensor>& WxT,
                      const c10::optional<at::Tensor>& xin, const c10::optional<at::Tensor>& bias,
                      bool cnt_zeroed, const c10::optional<at::Tensor>& clast32) {
  check_seq(WT, at::kBFloat16, "WT");
  check_seq(zx, at::kFloat, "zx");
  check_seq(hbuf, at::kBFloat16, "hbuf");
  check_seq(cbuf, at::kFloat, "cbuf");
  check_seq(hlast32, at::kFloat, "hlast32");
  check_opt(gates, at::kBFloat16, "gates");
  check_opt(ids, at::kInt, "ids");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == at::kInt && err.scalar_type() == at::kInt,
              "cnt/err must be int32 GPU tensors");
  const int T = (int)hbuf.size(0) - 1, B = (int)hbuf.size(1), H = (int)hbuf.size(2);
  TORCH_CHECK(dcr::lstm_persist_supported(H, B, num_cus()), "persistent LSTM unsupported for this shape");
  TORCH_CHECK(WT.size(0) == 4 * H && WT.size(1) == H, "WT must be [4H, H]");
  TORCH_CHECK(zx.size(-1) == 4 * H, "zx rows must be 4H wide");
  const bool xfuse = has(WxT);
  if (xfuse) {
    check_seq(*WxT, at::kBFloat16, "WxT");
    TORCH_CHECK(has(xin) && has(bias), "fused input projection needs xin and bias");
    check_seq(*xin, at::kBFloat16, "xin");
    check_seq(*bias, at::kFloat, "bias");
    TORCH_CHECK(WxT->size(0) == 4 * H && WxT->size(1) == H, "WxT must be [4H, H]");
    TORCH_CHECK(xin->numel() == (int64_t)T * B * H && bias->numel() == 4 * H, "xin/bias shape");
    TORCH_CHECK(dcr::lstm_persist_xfuse_supported(H, B, num_cus()), "fused-input persistent LSTM unsupported");
  } else if (has(ids)) {
    TORCH_CHECK(ids->numel() == (int64_t)T * B, "ids must be [T, B]");
  } else {
    TORCH_CHECK(zx.numel() == (int64_t)T * B * 4 * H, "zx must be [T, B, 4H]");
  }
  if (!xfuse && has(bias)) {  // input bias added in the cell epilogue (H > 1024 kernels)
    TORCH_CHECK(H > 1024, "an in-kernel input bias without the fused projection needs H > 1024");
    check_seq(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == 4 * H, "bias must be [4H]");
  }
  if (has(gates)) TORCH_CHECK(gates->numel() == (int64_t)T * B * 4 * H, "gates must be [T, B, 4H]");
  TORCH_CHECK(cnt.numel() >= (int64_t)((B + 15) / 16) * (T + 1) * 4, "counter buffer too small");
  dcr::PersistArgs a{};
  a.W = ptr<bf16>(WT);
  a.zx = ptr<float>(zx);
  a.ids = optr<int>(ids);
  a.zx_ld = 4 * H;
  a.hbuf = ptr<bf16>(hbuf);
  a.cbuf = ptr<float>(cbuf);
  a.gates = optr<bf16>(gates);
  a.hlast32 = ptr<float>(hlast32);
  a.cnt = reinterpret_cast<unsigned*>(cnt.data_ptr());
  a.err = reinterpret_cast<unsigned*>(err.data_ptr());
  a.B = B; a.H = H; a.T = T;
  a.forget_bias = (float)forget_bias;
  a.spin_limit = (unsigned)spin_limit;
  if (xfuse) {
    a.Wx = optr<bf16>(WxT);
    a.xin = optr<bf16>(xin);
  }
  a.bias = optr<float>(bias);
  if (has(diag)) {
    TORCH_CHECK(diag->element_size() == 8 && diag->numel() >= (int64_t)T * 8, "diag must hold [T, 8] int64");
    a.diag = reinterpret_cast<unsigned long long*>(diag->data_ptr());
  }
  a.cnt_zeroed = cnt_zeroed ? 1 : 0;
  if (has(clast32)) {
    check_seq(*clast32, at::kFloat, "clast32");
    TORCH_CHECK(clast32->numel() == (int64_t)B * H, "clast32 must be [B, H]");
    a.clast32 = ptr<float>(*clast32);
  }
  check_seq(hring, at::kBFloat16, "hring");
  TORCH_CHECK(hring.numel() >= (int64_t)2 * ((B + 15) / 16 * 16) * H, "hring must hold [2, ceil16(B), H]");
  a.hring = ptr<bf16>(hring);
  const int rc = dcr::launch_lstm_fwd_persist(a, num_cus(), cur_stream());
  TORCH_CHECK(rc == 0, "persistent LSTM forward not launched (", rc,
              "): grid cannot be co-resident on this GPU for H=", H, " B=", B);
}

void lstm_persist_bwd(const at::Tensor& W, const at::Tensor& dtop, at::Tensor& dz,
                      const at::Tensor& gates, const at::Tensor& cbuf, at::Tensor& cnt,
                      at::Tensor& err, int64_t spin_limit, at::Tensor& zring,
                      const c10::optional<at::Tensor>& db_part, const c10::optional<at::Tensor>& ids,
                      const c10::optional<at::Tensor>& dew_part, int64_t V,
                      const c10::optional<at::Tensor>& diag, bool exclusive, bool cnt_zeroed) {
  check_seq(W, at::kBFloat16, "W");
  check_seq(dtop, at::kFloat, "dtop");
  check_seq(dz, at::kBFloat16, "dz");
  check_seq(gates, at::kBFloat16, "gates");
  check_seq(cbuf, at::kFloat, "cbuf");
  const int T = (int)dtop.size(0), B = (int)dtop.size(1), H = (int)dtop.size(2);
  TORCH_CHECK(dcr::lstm_persist_supported(H, B, num_cus()), "persistent LSTM unsupported for this shape");
  TORCH_CHECK(W.size(0) == H && W.size(1) == 4 * H, "W must be [H, 4H]");
  TORCH_CHECK(dz.numel() == (int64_t)T * B * 4 * H && gates.numel() == (int64_t)T * B * 4 * H, "dz/gates shape");
  TORCH_CHECK(cbuf.numel() == (int64_t)(T + 1) * B * H, "cbuf shape");
  TORCH_CHECK(cnt.numel() >= (int64_t)((B + 15) / 16) * (T + 1) * 4, "counter buffer too small");
  dcr::PersistArgs a{};
  a.W = ptr<bf16>(W);
  a.dtop = ptr<float>(dtop);
  a.dz = ptr<bf16>(dz);
  a.gates = ptr<bf16>(gates);
  a.cbuf = ptr<float>(cbuf);
  a.cnt = reinterpret_cast<unsigned*>(cnt.data_ptr());
  a.err = reinterpret_cast<unsigned*>(err.data_ptr());
  a.B = B; a.H = H; a.T = T;
  a.spin_limit = (unsigned)spin_limit;
  check_opt(db_part, at::kFloat, "db_part");
  check_opt(dew_part, at::kFloat, "dew_part");
  check_opt(ids, at::kInt, "ids");
  if (has(db_part))
    TORCH_CHECK(db_part->numel() == (int64_t)((B + 15) / 16) * 4 * H, "db_part must be [ceil(B/16), 4H]");
  a.db_part = optr<float>(db_part);
  if (has(dew_part)) {
    TORCH_CHECK(has(ids) && ids->numel() == (int64_t)T * B, "dew_part needs ids [T, B]");
    TORCH_CHECK(V >= 1 && V <= 128, "fused dEW supports V <= 128");
    TORCH_CHECK(dew_part->numel() == (int64_t)((B + 15) / 16) * V * 4 * H,
                "dew_part must be [ceil(B/16), V, 4H]");
    a.dew_part = optr<float>(dew_part);
    a.ids = optr<int>(ids);
    a.V = (int)V;
  }
  if (has(diag)) {
    TORCH_CHECK(diag->element_size() == 8 && diag->numel() >= (int64_t)T * 8, "diag must hold [T, 8] int64");
    a.diag = reinterpret_cast<unsigned long long*>(diag->data_ptr());
  }
  a.excl = exclusive ? 1 : 0;
  a.cnt_zeroed = cnt_zeroed ? 1 : 0;
  check_seq(zring, at::kBFloat16, "zring");
  TORCH_CHECK(zring.numel() >= (int64_t)2 * ((B + 15) / 16 * 16) * 4 * H,
              "zring must hold [2, ceil16(B), 4H]");
  a.zring = ptr<bf16>(zring);
  const int rc = dcr::launch_lstm_bwd_persist(a, num_cus(), cur_stream());
  TORCH_CHECK(rc == 0, "persistent LSTM BPTT not launched (", rc,
              "): grid cannot be co-resident on this GPU for H=", H, " B=", B);
}

// two-layer wavefront LSTM forward (lstm2_persist.hip)
// ------------------------------------------------------------------------------------------
static int lstm2_nbg(int B, int G) { return ((B + 31) / 32 + G - 1) / G * G; }

// dropout bit masks (dropout.hip): [T, B, H/8] uint8, time-major rows
static const uint8_t* drop_bits(const c10::optional<at::Tensor>& m, int T, int B, int H,
                                const char* name) {
  if (!has(m)) return nullptr;
  TORCH_CHECK(m->is_cuda() && m->is_contiguous() && m->scalar_type() == at::kByte, name,
              " must be a contiguous uint8 GPU tensor");
  TORCH_CHECK(m->numel() == (int64_t)T * B * (H / 8), name, " must be [T, B, H/8]");
  return reinterpret_cast<const uint8_t*>(m->data_ptr());
}

void dropout_bits(at::Tensor& bits, int64_t seed, int64_t stream, double keep) {
  TORCH_CHECK(bits.is_cuda() && bits.is_contiguous() && bits.scalar_type() == at::kByte,
              "bits must be a contiguous uint8 GPU tensor");
  TORCH_CHECK(bits.numel() % 4 == 0 && (reinterpret_cast<uintptr_t>(bits.data_ptr()) & 3) == 0,
              "bits: a whole number of aligned 32-bit words");
  dcr::DropSegs d{};
  d.n = 1;
  d.nwords = bits.numel() / 4;
  d.stream[0] = (uint64_t)stream;
  d.kt[0] = dcr::drop_threshold((float)keep);
  dcr::launch_dropout_bits(reinterpret_cast<uint8_t*>(bits.data_ptr()), d, (uint64_t)seed,
                           cur_stream());
}

// all masks of a step in one launch: bits [n, ...] (segment m = bits[m]), streams / keeps per m
void dropout_bits_multi(at::Tensor& bits, int64_t seed, at::IntArrayRef streams,
                        at::ArrayRef<double> keeps, const c10::optional<at::Tensor>& ids,
                        const c10::optional<at::Tensor>& E, double scale,
                        const c10::optional<at::Tensor>& out) {
  TORCH_CHECK(bits.is_cuda() && bits.is_contiguous() && bits.scalar_type() == at::kByte &&
                  bits.dim() >= 1, "bits must be a contiguous uint8 GPU tensor [n, ...]");
  const int n = (int)bits.size(0);
  TORCH_CHECK(n >= 1 && n <= dcr::kDropMaxSegs && (int)streams.size() == n &&
                  (int)keeps.size() == n, "dropout_bits_multi: 1..", dcr::kDropMaxSegs, " masks");
  const int64_t per = bits.numel() / n;
  TORCH_CHECK(per % 4 == 0 && (reinterpret_cast<uintptr_t>(bits.data_ptr()) & 3) == 0,
              "bits: a whole number of aligned 32-bit words per mask");
  dcr::DropSegs d{};
  d.n = n;
  d.nwords = per / 4;
  for (int i = 0; i < n; ++i) {
    d.stream[i] = (uint64_t)streams[i];
    d.kt[i] = dcr::drop_threshold((float)keeps[i]);
  }
  dcr::DropEmbed e{};
  if (has(out)) {  // segment 0 is layer 0's input mask: its masked embedding rows too
    TORCH_CHECK(has(ids) && has(E), "dropout_bits_multi: out needs ids and E");
    check_seq(*ids, at::kInt, "ids");
    check_seq(*E, at::kFloat, "E");
    check_seq(*out, at::kBFloat16, "out");
    const int64_t R = ids->numel();
    const int K = (int)E->size(1);
    TORCH_CHECK(K % 32 == 0 && out->numel() == R * K && per == R * (K / 8),
                "dropout_bits_multi: out [rows, K] (K % 32 == 0) over segment 0's [rows, K/8] bits");
    e.ids = ptr<int>(*ids); e.E = ptr<float>(*E); e.out = ptr<bf16>(*out);
    e.K = K; e.scale = (float)scale;
  }
  dcr::launch_dropout_bits(reinterpret_cast<uint8_t*>(bits.data_ptr()), d, (uint64_t)seed,
                           cur_stream(), e);
}

void mask_apply(const at::Tensor& in, const at::Tensor& bits, double scale, at::Tensor& out) {
  TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.dim() == 2 && out.dim() == 2 &&
                  in.sizes() == out.sizes(), "mask_apply: 2-D GPU tensors of equal shape");
  TORCH_CHECK(in.stride(1) == 1 && out.stride(1) == 1, "mask_apply: unit column stride");
  TORCH_CHECK(in.stride(0) % 8 == 0 && out.stride(0) % 8 == 0 &&
                  (reinterpret_cast<uintptr_t>(in.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15) == 0,
              "mask_apply: 16-byte aligned rows (8-vector loads)");
  const int64_t R = in.size(0);
  const int K = (int)in.size(1);
  TORCH_CHECK(K % 8 == 0, "mask_apply: K % 8 == 0");
  for (const at::Tensor* t : {&in, (const at::Tensor*)&out})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 || t->scalar_type() == at::kFloat,
                "mask_apply: bf16 or fp32");
  TORCH_CHECK(bits.is_cuda() && bits.is_contiguous() && bits.scalar_type() == at::kByte &&
                  bits.numel() == R * (K / 8), "mask_apply: bits must be [rows, K/8] uint8");
  dcr::launch_mask_apply(in.data_ptr(), in.scalar_type() == at::kBFloat16, in.stride(0),
                         out.data_ptr(), out.scalar_type() == at::kBFloat16, out.stride(0),
                         reinterpret_cast<const uint8_t*>(bits.data_ptr()), R, K, (float)scale,
                         cur_stream());
}

void embed_dropout(const at::Tensor& ids, const at::Tensor& E, const c10::optional<at::Tensor>& bits,
                   double scale, at::Tensor& out) {
  check_seq(ids, at::kInt, "ids");
  check_seq(E, at::kFloat, "E");
  check_seq(out, at::kBFloat16, "out");
  const int64_t R = ids.numel();
  const int K = (int)E.size(1);
  TORCH_CHECK(K % 8 == 0 && out.numel() == R * K, "embed_dropout: out [rows, K], K % 8 == 0");
  if (has(bits))
    TORCH_CHECK(bits->is_cuda() && bits->is_contiguous() && bits->scalar_type() == at::kByte &&
                    bits->numel() == R * (K / 8), "embed_dropout: bits [rows, K/8] uint8");
  dcr::launch_embed_dropout(ptr<int>(ids), ptr<float>(E),
                            has(bits) ? reinterpret_cast<const uint8_t*>(bits->data_ptr()) : nullptr,
                            ptr<bf16>(out), R, K, (float)scale, cur_stream());
}

static void check_lstm2_counters(const at::Tensor& c, int nbg, int T) {
  TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kInt && c.is_contiguous() &&
                  c.numel() >= (int64_t)nbg * (T + 1) * 4, "counter buffer too small");
}

void lstm2_persist_fwd(const at::Tensor& W0T, const at::Tensor& W1T, const at::Tensor& X1T,
                       const at::Tensor& zx0, const c10::optional<at::Tensor>& ids,
                       const at::Tensor& bias1, at::Tensor& hbuf0, at::Tensor& cbuf0,
                       const c10::optional<at::Tensor>& gates0, at::Tensor& hlast0,
                       at::Tensor& hbuf1, at::Tensor& cbuf1,
                       const c10::optional<at::Tensor>& gates1, at::Tensor& hlast1,
                       at::Tensor& cnt0, at::Tensor& cnt1, at::Tensor& err, double forget_bias,
                       int64_t spin_limit, at::Tensor& hring0, at::Tensor& hring1, int64_t G,
                       const c10::optional<at::Tensor>& clast0,
                       const c10::optional<at::Tensor>& clast1,
                       const c10::optional<at::Tensor>& diag,
                       const c10::optional<at::Tensor>& xmask, double xscale,
                       const c10::optional<at::Tensor>& bias0,
                       const c10::optional<at::Tensor>& x0,
                       const c10::optional<at::Tensor>& X0T,
                       const c10::optional<at::Tensor>& xdst,
                       const c10::optional<at::Tensor>& omask, double oscale,
                       const c10::optional<at::Tensor>& odst) {
  for (auto* t : {&W0T, &W1T, &X1T}) check_seq(*t, at::kBFloat16, "W");
  TORCH_CHECK(has(x0) == has(X0T), "pass x0 and X0T together");
  const bool xin = has(x0);
  if (!xin) check_seq(zx0, at::kFloat, "zx0");
  check_seq(bias1, at::kFloat, "bias1");
  for (auto* t : {&hring0, &hring1}) check_seq(*t, at::kBFloat16, "hring");
  // hbuf0 / hbuf1: [T+1, B, H] with rows of stride hld >= H (the pair-interleaved layout of
  // engine/native/buffers.py puts both layers in one [T+2, B, 2H] buffer: hld = 2H)
  for (auto* t : {&hbuf0, &hbuf1}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 3,
                "hbuf must be a bf16 GPU tensor [T+1, B, H]");
    TORCH_CHECK(t->stride(2) == 1 && t->stride(1) >= t->size(2) && t->stride(1) % 8 == 0 &&
                    t->stride(0) == t->size(1) * t->stride(1) &&
                    (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                "hbuf rows must be unit-stride, 16-B aligned, stride a multiple of 8, slot-dense");
  }
  TORCH_CHECK(hbuf1.stride(1) == hbuf0.stride(1), "hbuf0 and hbuf1 must share the row stride");
  for (auto* t : {&cbuf0, &cbuf1, &hlast0, &hlast1}) check_seq(*t, at::kFloat, "state");
  check_opt(gates0, at::kBFloat16, "gates0");
  check_opt(gates1, at::kBFloat16, "gates1");
  check_opt(ids, at::kInt, "ids");
  const int T = (int)hbuf0.size(0) - 1, B = (int)hbuf0.size(1), H = (int)hbuf0.size(2);
  TORCH_CHECK(G >= 1 && dcr::lstm2_plan_g(H, B, num_cus(), (int)G) == G,
              "two-layer persistent LSTM: no co-resident grid for H=", H, " B=", B, " G=", G);
  const int nbg = lstm2_nbg(B, (int)G);
  TORCH_CHECK(hbuf1.sizes() == hbuf0.sizes(), "hbuf1 must match hbuf0");
  TORCH_CHECK(cbuf0.numel() == (int64_t)(T + 1) * B * H && cbuf1.numel() == cbuf0.numel(),
              "cbuf shape");
  TORCH_CHECK(hlast0.numel() == (int64_t)B * H && hlast1.numel() == (int64_t)B * H, "hlast shape");
  for (auto* t : {&W0T, &W1T, &X1T})
    TORCH_CHECK(t->size(0) == 4 * H && t->size(1) == H, "weights must be [4H, H]");
  TORCH_CHECK(bias1.numel() == 4 * H, "bias1 must be [4H]");
  if (xin) {
    check_seq(*x0, at::kBFloat16, "x0");
    check_seq(*X0T, at::kBFloat16, "X0T");
    TORCH_CHECK(x0->numel() == (int64_t)T * B * H && X0T->size(0) == 4 * H && X0T->size(1) == H,
                "x0 must be [T*B, H], X0T [4H, H]");
    TORCH_CHECK(!has(ids) && G == 1 && dcr::lstm2_xin_ok(H, num_cus()),
                "in-kernel input projection: dense rows, one batch group per workgroup");
  } else {
    TORCH_CHECK(zx0.size(-1) == 4 * H, "zx0 rows must be 4H wide");
    if (has(ids)) {
      TORCH_CHECK(ids->numel() == (int64_t)T * B, "ids must be [T, B]");
    } else {
      TORCH_CHECK(zx0.numel() == (int64_t)T * B * 4 * H, "zx0 must be [T, B, 4H]");
    }
  }
  for (auto* g : {&gates0, &gates1})
    if (has(*g)) TORCH_CHECK((*g)->numel() == (int64_t)T * B * 4 * H, "gates must be [T, B, 4H]");
  for (auto* c : {&cnt0, &cnt1}) check_lstm2_counters(*c, nbg, T);
  for (auto* r : {&hring0, &hring1})
    TORCH_CHECK(r->numel() >= (int64_t)2 * nbg * 32 * H, "hring must hold [2, ", nbg * 32, ", H]");
  dcr::Lstm2Args a{};
  a.W0T = ptr<bf16>(W0T); a.W1T = ptr<bf16>(W1T); a.X1T = ptr<bf16>(X1T);
  a.zx0 = xin ? nullptr : ptr<float>(zx0); a.ids = optr<int>(ids); a.zx_ld = 4 * H;
  a.zx_rows = (!xin && has(ids)) ? (int)(zx0.numel() / (4 * H)) : 0;
  a.x0 = optr<bf16>(x0); a.X0T = optr<bf16>(X0T);
  a.hld = (int)hbuf0.stride(1);
  a.bias1 = ptr<float>(bias1);
  if (has(bias0)) {
    check_seq(*bias0, at::kFloat, "bias0");
    TORCH_CHECK(bias0->numel() == 4 * H && !has(ids), "bias0: [4H], dense zx0 only");
  }
  a.bias0 = optr<float>(bias0);
  a.hbuf0 = ptr<bf16>(hbuf0); a.cbuf0 = ptr<float>(cbuf0); a.gates0 = optr<bf16>(gates0);
  a.hlast0 = ptr<float>(hlast0);
  a.hbuf1 = ptr<bf16>(hbuf1); a.cbuf1 = ptr<float>(cbuf1); a.gates1 = optr<bf16>(gates1);
  a.hlast1 = ptr<float>(hlast1);
  a.cnt0 = reinterpret_cast<unsigned*>(cnt0.data_ptr());
  a.cnt1 = reinterpret_cast<unsigned*>(cnt1.data_ptr());
  a.err = reinterpret_cast<unsigned*>(err.data_ptr());
  a.B = B; a.H = H; a.T = T; a.G = (int)G; a.nbg = nbg;
  a.forget_bias = (float)forget_bias;
  a.spin_limit = (unsigned)spin_limit;
  a.wgarr = dcr::debug_int("wgarr", 1);  // one hand-off add per workgroup and layer
  a.xcdloc = dcr::debug_int("xcdloc", 1);  // XCD-resident hand-offs where placement allows
  a.steady = dcr::debug_int("fwd_steady", 1);
  if (has(diag)) {
    TORCH_CHECK(diag->element_size() == 8 && diag->numel() >= (int64_t)(T + 2) * G * 8,
                "diag must hold [T+2, G, 8] int64 (ticks 0..T+1)");
    a.diag = reinterpret_cast<unsigned long long*>(diag->data_ptr());
  }
  a.hring0 = ptr<bf16>(hring0);
  a.hring1 = ptr<bf16>(hring1);
  for (auto* c : {&clast0, &clast1})
    if (has(*c)) {
      check_seq(**c, at::kFloat, "clast");
      TORCH_CHECK((*c)->numel() == (int64_t)B * H, "clast must be [B, H]");
    }
  a.clast0 = optr<float>(clast0);
  a.clast1 = optr<float>(clast1);
  a.xmask = drop_bits(xmask, T, B, H, "xmask");
  a.xscale = (float)xscale;
  if (has(xdst)) {  // layer l+1's masked input rows, written beside layer l's row-major h
    TORCH_CHECK(has(xmask) && G == 1, "xdst: dropout (xmask) with one batch group per workgroup");
    TORCH_CHECK(xdst->is_cuda() && xdst->scalar_type() == at::kBFloat16 && xdst->dim() == 2 &&
                    xdst->size(0) == (int64_t)T * B && xdst->size(1) == H && xdst->stride(1) == 1 &&
                    xdst->stride(0) >= H && xdst->stride(0) % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(xdst->data_ptr()) & 7) == 0,
                "xdst must be bf16 [T*B, H] rows, unit-stride, 8-B aligned, stride a multiple of 4");
    a.xdst = ptr<bf16>(*xdst);
    a.xdld = (int)xdst->stride(0);
  }
  if (has(odst)) {  // layer l+1's output-dropout rows (the head's input), written beside its h
    TORCH_CHECK(has(xmask) && G == 1 && has(omask),
                "odst: dropout (xmask, omask) with one batch group per workgroup");
    check_seq(*odst, at::kBFloat16, "odst");
    TORCH_CHECK(odst->numel() == (int64_t)T * B * H, "odst must be [T*B, H]");
    a.omask = drop_bits(omask, T, B, H, "omask");
    a.oscale = (float)oscale;
    a.odst = ptr<bf16>(*odst);
  }
  const int rc = dcr::launch_lstm2_fwd_persist(a, num_cus(), cur_stream());
  TORCH_CHECK(rc == 0, "two-layer persistent LSTM forward not launched (", rc, ")");
}

// two-layer wavefront LSTM BPTT (lstm2_persist.hip)
void lstm2_persist_bwd(const at::Tensor& Wh0, const at::Tensor& Wh1, const at::Tensor& Wx1,
                       const at::Tensor& dtop1, const at::Tensor& gates0, const at::Tensor& cbuf0,
                       const at::Tensor& gates1, const at::Tensor& cbuf1, at::Tensor& dz0,
                       at::Tensor& dz1, at::Tensor& zring0, at::Tensor& zring1,
                       const c10::optional<at::Tensor>& db_part0,
                       const c10::optional<at::Tensor>& db_part1, at::Tensor& cnt0,
                       at::Tensor& cnt1, at::Tensor& err, int64_t spin_limit, int64_t G,
                       const c10::optional<at::Tensor>& diag,
                       const c10::optional<at::Tensor>& xmask, double xscale,
                       const c10::optional<at::Tensor>& pring) {
  for (auto* t : {&Wh0, &Wh1, &Wx1}) check_seq(*t, at::kBFloat16, "W");
  check_seq(dtop1, at::kFloat, "dtop1");
  for (const at::Tensor* t : {&gates0, &gates1, (const at::Tensor*)&dz0, (const at::Tensor*)&dz1,
                              (const at::Tensor*)&zring0, (const at::Tensor*)&zring1})
    check_seq(*t, at::kBFloat16, "bf16 buffer");
  for (auto* t : {&cbuf0, &cbuf1}) check_seq(*t, at::kFloat, "cbuf");
  const int T = (int)dtop1.size(0), B = (int)dtop1.size(1), H = (int)dtop1.size(2);
  TORCH_CHECK(G >= 1 && dcr::lstm2_plan_g(H, B, num_cus(), (int)G) == G,
              "two-layer persistent LSTM BPTT: no co-resident grid for H=", H, " B=", B, " G=", G);
  const int nbg = lstm2_nbg(B, (int)G);
  for (auto* t : {&Wh0, &Wh1, &Wx1})
    TORCH_CHECK(t->size(0) == H && t->size(1) == 4 * H, "weights must be [H, 4H]");
  const int64_t n4 = (int64_t)T * B * 4 * H;
  for (const at::Tensor* t : {&gates0, &gates1, (const at::Tensor*)&dz0, (const at::Tensor*)&dz1})
    TORCH_CHECK(t->numel() == n4, "gates/dz must be [T, B, 4H]");
  for (auto* t : {&cbuf0, &cbuf1})
    TORCH_CHECK(t->numel() == (int64_t)(T + 1) * B * H, "cbuf must be [T+1, B, H]");
  for (auto* t : {&zring0, &zring1})
    TORCH_CHECK(t->numel() >= (int64_t)2 * nbg * 32 * 4 * H, "zring must hold [2, ", nbg * 32, ", 4H]");
  for (auto* c : {&cnt0, &cnt1}) check_lstm2_counters(*c, nbg, T);
  for (auto* d : {&db_part0, &db_part1}) {
    check_opt(*d, at::kFloat, "db_part");
    if (has(*d))
      TORCH_CHECK((*d)->numel() == (int64_t)(2 * nbg / G) * 4 * H,
                  "db_part must be [2*nbg/G, 4H] = [", 2 * nbg / G, ", ", 4 * H, "]");
  }
  dcr::Lstm2BwdArgs a{};
  a.Wh0 = ptr<bf16>(Wh0); a.Wh1 = ptr<bf16>(Wh1); a.Wx1 = ptr<bf16>(Wx1);
  a.dtop1 = ptr<float>(dtop1);
  a.gates0 = ptr<bf16>(gates0); a.cbuf0 = ptr<float>(cbuf0);
  a.gates1 = ptr<bf16>(gates1); a.cbuf1 = ptr<float>(cbuf1);
  a.dz0 = ptr<bf16>(dz0); a.dz1 = ptr<bf16>(dz1);
  a.zring0 = ptr<bf16>(zring0); a.zring1 = ptr<bf16>(zring1);
  a.db_part0 = optr<float>(db_part0); a.db_part1 = optr<float>(db_part1);
  a.cnt0 = reinterpret_cast<unsigned*>(cnt0.data_ptr());
  a.cnt1 = reinterpret_cast<unsigned*>(cnt1.data_ptr());
  a.err = reinterpret_cast<unsigned*>(err.data_ptr());
  a.B = B; a.H = H; a.T = T; a.G = (int)G; a.nbg = nbg;
  a.spin_limit = (unsigned)spin_limit;
  a.wgarr = dcr::debug_int("wgarr", 1);  // one hand-off add per workgroup and layer
  a.xcdloc = dcr::debug_int("xcdloc", 1);  // XCD-resident hand-offs where placement allows
  if (has(diag)) {
    TORCH_CHECK(diag->element_size() == 8 && diag->numel() >= (int64_t)(T + 2) * G * 8,
                "diag must hold [T+2, G, 8] int64 (ticks 0..T+1)");
    a.diag = reinterpret_cast<unsigned long long*>(diag->data_ptr());
    // [grid, T+2, 8]: every workgroup stamps (the wide kernel's skew diagnostics)
    a.diag_all = diag->numel() >= (int64_t)(H / 32) * ((B + 15) / 16) * (T + 2) * 8 &&
                 diag->numel() > (int64_t)(T + 2) * G * 8;
  }
  a.xmask = drop_bits(xmask, T, B, H, "xmask");
  a.xscale = (float)xscale;
  a.db_rows = 2 * nbg / (int)G;
  int rc;
  // (the wide kernel addresses its activation operands with 32-bit buffer offsets)
  // (the reduce-scatter form is opt-in, DCR_DEBUG=bwd_rs=1: 7.1 vs 4.6 us per tick at the
  // headline shape, BASELINE.md "Measured and rejected")
  const bool rs = G == 1 && has(pring) && !a.xmask && dcr::debug_int("bwd_rs", 0) == 1 &&
                  dcr::lstm2_bwd_rs_ok(H, B, num_cus()) && n4 * 2 < ((int64_t)1 << 32);
  if (rs) {
    // reduce-scatter hand-off: each workgroup sends every unit block its [16 x 32] fp32 slice
    // of dZ_own·Wᵀ instead of every workgroup reading the column's whole dZ rows
    check_seq(*pring, at::kFloat, "pring");
    TORCH_CHECK(pring->numel() >= (int64_t)dcr::lstm2_bwd_rs_ring_floats(H, B),
                "pring must hold ", dcr::lstm2_bwd_rs_ring_floats(H, B), " floats");
    a.pring = ptr<float>(*pring);
    a.nbg = (B + 15) / 16;
    check_lstm2_counters(cnt0, a.nbg, T);
    rc = dcr::launch_lstm2_bwd_rs(a, num_cus(), cur_stream());
  } else if (G == 1 && dcr::lstm2_bwd_wide_ok(H, B, num_cus()) && n4 * 2 < ((int64_t)1 << 32)) {
    // 32-unit x 16-row workgroups: half the dZ payload per workgroup and tick
    a.nbg = (B + 15) / 16;
    for (auto* c : {&cnt0, &cnt1}) check_lstm2_counters(*c, a.nbg, T);
    rc = dcr::launch_lstm2_bwd_wide(a, num_cus(), cur_stream());
  } else {
    rc = dcr::launch_lstm2_bwd_persist(a, num_cus(), cur_stream());
  }
  TORCH_CHECK(rc == 0, "two-layer persistent LSTM BPTT not launched (", rc, ")");
}

// on-device sampling step (sample.hip)
void sample_step(const at::Tensor& O, const at::Tensor& WsT, const at::Tensor& bs, at::Tensor& cur,
                 at::Tensor& out, at::Tensor& pos, at::Tensor& ctr,
                 const c10::optional<at::Tensor>& u, const c10::optional<at::Tensor>& logits,
                 int64_t mode, int64_t space_id, int64_t seed) {
  check_seq(O, at::kBFloat16, "O");
  check_seq(WsT, at::kBFloat16, "WsT");
  check_seq(bs, at::kFloat, "bs");
  for (auto* t : {&cur, &out, &pos, &ctr}) check_seq(*t, at::kInt, "sampling state");
  const int S = (int)O.size(0), H = (int)O.size(1), V = (int)WsT.size(0);
  TORCH_CHECK(O.dim() == 2 && WsT.dim() == 2 && WsT.size(1) == H, "O [S, H], WsT [V, H]");
  TORCH_CHECK(bs.numel() == V, "bs must be [V]");
  TORCH_CHECK(dcr::sample_supported(V, H), "sampling kernel: V <= 8192, H % 8 == 0, H <= 4096");
  TORCH_CHECK(cur.numel() == S && pos.numel() == S && ctr.numel() == S, "per-stream state must be [S]");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == S, "out must be [S, n]");
  TORCH_CHECK(mode >= 0 && mode <= 2, "sampling_type must be 0, 1 or 2");
  dcr::SampleArgs a{};
  a.O = ptr<bf16>(O); a.WsT = ptr<bf16>(WsT); a.bs = ptr<float>(bs);
  a.cur = ptr<int>(cur); a.out = ptr<int>(out); a.pos = ptr<int>(pos);
  a.ctr = reinterpret_cast<unsigned*>(ctr.data_ptr());
  if (has(u)) {
    check_seq(*u, at::kFloat, "u");
    TORCH_CHECK(u->numel() == S, "u must be [S]");
    a.u = ptr<float>(*u);
  }
  if (has(logits)) {
    check_seq(*logits, at::kFloat, "logits");
    TORCH_CHECK(logits->numel() == (int64_t)S * V, "logits must be [S, V]");
    a.logits_out = ptr<float>(*logits);
  }
  a.S = S; a.H = H; a.V = V; a.ld = (int)out.size(1);
  a.mode = (int)mode; a.space_id = (int)space_id;
  a.seed = (unsigned long long)seed;
  dcr::launch_sample_step(a, cur_stream());
}

// ------------------------------------------------------------------------------------------
// persistent GRU recurrence (gru_persist.hip)
// ------------------------------------------------------------------------------------------
static void gru_common(dcr::GruPersistArgs& a, const at::Tensor& gates, const at::Tensor& h32,
                       at::Tensor& cnt, at::Tensor& err, int64_t spin_limit, bool cnt_zeroed,
                       int T, int B, int H, const c10::optional<at::Tensor>& ring0,
                       const c10::optional<at::Tensor>& ring1, int64_t w1) {
  TORCH_CHECK(has(ring0) == has(ring1), "pass both hand-off rings or neither");
  if (has(ring0)) {
    check_seq(*ring0, at::kBFloat16, "ring0");
    check_seq(*ring1, at::kBFloat16, "ring1");
    const int64_t Bp = dcr::gru_persist_rows(H, B, num_cus());  // padded batch rows
    TORCH_CHECK(ring0->numel() >= (int64_t)2 * Bp * H && ring1->numel() >= 2 * Bp * w1,
                "hand-off rings too small (", 2 * Bp, " padded rows)");
    a.ring0 = ptr<bf16>(*ring0);
    a.ring1 = ptr<bf16>(*ring1);
  }
  check_seq(gates, at::kBFloat16, "gates");
  check_seq(h32, at::kFloat, "h32");
  TORCH_CHECK(gates.numel() == (int64_t)T * B * 3 * H, "gates must be [T, B, 3H]");
  TORCH_CHECK(h32.numel() == (int64_t)(T + 1) * B * H, "h32 must be [T+1, B, H]");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == at::kInt && err.scalar_type() == at::kInt,
              "cnt/err must be int32 GPU tensors");
  TORCH_CHECK(cnt.numel() >= (int64_t)2 * ((B + 15) / 16) * (T + 1) * 4, "counter buffer too small");
  TORCH_CHECK(B % 16 == 0 || has(ring0), "a ragged batch (B % 16 != 0) needs the hand-off rings");
  TORCH_CHECK(dcr::gru_persist_ub(H, B, num_cus()) > 0, "persistent GRU unsupported for H=", H,
              " B=", B, " (grid cannot be co-resident)");
  a.gates = ptr<bf16>(gates);
  a.h32 = ptr<float>(h32);
  a.cnt = reinterpret_cast<unsigned*>(cnt.data_ptr());
  a.err = reinterpret_cast<unsigned*>(err.data_ptr());
  a.B = B; a.H = H; a.T = T;
  a.spin_limit = (unsigned)spin_limit;
  a.cnt_zeroed = cnt_zeroed ? 1 : 0;
  a.xcdloc = dcr::debug_int("xcdloc", 1);  // XCD-resident hand-offs where placement allows
}

void gru_persist_fwd(const at::Tensor& WgT, const at::Tensor& WcT, const at::Tensor& zx,
                     const c10::optional<at::Tensor>& ids, at::Tensor& hbuf, at::Tensor& h32,
                     at::Tensor& rh, at::Tensor& gates, const c10::optional<at::Tensor>& hlast32,
                     at::Tensor& cnt, at::Tensor& err, int64_t spin_limit, bool cnt_zeroed,
                     const c10::optional<at::Tensor>& ring0, const c10::optional<at::Tensor>& ring1,
                     const c10::optional<at::Tensor>& bias_x) {
  check_seq(WgT, at::kBFloat16, "WgT");
  check_seq(WcT, at::kBFloat16, "WcT");
  check_seq(zx, at::kFloat, "zx");
  check_seq(hbuf, at::kBFloat16, "hbuf");
  check_seq(rh, at::kBFloat16, "rh");
  check_opt(ids, at::kInt, "ids");
  check_opt(hlast32, at::kFloat, "hlast32");
  const int T = (int)hbuf.size(0) - 1, B = (int)hbuf.size(1), H = (int)hbuf.size(2);
  TORCH_CHECK(WgT.size(0) == 2 * H && WgT.size(1) == H, "WgT must be [2H, H]");
  TORCH_CHECK(WcT.size(0) == H && WcT.size(1) == H, "WcT must be [H, H]");
  TORCH_CHECK(zx.size(-1) == 3 * H, "zx rows must be 3H wide");
  if (has(ids)) {
    TORCH_CHECK(ids->numel() == (int64_t)T * B, "ids must be [T, B]");
  } else {
    TORCH_CHECK(zx.numel() == (int64_t)T * B * 3 * H, "zx must be [T, B, 3H]");
  }
  TORCH_CHECK(rh.numel() == (int64_t)T * B * H, "rh must be [T, B, H]");
  if (has(hlast32)) TORCH_CHECK(hlast32->numel() == (int64_t)B * H, "hlast32 must be [B, H]");
  dcr::GruPersistArgs a{};
  gru_common(a, gates, h32, cnt, err, spin_limit, cnt_zeroed, T, B, H, ring0, ring1, H);
  a.WgT = ptr<bf16>(WgT);
  a.WcT = ptr<bf16>(WcT);
  a.zx = ptr<float>(zx);
  a.ids = optr<int>(ids);
  a.zx_ld = 3 * H;
  if (has(bias_x)) {
    check_seq(*bias_x, at::kFloat, "bias_x");
    TORCH_CHECK(bias_x->numel() == 3 * H && !has(ids), "bias_x: [3H], dense zx only");
  }
  a.bias_x = optr<float>(bias_x);
  a.hbuf = ptr<bf16>(hbuf);
  a.rh = ptr<bf16>(rh);
  a.hlast32 = optr<float>(hlast32);
  const int rc = dcr::launch_gru_persist(0, a, num_cus(), cur_stream());
  TORCH_CHECK(rc == 0, "persistent GRU forward not launched (", rc, ")");
}

void gru_persist_bwd(const at::Tensor& Wg, const at::Tensor& Wc, const at::Tensor& dtop,
                     at::Tensor& dz, const at::Tensor& gates, const at::Tensor& h32,
                     at::Tensor& cnt, at::Tensor& err, int64_t spin_limit, bool cnt_zeroed,
                     const c10::optional<at::Tensor>& ring0, const c10::optional<at::Tensor>& ring1,
                     const c10::optional<at::Tensor>& db_part) {
  check_seq(Wg, at::kBFloat16, "Wg");
  check_seq(Wc, at::kBFloat16, "Wc");
  check_seq(dtop, at::kFloat, "dtop");
  check_seq(dz, at::kBFloat16, "dz");
  TORCH_CHECK(dtop.dim() == 3, "dtop must be [T, B, H]");
  const int T = (int)dtop.size(0), B = (int)dtop.size(1), H = (int)dtop.size(2);
  TORCH_CHECK(Wg.size(0) == H && Wg.size(1) == 2 * H, "Wg must be [H, 2H]");
  TORCH_CHECK(Wc.size(0) == H && Wc.size(1) == H, "Wc must be [H, H]");
  TORCH_CHECK(dz.numel() == (int64_t)T * B * 3 * H, "dz must be [T, B, 3H]");
  dcr::GruPersistArgs a{};
  gru_common(a, gates, h32, cnt, err, spin_limit, cnt_zeroed, T, B, H, ring0, ring1, 2 * H);
  a.Wg = ptr<bf16>(Wg);
  a.Wc = ptr<bf16>(Wc);
  a.dtop = ptr<float>(dtop);
  a.dz = ptr<bf16>(dz);
  check_opt(db_part, at::kFloat, "db_part");
  if (has(db_part)) {
    TORCH_CHECK(db_part->numel() >= (int64_t)((B + 15) / 16) * 3 * H,
                "db_part must hold [ceil(B/16), 3H]");
    a.db_part = optr<float>(db_part);
  }
  const int rc = dcr::launch_gru_persist(1, a, num_cus(), cur_stream());
  TORCH_CHECK(rc == 0, "persistent GRU BPTT not launched (", rc, ")");
}

// ------------------------------------------------------------------------------------------
// fused softmax head (head.hip)
// ------------------------------------------------------------------------------------------
void head(const at::Tensor& O, const at::Tensor& WsT, const c10::optional<at::Tensor>& Wsk,
          const at::Tensor& bias, const c10::optional<at::Tensor>& targets, double grad_scale,
          const c10::optional<at::Tensor>& logits, const c10::optional<at::Tensor>& row_loss,
          const c10::optional<at::Tensor>& dlogits, const c10::optional<at::Tensor>& dtop,
          const c10::optional<at::Tensor>& db, at::Tensor& part,
          const c10::optional<at::Tensor>& loss, const c10::optional<at::Tensor>& omask,
          double oscale) {
  TORCH_CHECK(O.is_cuda() && O.dim() == 2 && O.scalar_type() == at::kBFloat16 && O.stride(1) == 1,
              "O must be a row-major bf16 [N, H] GPU tensor");
  const int N = (int)O.size(0), H = (int)O.size(1), V = (int)bias.numel();
  TORCH_CHECK(dcr::head_supported(V, H), "fused head supports V <= 256 and H % 32 == 0");
  const int VP = dcr::head_vpad(V), VK = dcr::head_kpad(V);
  check_seq(WsT, at::kBFloat16, "WsT");
  check_seq(bias, at::kFloat, "bias");
  TORCH_CHECK(WsT.numel() == (int64_t)VP * H, "WsT must be [head_vpad(V), H]");
  const bool train = has(dlogits) || has(dtop);
  if (has(dtop)) {
    TORCH_CHECK(has(Wsk), "dtop needs Wsk");
    check_seq(*Wsk, at::kBFloat16, "Wsk");
    TORCH_CHECK(Wsk->numel() == (int64_t)H * VK, "Wsk must be [H, head_kpad(V)]");
    check_seq(*dtop, at::kFloat, "dtop");
    TORCH_CHECK(dtop->numel() == (int64_t)N * H, "dtop must be [N, H]");
  }
  if (train || has(loss) || has(row_loss)) {
    TORCH_CHECK(has(targets), "loss / gradients need targets");
  }
  if (has(targets)) {
    check_seq(*targets, at::kInt, "targets");
    TORCH_CHECK(targets->numel() == N, "targets must be [N]");
  }
  if (has(logits)) { check_seq(*logits, at::kFloat, "logits"); TORCH_CHECK(logits->numel() == (int64_t)N * V, "logits must be [N, V]"); }
  if (has(row_loss)) { check_seq(*row_loss, at::kFloat, "row_loss"); TORCH_CHECK(row_loss->numel() == N, "row_loss must be [N]"); }
  int ldl = V;
  if (has(dlogits)) {
    // contiguous [N, V], or a [N, V] view of zero-padded rows (row stride ldl >= V)
    const at::Tensor& d = *dlogits;
    TORCH_CHECK(d.is_cuda() && d.scalar_type() == at::kBFloat16, "dlogits must be bf16 on the GPU");
    if (d.dim() == 2 && d.size(0) == N && d.size(1) == V && d.stride(1) == 1) {
      ldl = (int)d.stride(0);
      TORCH_CHECK(ldl >= V, "dlogits: row stride below V");
    } else {
      TORCH_CHECK(d.is_contiguous() && d.numel() == (int64_t)N * V, "dlogits must be [N, V]");
    }
  }
  if (has(db)) { check_seq(*db, at::kFloat, "db"); TORCH_CHECK(db->numel() == V, "db must be [V]"); }
  if (has(loss)) { check_seq(*loss, at::kFloat, "loss"); TORCH_CHECK(loss->numel() >= 1, "loss must hold 1 float"); }
  check_seq(part, at::kFloat, "part");
  TORCH_CHECK(part.numel() >= (int64_t)dcr::head_num_partials(N, num_cus()) * (VP + 1),
              "partials workspace too small (head_num_partials)");
  dcr::HeadArgs a{};
  a.O = ptr<bf16>(O);
  a.ldo = (int)O.stride(0);
  a.WsT = ptr<bf16>(WsT);
  a.Wsk = optr<bf16>(Wsk);
  a.bias = ptr<float>(bias);
  a.targets = optr<int>(targets);
  a.N = N; a.H = H; a.V = V;
  a.grad_scale = (float)grad_scale;
  a.logits = optr<float>(logits);
  a.row_loss = optr<float>(row_loss);
  a.dlogits = optr<bf16>(dlogits);
  a.ldl = ldl;
  a.dtop = optr<float>(dtop);
  a.part = ptr<float>(part);
  if (has(omask)) {
    TORCH_CHECK(has(dtop) && omask->is_cuda() && omask->scalar_type() == at::kByte &&
                    omask->is_contiguous() && omask->numel() == (int64_t)N * (H / 8) && H % 8 == 0,
                "omask: uint8 [N, H/8] bits, with dtop");
    a.omask = omask->data_ptr<uint8_t>();
    a.oscale = (float)oscale;
  }
  TORCH_CHECK(dcr::launch_head(a, num_cus(), optr<float>(db), optr<float>(loss), cur_stream()) == 0,
              "fused head launch failed");
}

// ------------------------------------------------------------------------------------------
// batched per-step data movement (prep.hip)
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// token-reduction weight-gradient GEMMs (wgrad.hip): part[p][s] = A_p[chunk s]ᵀ · B_p[chunk s]
// ------------------------------------------------------------------------------------------
void wgrad(at::TensorList A, at::TensorList B, at::TensorList part) {
  const int np = (int)A.size();
  TORCH_CHECK(np >= 1 && np <= dcr::kWgradMaxProblems && (int)B.size() == np &&
                  (int)part.size() == np, "wgrad: 1..", dcr::kWgradMaxProblems, " problems");
  const int K = (int)A[0].size(0);
  dcr::WgradArgs a{};
  for (int i = 0; i < np; ++i) {
    const at::Tensor& x = A[i];
    const at::Tensor& y = B[i];
    const at::Tensor& c = part[i];
    for (const at::Tensor* t : {&x, &y}) {
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 2 &&
                      t->stride(1) == 1 && t->stride(0) % 8 == 0 &&
                      reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                  "wgrad operands: bf16 [K, *] views with unit column stride, 16-B aligned rows");
    }
    check_seq(c, at::kFloat, "part");
    TORCH_CHECK(c.dim() == 3, "wgrad: part[p] must be [S, M, N]");
    const int S = (int)c.size(0), M = (int)c.size(1), N = (int)c.size(2);
    TORCH_CHECK(S >= 1 && S <= dcr::kWgradMaxSplit, "wgrad: 1..", dcr::kWgradMaxSplit, " slabs");
    TORCH_CHECK(x.size(0) == K && y.size(0) == K && x.size(1) == M && y.size(1) == N,
                "wgrad: A_p must be [K, M], B_p [K, N] (one K for every problem)");
    TORCH_CHECK(dcr::wgrad_supported(M, N, K), "wgrad: unsupported shape M=", M, " N=", N, " K=", K);
    a.p[i].A = ptr<bf16>(x); a.p[i].lda = x.stride(0);
    a.p[i].B = ptr<bf16>(y); a.p[i].ldb = y.stride(0);
    a.p[i].C = c.data_ptr<float>();
    a.p[i].ldc = N;
    a.p[i].slab = (long)M * N;
    a.p[i].M = M; a.p[i].N = N; a.p[i].S = S;
  }
  a.np = np; a.K = K;
  dcr::launch_wgrad(a, cur_stream());
}

// ------------------------------------------------------------------------------------------
// the step's tail (tail.hip): FINALIZE (phase 0) / ADAM with the bf16 layouts (phase 1).  The
// tasks arrive as kTailWords int64 words each (engine/native/tail.py builds them from tensors
// it keeps alive; pointers as data_ptr integers), checked here before the launch.
// ------------------------------------------------------------------------------------------
constexpr int kTailWords = 27;
void tail(at::IntArrayRef words, int64_t phase, at::Tensor& part, at::Tensor& sync, at::Tensor& dep,
          at::Tensor& err, int64_t spin_limit, const c10::optional<at::Tensor>& total_out,
          const c10::optional<at::Tensor>& total_in, const c10::optional<at::Tensor>& extra,
          const c10::optional<at::Tensor>& p, const c10::optional<at::Tensor>& g,
          const c10::optional<at::Tensor>& m, const c10::optional<at::Tensor>& v,
          const c10::optional<at::Tensor>& mirror, int64_t n_norm, double lr_t, double b1,
          double b2, double eps, double clip, double gscale, const c10::optional<at::Tensor>& lr_dev,
          const c10::optional<at::Tensor>& skip_if, const c10::optional<at::Tensor>& norm_out,
          bool dynamic) {
  TORCH_CHECK(words.size() % kTailWords == 0, "tail: ", kTailWords, " words per task");
  const int n = (int)(words.size() / kTailWords);
  TORCH_CHECK(n >= 1 && n <= dcr::kTailMaxTasks, "tail: 1..", dcr::kTailMaxTasks, " tasks");
  TORCH_CHECK(phase == 0 || phase == 1, "tail: phase 0 or 1");
  CHECK_DEV(part); CHECK_F32(part);
  TORCH_CHECK(part.numel() >= dcr::kTailMaxTiles, "tail: part needs ", dcr::kTailMaxTiles, " floats");
  CHECK_DEV(sync); CHECK_I32(sync); TORCH_CHECK(sync.numel() >= dcr::kTailSyncWords, "tail: sync needs ", dcr::kTailSyncWords, " words");
  CHECK_DEV(dep); CHECK_I32(dep);
  TORCH_CHECK(dep.numel() >= dcr::kTailDepWords, "tail: dep needs ", dcr::kTailDepWords, " words");
  CHECK_DEV(err); CHECK_I32(err);
  auto opt_ptr = [](const c10::optional<at::Tensor>& t) -> void* {
    return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
  };
  dcr::TailArgs a{};
  a.n = n;
  a.phase = (int)phase;
  a.part = ptr<float>(part);
  a.sync = reinterpret_cast<unsigned*>(sync.data_ptr());
  a.dep = reinterpret_cast<unsigned*>(dep.data_ptr());
  a.err = reinterpret_cast<unsigned*>(err.data_ptr());
  a.spin_limit = (unsigned)spin_limit;
  a.dynamic = dynamic ? 1 : 0;
  a.total_out = static_cast<float*>(opt_ptr(total_out));
  a.total_in = static_cast<const float*>(opt_ptr(total_in));
  a.extra = static_cast<const float*>(opt_ptr(extra));
  if (phase == 1) {
    TORCH_CHECK(p && g && m && v && p->defined() && g->defined() && m->defined() && v->defined(),
                "tail ADAM: p, g, m, v");
    for (const at::Tensor* t : {&*p, &*g, &*m, &*v}) {
      CHECK_DEV(*t); CHECK_CONTIG(*t); CHECK_F32(*t); CHECK_ALIGN16(*t);
      TORCH_CHECK(t->numel() == p->numel(), "tail ADAM: p, g, m, v sizes differ");
    }
    TORCH_CHECK(n_norm >= 0 && n_norm <= p->numel(), "tail ADAM: n_norm out of range");
    TORCH_CHECK(total_in && total_in->defined(), "tail ADAM: the global sum of squares (total_in)");
    a.p = ptr<float>(*p); a.g = ptr<float>(*g); a.m = ptr<float>(*m); a.v = ptr<float>(*v);
    if (mirror && mirror->defined()) {
      CHECK_BF16(*mirror); CHECK_CONTIG(*mirror); CHECK_ALIGN16(*mirror);
      TORCH_CHECK(mirror->numel() >= p->numel(), "tail ADAM: mirror too small");
      a.mirror = ptr<bf16>(*mirror);
    }
  }
  a.n_norm = n_norm;
  a.lr_t = (float)lr_t; a.b1 = (float)b1; a.b2 = (float)b2; a.eps = (float)eps;
  a.clip = (float)clip; a.gscale = (float)gscale;
  a.lr_dev = static_cast<const float*>(opt_ptr(lr_dev));
  a.skip_if = static_cast<const unsigned*>(opt_ptr(skip_if));
  a.norm_out = static_cast<float*>(opt_ptr(norm_out));
  auto a16 = [](int64_t x) { return (x & 15) == 0; };
  for (int i = 0; i < n; ++i) {
    const int64_t* w = words.data() + (size_t)i * kTailWords;
    dcr::TailTask& T = a.t[i];
    T.op = (int)w[0]; T.rows = (int)w[1]; T.cols = (int)w[2]; T.norm = (int)w[3];
    T.wait = (int)w[4]; T.need = (int)w[5]; T.sig = (int)w[6]; T.vec4 = (int)w[7];
    T.nslab = (int)w[8]; T.k = (int)w[9]; T.o1_t = (int)w[10]; T.o2_t = (int)w[11];
    T.a = reinterpret_cast<const float*>(w[12]); T.ar = w[13]; T.ak = w[14];
    T.b = reinterpret_cast<const float*>(w[15]); T.bk = w[16]; T.bc = w[17];
    T.bias = reinterpret_cast<const float*>(w[18]);
    T.dst = reinterpret_cast<float*>(w[19]); T.dst_ld = w[20];
    T.off = w[21]; T.ld = w[22];
    T.o1 = reinterpret_cast<bf16*>(w[23]); T.o1_ld = w[24];
    T.o2 = reinterpret_cast<bf16*>(w[25]); T.o2_ld = w[26];
    TORCH_CHECK(T.op >= dcr::TAIL_SUM && T.op <= dcr::TAIL_ADAM, "tail: unknown op ", T.op);
    TORCH_CHECK((T.op == dcr::TAIL_ADAM) == (phase == 1) || T.op == dcr::TAIL_MM ||
                    (T.op == dcr::TAIL_SUM && !T.norm),
                "tail: ADAM tasks only in phase 1, COLSUM / SUMSQ / norm SUMs only in phase 0");
    TORCH_CHECK(T.rows > 0 && T.cols > 0, "tail: empty task");
    TORCH_CHECK(T.wait < dcr::kTailMaxDeps && T.sig < dcr::kTailMaxDeps, "tail: dep index");
    TORCH_CHECK(T.wait < 0 || T.need > 0, "tail: a waiting task needs a positive count");
    if (T.op != dcr::TAIL_ADAM) TORCH_CHECK(T.a != nullptr, "tail: task without a source");
    if (T.op == dcr::TAIL_SUM || T.op == dcr::TAIL_COLSUM || T.op == dcr::TAIL_MM)
      TORCH_CHECK(T.dst != nullptr, "tail: task without a destination");
    if (T.op == dcr::TAIL_SUM) {
      TORCH_CHECK(T.nslab >= 1, "tail SUM: slabs");
      if (T.vec4)
        TORCH_CHECK(a16(w[12]) && a16(w[19]) && T.ar % 4 == 0 && T.ak % 4 == 0 && T.dst_ld % 4 == 0 &&
                    T.cols % 4 == 0, "tail SUM: float4 path needs 16-B aligned rows");
    }
    if (T.op == dcr::TAIL_COLSUM) TORCH_CHECK(T.k >= 1, "tail COLSUM: partial rows in k");
    if (T.op == dcr::TAIL_MM) {
      TORCH_CHECK(T.b != nullptr && T.k >= 1, "tail MM: B and k");
      if (T.k > 128)  // the long path: float4 loads of A along k, k in whole 4-element groups
        TORCH_CHECK(T.ak == 1 && T.k % 4 == 0 && (w[12] & 15) == 0 && T.ar % 4 == 0 &&
                        (T.bk != 1 || ((w[15] & 15) == 0 && T.bc % 4 == 0)),
                    "tail MM (k > 128): A k-contiguous, 16-B aligned rows, k % 4 == 0");
      if (T.nslab > 1)  // k-slabs (long path only) into dst + s * off, summed by a later SUM
        TORCH_CHECK(T.k > 128 && !T.norm && T.off >= (int64_t)(T.rows - 1) * T.dst_ld + T.cols &&
                        T.nslab <= T.k / 64,
                    "tail MM: k-slabs need k > 128, no norm, a slab stride covering a slab and "
                    "at least 64 k per slab");
    }
    if (T.op == dcr::TAIL_ADAM) {
      TORCH_CHECK(phase == 1, "tail ADAM in phase 1");
      TORCH_CHECK(T.off >= 0 && T.off + (T.rows - 1) * T.ld + T.cols <= p->numel(),
                  "tail ADAM: region outside the parameter buffer");
      if (T.vec4)
        TORCH_CHECK(T.off % 4 == 0 && T.ld % 4 == 0 && T.cols % 4 == 0 &&
                    (!T.o1 || T.o1_t || (T.o1_ld % 4 == 0 && (w[23] & 7) == 0)) &&
                    (!T.o2 || T.o2_t || (T.o2_ld % 4 == 0 && (w[25] & 7) == 0)),
                    "tail ADAM: float4 path alignment");
    }
  }
  const int rc = dcr::launch_tail(a, num_cus(), cur_stream());
  TORCH_CHECK(rc == 0, "tail: launch failed (", rc, ")");
}

int64_t tail_words() { return kTailWords; }

// single-launch generation (generate.hip)
void generate(at::TensorList Wh, at::TensorList Wx, at::TensorList bias, const at::Tensor& table,
              const at::Tensor& WsT, const at::Tensor& bs, double forget_bias, const at::Tensor& h0,
              const at::Tensor& c0, at::Tensor& h_out, at::Tensor& c_out, const at::Tensor& prime,
              int64_t num, at::Tensor& out, at::Tensor& hx, int64_t mode, int64_t space_id,
              int64_t seed, const at::Tensor& ctr0, const c10::optional<at::Tensor>& logits_out,
              at::Tensor& err, int64_t spin_limit, const c10::optional<at::Tensor>& stamps) {
  const int L = (int)Wh.size();
  TORCH_CHECK(L >= 1 && L <= dcr::kGenMaxLayers && (int)Wx.size() == L && (int)bias.size() == L,
              "generate: 1..", dcr::kGenMaxLayers, " layers");
  CHECK_DEV(table); CHECK_F32(table); CHECK_CONTIG(table);
  CHECK_DEV(WsT); CHECK_BF16(WsT); CHECK_CONTIG(WsT); CHECK_ALIGN16(WsT);
  const int V = (int)WsT.size(0), H = (int)WsT.size(1);
  TORCH_CHECK(table.dim() == 2 && table.size(0) == V && table.size(1) == 4 * H, "generate: table [V, 4H]");
  CHECK_DEV(bs); CHECK_F32(bs); TORCH_CHECK(bs.numel() == V, "generate: bs [V]");
  dcr::GenArgs a{};
  a.L = L; a.H = H; a.V = V;
  for (int l = 0; l < L; ++l) {
    for (const at::Tensor* t : {&Wh[l], &Wx[l]}) {
      CHECK_DEV(*t); CHECK_BF16(*t); CHECK_CONTIG(*t);
      TORCH_CHECK(t->dim() == 2 && t->size(0) == H && t->size(1) == 4 * H, "generate: W [H, 4H]");
    }
    CHECK_DEV(bias[l]); CHECK_F32(bias[l]); CHECK_CONTIG(bias[l]);
    TORCH_CHECK(bias[l].numel() == 4 * H, "generate: bias [4H]");
    a.Wh[l] = ptr<bf16>(Wh[l]); a.Wx[l] = ptr<bf16>(Wx[l]); a.bias[l] = ptr<float>(bias[l]);
  }
  for (const at::Tensor* t : {&h0, &c0, (const at::Tensor*)&h_out, (const at::Tensor*)&c_out}) {
    CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t);
    TORCH_CHECK(t->dim() == 3 && t->size(0) == L && t->size(2) == H && t->size(1) == h0.size(1),
                "generate: state [L, S, H]");
  }
  a.S = (int)h0.size(1);
  CHECK_DEV(prime); CHECK_I32(prime); CHECK_CONTIG(prime);
  a.P = (int)prime.numel();
  TORCH_CHECK(a.P >= 1 && num >= 1, "generate: a prime of >= 1 ids and num >= 1");
  CHECK_DEV(out); CHECK_I32(out); CHECK_CONTIG(out);
  TORCH_CHECK(out.numel() == (int64_t)a.S * num, "generate: out [S, num]");
  CHECK_DEV(hx); CHECK_CONTIG(hx);
  TORCH_CHECK(hx.element_size() == 8 && hx.numel() >= (int64_t)L * 2 * a.S * H, "generate: hx [L, 2, S, H] of 8-B granules");
  CHECK_DEV(ctr0); CHECK_I32(ctr0); TORCH_CHECK(ctr0.numel() >= a.S, "generate: ctr0 [S]");
  CHECK_DEV(err); CHECK_I32(err);
  a.table = ptr<float>(table); a.WsT = ptr<bf16>(WsT); a.bs = ptr<float>(bs);
  if (stamps && stamps->defined()) {
    CHECK_DEV(*stamps); TORCH_CHECK(stamps->element_size() == 8 && stamps->numel() >= 256, "generate: stamps [256] of 8 B");
    a.stamps = reinterpret_cast<unsigned long long*>(stamps->data_ptr());
  }
  a.forget_bias = (float)forget_bias;
  a.h0 = ptr<float>(h0); a.c0 = ptr<float>(c0); a.h_out = ptr<float>(h_out); a.c_out = ptr<float>(c_out);
  a.prime = ptr<int>(prime); a.num = (int)num; a.out = ptr<int>(out);
  a.hx = reinterpret_cast<unsigned long long*>(hx.data_ptr());
  a.mode = (int)mode; a.space_id = (int)space_id; a.seed = (unsigned long long)seed;
  a.ctr0 = reinterpret_cast<const unsigned*>(ctr0.data_ptr());
  if (logits_out.has_value() && logits_out->defined()) {
    CHECK_DEV(*logits_out); CHECK_F32(*logits_out); CHECK_CONTIG(*logits_out);
    TORCH_CHECK(logits_out->numel() >= num * a.S * V, "generate: logits_out [num, S, V]");
    a.logits_out = ptr<float>(*logits_out);
  }
  a.err = reinterpret_cast<unsigned*>(err.data_ptr());
  a.spin_limit = (unsigned)spin_limit;
  // the hand-off tags must not match stale granules of an earlier launch
  TORCH_CHECK(hipMemsetAsync(hx.data_ptr(), 0, (size_t)L * 2 * a.S * H * 8, cur_stream()) == hipSuccess,
              "generate: clearing the hand-off buffer failed");
  const int rc = dcr::launch_generate(a, num_cus(), cur_stream());
  TORCH_CHECK(rc == 0, "generate: unsupported shape or launch failure (", rc, ")");
}
// TF token-norm term (tokennorm.hip): out[0] = sum_tok ||dz[tok] · wᵀ||²
void tokennorm(const at::Tensor& dz, const at::Tensor& w, at::Tensor& part, at::Tensor& ticket,
               at::Tensor& out) {
  for (const at::Tensor* t : {&dz, &w}) {
    CHECK_DEV(*t); CHECK_BF16(*t);
    TORCH_CHECK(t->dim() == 2 && t->stride(1) == 1 && t->stride(0) % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                "tokennorm: 2-D bf16 views with 16-B aligned rows");
  }
  const int N = (int)dz.size(0), K = (int)dz.size(1), H = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K, "tokennorm: dz [N, K], w [H, K]");
  TORCH_CHECK(dcr::tokennorm_supported(N, H, K), "tokennorm: unsupported shape N=", N, " H=", H,
              " K=", K);
  CHECK_DEV(part); CHECK_F32(part);
  TORCH_CHECK(part.numel() >= dcr::kTokenNormMaxGrid, "tokennorm: part too small");
  CHECK_DEV(ticket); CHECK_I32(ticket); CHECK_DEV(out); CHECK_F32(out);
  dcr::TokenNormArgs a{};
  a.dz = ptr<bf16>(dz); a.ld_dz = dz.stride(0);
  a.w = ptr<bf16>(w); a.ld_w = w.stride(0);
  a.N = N; a.N_units = H; a.K = K;
  a.part = ptr<float>(part);
  a.ticket = reinterpret_cast<unsigned*>(ticket.data_ptr());
  a.out = ptr<float>(out);
  dcr::launch_tokennorm(a, cur_stream());
}

// dropout route's embedding input gradient (tokennorm.hip, masked form): dx [N, H] bf16 =
// (dz · wᵀ) ⊙ mask · scale and out[0] = sum of the squares of dx's values, in one launch
void tokennorm_masked(const at::Tensor& dz, const at::Tensor& w, const at::Tensor& mask,
                      double scale, at::Tensor& dx, at::Tensor& part, at::Tensor& ticket,
                      at::Tensor& out) {
  for (const at::Tensor* t : {&dz, &w}) {
    CHECK_DEV(*t); CHECK_BF16(*t);
    TORCH_CHECK(t->dim() == 2 && t->stride(1) == 1 && t->stride(0) % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                "tokennorm_masked: 2-D bf16 views with 16-B aligned rows");
  }
  const int N = (int)dz.size(0), K = (int)dz.size(1), H = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K, "tokennorm_masked: dz [N, K], w [H, K]");
  TORCH_CHECK(dcr::tokennorm_supported(N, H, K), "tokennorm_masked: unsupported shape N=", N,
              " H=", H, " K=", K);
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.is_contiguous() &&
                  mask.numel() == (int64_t)N * (H / 8) &&
                  (reinterpret_cast<uintptr_t>(mask.data_ptr()) & 7) == 0,
              "tokennorm_masked: mask must be uint8 [N, H/8] bits, 8-B aligned");
  CHECK_DEV(dx); CHECK_BF16(dx);
  TORCH_CHECK(dx.dim() == 2 && dx.size(0) == N && dx.size(1) == H && dx.stride(1) == 1,
              "tokennorm_masked: dx [N, H] with unit column stride");
  CHECK_DEV(part); CHECK_F32(part);
  TORCH_CHECK(part.numel() >= dcr::kTokenNormMaxGrid, "tokennorm_masked: part too small");
  CHECK_DEV(ticket); CHECK_I32(ticket); CHECK_DEV(out); CHECK_F32(out);
  dcr::TokenNormArgs a{};
  a.dz = ptr<bf16>(dz); a.ld_dz = dz.stride(0);
  a.w = ptr<bf16>(w); a.ld_w = w.stride(0);
  a.N = N; a.N_units = H; a.K = K;
  a.part = ptr<float>(part);
  a.ticket = reinterpret_cast<unsigned*>(ticket.data_ptr());
  a.out = ptr<float>(out);
  a.mask = mask.data_ptr<uint8_t>();
  a.cb = ptr<bf16>(dx); a.ldc = dx.stride(0); a.mscale = (float)scale;
  dcr::launch_tokennorm(a, cur_stream());
}

// wide-vocabulary route's embedding input gradient (tokennorm.hip, storing form): dx [N, H]
// fp32 = dz · wᵀ and out[0] = sum of its squares, in one launch
void tokennorm_store(const at::Tensor& dz, const at::Tensor& w, at::Tensor& dx, at::Tensor& part,
                     at::Tensor& ticket, at::Tensor& out) {
  for (const at::Tensor* t : {&dz, &w}) {
    CHECK_DEV(*t); CHECK_BF16(*t);
    TORCH_CHECK(t->dim() == 2 && t->stride(1) == 1 && t->stride(0) % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                "tokennorm_store: 2-D bf16 views with 16-B aligned rows");
  }
  const int N = (int)dz.size(0), K = (int)dz.size(1), H = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K, "tokennorm_store: dz [N, K], w [H, K]");
  TORCH_CHECK(dcr::tokennorm_supported(N, H, K), "tokennorm_store: unsupported shape N=", N,
              " H=", H, " K=", K);
  CHECK_DEV(dx); CHECK_F32(dx);
  TORCH_CHECK(dx.dim() == 2 && dx.size(0) == N && dx.size(1) == H && dx.stride(1) == 1,
              "tokennorm_store: dx [N, H] with unit column stride");
  CHECK_DEV(part); CHECK_F32(part);
  TORCH_CHECK(part.numel() >= dcr::kTokenNormMaxGrid, "tokennorm_store: part too small");
  CHECK_DEV(ticket); CHECK_I32(ticket); CHECK_DEV(out); CHECK_F32(out);
  dcr::TokenNormArgs a{};
  a.dz = ptr<bf16>(dz); a.ld_dz = dz.stride(0);
  a.w = ptr<bf16>(w); a.ld_w = w.stride(0);
  a.N = N; a.N_units = H; a.K = K;
  a.part = ptr<float>(part);
  a.ticket = reinterpret_cast<unsigned*>(ticket.data_ptr());
  a.out = ptr<float>(out);
  a.c = ptr<float>(dx); a.ldc = dx.stride(0);
  dcr::launch_tokennorm(a, cur_stream());
}

// C [M, N] fp32 = a [M, K] · bᵀ (b [N, K]), both bf16 K-contiguous (tokennorm.hip's pipeline)
void gemm_nt(const at::Tensor& a_, const at::Tensor& b, at::Tensor& c,
             const c10::optional<at::Tensor>& bias) {
  for (const at::Tensor* t : {&a_, &b}) {
    CHECK_DEV(*t); CHECK_BF16(*t);
    TORCH_CHECK(t->dim() == 2 && t->stride(1) == 1 && t->stride(0) % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                "gemm_nt: 2-D bf16 views with 16-B aligned rows");
  }
  const int M = (int)a_.size(0), K = (int)a_.size(1), N = (int)b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_nt: a [M, K], b [N, K]");
  TORCH_CHECK(dcr::gemm_nt_supported(M, N, K), "gemm_nt: unsupported shape M=", M, " N=", N,
              " K=", K);
  // the DMA offsets are 32-bit buffer offsets
  TORCH_CHECK((double)(M - 1) * a_.stride(0) * 2 + (double)K * 2 < 2147483632.0 &&
                  (double)(N - 1) * b.stride(0) * 2 + (double)K * 2 < 2147483632.0,
              "gemm_nt: operands beyond the 2 GB buffer range");
  CHECK_DEV(c); CHECK_F32(c);
  TORCH_CHECK(c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1,
              "gemm_nt: c [M, N] with unit column stride");
  dcr::TokenNormArgs a{};
  a.dz = ptr<bf16>(a_); a.ld_dz = a_.stride(0);
  a.w = ptr<bf16>(b); a.ld_w = b.stride(0);
  a.N = M; a.N_units = N; a.K = K;
  a.c = ptr<float>(c); a.ldc = c.stride(0);
  if (has(bias)) {
    CHECK_DEV(*bias); CHECK_F32(*bias);
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N, "gemm_nt: bias must be [N]");
    a.cbias = ptr<float>(*bias);
  }
  dcr::launch_gemm_nt(a, cur_stream());
}

void prep(at::TensorList src, at::TensorList dst, at::IntArrayRef mode, at::TensorList extra) {
  TORCH_CHECK(src.size() == dst.size() && dst.size() == mode.size(), "prep: list lengths differ");
  TORCH_CHECK((int)dst.size() <= dcr::kPrepMaxTasks, "prep: too many tasks");
  dcr::PrepTable tab{};
  tab.n = (int)dst.size();
  size_t xi = 0;  // next unused tensor of `extra` (TABLE: W, bias)
  auto ld = [](const at::Tensor& t) -> int {
    TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, "prep: views must be 2-D with unit column stride");
    return (int)t.stride(0);
  };
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  for (int i = 0; i < tab.n; ++i) {
    const at::Tensor& d = dst[i];
    const at::Tensor& s = src[i];
    TORCH_CHECK(d.is_cuda(), "prep: destinations must be GPU tensors");
    dcr::PrepTask& T = tab.t[i];
    T.mode = (int)mode[i];
    T.dst = d.data_ptr();
    if (T.mode == dcr::PREP_COLSUM) {
      // bias partials [R, cols] -> [cols]
      TORCH_CHECK(s.is_cuda() && s.scalar_type() == at::kFloat && d.scalar_type() == at::kFloat,
                  "prep COLSUM: fp32");
      TORCH_CHECK(d.is_contiguous() && d.numel() == s.size(-1), "prep COLSUM: dst must be [cols]");
      T.src = s.data_ptr();
      T.src_ld = ld(s);
      T.rows = (int)s.size(0);
      T.cols = (int)s.size(1);
      T.dst_ld = T.cols;
      continue;
    }
    T.dst_ld = ld(d);
    T.rows = (int)d.size(0);
    T.cols = (int)d.size(1);
    if (T.mode == dcr::PREP_ZERO) {
      TORCH_CHECK(d.element_size() == 4, "prep: ZERO needs 4-byte elements");
      continue;
    }
    TORCH_CHECK(s.is_cuda(), "prep: sources must be GPU tensors");
    T.src = s.data_ptr();
    if (T.mode == dcr::PREP_SUM) {
      // split-K slabs [S, rows, cols] -> [rows, cols]
      TORCH_CHECK(s.scalar_type() == at::kFloat && d.scalar_type() == at::kFloat, "prep SUM: fp32");
      TORCH_CHECK(s.dim() == 3 && s.stride(2) == 1 && s.size(1) == d.size(0) && s.size(2) == d.size(1),
                  "prep SUM: src must be [S, rows, cols] over dst [rows, cols]");
      TORCH_CHECK(s.stride(0) < (int64_t)1 << 31, "prep SUM: slab too large");
      T.src_ld = (int)s.stride(1);
      T.slab = (int)s.stride(0);
      T.nslab = (int)s.size(0);
      T.vec4 = (T.cols % 4 == 0 && T.src_ld % 4 == 0 && T.dst_ld % 4 == 0 && T.slab % 4 == 0 &&
                a16(T.src) && a16(T.dst)) ? 1 : 0;
      continue;
    }
    if (T.mode == dcr::PREP_ONEHOT) {
      // batch-major ids [B, T] -> time-major one-hot rows [T*B, VP] (bf16)
      TORCH_CHECK(s.scalar_type() == at::kInt && d.scalar_type() == at::kBFloat16, "prep ONEHOT: int32 -> bf16");
      T.src_ld = ld(s);
      T.kdim = (int)s.size(0);
      TORCH_CHECK(s.size(0) * s.size(1) == d.size(0), "prep ONEHOT: dst rows must be B*T");
      T.vec4 = (T.cols % 8 == 0 && T.cols <= 256 && T.dst_ld % 8 == 0 && a16(T.dst)) ? 1 : 0;
      continue;
    }
    if (T.mode == dcr::PREP_GATHER) {
      // batch-major ids [B, T] -> time-major bf16 rows E[id] [T*B, cols] (E fp32 [V, cols] in
      // `extra`; the ids must be < V: they index E unchecked)
      TORCH_CHECK(xi + 1 <= extra.size(), "prep GATHER: needs E in `extra`");
      const at::Tensor& E = extra[xi];
      xi += 1;
      TORCH_CHECK(s.scalar_type() == at::kInt && E.scalar_type() == at::kFloat &&
                  d.scalar_type() == at::kBFloat16, "prep GATHER: int32 ids, fp32 E -> bf16");
      TORCH_CHECK(E.is_cuda() && E.dim() == 2 && E.size(1) == d.size(1) &&
                  s.size(0) * s.size(1) == d.size(0), "prep GATHER: shape mismatch");
      T.src_ld = ld(s);
      T.src2 = E.data_ptr<float>();
      T.src2_ld = ld(E);
      T.kdim = (int)s.size(0);
      T.kind = dcr::PREP_BF16;
      T.vec4 = (T.cols % 4 == 0 && T.src2_ld % 4 == 0 && T.dst_ld % 4 == 0 && a16(T.src2) &&
                (reinterpret_cast<uintptr_t>(T.dst) & 7) == 0) ? 1 : 0;
      continue;
    }
    if (T.mode == dcr::PREP_TABLE) {
      // E [rows, K] · W [K, cols] + bias [cols], fp32
      TORCH_CHECK(xi + 2 <= extra.size(), "prep TABLE: needs W and bias in `extra`");
      const at::Tensor& W = extra[xi];
      const at::Tensor& bias = extra[xi + 1];
      xi += 2;
      TORCH_CHECK(s.scalar_type() == at::kFloat && W.scalar_type() == at::kFloat &&
                  d.scalar_type() == at::kFloat && bias.scalar_type() == at::kFloat, "prep TABLE: fp32");
      TORCH_CHECK(s.size(0) == d.size(0) && W.size(0) == s.size(1) && W.size(1) == d.size(1) &&
                  bias.is_contiguous() && bias.numel() == d.size(1), "prep TABLE: shape mismatch");
      T.src_ld = ld(s);
      T.src2 = W.data_ptr<float>();
      T.src2_ld = ld(W);
      T.aux = bias.data_ptr<float>();
      T.kdim = (int)s.size(1);
      continue;
    }
    T.src_ld = ld(s);
    T.rows = (int)s.size(0);
    T.cols = (int)s.size(1);
    if (s.scalar_type() == at::kInt) {
      TORCH_CHECK(d.scalar_type() == at::kInt, "prep: int32 sources copy to int32");
      T.kind = dcr::PREP_RAW32;
    } else {
      TORCH_CHECK(s.scalar_type() == at::kFloat, "prep: sources must be fp32 or int32");
      TORCH_CHECK(d.scalar_type() == at::kBFloat16 || d.scalar_type() == at::kFloat,
                  "prep: destinations must be bf16 or fp32");
      T.kind = d.scalar_type() == at::kBFloat16 ? dcr::PREP_BF16 : dcr::PREP_F32;
    }
    // float4 reads / 4-element writes (the weight-layout refresh of every step: 27 us in scalar
    // form at the headline shape, profiles/r2_s5_prep_split.txt)
    const bool al = T.src_ld % 4 == 0 && T.dst_ld % 4 == 0 && a16(T.src) &&
                    (reinterpret_cast<uintptr_t>(T.dst) & 7) == 0 && T.kind != dcr::PREP_RAW32 &&
                    (T.kind == dcr::PREP_BF16 || a16(T.dst));
    if (T.mode == dcr::PREP_COPY) {
      TORCH_CHECK(d.size(0) == s.size(0) && d.size(1) == s.size(1), "prep: copy shape mismatch");
      T.vec4 = (al && T.cols % 4 == 0) ? 1 : 0;
    } else if (T.mode == dcr::PREP_TRANSPOSE) {
      TORCH_CHECK(d.size(0) == s.size(1) && d.size(1) == s.size(0), "prep: transpose shape mismatch");
      T.vec4 = (al && T.cols % 4 == 0 && T.rows % 4 == 0) ? 1 : 0;
    } else {
      TORCH_CHECK(false, "prep: unknown mode");
    }
  }
  dcr::launch_prep(tab, cur_stream());
}

}  // namespace

TORCH_LIBRARY(dcr, m) {
  m.def("opt_num_partials(int n) -> int", [](int64_t n) -> int64_t { return dcr::opt_num_partials(n); });
  m.def("global_norm(Tensor g, Tensor(a!) partials, Tensor(b!) norm_out) -> ()");
  m.def(
      "adam_clip(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor(d!)? pbf, "
      "Tensor(e!) partials, Tensor(f!) norm_out, float lr_t, float b1, float b2, float eps, "
      "float clip, float gscale=1.0, int n_norm=-1, Tensor? extra_sq=None, "
      "Tensor? skip_if=None, Tensor? lr_dev=None) -> ()");
  m.def("sumsq(Tensor x, Tensor(a!) partials, Tensor(b!) out, Tensor(c!)? ticket=None, "
        "Tensor? extra=None, Tensor? guard=None) -> ()");
  m.def(
      "lstm_step_ew_fwd(Tensor zrec, Tensor zx, Tensor? ids, Tensor cprev, Tensor(a!) hout, "
      "Tensor(b!)? hout32, Tensor(c!) cout, Tensor(d!) gates, float forget_bias, "
      "Tensor? bias=None) -> ()");
  m.def(
      "lstm_step_ew_bwd(Tensor dtop, Tensor? dhrec, Tensor gates, Tensor c, Tensor cprev, "
      "Tensor(a!) dc, Tensor(b!) dz_out) -> ()");
  m.def(
      "lstm_big_step_fwd(Tensor WhT, Tensor hprev, Tensor zx, Tensor? ids, Tensor cprev, "
      "Tensor(a!) hout, Tensor(b!)? hout32, Tensor(c!) cout, Tensor(d!) gates, Tensor(e!) ws, "
      "Tensor(f!) cnt, float forget_bias, int force_S=0, Tensor? bias=None) -> int");
  m.def(
      "lstm_big_step_bwd(Tensor Wh, Tensor dznext, Tensor dtop, Tensor gates, Tensor c, "
      "Tensor cprev, Tensor(a!) dc, Tensor(b!) dz_out, Tensor(c!) ws, Tensor(d!) cnt, "
      "int force_S=0) -> int");
  m.def("big_step_workspace(bool bwd, int B, int H, int force_S=0) -> int[]",
        [](bool bwd, int64_t B, int64_t H, int64_t force_S) -> std::vector<int64_t> {
          int64_t wf = 0, nt = 0;
          dcr::big_step_workspace(bwd, (int)B, (int)H, num_cus(), (int)force_S, &wf, &nt);
          return {wf, nt};
        });
  m.def("big_step_supported(int B, int H) -> bool", [](int64_t B, int64_t H) -> bool {
    return dcr::big_step_supported((int)B, (int)H);
  });
  m.def("f32_fwd_seq(int cell, Tensor WT, Tensor? WT2, Tensor zx, Tensor(a!) hs, Tensor(b!)? cs, "
        "Tensor(c!)? gates, Tensor(d!)? rh, float forget_bias) -> ()");
  m.def("f32_bwd_seq(int cell, Tensor W, Tensor? W2, Tensor? dtop, Tensor hs, Tensor? cs, "
        "Tensor? gates, Tensor(a!) dz, Tensor(b!) work0, Tensor(c!) work1) -> ()");
  m.def("f32_seq_supported(int cell, int H) -> bool", [](int64_t c, int64_t H) -> bool {
    return dcr::f32_seq_supported((int)c, (int)H);
  });
  m.def(
      "rnn_fwd_seq(int cell, Tensor WT, Tensor? WT2, Tensor zx, Tensor? ids, Tensor(a!) hbuf, "
      "Tensor(b!)? h32, Tensor(c!)? cbuf, Tensor(d!)? gates, Tensor(e!)? pre, Tensor(f!)? aux, "
      "Tensor(g!)? rh, Tensor(h!)? hlast32, float forget_bias) -> ()");
  m.def(
      "rnn_bwd_seq(int cell, Tensor W, Tensor? W2, Tensor dtop, Tensor(a!) dz, Tensor(b!)? dzx, "
      "Tensor? gates, Tensor? pre, Tensor? aux, Tensor? zx, Tensor? cbuf, Tensor? h32, "
      "Tensor? hbuf, Tensor(c!) dc, Tensor(d!)? partial) -> ()");
  m.def(
      "xent(Tensor logits, Tensor targets, float grad_scale, Tensor(a!)? row_loss, "
      "Tensor(b!)? dlogits, Tensor(c!) partial, Tensor(d!) loss_out) -> ()");
  m.def(
      "xent_wide(Tensor logits, Tensor? bias, Tensor targets, float grad_scale, Tensor(a!)? row_loss, "
      "Tensor(b!)? dlogits, Tensor(c!)? colpart, Tensor(d!)? db, Tensor(e!) partial, "
      "Tensor(f!) loss_out) -> ()");
  m.def(
      "head_wide(Tensor O, Tensor WsT, Tensor? bias, Tensor? targets, float grad_scale, "
      "Tensor(a!)? row_loss, Tensor(b!)? dlogits, Tensor(c!)? logits, Tensor(d!)? colpart, "
      "Tensor(e!)? db, Tensor(f!) ws, Tensor(g!) loss_out) -> ()");
  m.def("head_wide_supported(int V, int H) -> int", [](int64_t V, int64_t H) -> int64_t {
    return dcr::head_wide_supported((int)V, (int)H);
  });
  m.def("head_wide_blocks(int N) -> int",
        [](int64_t N) -> int64_t { return dcr::head_wide_blocks((int)N); });
  m.def("head_wide_colpart_rows(int N) -> int",
        [](int64_t N) -> int64_t { return dcr::head_wide_colpart_rows((int)N); });
  m.def("head_wide_workspace(int N) -> int", [](int64_t N) -> int64_t {
    return (dcr::head_wide_blocks((int)N) + 3) / 4 * 4 + (int64_t)dcr::head_wide_stats_floats((int)N);
  });
  m.def("xent_wide_supported(int V) -> int",
        [](int64_t V) -> int64_t { return dcr::xent_wide_supported((int)V); });
  m.def("xent_wide_waves(int n) -> int",
        [](int64_t n) -> int64_t { return dcr::xent_wide_waves((int)n); });
  m.def("xent_num_partials(int n) -> int",
        [](int64_t n) -> int64_t { return dcr::xent_num_partials((int)n); });
  m.def("lstm_persist_supported(int H, int B) -> int", &lstm_persist_supported);
  m.def("lstm_persist_nt_tiles(int H, int B) -> int", &lstm_persist_nt_tiles);
  m.def("num_cus() -> int", []() -> int64_t { return num_cus(); });
  m.def("lstm_persist_grid(int H, int B) -> int", [](int64_t H, int64_t B) -> int64_t {
    return dcr::lstm_persist_grid((int)H, (int)B, num_cus());
  });
  m.def("lstm_persist_occupancy(int bwd, int H, int B, int V, int flags) -> int",
        [](int64_t bwd, int64_t H, int64_t B, int64_t V, int64_t flags) -> int64_t {
          return dcr::lstm_persist_occupancy((int)bwd, (int)H, (int)B, (int)V, (int)flags, num_cus());
        });
  m.def("lstm_persist_xfuse_supported(int H, int B) -> int", [](int64_t H, int64_t B) -> int64_t {
    return dcr::lstm_persist_xfuse_supported((int)H, (int)B, num_cus());
  });
  m.def(
      "lstm_persist_fwd(Tensor WT, Tensor zx, Tensor? ids, Tensor(a!) hbuf, Tensor(b!) cbuf, "
      "Tensor(c!)? gates, Tensor(d!) hlast32, Tensor(e!) cnt, Tensor(f!) err, float forget_bias, "
      "int spin_limit, Tensor(g!) hring, Tensor(h!)? diag=None, Tensor? WxT=None, "
      "Tensor? xin=None, Tensor? bias=None, bool cnt_zeroed=False, "
      "Tensor(i!)? clast32=None) -> ()");
  m.def(
      "lstm_persist_bwd(Tensor W, Tensor dtop, Tensor(a!) dz, Tensor gates, Tensor cbuf, "
      "Tensor(b!) cnt, Tensor(c!) err, int spin_limit, Tensor(d!) zring, Tensor(e!)? db_part=None, "
      "Tensor? ids=None, Tensor(f!)? dew_part=None, int V=0, Tensor(g!)? diag=None, "
      "bool exclusive=False, bool cnt_zeroed=False) -> ()");
  m.def("head_supported(int V, int H) -> int", [](int64_t V, int64_t H) -> int64_t {
    return dcr::head_supported((int)V, (int)H);
  });
  m.def("head_pads(int V) -> int[]", [](int64_t V) -> std::vector<int64_t> {
    return {dcr::head_vpad((int)V), dcr::head_kpad((int)V)};
  });
  m.def("head_workspace(int N, int V) -> int", [](int64_t N, int64_t V) -> int64_t {
    return (int64_t)dcr::head_num_partials((int)N, num_cus()) * (dcr::head_vpad((int)V) + 1);
  });
  m.def(
      "head(Tensor O, Tensor WsT, Tensor? Wsk, Tensor bias, Tensor? targets, float grad_scale, "
      "Tensor(a!)? logits, Tensor(b!)? row_loss, Tensor(c!)? dlogits, Tensor(d!)? dtop, "
      "Tensor(e!)? db, Tensor(f!) part, Tensor(g!)? loss, Tensor? omask=None, "
      "float oscale=1.0) -> ()");
  m.def("prep(Tensor[] src, Tensor(a!)[] dst, int[] mode, Tensor[] extra) -> ()");
  m.def("prep_max_tasks() -> int", []() -> int64_t { return dcr::kPrepMaxTasks; });
  m.def("tail(int[] words, int phase, Tensor(a!) part, Tensor(b!) sync, Tensor(c!) dep, "
        "Tensor(d!) err, int spin_limit, Tensor(e!)? total_out, Tensor? total_in, Tensor? extra, "
        "Tensor(f!)? p, Tensor? g, Tensor(g!)? m, Tensor(h!)? v, Tensor(i!)? mirror, int n_norm, "
        "float lr_t, float b1, float b2, float eps, float clip, float gscale, Tensor? lr_dev, "
        "Tensor? skip_if, Tensor(j!)? norm_out, bool dynamic=True) -> ()");
  m.def("tail_words() -> int", []() -> int64_t { return kTailWords; });
  m.def("generate(Tensor[] Wh, Tensor[] Wx, Tensor[] bias, Tensor table, Tensor WsT, Tensor bs, "
        "float forget_bias, Tensor h0, Tensor c0, Tensor(a!) h_out, Tensor(b!) c_out, Tensor prime, "
        "int num, Tensor(c!) out, Tensor(d!) hx, int mode, int space_id, int seed, Tensor ctr0, "
        "Tensor(e!)? logits_out, Tensor(f!) err, int spin_limit, Tensor(g!)? stamps=None) -> ()");
  m.def("generate_supported(int L, int H, int V, int S) -> int",
        [](int64_t L, int64_t H, int64_t V, int64_t S) -> int64_t {
          return dcr::generate_supported((int)L, (int)H, (int)V, (int)S, num_cus()); });
  m.def("tokennorm(Tensor dz, Tensor w, Tensor(a!) part, Tensor(b!) ticket, Tensor(c!) out) -> ()");
  m.def("gemm_nt(Tensor a, Tensor b, Tensor(a!) c, Tensor? bias=None) -> ()");
  m.def("tokennorm_store(Tensor dz, Tensor w, Tensor(a!) dx, Tensor(b!) part, Tensor(c!) ticket, "
        "Tensor(d!) out) -> ()");
  m.def("tokennorm_masked(Tensor dz, Tensor w, Tensor mask, float scale, Tensor(a!) dx, "
        "Tensor(b!) part, Tensor(c!) ticket, Tensor(d!) out) -> ()");
  m.def("id_sort(Tensor ids, int V, Tensor(a!) ws, Tensor(b!) sid, Tensor(c!) perm, "
        "Tensor(d!)? zero=None) -> bool");
  m.def("id_sort_workspace(int N, int V) -> int", [](int64_t N, int64_t V) -> int64_t {
    return V > 0 && V <= 16384 && N > 0 && N <= 65535
               ? (int64_t)dcr::id_sort_workspace((int)N, (int)V) : 0; });
  m.def("gemm_nt_supported(int M, int N, int K) -> int", [](int64_t M, int64_t N, int64_t K) -> int64_t {
    return dcr::gemm_nt_supported((int)M, (int)N, (int)K) ? 1 : 0; });
  m.def("tokennorm_supported(int N, int H, int K) -> int", [](int64_t N, int64_t H, int64_t K) -> int64_t {
    return dcr::tokennorm_supported((int)N, (int)H, (int)K) ? 1 : 0; });
  m.def("tail_max_tasks() -> int", []() -> int64_t { return dcr::kTailMaxTasks; });
  m.def("tail_ws_words() -> int[]", []() -> std::vector<int64_t> {
    return {dcr::kTailSyncWords, dcr::kTailDepWords};
  });
  m.def("tail_grid() -> int", []() -> int64_t { return dcr::tail_grid(num_cus()); });
  m.def("wgrad(Tensor[] A, Tensor[] B, Tensor(a!)[] part) -> ()");
  m.def("wgrad_plan_tiles(int tiles, int K) -> int", [](int64_t tiles, int64_t K) -> int64_t {
    return dcr::wgrad_splits_tiles((int)tiles, (int)K, num_cus()); });
  m.def("wgrad_plan_cost(int tiles, int K) -> float", [](int64_t tiles, int64_t K) -> double {
    double c = 0.0;
    dcr::wgrad_splits_tiles((int)tiles, (int)K, num_cus(), &c);
    return c; });
  m.def("wgrad_plan(int np, int M, int N, int K) -> int",
        [](int64_t np, int64_t M, int64_t N, int64_t K) -> int64_t {
          if (!dcr::wgrad_supported((int)M, (int)N, (int)K)) return 0;
          return dcr::wgrad_splits((int)np, (int)M, (int)N, (int)K, num_cus());
        });
  m.def("lstm2_plan(int H, int B, int force=0) -> int",
        [](int64_t H, int64_t B, int64_t force) -> int64_t {
          return dcr::lstm2_plan_g((int)H, (int)B, num_cus(), (int)force);
        });
  m.def("lstm2_xin_ok(int H) -> bool",
        [](int64_t H) -> bool { return dcr::lstm2_xin_ok((int)H, num_cus()); });
  m.def("lstm2_bwd_rs_ring_floats(int H, int B) -> int", [](int64_t H, int64_t B) -> int64_t {
    return (int64_t)dcr::lstm2_bwd_rs_ring_floats((int)H, (int)B);
  });
  m.def("lstm2_bwd_rs_ok(int H, int B) -> bool", [](int64_t H, int64_t B) -> bool {
    return dcr::lstm2_bwd_rs_ok((int)H, (int)B, num_cus());
  });
  m.def("lstm2_bwd_wide_ok(int H, int B) -> bool", [](int64_t H, int64_t B) -> bool {
    return dcr::lstm2_bwd_wide_ok((int)H, (int)B, num_cus());
  });
  m.def("lstm2_nbg(int B, int G) -> int",
        [](int64_t B, int64_t G) -> int64_t { return lstm2_nbg((int)B, (int)G); });
  m.def(
      "lstm2_persist_fwd(Tensor W0T, Tensor W1T, Tensor X1T, Tensor zx0, Tensor? ids, "
      "Tensor bias1, Tensor(a!) hbuf0, Tensor(b!) cbuf0, Tensor(c!)? gates0, Tensor(d!) hlast0, "
      "Tensor(e!) hbuf1, Tensor(f!) cbuf1, Tensor(g!)? gates1, Tensor(h!) hlast1, "
      "Tensor(i!) cnt0, Tensor(j!) cnt1, Tensor(k!) err, float forget_bias, int spin_limit, "
      "Tensor(l!) hring0, Tensor(m!) hring1, int G, Tensor(o!)? clast0=None, "
      "Tensor(p!)? clast1=None, Tensor(q!)? diag=None, Tensor? xmask=None, "
      "float xscale=1.0, Tensor? bias0=None, Tensor? x0=None, Tensor? X0T=None, "
      "Tensor(r!)? xdst=None, Tensor? omask=None, float oscale=1.0, Tensor(s!)? odst=None) -> ()");
  m.def(
      "lstm2_persist_bwd(Tensor Wh0, Tensor Wh1, Tensor Wx1, Tensor dtop1, Tensor gates0, "
      "Tensor cbuf0, Tensor gates1, Tensor cbuf1, Tensor(a!) dz0, Tensor(b!) dz1, "
      "Tensor(c!) zring0, Tensor(d!) zring1, Tensor(e!)? db_part0, Tensor(f!)? db_part1, "
      "Tensor(g!) cnt0, Tensor(h!) cnt1, Tensor(i!) err, int spin_limit, int G, "
      "Tensor(j!)? diag=None, Tensor? xmask=None, float xscale=1.0, Tensor(k!)? pring=None) -> ()");
  m.def("dropout_bits(Tensor(a!) bits, int seed, int stream, float keep) -> ()");
  m.def(
      "dropout_bits_multi(Tensor(a!) bits, int seed, int[] streams, float[] keeps, "
      "Tensor? ids=None, Tensor? E=None, float scale=1.0, Tensor(b!)? out=None) -> ()");
  m.def("mask_apply(Tensor input, Tensor bits, float scale, Tensor(a!) out) -> ()");
  m.def("embed_dropout(Tensor ids, Tensor E, Tensor? bits, float scale, Tensor(a!) out) -> ()");
  m.def("sample_supported(int V, int H) -> int", [](int64_t V, int64_t H) -> int64_t {
    return dcr::sample_supported((int)V, (int)H);
  });
  m.def(
      "sample_step(Tensor O, Tensor WsT, Tensor bs, Tensor(a!) cur, Tensor(b!) out, "
      "Tensor(c!) pos, Tensor(d!) ctr, Tensor? u, Tensor(e!)? logits, int mode, int space_id, "
      "int seed) -> ()");
  m.def("gru_persist_ub(int H, int B) -> int", [](int64_t H, int64_t B) -> int64_t {
    return dcr::gru_persist_ub((int)H, (int)B, num_cus());
  });
  m.def(
      "gru_persist_fwd(Tensor WgT, Tensor WcT, Tensor zx, Tensor? ids, Tensor(a!) hbuf, "
      "Tensor(b!) h32, Tensor(c!) rh, Tensor(d!) gates, Tensor(e!)? hlast32, Tensor(f!) cnt, "
      "Tensor(g!) err, int spin_limit, bool cnt_zeroed=False, Tensor(h!)? ring0=None, "
      "Tensor(i!)? ring1=None, Tensor? bias_x=None) -> ()");
  m.def(
      "gru_persist_bwd(Tensor Wg, Tensor Wc, Tensor dtop, Tensor(a!) dz, Tensor gates, "
      "Tensor h32, Tensor(b!) cnt, Tensor(c!) err, int spin_limit, bool cnt_zeroed=False, "
      "Tensor(d!)? ring0=None, Tensor(e!)? ring1=None, Tensor(f!)? db_part=None) -> ()");
  m.def("segsum(Tensor X, Tensor? ids, int V, Tensor(a!) out, Tensor(b!) workspace, bool accumulate, "
        "Tensor? perm=None) -> ()");
  m.def("segsum_workspace(int N, int W, int V) -> int", [](int64_t N, int64_t W, int64_t V) -> int64_t {
    return (int64_t)dcr::segsum_workspace_floats((int)N, (int)W, (int)V);
  });
}

TORCH_LIBRARY_IMPL(dcr, CUDA, m) {
  m.impl("global_norm", &global_norm);
  m.impl("sumsq", &sumsq);
  m.impl("lstm_step_ew_fwd", &lstm_step_ew_fwd);
  m.impl("lstm_step_ew_bwd", &lstm_step_ew_bwd);
  m.impl("lstm_big_step_fwd", &lstm_big_step_fwd);
  m.impl("lstm_big_step_bwd", &lstm_big_step_bwd);
  m.impl("head_wide", &head_wide);
  m.impl("adam_clip", &adam_clip);
  m.impl("rnn_fwd_seq", &rnn_fwd_seq);
  m.impl("f32_fwd_seq", &f32_fwd_seq);
  m.impl("f32_bwd_seq", &f32_bwd_seq);
  m.impl("rnn_bwd_seq", &rnn_bwd_seq);
  m.impl("xent", &xent);
  m.impl("xent_wide", &xent_wide);
  m.impl("segsum", &segsum);
  m.impl("lstm_persist_fwd", &lstm_persist_fwd);
  m.impl("lstm_persist_bwd", &lstm_persist_bwd);
  m.impl("head", &head);
  m.impl("prep", &prep);
  m.impl("tail", &tail);
  m.impl("generate", &generate);
  m.impl("tokennorm", &tokennorm);
  m.impl("gemm_nt", &gemm_nt);
  m.impl("tokennorm_masked", &tokennorm_masked);
  m.impl("tokennorm_store", &tokennorm_store);
  m.impl("id_sort", &id_sort);
  m.impl("wgrad", &wgrad);
  m.impl("gru_persist_fwd", &gru_persist_fwd);
  m.impl("lstm2_persist_fwd", &lstm2_persist_fwd);
  m.impl("lstm2_persist_bwd", &lstm2_persist_bwd);
  m.impl("dropout_bits", &dropout_bits);
  m.impl("dropout_bits_multi", &dropout_bits_multi);
  m.impl("mask_apply", &mask_apply);
  m.impl("embed_dropout", &embed_dropout);
  m.impl("sample_step", &sample_step);
  m.impl("gru_persist_bwd", &gru_persist_bwd);
}
