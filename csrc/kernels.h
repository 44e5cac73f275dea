// Host-side launcher declarations for the gfx950 kernels.  Implemented in the *.hip files,
// bound to torch in ops.cpp.  All launchers are asynchronous on `stream`, allocate nothing and
// never synchronise (hipGraph-capturable, cdna_hip_programming.md Guideline 9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcr {
typedef __bf16 bf16;

// ---- optim.hip -------------------------------------------------------------------------
int opt_num_partials(int64_t n);
void launch_global_norm(const float* g, int64_t n, float* partials, float* norm_out,
                        hipStream_t stream);
void launch_sumsq(const void* x, bool is_bf16, int64_t n, float* partials, float* out,
                  unsigned* ticket, hipStream_t stream, const float* extra = nullptr,
                  const int* guard = nullptr);
void launch_adam_clip(float* p, const float* g, float* m, float* v, bf16* pbf, int64_t n,
                      float* partials, float* norm_out, float lr_t, float b1, float b2, float eps,
                      float clip, float gscale, int64_t n_norm, const float* extra_sq,
                      const unsigned* skip_if, const float* lr_dev, hipStream_t stream);

// ---- rnn_step.hip -----------------------------------------------------------------------
enum CellKind { CELL_LSTM = 0, CELL_GRU_A = 1, CELL_GRU_B = 2, CELL_RNN = 3, CELL_NAS = 4 };

struct FwdStepArgs {
  const bf16* WT;        // [G*H, H] bf16: transposed recurrent weights (row = gate column)
  const float* zx;       // [B, zx_ld] fp32 input projection (+bias) of this step, or the
                         // [V, zx_ld] E·W_x table when ids != nullptr (layer-0 gather mode)
  const int* ids;        // [B] token ids of this step (gather mode) or nullptr
  int zx_ld, zx_off;     // row stride and column offset of this cell's gate block in zx
  const bf16* hop;       // [B, H] bf16 MFMA B-operand (h_{t-1}; r*h for GRU_B)
  const float* hprev32;  // [B, H] fp32 h_{t-1} (GRU)
  const float* cprev;    // [B, H] fp32 c_{t-1} (LSTM, NAS)
  bf16* hout;            // [B, H] bf16 h_t
  float* hout32;         // [B, H] fp32 h_t (GRU always; others optional)
  float* cout;           // [B, H] fp32 c_t (LSTM, NAS)
  bf16* gates;           // [B, gates_ld] bf16 activation cache for backward
  float* pre;            // NAS: [B, gates_ld] fp32 pre-activations
  float* aux;            // NAS: [B, H] fp32 recurrent branch-3 pre-activation
  bf16* rh;              // GRU_A: [B, H] bf16 r*h_{t-1}
  int gates_ld;
  int B, H;
  float forget_bias;
  // no-GEMM mode (WT == nullptr; LSTM / RNN): the recurrent pre-activation h_{t-1}·W_h was
  // computed elsewhere (library GEMM, large H) into zrec [B, zrec_ld] fp32; epilogue only
  const float* zrec;
  int zrec_ld;
  int nsplit;            // zrec holds nsplit split-K partial slabs of [B, zrec_ld] (0 = 1)
};

struct BwdStepArgs {
  const bf16* W;         // [H, K] bf16 recurrent weights in TF layout (row = unit, k contiguous)
  const bf16* dz_next;   // [B, dz_ld] bf16 GEMM operand (dZ of step t+1), nullptr => no GEMM
  int K, dz_ld;
  const float* dtop;     // [B, H] fp32 gradient arriving from above/the loss at this step
  const bf16* gates;     // [B, gates_ld] activation cache
  const float* pre;      // NAS pre-activations [B, gates_ld]
  const float* aux;      // NAS zm3 [B, H]
  const float* zx3;      // NAS: input branch 3 pre-activation, row stride zx3_ld
  int zx3_ld;
  const float* c;        // [B, H] c_t
  const float* cprev;    // [B, H] c_{t-1}
  const float* hprev32;  // GRU h_{t-1}
  const bf16* hcur;      // RNN h_t
  float* dc;             // [B, H] fp32 carry: dc (LSTM/NAS), dh' (GRU)
  float* partial;        // GRU [B, H] fp32 partial dh_{t-1}
  bf16* dz_out;          // [B, dz_out_ld] bf16 dZ_t (NAS: recurrent-branch dZm)
  bf16* dzx_out;         // NAS: input-branch dZx
  int dz_out_ld, gates_ld;
  int B, H;
  int nsplit;            // LSTM epilogue-only: `partial` = nsplit [B, H] slabs (0 = 1)
};

// ---- lstm_ew.hip: epilogue-only LSTM cell steps (large-H library-step path) -------------
struct LstmEwArgs {
  int B, H, nsplit;        // nsplit: zrec / dhrec slabs ([nsplit, B, 4H] / [nsplit, B, H])
  float forget_bias;
  // forward
  const float* zrec;       // recurrent pre-activation slabs
  const float* zx;         // [B, 4H] input projection + bias, or the [V, 4H] table with ids
  const int* ids;          // [B] or nullptr
  const float* bias;       // optional [4H]: input bias not folded into a dense zx
  const float* cprev;      // [B, H]
  bf16* hout;              // [B, H]
  float* hout32;           // optional [B, H]
  float* cout;             // [B, H]
  bf16* gates;             // [B, 4H] (sigma i, tanh j, sigma f, sigma o)
  // backward
  const float* dtop;       // [B, H]
  const float* dhrec;      // recurrent dh slabs (nsplit may be 0)
  const bf16* gates_in;    // [B, 4H]
  const float* c;          // [B, H] c_t
  float* dc;               // [B, H] carry (in/out)
  bf16* dz_out;            // [B, 4H]
};
void launch_lstm_ew(bool bwd, const LstmEwArgs& a, hipStream_t s);

// ---- lstm_gemm_step.hip: fused large-H LSTM step (MFMA GEMM + cell epilogue) -------------
struct BigStepArgs {
  int B, H, S;             // S: split-K slices (set by the launcher)
  const bf16* A;           // forward: W_hᵀ [4H, H]; backward: W_h [H, 4H]
  const bf16* X;           // forward: h_{t-1} [B, H]; backward: dZ_{t+1} [B, 4H]
  float* ws;               // split-K slabs (big_step_workspace floats)
  unsigned* cnt;           // [tiles] arrival tickets, zero between launches
  LstmEwArgs ew;           // epilogue operands (forward / backward fields as in lstm_ew.hip)
};
bool big_step_supported(int B, int H);
void big_step_workspace(bool bwd, int B, int H, int cus, int force_S, int64_t* ws_floats,
                        int64_t* tickets);
int launch_big_step(bool bwd, const BigStepArgs& a, int cus, int force_S, hipStream_t s);

void launch_fwd_step(int cell, const FwdStepArgs& a, hipStream_t s);
void launch_bwd_step(int cell, const BwdStepArgs& a, hipStream_t s);

// ---- cell_f32.hip: fp32-operand sequences (--dtype fp32) ------------------------------------
struct F32Seq {
  int cell;              // CELL_LSTM, CELL_GRU_A (the GRU), CELL_RNN
  const float* WT;       // fwd: W_hᵀ [G·H, H] (GRU: Wg_hᵀ [2H, H])
  const float* WT2;      // fwd GRU: Wc_hᵀ [H, H]
  const float* W;        // bwd: W_h [H, GW] TF layout (GRU: Wc_h [H, H])
  const float* W2;       // bwd GRU: Wg_h [H, 2H]
  const float* zx;       // [T, B, GW] input projection + bias
  const float* dtop;     // [T, B, H] or null
  float* hs;             // [T+1, B, H]
  float* cs;             // [T+1, B, H] (LSTM)
  float* gates;          // [T, B, GW] (LSTM, GRU)
  float* rh;             // [T, B, H] (GRU)
  float* dz;             // [T, B, GW]
  float* work0;          // [B, H]
  float* work1;          // [B, H]
  int T, B, H, GW;
  float forget_bias;
};
bool f32_seq_supported(int cell, int H);
void launch_f32_fwd_seq(const F32Seq& q, hipStream_t s);
void launch_f32_bwd_seq(const F32Seq& q, hipStream_t s);

// ---- xent.hip ---------------------------------------------------------------------------
int xent_num_partials(int N);
void launch_xent(const float* logits, const int* targets, int N, int V, float grad_scale,
                 float* row_loss, bf16* dlogits, float* partial, float* loss_out, hipStream_t s);

// ---- dropout.hip: bit masks ([rows, K/8] bytes) -----------------------------------------------
constexpr int kDropMaxSegs = 16;
struct DropSegs {             // n masks of nwords 32-bit words each, consecutive in memory
  int n;
  int64_t nwords;
  uint64_t stream[kDropMaxSegs];
  unsigned kt[kDropMaxSegs];  // keep threshold on a 16-bit uniform (drop_threshold)
};
struct DropEmbed {            // optional: segment 0's masked embedding rows (embed_dropout)
  const int* ids = nullptr;   // [rows] ids of the rows (time-major)
  const float* E = nullptr;   // [V, K] fp32 embedding
  bf16* out = nullptr;        // [rows, K] bf16 (null: bits only)
  int K = 0;                  // row width, a multiple of 32
  float scale = 1.f;
};
unsigned drop_threshold(float keep);
void launch_dropout_bits(uint8_t* bits, const DropSegs& d, uint64_t seed, hipStream_t s,
                         const DropEmbed& e = DropEmbed{});
void launch_mask_apply(const void* in, bool in_bf16, int64_t ld_in, void* out, bool out_bf16,
                       int64_t ld_out, const uint8_t* bits, int64_t rows, int K, float scale,
                       hipStream_t s);
void launch_embed_dropout(const int* ids, const float* E, const uint8_t* bits, bf16* out,
                          int64_t rows, int K, float scale, hipStream_t s);

// ---- embed.hip --------------------------------------------------------------------------
// stable counting sort of N <= 65535 ids in [0, V), V <= 16384: sid = sorted ids, perm = their
// positions; ws holds id_sort_workspace(N, V) ints; returns -1 for other shapes
int id_sort_blocks(int N);
int id_sort_cols(int V);
size_t id_sort_workspace(int N, int V);
// zero (optional): zero_n floats (16-B aligned, zero_n % 4 == 0) cleared by the first launch
int launch_id_sort(const int* ids, int N, int V, int* ws, int* sid, int* perm, hipStream_t s,
                   float* zero = nullptr, size_t zero_n = 0);
int segsum_rows_per_chunk(int N);
size_t segsum_workspace_floats(int N, int W, int V);
// perm (atomic route only): ids are sorted and perm[n] is the source row of position n
void launch_segsum_bf16(const bf16* X, int ldx, const int* ids, int N, int W, int V, float* out,
                        float* workspace, int accumulate, hipStream_t s,
                        const int* perm = nullptr);
void launch_segsum_f32(const float* X, int ldx, const int* ids, int N, int W, int V, float* out,
                       float* workspace, int accumulate, hipStream_t s,
                       const int* perm = nullptr);

// ---- lstm_persist.hip -------------------------------------------------------------------
struct PersistArgs {
  const bf16* W;         // fwd: W_hᵀ [4H, H]; bwd: W_h [H, 4H] (TF layout)
  const float* zx;       // fwd: [T, B, zx_ld] input projection, or [V, zx_ld] table with ids
  const int* ids;        // fwd gather mode: [T, B] token ids
  int zx_ld;
  bf16* hbuf;            // [T+1, B, H] bf16 (slot 0 = h_0)
  float* cbuf;           // [T+1, B, H] fp32 (slot 0 = c_0)
  bf16* gates;           // [T, B, 4H] bf16 activation cache (sigma(i), tanh(j), sigma(f), sigma(o))
  float* hlast32;        // [B, H] fp32 final h
  float* clast32;        // optional [B, H] fp32 final c (the new TBPTT state without a copy)
  const float* dtop;     // bwd: [T, B, H] fp32 gradient from above
  bf16* dz;              // bwd: [T, B, 4H] bf16 gate-pre-activation gradients
  float* db_part;        // bwd: [B/16, 4H] per-batch-group bias-gradient partials (or nullptr)
  float* dew_part;       // bwd layer-0 gather mode: [B/16, V, 4H] dEW partials (or nullptr)
  int V;
  const bf16* Wx;        // fwd: W_xᵀ [4H, H] fused input projection (or nullptr)
  const bf16* xin;       // fwd fused input: [T, B, H] bf16 layer input
  const float* bias;     // fwd fused input: [4H] fp32
  unsigned* cnt;         // [B/16, T+1] arrival counters (zeroed by the launcher)
  unsigned* err;         // timeout / error word (0 = ok)
  unsigned long long* diag;  // optional [T, 8] s_memtime stamps of workgroup 0 (diagnostics)
  int B, H, T;
  float forget_bias;
  unsigned spin_limit;
  int excl;              // bwd: all-loads-in-flight variant (one WG per CU: nothing may run beside it)
  int cnt_zeroed;        // counters already zeroed by the caller (batched prep launch)
  int poller;            // H > 1024 kernels: thread that polls the hand-off counters (launcher)
  bf16* hring;           // fwd: [2, B, H] fragment-tiled h hand-off ring
  bf16* zring;           // bwd: [2, B, 4H] fragment-tiled dZ hand-off ring
                         //   (persist_common.h frag_index); dz stays row-major for the GEMMs
};
int lstm_persist_supported(int H, int B, int cus);
// H > 1024 (lstm_persist_nt.hip): 16-unit workgroups over NT 16-row batch tiles
int lstm_persist_nt_tiles(int H, int B, int cus);
int lstm_persist_nt_grid(int H, int B, int cus);
const void* lstm_persist_nt_fn(int bwd, int H, int B, int cus, int diag = 0);
int lstm_persist_grid(int H, int B, int cus);
int lstm_persist_xfuse_supported(int H, int B, int cus);
// max co-resident workgroups per CU of the instantiation a launch with these flags would use
// (flags: 1 fused input projection (fwd), 2 diag stamps, 4 exclusive bwd; V>0: fused dEW LDS)
int lstm_persist_occupancy(int bwd, int H, int B, int V, int flags, int cus);
// return 0 on success, <0 if the grid cannot be co-resident or the shape is unsupported
int launch_lstm_fwd_persist(const PersistArgs& a, int cus, hipStream_t s);
int launch_lstm_bwd_persist(const PersistArgs& a, int cus, hipStream_t s);

// wide-vocabulary softmax CE (xent.hip): bias added in-kernel, fused d softmax_b, V % 4 == 0,
// V <= 8192
int xent_wide_waves(int N);
// loss = sum(partial[0:nb]) / N; db = column sums of colpart [ncp, V] (when both given)
void launch_xent_finalize(const float* partial, int nb, int N, float* loss_out,
                          const float* colpart, int ncp, int V, float* db, hipStream_t s);

// fused wide-vocabulary head (head_wide.hip): logits -> lse -> loss, bf16 dlogits, d softmax_b
// partials, without writing fp32 logits
struct HeadWideArgs {
  const bf16* O; int ldo;      // [N, H] top-layer outputs (bf16, row stride ldo)
  const bf16* WsT;             // [V, H] softmax_wᵀ (bf16)
  const float* bias;           // [V] softmax_b (or nullptr)
  const int* targets;          // [N] (or nullptr: no loss)
  int N, V, H;
  float grad_scale;            // 1 / N
  float* row_loss;             // [N] (optional)
  bf16* dlogits;               // [N, V] (optional: training)
  float* logits;               // [N, V] fp32 (optional: summaries / eval)
  float* colpart;              // [head_wide_colpart_rows(N), V] d softmax_b partials (optional)
  float* partial;              // [head_wide_blocks(N)] loss partials
  float* stats;                // [head_wide_stats_floats(N)] per-half softmax stats (8-B aligned)
};
int head_wide_blocks(int N);
int head_wide_colpart_rows(int N);
size_t head_wide_stats_floats(int N);
int head_wide_supported(int V, int H);
int launch_head_wide(const HeadWideArgs& a, float* db, float* loss_out, hipStream_t s);
int xent_wide_blocks(int N);
int xent_wide_supported(int V);
void launch_xent_wide(const float* logits, const float* bias, const int* targets, int N, int V,
                      float grad_scale, float* row_loss, bf16* dlogits, float* colpart, float* db,
                      float* partial, float* loss_out, hipStream_t s);

// two-layer wavefront LSTM forward (lstm2_persist.hip)
struct Lstm2Args {
  const bf16* W0T;      // layer l   W_hᵀ [4H, H]
  const bf16* W1T;      // layer l+1 W_hᵀ [4H, H]
  const bf16* X1T;      // layer l+1 W_xᵀ [4H, H]
  const float* zx0;     // layer l input projections (+bias): [T, B, zx_ld] or [V, zx_ld] table
  const int* ids;       // gather mode: [T, B]
  int zx_ld;
  const float* bias1;   // layer l+1 bias [4H]
  const float* bias0;   // optional layer l bias [4H], added in-kernel to a dense zx0 written
                        // without it (null: zx0 / the gather table already holds it)
  bf16* hbuf0; float* cbuf0; bf16* gates0; float* hlast0;   // layer l   [T+1,B,H] ...
  bf16* hbuf1; float* cbuf1; bf16* gates1; float* hlast1;   // layer l+1
  unsigned* cnt0;       // [nbg, T+1, 4] arrivals of layer l   (zeroed by the caller)
  unsigned* cnt1;       // [nbg, T+1, 4] arrivals of layer l+1
  unsigned* err;
  unsigned long long* diag;  // optional [T+1, 8] s_memtime stamps of workgroup 0 (diagnostics)
  float* clast0;        // optional [B, H] final c of layers l and l+1
  float* clast1;
  bf16* hring0;         // [2, nbg*32, H] fragment-tiled h hand-off rings (persist_common.h)
  bf16* hring1;
  int B, H, T;          // B: real batch rows (row-major buffers); rows up to nbg*32 are padding
  int G, nbg;           // batch groups per workgroup; 32-row batch groups (multiple of G)
  float forget_bias;
  unsigned spin_limit;
  const uint8_t* xmask; // optional dropout bits of layer l+1's input [T, B, H/8] (dropout.hip)
  float xscale;         //   and their 1/keep
  const bf16* x0;       // optional (G = 1): layer l's bf16 input rows [T·B, H]; the input
  const bf16* X0T;      //   projection x0·W_x,l (W_x,lᵀ [4H, H]) then runs in-kernel (zx0 unused)
  int wgarr;            // 1: one counter add per workgroup and layer (the layer's last epilogue
                        //   wave signals for both, persist_common.h wg_arrive); 0: one per wave
  int hld;              // row stride (elements) of hbuf0 / hbuf1: H, or 2H when both layers' h
                        //   live interleaved in one [T+2, B, 2H] buffer (row t+1 = [h_l(t),
                        //   h_l+1(t-1)]: the operand of layer l+1's merged weight gradient)
  int xcdloc;           // 1: XCD-resident hand-offs for columns found on one XCD (persist_common.h;
                        //   exchange word: dwords 2-3 of cnt0's slot 0 per column); 0: write-through
  int zx_rows;          // gather mode: rows of the zx0 table (the vocabulary), else 0
  int steady;           // forward: ticks LAG+1 .. T-3 on the steady-state (constant-condition) body
  bf16* xdst;           // optional (dropout, G = 1): layer l+1's masked input rows h_l ⊙ mask /
  int xdld;             //   keep [T·B, H] (row stride xdld), written with layer l's row-major h
  const uint8_t* omask; // optional (dropout, G = 1): layer l+1's output dropout bits [T, B, H/8],
  float oscale;         //   their 1/keep and the masked rows h_l+1 ⊙ mask / keep [T·B, H]
  bf16* odst;           //   (dense) written with layer l+1's row-major h
};
// batch groups per workgroup for the two-layer kernels at (H, B) (force > 0: only that value),
// 0 = unsupported
int lstm2_plan_g(int H, int B, int cus, int force);
int launch_lstm2_fwd_persist(const Lstm2Args& a, int cus, hipStream_t s);
bool lstm2_xin_ok(int H, int cus);

// two-layer wavefront LSTM BPTT (lstm2_persist.hip): layers l and l+1 in one launch, layer l
// one step behind layer l+1; layer l's dtop = dZ_{l+1}·W_x,l+1ᵀ is computed in-kernel
struct Lstm2BwdArgs {
  const bf16* Wh0;      // layer l   W_h [H, 4H] (TF layout)
  const bf16* Wh1;      // layer l+1 W_h [H, 4H]
  const bf16* Wx1;      // layer l+1 W_x [H, 4H] (input rows of its kernel)
  const float* dtop1;   // [T, B, H] gradient arriving at layer l+1's output
  const bf16* gates0; const float* cbuf0;   // layer l   activation cache [T,B,4H], c [T+1,B,H]
  const bf16* gates1; const float* cbuf1;   // layer l+1
  bf16* dz0; bf16* dz1;                     // [T, B, 4H] row-major dZ (weight GEMM operands)
  bf16* zring0; bf16* zring1;               // [2, B, 4H] fragment-tiled dZ hand-off rings
  float* db_part0; float* db_part1;         // [2*nbg/G, 4H] bias-gradient partials (or nullptr)
  unsigned* cnt0;       // [nbg, T+1, 4] arrivals of layer l   (zeroed by the caller)
  unsigned* cnt1;       // [nbg, T+1, 4] arrivals of layer l+1
  unsigned* err;
  unsigned long long* diag;  // optional [T+2, 8] s_memtime stamps of workgroup 0
  int B, H, T;
  int G, nbg;           // as Lstm2Args; zring0/1 hold [2, nbg*32, 4H]
  unsigned spin_limit;
  const uint8_t* xmask; // optional dropout bits of layer l+1's input [T, B, H/8]: layer l's dtop
  float xscale;         //   (dtop1 arrives with layer l+1's output dropout already applied)
  int db_rows;          // rows of db_part0/1 (the wide kernel zeroes the ones past its columns)
  int wgarr;            // as Lstm2Args::wgarr
  int diag_all;         // diag holds [grid, T+2, 8] s_memrealtime stamps of every workgroup
  int xcdloc;           // as Lstm2Args::xcdloc (exchange word: dwords 2-3 of cnt0's slot 0)
  float* pring;         // optional reduce-scatter partial ring (lstm2_bwd_rs.hip), fp32
};
int launch_lstm2_bwd_persist(const Lstm2BwdArgs& a, int cus, hipStream_t s);
// the reduce-scatter form of the 32 x 16 BPTT (lstm2_bwd_rs.hip): no dropout, H in {128, 256,
// 512}; pring holds lstm2_bwd_rs_ring_floats(H, B) floats
size_t lstm2_bwd_rs_ring_floats(int H, int B);
bool lstm2_bwd_rs_ok(int H, int B, int cus);
int launch_lstm2_bwd_rs(const Lstm2BwdArgs& a, int cus, hipStream_t s);
// the 32-unit x 16-row form of the same BPTT (lstm2_bwd_wide.hip): nbg = ceil(B / 16) 16-row
// columns, G = 1
bool lstm2_bwd_wide_ok(int H, int B, int cus);
int launch_lstm2_bwd_wide(const Lstm2BwdArgs& a, int cus, hipStream_t s);

// persistent GRU recurrence (gru_persist.hip)
struct GruPersistArgs {
  const bf16* WgT;      // fwd: W_g,hᵀ [2H, H] (r rows, then u rows)
  const bf16* WcT;      // fwd: W_c,hᵀ [H, H]
  const float* zx;      // fwd: [T, B, zx_ld] input projections (+bias) or [V, zx_ld] table
  const float* bias_x;  // fwd: optional [3H] bias added in-kernel (zx written without it)
  const int* ids;       // fwd gather mode: [T, B]
  int zx_ld;            // 3H
  bf16* hbuf;           // [T+1, B, H] bf16 (slot 0 = h_0)
  float* h32;           // [T+1, B, H] fp32 (slot 0 = h_0)
  bf16* rh;             // fwd: [T, B, H] r ⊙ h_{t-1}
  bf16* gates;          // [T, B, 3H] r, u, c~
  float* hlast32;       // fwd: [B, H] (optional)
  const bf16* Wg;       // bwd: W_g,h [H, 2H] (TF layout)
  const bf16* Wc;       // bwd: W_c,h [H, H]
  const float* dtop;    // bwd: [T, B, H]
  bf16* dz;             // bwd: [T, B, 3H] dZr, dZu, dZc
  unsigned* cnt;        // 2 sets x [B/16, T+1, 4] counters
  unsigned* err;
  bf16* ring0;          // optional fragment-tiled hand-off rings (persist_common.h):
  bf16* ring1;          //   fwd: h [2,B,H], r⊙h [2,B,H];  bwd: dZc [2,B,H], dZg [2,B,2H]
  int B, H, T;
  unsigned spin_limit;
  int cnt_zeroed;
  int xcdloc;           // as Lstm2Args::xcdloc (exchange word: dwords 2-3 of slot 0 of the fwd's
                        //   h set / the bwd's dZg set, which no counter uses)
  float* db_part;       // bwd (optional): [ceil(B/16), 3H] bias-gradient partials, one row per
                        //   16-row batch tile (sums of the bf16-rounded dZr, dZu, dZc)
};
// token-reduction weight-gradient GEMM (wgrad.hip): C_s = A_chunkᵀ · B_chunk per split-K slab
constexpr int kWgradMaxProblems = 4;
constexpr int kWgradMaxSplit = 32;
struct WgradProblem {
  const bf16* A; long lda;   // [K, M] token-major rows (row stride lda elements)
  const bf16* B; long ldb;   // [K, N]
  float* C; long ldc;        // slab 0 of [S, M, N] fp32 partials (row stride ldc)
  long slab;                 // elements between slabs
  int M, N, S;               // this problem's shape and split count
  int tiles, item0;          // set by the launcher
};
struct WgradArgs {
  WgradProblem p[kWgradMaxProblems];
  int np, K, items;          // items: set by the launcher
};
bool wgrad_supported(int M, int N, int K);
int wgrad_splits(int np, int M, int N, int K, int cus);
int wgrad_splits_tiles(int tiles, int K, int cus, double* cost_out = nullptr);  // (+ modelled us)
void launch_wgrad(WgradArgs& a, hipStream_t s);
int gru_persist_ub(int H, int B, int cus);
int gru_persist_rows(int H, int B, int cus);  // padded batch rows of the launch plan (rings)
int launch_gru_persist(int bwd, const GruPersistArgs& a, int cus, hipStream_t s);

// fused softmax head (head.hip)
struct HeadArgs {
  const bf16* O;        // [N, ldo] bf16 top-layer outputs
  int ldo;
  const bf16* WsT;      // [VP, H] bf16 softmax_wᵀ, rows >= V zero (VP = head_vpad(V))
  const bf16* Wsk;      // [H, VK] bf16 softmax_w, columns >= V zero (VK = head_kpad(V))
  const float* bias;    // [V]
  const int* targets;   // [N] or nullptr (logits-only)
  int N, H, V;
  float grad_scale;     // d loss / d logit scale (1/N for cost = sum/B/T)
  float* logits;        // [N, V] fp32 or nullptr
  float* row_loss;      // [N] or nullptr
  bf16* dlogits;        // [N, ldl] bf16 (columns < V written) or nullptr
  int ldl;              // dlogits row stride (V, or 256: the zero-padded operand of the
                        //   softmax_w gradient's wgrad tile)
  float* dtop;          // [N, H] fp32 or nullptr
  float* part;          // [grid, VP+1] partials workspace
  const uint8_t* omask; // optional dropout bits of O ([N, H/8], dropout.hip): dtop is written
  float oscale;         //   masked and scaled by 1/keep (the output dropout's backward)
  int lds_wst;          // set by the launcher: softmax_wᵀ staged in (dynamic) LDS
};
int head_vpad(int V);
int head_kpad(int V);
int head_supported(int V, int H);
int head_num_partials(int N, int cus);
int launch_head(const HeadArgs& a, int cus, float* db_out, float* loss_out, hipStream_t s);

// batched per-step data movement (prep.hip)
enum PrepMode : int {
  PREP_COPY = 0, PREP_TRANSPOSE = 1, PREP_ZERO = 2, PREP_SUM = 3, PREP_COLSUM = 4,
  PREP_ONEHOT = 5, PREP_TABLE = 6, PREP_GATHER = 7
};
enum PrepKind : int { PREP_F32 = 0, PREP_BF16 = 1, PREP_RAW32 = 2 };  // destination element
struct PrepTask {
  const void* src;      // fp32 row-strided source (RAW32: any 32-bit; ONEHOT: int32 [B, T] ids)
  void* dst;            // bf16 / fp32 / raw 32-bit (ZERO: any 4-byte element type)
  const float* src2;    // TABLE: W [kdim, cols]
  const float* aux;     // TABLE: bias [cols] (optional)
  int rows, cols;       // source shape (ZERO, ONEHOT, SUM, TABLE: destination shape)
  int src_ld, dst_ld;   // row strides in elements
  int src2_ld;          // TABLE: row stride of W
  int slab;             // SUM: elements between consecutive slabs
  int nslab;            // SUM: number of slabs
  int kdim;             // TABLE: reduction length; ONEHOT: batch B
  int mode;             // PrepMode
  int kind;             // PrepKind
  int vec4;             // SUM: float4 path (all strides and pointers 16-B aligned)
  int tile0;            // first tile (set by launch_prep)
};
constexpr int kPrepMaxTasks = 40;  // keeps the by-value table (kernel arguments) near 3 KB
struct PrepTable {
  PrepTask t[kPrepMaxTasks];
  int n;
};
void launch_prep(PrepTable& tab, hipStream_t s);


// TF token-norm term sum_tok ||dZ0_tok · W_x0ᵀ||² without materialising dx (tokennorm.hip)
constexpr int kTokenNormMaxGrid = 1024;
struct TokenNormArgs {
  const bf16* dz; long ld_dz;   // [N, K] bf16, K-contiguous rows
  const bf16* w; long ld_w;     // [N_units, K] bf16 (W_x0 in TF layout [H, 4H])
  int N, N_units, K;
  float* part;                  // [grid] partials
  unsigned* ticket;             // zeroed, reset by the kernel
  float* out;                   // [1] the sum of squares
  float* c; long ldc;           // gemm_nt: C [N, N_units] fp32 (the products themselves)
  const float* cbias;           // gemm_nt: optional [N_units] added to every row of C
  const uint8_t* mask;          // masked form: dropout bits [N, N_units / 8] (dropout.hip), and
  bf16* cb; float mscale;       //   C [N, N_units] bf16 (row stride ldc) = products ⊙ mask · mscale
};
bool tokennorm_supported(int N, int H, int K);
void launch_tokennorm(const TokenNormArgs& a, hipStream_t s);
// the same pipeline storing C = dz · wᵀ (config 5's dtop = dlogits · softmax_wᵀ)
bool gemm_nt_supported(int M, int N, int K);
void launch_gemm_nt(const TokenNormArgs& a, hipStream_t s);

// single-launch autoregressive generation (generate.hip): LSTM layers + head + draw per char
constexpr int kGenMaxLayers = 4;
constexpr int kGenMaxStreams = 16;
struct GenArgs {
  int L, H, V, S;
  const bf16* Wh[kGenMaxLayers];     // [H, 4H] bf16 TF layout (recurrent rows)
  const bf16* Wx[kGenMaxLayers];     // [H, 4H] bf16 (input rows; layer 0 unused: the table)
  const float* bias[kGenMaxLayers];  // [4H] fp32 (layer 0 unused: inside the table)
  const float* table;                // [V, 4H] fp32 E·W_x0 + b0
  const bf16* WsT;                   // [V, H] bf16 softmax_wᵀ
  const float* bs;                   // [V]
  float forget_bias;
  const float* h0; const float* c0;  // [L, S, H] initial state
  float* h_out; float* c_out;        // [L, S, H] final state
  const int* prime; int P;           // prime ids (P >= 1); prime[:-1] warms the state
  int num;                           // characters drawn
  int* out;                          // [S, num]
  unsigned long long* hx;            // [L, 2, S, H] tagged hand-off granules (zeroed per launch)
  int mode, space_id;
  unsigned long long seed;
  const unsigned* ctr0;              // [S] first RNG counter of each stream
  float* logits_out;                 // optional [num, S, V]
  unsigned* err; unsigned spin_limit;
  int ws_lds;                        // set by the launcher: softmax_wᵀ resident in LDS
  unsigned long long* stamps;        // optional [2][8][16] phase timestamps (diagnostics)
  int dbg;                           // diagnostics (DCR_DEBUG=gen_dbg): 1 no head, 2 head w/o h
};
int generate_supported(int L, int H, int V, int S, int cus);
int launch_generate(GenArgs& a, int cus, hipStream_t s);

// the training step's tail (tail.hip): gradient finalize + fused Adam with the bf16 layouts
enum TailOp : int { TAIL_SUM = 0, TAIL_COLSUM = 1, TAIL_SUMSQ = 2, TAIL_MM = 3, TAIL_ADAM = 4 };
struct TailTask {
  int op, rows, cols, tile0;   // output (SUM / COLSUM / MM) or region (SUMSQ / ADAM) shape
  int norm;                    // FINALIZE: square the outputs into the global norm
  int wait, need;              // wait until dep[wait] >= need (-1: none; producers come first)
  int sig;                     // dep counter each finished tile adds 1 to (-1: none)
  int vec4, nslab, k;          // float4 path; SUM slabs; MM reduction length
  int o1_t, o2_t;              // ADAM layout outputs: 1 = transposed (o[c][r])
  // SUM: a = slab 0 of [S, rows, cols] (row stride ar, slab stride ak); COLSUM: a = [k, cols]
  // partials (row stride ar); SUMSQ: a = rows * cols contiguous floats;
  // MM: dst[r, c] = bias[c] + sum_k a[r ar + k ak] * b[k bk + c bc]
  const float* a; long ar, ak;
  const float* b; long bk, bc;
  const float* bias;
  float* dst; long dst_ld;
  long off, ld;                // ADAM: region flat[off + r ld + c] of p / g / m / v / mirror
  bf16* o1; long o1_ld;
  bf16* o2; long o2_ld;
};
constexpr int kTailMaxTasks = 16;  // the by-value table stays under 3 KB of kernel arguments
constexpr int kTailMaxDeps = 4;
constexpr int kTailMaxGrid = 1024;
constexpr int kTailMaxTiles = 16384;  // per-tile norm partials (the part buffer)
// every counter of the tail on its own 256-B line: agent-scope atomics to one line serialise
// (~90 per us), and the ticket / queue / dependency words are hit by different workgroup sets
constexpr int kTailLine = 64;                          // words
constexpr int kTailTop = 0, kTailQueue = 1, kTailGroup0 = 2;  // line indices in sync
constexpr int kTailSyncWords = (kTailGroup0 + 8) * kTailLine;
constexpr int kTailDepWords = kTailMaxDeps * kTailLine;
struct TailArgs {
  TailTask t[kTailMaxTasks];
  int n, ntiles, phase;        // phase 0 FINALIZE, 1 ADAM
  int static_tiles;            // set by the launcher: tiles before the first waiting task's
  int dynamic;                 // 1: atomic tile queue (the GPU may be shared); 0: static tiles
  float* part;                 // [kTailMaxTiles] per-tile sums of squares (norm)
  unsigned* sync;              // [kTailSyncWords] top ticket, tile queue head, 8 group tickets
                               //   (one line each); zeroed, reset by the kernel
  unsigned* dep;               // [kTailDepWords] dependency counters (line i: counter i)
  unsigned* err;
  unsigned spin_limit;
  float* total_out;            // FINALIZE: global sum of squares (+ extra)
  const float* total_in;       // ADAM: that sum
  const float* extra;          // one more norm term (the TF per-token embedding slot)
  float* p; const float* g; float* m; float* v; bf16* mirror;
  long n_norm;
  float lr_t, b1, b2, eps, clip, gscale;
  const float* lr_dev;
  const unsigned* skip_if;
  float* norm_out;
};
int tail_grid(int cus);
int launch_tail(TailArgs& a, int cus, hipStream_t s);

// on-device sampling step (sample.hip): softmax head + categorical draw, one workgroup per stream
struct SampleArgs {
  const bf16* O;          // [S, H] top-layer output of this step
  const bf16* WsT;        // [V, H] softmax_wᵀ (bf16)
  const float* bs;        // [V] softmax_b
  int* cur;               // [S] in: previous ids (sampling_type 2); out: the picks
  int* out;               // [S, ld] generated ids; row s written at pos[s]
  int* pos;               // [S] write positions (incremented)
  unsigned* ctr;          // [S] RNG counters (incremented)
  const float* u;         // optional [S] explicit uniforms in [0, 1) (tests)
  float* logits_out;      // optional [S, V] fp32 logits (tests)
  int S, H, V, ld, mode, space_id;
  unsigned long long seed;
};
int sample_supported(int V, int H);
void launch_sample_step(const SampleArgs& a, hipStream_t s);

}  // namespace dcr
