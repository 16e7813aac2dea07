// Host-callable launchers of the gfx950 kernels (defined in csrc/kernels/*.hip).
// None of them allocates or synchronises: they only enqueue on `stream`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cst {

// beam.hip: fused beam step (LSE + candidate top-K + selection + next cell)
struct BeamFusedArgs {
  const struct VocabPartial* part;  // (n_vt, R) tile partials of the vocab launch
  const float2* cand;               // (n_vt, R, K) tile candidates (VF_TOPK)
  int n_vt, R, K, B, T;
  float* beam_sum;
  int64_t* seq_hist;  // (2, R, T)
  float* lp_hist;
  float* best_ppl;
  int64_t* best_seq;
  float* best_lp;
  int64_t* tok_out;
  const float* pre;   // (R, 4H) h_t W_hh^T + video gates; nullptr = no cell (last step)
  const uint16_t* ptab;  // (V, 4H) fp16
  const float* c_in;  // (R, H)
  float* c_out;
  uint16_t* h_out;    // (R, H) bf16
  int H, cell;
  const uint16_t* vg16;  // nullable (R, 4H) bf16 video gates of every current row (attention)
};
void launch_beam_fused_step(const BeamFusedArgs& a, int t, hipStream_t stream);

// cider_d.hip
void launch_cider_d(const int64_t* hyps, int T, const int64_t* hyp_video, int N,
                    const int64_t* ht_keys, const float* ht_vals, uint32_t ht_cap,
                    const int32_t* vid_ref_off, const int32_t* ref_ng_off,
                    const float* ref_norm, const int32_t* ref_len, const int64_t* ng_key,
                    const float* ng_val, float log_ref_len, int use_eos, float* out,
                    hipStream_t stream);

// adam.hip
// bf16 shadow copies of decoder weights written by the optimizer pass
// (GATES kinds: a recurrent cell's W_ih / W_hh, rows scattered into the packed
// 4-slot gate layout, see common.h "recurrent cells")
enum ShadowKind : int { SHADOW_PLAIN = 0, SHADOW_GATES_IH = 1, SHADOW_GATES_HH = 2 };
constexpr int SHADOW_MAX_SEGS = 12;
struct ShadowSeg {
  int64_t off, n;   // range of the flat parameter buffer
  int kind;         // ShadowKind
  int cols;         // row length of the source matrix (GATES kinds)
  int H, E;         // cell sizes: packed wx is (4H, E + H)
  uint16_t* dst;    // PLAIN: dst[j]; GATES kinds: packed wx
  uint16_t* dst2;   // GATES_HH: packed W_hh copy; GATES_IH: packed video columns
                    // [E, cols) of W_ih (nullable); row stride ld2
  int ld2;
  int slots;        // GATES kinds: packed slot of source gate g = bits [2g, 2g + 2)
};
struct ShadowSegs {
  ShadowSeg s[SHADOW_MAX_SEGS];
  int n;
};
// hyper (device): [lr, step before, skipped count, step after] (adam.hip)
void launch_flat_adam(float* p, const float* g, float* m, float* v, int64_t n, float* partials,
                      const bool* skip, float* scal, float* hyper, float b1, float b2,
                      float eps, float clip, float gscale, int phase, const ShadowSegs& ss,
                      hipStream_t stream);
void launch_shadow_refresh(const float* p, const ShadowSegs& ss, hipStream_t stream);

// vocab.hip
enum SelModeHost : int { SEL_GT_H = 0, SEL_SAMPLE_H = 1, SEL_GREEDY_H = 2, SEL_SS_H = 3 };
// vocab flag of the beam search's per-tile top-K candidates (kernels/vocab_common.h
// VF_TOPK; the beam size in bits 8..11)
constexpr int VF_TOPK_H = 32;
int vocab_num_tiles(int V);
void launch_vocab_fwd_variant(int variant, const uint16_t* hd, int ldh, int R, int H,
                              const uint16_t* W, const float* bias, int V, uint16_t* logits16,
                              int64_t ldl, void* part, const int64_t* tgt, int64_t tgt_stride,
                              int flags, float inv_temp, const uint32_t* rng, int step,
                              hipStream_t stream);
int vocab_partial_bytes();
// rng (device, nullable): int32[2] seeds {dropout, sampling}, see common.h
void launch_vocab_fwd(const uint16_t* hd, int ldh, int R, int H, const uint16_t* W,
                      const float* bias,
                      int V, uint16_t* logits16, int64_t ldl, void* part, const int64_t* tgt,
                      int64_t tgt_stride, int flags, float inv_temp, const uint32_t* rng,
                      int step, hipStream_t stream,
                      const float* eoff = nullptr);  // flags: 1 = sample, 2 = argmax, 8 = fp32 logits, 16 = exp store
// Cell epilogue of the next step, fused into the combine (see lstm_gemm.h).
struct CellLaunch {
  const void* pre;        // (R, 4H) fp32, or fp16 with pre_half
  const uint16_t* ptab;   // (V, 4H) fp16 projected embedding table
  const float* c_prev;
  float* c_out;
  uint16_t* h_out;
  uint16_t* hdrop_out;
  int ldh;
  uint16_t* gates_out;
  int H;
  float drop_p;
  int step;
  int cell;  // CellType (common.h)
  const uint16_t* vg16;  // nullable (R, 4H) bf16 per-row video gates (attention)
  int pre_half;
};
// temporal-attention forward operands (kernels/att_fwd.h)
struct AttFwdArgs {
  const float* gv;       // (Bv, C, G4) per-frame gate tables
  const float* pre;      // (Bv, C, A) projected frames P
  const float* q;        // (rows, A) queries (nullptr: q = 0)
  const int* q_rowmap;   // nullable: query row of each row
  const float* wa;       // scorer weights (A) or (C, A) per frame
  const float* ba;       // scorer bias (1) or (C)
  int wa_ld, ba_ld, vdiv, ngroups, C, A, G4;
  float* vg_out;         // (rows, G4): per-row video gate term
  float* alpha_out;      // nullable (rows, C)
  int accumulate;        // 1: vg_out += (else =)
};
// MFMA temporal attention of one decode step, one workgroup per video
// (kernels/att_mfma.h), run as extra workgroups of the merged decode launch
struct AttMfmaArgs {
  const uint16_t* h;     // (R, H) bf16 query input h_t
  const uint16_t* wq;    // (A, H) bf16
  const float* P;        // (Bv, C, A) projected frames
  const float* wa;       // (A) scorer weights
  const float* ba;       // (1) scorer bias
  const uint16_t* gv16;  // (Bv, 4H, CP) bf16 per-frame gate tables, frame-minor
  int H, A, C, CP, G4, vdiv, Bv;
  uint16_t* vg_out;      // (R, 4H) bf16 per-row video gates
  float* alpha_out;      // nullable (R, C)
  float* q_out;          // nullable (R, A) fp32
  float* e_part;         // (Bv, A / 64, 32, CP) partial-score slots
  int* cnt;              // (Bv) tickets, zero at the first launch (re-armed by the kernel)
  uint16_t* u_out;       // nullable (R, C, A) fp16 scorer values tanh(P + q) (training:
                         // the fused attention backward reads them instead of recomputing)
  int64_t* dbg;          // nullable (workgroups, 8) wall-clock phase stamps (microbenchmark)
  int whole;             // 1: one workgroup per video loops over the A / 64 query slices
                         // (att_mfma.h att_mfma_fwd_video: no slots / ticket)
};
// the MFMA attention path applies: rows per video 2..32, C <= 16, A % 64 == 0,
// A <= 1024, H % 32 == 0, 64 <= H <= 512, the shared scorer (not per frame)
bool att_mfma_ok(int vdiv, int C, int A, int H, int per_frame);
// the same for a forward that saves nothing for a backward (the SCST greedy
// baseline, evaluation): one row per video allowed
bool att_mfma_fwd_ok(int vdiv, int C, int A, int H, int per_frame);
// standalone launch of the same workgroups (tests / microbenchmarks)
void launch_att_mfma_fwd(const AttMfmaArgs& a, hipStream_t stream);
// AttMfmaArgs::whole for a shape (1 with CSTCAP_ATT_WHOLE=1 where its LDS fits)
int att_mfma_whole_default(int C, int H);
// size of the end-of-sequence flag area per decode step (ints) of `counts`
int combine_count_ints_per_step();
void launch_vocab_combine(const void* part, int n_vt, int R, float* lse_out, int64_t* tok_out,
                          int64_t tok_stride, float* g_sel, int64_t gsel_stride, float* g_xe,
                          int64_t gxe_stride, const int64_t* gt, int64_t gt_stride, int mode,
                          float ss_prob, const uint32_t* rng, int step, int* counts, int count_step,
                          uint8_t* unfinished, hipStream_t stream, const CellLaunch* cell = nullptr,
                          int rows_per_step = 0);
// (rows_per_step > 0: the partials are per-step blocks [R / rows_per_step]
// [n_vt][rows_per_step] -- the XE all-rows forward combines every step's rows
// in one launch; 0: one block [n_vt][R])
// vocab projection of step t + recurrent GEMM of step t+1 in one launch
// (tiled transposed-epilogue kernel; pre == nullptr: vocab only).  NQ > 0:
// whh has 4H + NQ rows, the last NQ (W_q) produce the attention query q_out
// (R x NQ) and vgate must be nullptr.  Returns the number of partial slots
// per row it wrote into part (the combine's n_vt); part must hold
// vocab_part_slots(V) x R.
int vocab_part_slots(int V);
int launch_vocab_lstm_fwd(const uint16_t* hd, int ldh, int R, int H, const uint16_t* W,
                           const float* bias, int V, uint16_t* logits16, int64_t ldl, void* part,
                           const int64_t* tgt, int64_t tgt_stride, int flags, float inv_temp,
                           const uint32_t* rng, int step, const uint16_t* h_t, const uint16_t* whh,
                           const float* vgate, int vdiv, float* pre, hipStream_t stream,
                           int NQ = 0, float* q_out = nullptr, const float* eoff = nullptr,
                           const AttMfmaArgs* att = nullptr, int pre_half = 0);
// exp store of step 0: fp16 logits rows -> bf16 exp(x - lse_r), in place
void launch_vocab_exp_convert(uint16_t* buf, int64_t ldl, int V, int R, const float* lse,
                              hipStream_t stream);

// vocab_grad.hip: vocab-head backward from the exp store (see that file).
// Row weights of the NR = n_steps * R rollout rows: sampled / chosen tokens
// (weight dg_sel) and XE targets (weight dg_xe)
// XE all rows (engine.cpp): the cell operands of a whole-step LSTM tile
// (lstm_gemm.h lstm_cell_block) inside the previous step's decode launch
struct XeCell {
  const int64_t* tok;  // input tokens of the step (row stride tok_stride)
  int64_t tok_stride;
  const uint16_t* ptab;  // fp16 (V, 4H) projected-embedding gate table
  const float* c_prev;   // (R, H)
  uint16_t* h_out;       // (R, H) bf16
  float* c_out;          // (R, H)
  uint16_t* hd_out;      // (R, H) bf16 dropout(h)
  uint16_t* gates_out;   // (R, 4H) bf16 packed cell gates (saved for the backward)
  float drop_p;
  int key;   // dropout key of the step
  int cell;  // CellType
};

// one decode launch of the XE all-rows forward: the whole LSTM step of h_t's
// successor (xc non-null: h_t W_hh^T + vgate + P[tok] -> cell) and the
// vocabulary tiles of the rows hd (non-null): E = exp(x) (offset 0, bf16) into
// logits16 and the per-tile partials (target logit tgt), no token choice
void launch_vocab_lstm_xe(const uint16_t* hd, int R, int H, const uint16_t* W, const float* bias,
                          int V, uint16_t* logits16, int64_t ldl, void* part, const int64_t* tgt,
                          const uint32_t* rng, const uint16_t* h_t, const uint16_t* whh,
                          const float* vgate, int vdiv, const XeCell* xc, hipStream_t stream);

struct VGradRows {
  int R, n_steps, T_sel, H, V;
  const float* lse;       // (n_steps, R)
  const int64_t* y_sel;   // (R, T_sel) sampled / chosen tokens, nullable
  const float* dg_sel;    // (R, T_sel), nullable
  const int64_t* y_xe;    // labels + 1, row stride yxe_rs, nullable
  int64_t yxe_rs;
  const float* dg_xe;     // row stride dgxe_rs, nullable
  int64_t dgxe_rs;
  // exp-store range guard (nullable): rows whose LSE moved by more than
  // EXP_SAFE_LSE_JUMP from the previous step are listed here by
  // vgrad_onehot ([0] = count, then flat row ids) and recomputed by vgrad_fix
  int* fix;
  // forward-computed X = E W (engine.cpp "X in the rollout"): vgrad_onehot also
  // writes each row's one-hot weights / tokens (nullable outputs, NR each;
  // token -1 = none), so the loop forms dHd = alpha X + a W[ys] + b W[yx]
  // without the folded E', and vgrad_fix recomputes the listed rows of X
  float* oh_a;
  int* oh_ys;
  float* oh_b;
  int* oh_yx;
  float* X;  // (NR, H) fp32, nullable
  // the forward wrote E = exp(x) (offset 0: the XE all-rows forward) instead
  // of exp(x - the previous step's LSE): s = exp(-lse), and the range guard
  // lists rows with |lse| > EXP_SAFE_LSE_JUMP (step 0 included)
  int zero_off;
};
constexpr float EXP_SAFE_LSE_JUMP = 60.f;
// alpha (NR) and the one-hot terms folded into E (NR rows, stride ldl), in place
void launch_vgrad_onehot(const VGradRows& g, uint16_t* E, int64_t ldl, float* alpha,
                         hipStream_t stream);
// Exact recompute of the listed rows (fix[0] of them, flat ids fix[1..]):
// logits from the saved vocab input hd (NR x H bf16) and W / bias, the row's
// E rewritten with its own LSE as offset (scale 1), alpha and the one-hot
// terms set accordingly; fix_total[0] += fix[0] (a running count, nullable)
void launch_vgrad_fix(const VGradRows& g, const uint16_t* hd, const uint16_t* W,
                      const float* bias, uint16_t* E, int64_t ldl, float* alpha, int* fix_total,
                      hipStream_t stream);
// dhd = alpha . dhd in place (X = E' W -> dHd; dhd nullable: the consumer
// scales the rows itself), hs = bf16(alpha . hd)
void launch_vgrad_rows(const float* alpha, int64_t NR, int H, const uint16_t* hd, float* dhd,
                       uint16_t* hs, hipStream_t stream, int ldhs = 0);
// dblog = sum_r alpha_r E_rv (two launches: per-row-block partials, reduce);
// part: vgrad_colsum_blocks(NR) * V floats
int vgrad_colsum_blocks(int64_t NR);
void launch_vgrad_colsum(const uint16_t* E, int64_t ldl, int V, int64_t NR, const float* alpha,
                         float* part, float* dblog, hipStream_t stream);

// lstm.hip
void launch_lstm_step_fwd(const int64_t* tok, int64_t tok_stride, const uint16_t* ptab,
                          const uint16_t* h_prev, const float* c_prev, const float* vgate,
                          int vgate_div, int R, int H, const uint16_t* whh, uint16_t* h_out,
                          float* c_out, uint16_t* hdrop_out, int ldh, float drop_p,
                          const uint32_t* rng, int step, uint16_t* gates_out, hipStream_t stream,
                          const int* row_map, int cell);  // row_map: h/c source row (beam)

// dg_next / dG rows have stride KD: 4H gate columns (+ A attention-query
// columns, matched by extra whhT columns [W_hh^T | W_q^T] of width KD)
int lstm_bwd_tiles(int R, int H);
// Temporal-attention term of the backward step's epilogue (MFMA attention
// path): per 64-unit column tile, the partial dalpha[r][c] = sum over the
// tile's 256 packed gate columns of dG[r][n] Gv[video(r)][n][c] (kernels
// lstm.hip); kernels/attention.hip att_bwd_mfma sums the H/64 partials.
// One-hot part of the vocab head's h gradient when the loop reads the
// forward-computed X = E W instead of E' W: dh_logit row r gets
// + a[r] W[ys[r]] + b[r] W[yx[r]] (W: logit weights (V, H) bf16; a / ys, b /
// yx nullable, this step's R rows; token < 0: no term)
struct DhOneHot {
  const uint16_t* W;
  const float* a;
  const int* ys;
  const float* b;
  const int* yx;
};
struct AttBwdEpi {
  const uint16_t* gvb16;  // (Bv, H, CP, 4) bf16 gate tables, the 4 gates of a unit innermost
  int vdiv, C, CP;
  float* dal_part;       // (H / 64, R, CP) fp32, this step's partials
  // Attention backward of step t + 1 fused into step t's launch (flags != null):
  // Bv extra workgroups, dispatched first (blockIdx < Bv), turn step t + 1's
  // dalpha partials (dal_next) into dq_{t+1} (bf16, written through into the
  // tail columns [G4, G4 + A) of dg_next, the launch's own A operand) and
  // accumulate dP / dw_a / db_a; each then bumps flags[video].  The GEMM
  // workgroups stream the dG_{t+1} columns first and wait for their videos'
  // flags only before the tail K-tiles (lstm.hip).
  int* flags;             // (Bv) int32, zero before the launch (per step)
  const float* dal_next;  // (H / 64, R, CP): step t + 1's partials (other buffer)
  const float* alpha;     // (R, C) of step t + 1
  const uint16_t* u;      // (R, C, A) fp16 tanh(P + q) of step t + 1 (AttMfmaArgs::u_out)
  const float* wa;        // (A)
  int Bv, A, G4;
  float* dP_acc;    // (Bv, C, A)
  float* dwa_part;  // (Bv, A)
  float* dba_part;  // (Bv)
  // bounded flag poll of the GEMM workgroups: polls before giving up, and the
  // device error word a wait that gave up increments (nullable)
  int poll_bound;
  int* poll_err;
};
// fused attention backward (AttBwdEpi::flags) supported for this shape
bool att_bwd_fuse_ok(int vdiv, int C, int A, int H, int Bv, int R);
bool att_bwd_epi_ok(int vdiv, int C, int H);
void launch_lstm_step_bwd(const uint16_t* dg_next, const uint16_t* whhT, const float* dh_logit,
                          float* dc_carry, const uint16_t* gates, const float* c_t,
                          const float* c_prev, int R, int H, float drop_p, const uint32_t* rng,
                          int step, uint16_t* dG, int KD, hipStream_t stream, int cell,
                          const float* dh_scale = nullptr,  // dh_logit row scales (nullable)
                          const AttBwdEpi* att = nullptr,
                          const struct DhOneHot* oh = nullptr);

// lstm_loop.hip: the whole reverse recurrence of a one-layer decoder without
// attention / initial state in ONE persistent launch (see the file header)
struct BwdLoopArgs {
  uint16_t* dG;            // (T, R, 4H) bf16 out: gate gradients of every step
  const uint16_t* whhT;    // (H, 4H) bf16 W_hh^T (packed gate columns)
  const float* dh;         // (T, R, H) fp32 vocab-head h gradient (X or dHd); the row
                           // scales and one-hot terms are folded into it IN PLACE
  const float* scale;      // (T, R) row scales of dh (nullable)
  const uint16_t* oh_W;    // one-hot terms (DhOneHot, all steps; oh_a null: none)
  const float* oh_a;
  const int* oh_ys;
  const float* oh_b;
  const int* oh_yx;
  const uint16_t* gates;   // (T, R, 4H) bf16 saved gate activations
  const float* c_all;      // (T, R, H) fp32 cell states
  float* dc_out;           // (R, H) final state-gradient carry (nullable)
  int R, H, T, cell;
  float drop_p;
  const uint32_t* rng;
  int* cnt;                // team counters (lstm_bwd_loop_counter_ints), zeroed per launch
  int* err;                // device error word (nullable)
  int poll_bound;
  int nub, nrb, rows_per_group, rows_per_block;  // (set by the launcher)
  int64_t* phases;         // microbenchmark: (grid, T, 4) wall-clock stamps (nullable)
  int dbg;                 // microbenchmark variants of form 1: 1 plain B loads, 2 no B
                           // loads, 4 plain dG stores (results not valid)
  int form;                // 1: each workgroup reads its rows' whole dG_{t+1} (default);
                           // 0: K-split team GEMM, partials exchanged (lstm_loop.hip)
  float* xb;               // form 0: exchange slabs (lstm_bwd_loop_xb_floats)
};
bool lstm_bwd_loop_ok(int R, int H, int T);
int lstm_bwd_loop_counter_ints(int R, int H);
int64_t lstm_bwd_loop_xb_floats(int R, int H);
void launch_lstm_bwd_loop(BwdLoopArgs a, hipStream_t stream);

// attention.hip (temporal attention over num_chunks frames; MANet modal
// attention with per_frame = 1: scorer weights w_a (C, A), biases b_a (C))
// rows of one video per attention-backward workgroup (2 or 4; C > 8: 4)
constexpr int ATT_BWD_RPW = 4;
int att_groups(int vdiv, int rpw = ATT_BWD_RPW);  // backward workgroups per video
// dGv partials (att_dgv_chunks(n_steps), Bv, C, G4) fp32 of sum_{t, r in b}
// alpha[t, r, c] dG[t, r, 0:G4] (dG rows bf16, stride ldg; alpha (n, R, C))
int att_dgv_chunks(int n_steps);
void launch_att_dgv(const uint16_t* dG, int ldg, const float* alpha, int n_steps, int R, int Bv,
                    int vdiv, int C, int G4, float* part, hipStream_t stream);
// vg_out[r] = sum_c alpha_rc Gv[b, c]  (+= when accumulate: adds into pre)
// rows of one video per attention-forward workgroup: 0 = by the rows per
// video (4 at >= 4, e.g. the rollout's 20; 1 for the one-row greedy baseline:
// 16.6 vs 22.7 us at 1,280 rows, 9.2 vs 7.2 us at 64,
// profiles/r2/microbench_kernels_v11.json)
constexpr int ATT_FWD_RPW = 0;
void launch_att_fwd(const float* gv, const float* pre, const float* q, const int* q_rowmap,
                    const float* wa, const float* ba, int Bv, int vdiv, int C, int A, int G4,
                    float* vg_out, float* alpha_out, hipStream_t stream, int accumulate,
                    int per_frame, int rpw = ATT_FWD_RPW);
// MFMA attention path backward of one step, grid (Bv, A / 128): dalpha from
// the step kernel's partials, softmax backward, tanh-scorer backward; dq_t
// written as bf16 into columns [4H, 4H + A) of the dG rows (write_dq), dP
// accumulated in place (dP_acc (Bv, C, A)), dw_a / db_a into per-video slots
// (Bv, A) / (Bv).  q nullable (step 0: q = 0).
void launch_att_bwd_mfma(const float* dal_part, int n_ut, int R, const float* alpha,
                         const float* q, const float* P, const float* wa, int Bv, int vdiv, int C,
                         int CP, int A, int G4, uint16_t* dG, int ldg, int write_dq, float* dP_acc,
                         float* dwa_part, float* dba_part, hipStream_t stream);
// dwa_part / dba_part: per-workgroup slots of (A) / (1), or (C, A) / (C) per_frame
void launch_att_bwd(uint16_t* dG, int ldg, const float* gv, const float* pre, const float* q,
                    const float* alpha, const float* wa, int Bv, int vdiv, int C, int A, int G4,
                    int write_dq, float* dpre_part, float* dwa_part, float* dba_part,
                    hipStream_t stream, int per_frame, int rpw = ATT_BWD_RPW);

// featpool.hip: FeatPool (per modality Linear -> ReLU -> Dropout, concat)
constexpr int FEATPOOL_MAX_F = 8;
struct FeatPoolSeg {
  const float* x;  // (rows, d) features of modality f, row stride ld
  const float* w;  // (H, d) weight
  const float* b;  // (H) bias
  int d, ld;
  int blk0, bblk0;  // first forward / backward workgroup of the modality
};
struct FeatPoolArgs {
  FeatPoolSeg s[FEATPOOL_MAX_F];
  int nf, rows, H;
  int fwd_blocks, bwd_blocks;
};
struct FeatPoolGrads {
  float* dw[FEATPOOL_MAX_F];
  float* db[FEATPOOL_MAX_F];
};
void featpool_layout(FeatPoolArgs& a);  // fills blk0 / bblk0 / *_blocks
// ws: fwd_blocks * 64 * 64 floats; out: (rows, nf * H)
void launch_featpool_fwd(const FeatPoolArgs& a, float* ws, float* out, float drop_p,
                         const uint32_t* rng, hipStream_t stream);
void launch_featpool_bwd(const FeatPoolArgs& a, const float* dout, const float* out, float drop_p,
                         const FeatPoolGrads& gr, hipStream_t stream);

// loss.hip: SCST reward + reward mask + REINFORCE loss (out = {loss, mean
// sample, mean greedy, sum mask}), and its backward
// ws: scst_loss_ws_ints(R) ints, zero before the first launch (the kernel
// re-arms its ticket)
int scst_loss_ws_ints(int R);
// CST baseline of the fused loss (S == 0: SCST, the greedy scores)
struct CstBase {
  const float* bref;  // nullable (R) GT consensus scores (scb_baseline 1); null: the samples'
  int S;              // rows (scores) per video, <= 64
  int k;              // scb_captions: lowest scores averaged (0: no baseline)
};
void launch_scst_loss_fwd(const int64_t* seq, const float* lp, int R, int T, const float* sample,
                          const float* greedy, int gdiv, float* reward, float* out, float* loss,
                          int* ws, CstBase cb, hipStream_t stream);
void launch_scst_loss_bwd(const int64_t* seq, const float* reward, const float* out,
                          const float* dloss, int R, int T, float* dlp, hipStream_t stream);
// XE criterion with the loader's caption masks computed from the label rows
// (R x L int64): cnt (R) = counted log-probs per row, out = {loss, sum mask};
// ws as for the SCST loss
void launch_xe_loss_fwd(const int64_t* labels, int L, int off, const float* lp, int R, int T,
                        float* cnt, float* out, float* loss, int* ws, hipStream_t stream);
void launch_xe_loss_bwd(const float* cnt, const float* out, const float* dloss, int R, int T,
                        float* dlp, hipStream_t stream);

// embed_grad.hip
// per-token sums S[v] (bf16, V x C) of the bf16 rows x[srow[i]] (row stride ld)
// over a token sort (ws = its workspace: counts, group ends); S32 (V x C fp32
// scratch) must have been prepared by launch_token_long_zero after the sort
void launch_token_long_zero(const int* ws, int V, int C, float* S32, hipStream_t stream);
void launch_token_group_sum(const uint16_t* x, int C, int64_t ld, const int* stok,
                            const int* srow, int N, const int* ws, int V, uint16_t* S, float* S32,
                            hipStream_t stream);
// Weight-gradient GEMM C = A^T B of K-major bf16 operands (kernels/wgrad.hip):
// A (K x >= M, row stride lda), B (K x >= N, ldb); rows [0, M0) of C go to C0
// (row stride ldc0), rows [M0, M) to C1 (ldc1).  S > 1: split-K through the
// fp32 workspace ws (S x M x N) and a fixed-order reduce.  kts is set by the
// launcher (K-tiles per split).
struct WgradArgs {
  const uint16_t* A;
  int64_t lda;
  const uint16_t* B;
  int64_t ldb;
  int M, N, K, S, kts;
  float* ws;
  float* C0;
  int64_t ldc0;
  int M0;
  float* C1;
  int64_t ldc1;
  // fused weighted column sums (N == 512 only): db[m] = sum_k al[k] A[k][m]
  // (al: K floats; ws_db: S x M floats when S > 1); null: none
  const float* al;
  float* db;
  float* ws_db;
};
bool wgrad_tn_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* A,
                 const void* B);
int wgrad_tn_splits(int64_t M, int64_t N, int64_t K);
void launch_wgrad_tn(WgradArgs g, hipStream_t stream);
// d_vgate (Bv = R / vdiv, G4) fp32 = sum over the n_steps steps and the vdiv
// rows of each video of the bf16 rows dG (row stride ld, first G4 columns)
void launch_video_gate_grad(const uint16_t* dG, int64_t ld, int n_steps, int R, int vdiv, int G4,
                            float* out, hipStream_t stream);
// counting sort of N token ids (< V <= 65536) into (stok, srow); ws: 2V + 1 ints,
// ws[2V] = number of sorted entries (ids outside [0, V) are left out)
void launch_token_sort(const int64_t* toks, int N, int V, int* ws, int* stok, int* srow,
                       hipStream_t stream);

// stamp.hip: device timeline stamps (wall clock, 100 MHz) into a registered
// int64 buffer; no buffer registered = nothing is enqueued
void set_stamp_buffer(int64_t* buf, int slots);
bool stamps_enabled();
void launch_stamp(int slot, hipStream_t stream);
void launch_busy_copy(float* buf, int64_t n_floats, int blocks, double us, hipStream_t stream);
// slots written by the C++ executor, relative to the base the caller set
// (engine.cpp set_stamp_base): forward and backward phases
enum StampSlot : int {
  STAMP_FWD_BEGIN = 0,    // decoder_forward: before the first cell step
  STAMP_FWD_STEP0 = 1,    // after step 0's decode launch + combine
  STAMP_FWD_END = 2,      // after the last combine
  STAMP_BWD_BEGIN = 0,    // decoder_backward, main stream: entry
  STAMP_BWD_ONEHOT = 1,   // side: alpha / one-hot terms folded into E
  STAMP_BWD_DHD0 = 2,     // side: first dHd chunk
  STAMP_BWD_DHD = 3,      // side: all dHd chunks (+ scaled Hd rows)
  STAMP_BWD_LOOP0 = 4,    // main: first reverse step done
  STAMP_BWD_LOOP = 5,     // main: reverse loop done
  STAMP_BWD_DW = 6,       // side: dW_logit GEMM done
  STAMP_BWD_SIDE = 7,     // side: bias column sums + recurrent weight GEMMs done
  STAMP_BWD_TOKSUM = 8,   // main: per-token gate-gradient sums done
  STAMP_BWD_TOKGEMM = 9,  // main: embedding / input-weight GEMMs done
  STAMP_BWD_END = 10,     // main: video / attention gradients done (return)
};

// beam.hip
// the same top-K from the vocab launch's per-tile candidates (flags VF_TOPK)
void launch_beam_topk_cand(const void* cand, int n_vt, int R, int K, const float* lse,
                           float* top_v, int* top_i, hipStream_t stream);
void launch_beam_topk(const float* logits, int64_t ldl, int V, int R, int K, const float* lse,
                      float* top_v, int* top_i, hipStream_t stream);
void launch_beam_step(const float* top_v, const int* top_i, int B, int K, int T, int t,
                      float* beam_sum, int64_t* seq_hist, float* lp_hist, float* best_ppl,
                      int64_t* best_seq, float* best_lp, int64_t* tok_out, int* parent_out,
                      hipStream_t stream);

}  // namespace cst
