// Decoder executor: the time loops of the caption decoder in C++.
//
// The reference runs its time loops in Python (model.py:234-289 forward,
// 319-367 sample), one ATen/cuDNN call at a time, with a device->host sync per
// step (`it.sum() == 0`, model.py:269) and multinomial sampling on the CPU
// (model.py:331-337).  Here each step is three async launches -- fused LSTM
// step, fused vocab projection + statistics, row combine -- enqueued on the
// current HIP stream from C++; the end-of-sequence rules are evaluated on
// the device, so a whole rollout is enqueued without a single host sync (and
// is capturable in a HIP graph).
//
// decoder_forward : teacher forcing / scheduled sampling / MIXER rollout /
//                   greedy or multinomial sample(), optionally saving what the
//                   backward needs (fp16 logits, dropped h, gates, c, [x;h]).
// decoder_backward: batched vocab-head backward (dS in place, two
//                   hipBLASLt GEMMs over all T*R rows at once), then the
//                   reverse LSTM recurrence (cell kernel + one GEMM per step),
//                   then the batched weight-gradient GEMMs.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include "launchers.h"

namespace cst {

static hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// h_drop rows may carry HAUG extra columns [1, 0, ...] (written by the LSTM
// kernel) so that one GEMM dS^T [h | 1] also yields the bias gradient.  The
// MI355X measurement (hipBLASLt at N=528 vs 512) made the dS kernel's
// column-sum partials the faster route, so HAUG = 0.
constexpr int64_t HAUG = 0;

template <class T>
static T* ptr_or_null(const at::Tensor& t) {
  return t.defined() && t.numel() > 0 ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}

static void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// modes[t] = token-selection mode for token t+1 (see SelModeHost)
std::vector<at::Tensor> decoder_forward(at::Tensor wx, at::Tensor emb, at::Tensor ptab,
                                        at::Tensor whh, at::Tensor wlog,
                                        at::Tensor blog, at::Tensor vgate, int64_t vgate_div,
                                        at::Tensor labels, at::Tensor bos, int64_t R, int64_t T,
                                        std::vector<int64_t> modes, double ss_prob,
                                        double drop_p, double temperature, int64_t seed,
                                        bool save, bool want_xe, bool use_counts,
                                        bool use_unfinished) {
  check_cuda(wx, "wx");
  check_cuda(emb, "emb");
  check_cuda(wlog, "wlog");
  check_cuda(blog, "blog");
  check_cuda(vgate, "vgate");
  TORCH_CHECK(wx.scalar_type() == at::kBFloat16 && emb.scalar_type() == at::kBFloat16 &&
                  wlog.scalar_type() == at::kBFloat16,
              "decoder weights must be bf16");
  TORCH_CHECK(vgate.scalar_type() == at::kFloat, "vgate must be fp32");
  check_cuda(ptab, "ptab");
  check_cuda(whh, "whh");
  TORCH_CHECK(ptab.scalar_type() == at::kFloat && ptab.size(0) == emb.size(0) &&
                  ptab.size(1) == wx.size(0), "ptab must be fp32 (V, 4H)");
  TORCH_CHECK(whh.scalar_type() == at::kBFloat16 && whh.size(0) == wx.size(0) &&
                  whh.size(1) * 4 == wx.size(0), "whh must be bf16 (4H, H)");
  const int64_t H4 = wx.size(0), H = H4 / 4, E = emb.size(1), V = wlog.size(0);
  TORCH_CHECK(wx.size(1) == E + H, "wx must be (4H, E+H)");
  TORCH_CHECK(E % 64 == 0 && H % 64 == 0, "E and H must be multiples of 64");
  TORCH_CHECK(wlog.size(1) == H && blog.numel() == V, "logit weight shape");
  TORCH_CHECK(vgate.size(1) == H4 && vgate.size(0) * vgate_div >= R, "vgate shape");
  TORCH_CHECK(T >= 2 && (int64_t)modes.size() >= T - 1, "modes must cover T-1 steps");
  const bool have_labels = labels.defined() && labels.numel() > 0;
  int64_t L = 0;
  if (have_labels) {
    check_cuda(labels, "labels");
    TORCH_CHECK(labels.scalar_type() == at::kLong && labels.size(0) == R, "labels (R, L) int64");
    L = labels.size(1);
    TORCH_CHECK(L >= T + (want_xe ? 1 : 0), "labels too short for T steps");
  } else {
    TORCH_CHECK(!want_xe, "want_xe needs labels");
    check_cuda(bos, "bos");
  }
  const int64_t n_steps = want_xe ? T : T - 1;  // LSTM steps actually needed
  auto dev = wx.device();
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
  auto bf = at::TensorOptions().dtype(at::kBFloat16).device(dev);
  auto i64 = at::TensorOptions().dtype(at::kLong).device(dev);
  hipStream_t st = cur_stream();

  at::Tensor seq = at::zeros({R, T - 1}, i64);
  at::Tensor g_sel = at::zeros({R, T - 1}, f32);
  at::Tensor g_xe = want_xe ? at::zeros({R, T}, f32) : at::Tensor();
  at::Tensor lse = at::empty({n_steps, R}, f32);
  const int n_vt = vocab_num_tiles((int)V);
  at::Tensor part = at::empty({(int64_t)n_vt * R * vocab_partial_bytes() / 4}, f32);
  at::Tensor counts = at::zeros({T + 1}, at::TensorOptions().dtype(at::kInt).device(dev));
  at::Tensor unfinished =
      use_unfinished ? at::ones({R}, at::TensorOptions().dtype(at::kByte).device(dev))
                     : at::Tensor();
  const int64_t ldl = (V + 7) / 8 * 8;
  at::Tensor logits16, hdrop_all, gates_all, c_all, h_all;
  if (save) {
    logits16 = at::empty({n_steps, R, ldl}, at::TensorOptions().dtype(at::kHalf).device(dev));
    hdrop_all = at::empty({n_steps, R, H + HAUG}, bf);  // [h_drop | 1 | 0...]
    gates_all = at::empty({n_steps, R, H4}, bf);
    c_all = at::empty({n_steps, R, H}, f32);
    h_all = at::empty({n_steps, R, H}, bf);
  }
  at::Tensor h_a = at::zeros({R, H}, bf), h_b = at::empty({R, H}, bf);
  at::Tensor c_a = at::zeros({R, H}, f32), c_b = at::empty({R, H}, f32);
  at::Tensor hd_tmp = (!save && drop_p > 0) ? at::empty({R, H + HAUG}, bf) : at::Tensor();

  const uint32_t seed_drop = (uint32_t)(seed * 2654435761u + 17u);
  const uint32_t seed_samp = (uint32_t)(seed * 40503u + 0x9E37u);
  const float inv_temp = (float)(1.0 / temperature);
  const uint16_t* W = reinterpret_cast<const uint16_t*>(wlog.data_ptr());
  const uint16_t* WHH = reinterpret_cast<const uint16_t*>(whh.data_ptr());
  const int64_t* LAB = have_labels ? labels.data_ptr<int64_t>() : nullptr;

  for (int64_t t = 0; t < n_steps; ++t) {
    const int64_t* tok;
    int64_t tok_stride;
    if (t == 0) {
      tok = have_labels ? LAB : bos.data_ptr<int64_t>();
      tok_stride = have_labels ? L : 1;
    } else {
      tok = seq.data_ptr<int64_t>() + (t - 1);
      tok_stride = T - 1;
    }
    uint16_t* h_prev;
    uint16_t* h_out;
    if (save) {
      h_prev = reinterpret_cast<uint16_t*>(t == 0 ? h_a.data_ptr() : h_all[t - 1].data_ptr());
      h_out = reinterpret_cast<uint16_t*>(h_all[t].data_ptr());
    } else {
      h_prev = reinterpret_cast<uint16_t*>((t & 1 ? h_b : h_a).data_ptr());
      h_out = reinterpret_cast<uint16_t*>((t & 1 ? h_a : h_b).data_ptr());
    }
    const float* c_prev;
    float* c_out;
    if (save) {
      c_prev = t == 0 ? c_a.data_ptr<float>() : c_all[t - 1].data_ptr<float>();
      c_out = c_all[t].data_ptr<float>();
    } else {
      c_prev = (t & 1 ? c_b : c_a).data_ptr<float>();
      c_out = (t & 1 ? c_a : c_b).data_ptr<float>();
    }
    uint16_t* hd = nullptr;
    if (save) hd = reinterpret_cast<uint16_t*>(hdrop_all[t].data_ptr());
    else if (drop_p > 0) hd = reinterpret_cast<uint16_t*>(hd_tmp.data_ptr());
    launch_lstm_step_fwd(tok, tok_stride, ptab.data_ptr<float>(), h_prev, c_prev,
                         vgate.data_ptr<float>(), (int)vgate_div, (int)R, (int)H, WHH, h_out,
                         c_out, hd, (int)(H + HAUG), (float)drop_p, seed_drop, (int)t,
                         save ? reinterpret_cast<uint16_t*>(gates_all[t].data_ptr()) : nullptr,
                         st);
    const uint16_t* vin = hd ? hd : h_out;
    const int ldh = hd ? (int)(H + HAUG) : (int)H;
    const bool choose = t < T - 1;
    const int mode = choose ? (int)modes[t] : SEL_GT_H;
    const int do_sample = choose && (mode == SEL_SAMPLE_H || mode == SEL_SS_H);
    const int vflags = do_sample | ((choose && mode == SEL_GREEDY_H) ? 2 : 0);
    const int64_t* tgt = (have_labels && t + 1 < L) ? LAB + (t + 1) : nullptr;
    launch_vocab_fwd(vin, ldh, (int)R, (int)H, W, blog.data_ptr<float>(), (int)V,
                     save ? reinterpret_cast<uint16_t*>(logits16[t].data_ptr()) : nullptr, ldl,
                     part.data_ptr(), tgt, L, vflags, inv_temp, seed_samp, (int)t, st);
    launch_vocab_combine(part.data_ptr(), n_vt, (int)R, lse[t].data_ptr<float>(),
                         choose ? seq.data_ptr<int64_t>() + t : nullptr, T - 1,
                         choose ? g_sel.data_ptr<float>() + t : nullptr, T - 1,
                         want_xe ? g_xe.data_ptr<float>() + t : nullptr, T, tgt, L, mode,
                         (float)ss_prob, seed_samp, (int)t,
                         use_counts ? counts.data_ptr<int>() : nullptr, (int)(t + 1),
                         use_unfinished ? unfinished.data_ptr<uint8_t>() : nullptr, st);
  }
  std::vector<at::Tensor> out = {seq, g_sel, want_xe ? g_xe : at::Tensor(), lse};
  if (save) {
    out.push_back(logits16);
    out.push_back(hdrop_all);
    out.push_back(gates_all);
    out.push_back(c_all);
    out.push_back(h_all);
  }
  return out;
}

// Returns {dWx_packed (4H, E+H), dWlog (V, H), dblog (V), dX (n_steps*R, E), dvg_rows (R, 4H)}.
// toks: (n_steps*R) input token of every (step, row), step-major.
std::vector<at::Tensor> decoder_backward(at::Tensor wx, at::Tensor wlog, at::Tensor emb,
                                         at::Tensor lse, at::Tensor logits16,
                                         at::Tensor hdrop_all, at::Tensor gates_all,
                                         at::Tensor c_all, at::Tensor h_all, at::Tensor seq,
                                         at::Tensor labels, at::Tensor toks, at::Tensor dg_sel,
                                         at::Tensor dg_xe, double drop_p, int64_t seed) {
  const int64_t n_steps = logits16.size(0), R = logits16.size(1), ldl = logits16.size(2);
  const int64_t H4 = wx.size(0), H = H4 / 4, E = wx.size(1) - H, V = wlog.size(0);
  const int64_t T_sel = seq.size(1);
  hipStream_t st = cur_stream();
  auto dev = wx.device();
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
  const bool has_sel = dg_sel.defined() && dg_sel.numel() > 0;
  const bool has_xe = dg_xe.defined() && dg_xe.numel() > 0;
  if (has_sel) TORCH_CHECK(dg_sel.is_contiguous() && dg_sel.size(1) == T_sel, "dg_sel shape");
  if (has_xe) TORCH_CHECK(dg_xe.is_contiguous() && labels.defined(), "dg_xe needs labels");
  TORCH_CHECK(toks.numel() == n_steps * R, "toks must hold one token per (step, row)");
  const uint32_t seed_drop = (uint32_t)(seed * 2654435761u + 17u);

  // 1. dS = dG (onehot - softmax), in place (fp16 logits -> bf16 dS), plus
  //    per-block column sums of dS (bias gradient)
  TORCH_CHECK(V <= 8 * 2048, "vocab larger than the dS kernel's register tiling");
  at::Tensor colsum = at::empty({vocab_bwd_ds_blocks((int)n_steps, (int)R), V}, f32);
  launch_vocab_bwd_ds(reinterpret_cast<uint16_t*>(logits16.data_ptr()), ldl, (int)V, (int)R,
                      (int)n_steps, (int)T_sel, lse.data_ptr<float>(),
                      has_sel ? seq.data_ptr<int64_t>() : nullptr, T_sel,
                      has_sel ? dg_sel.data_ptr<float>() : nullptr, T_sel,
                      has_xe ? labels.data_ptr<int64_t>() + 1 : nullptr,
                      has_xe ? labels.size(1) : 0, has_xe ? dg_xe.data_ptr<float>() : nullptr,
                      has_xe ? dg_xe.size(1) : 0, colsum.data_ptr<float>(), st);
  at::Tensor dS = logits16.view(at::kBFloat16).view({n_steps * R, ldl}).narrow(1, 0, V);
  // 2. batched vocab-head GEMMs over all n_steps*R rows (hipBLASLt)
  at::Tensor dHd = at::mm(dS, wlog, at::kFloat);                        // (n*R, H)
  at::Tensor hd2 = hdrop_all.view({n_steps * R, H + HAUG}).narrow(1, 0, H);
  at::Tensor dWlog = at::mm(dS.t(), hd2, at::kFloat);                   // (V, H)
  at::Tensor dblog = colsum.sum(0);                                     // (V)
  // 3. reverse recurrence
  at::Tensor dG_all = at::empty({n_steps, R, H4}, wx.options());
  at::Tensor dc = at::zeros({R, H}, f32);
  at::Tensor whh = wx.narrow(1, E, H);  // (4H, H) packed rows, strided view
  at::Tensor dh_rec;
  for (int64_t t = n_steps - 1; t >= 0; --t) {
    launch_lstm_cell_bwd(dHd.data_ptr<float>() + t * R * H,
                         dh_rec.defined() ? dh_rec.data_ptr<float>() : nullptr,
                         dc.data_ptr<float>(),
                         reinterpret_cast<const uint16_t*>(gates_all[t].data_ptr()),
                         c_all[t].data_ptr<float>(),
                         t > 0 ? c_all[t - 1].data_ptr<float>() : nullptr, (int)R, (int)H,
                         (float)drop_p, seed_drop, (int)t,
                         reinterpret_cast<uint16_t*>(dG_all[t].data_ptr()), st);
    if (t > 0) dh_rec = at::mm(dG_all[t], whh, at::kFloat);  // (R, H)
  }
  // 4. batched weight gradients: dWx = dG^T [x ; h_prev] as two GEMMs
  at::Tensor dG2 = dG_all.view({n_steps * R, H4});
  at::Tensor x_in = emb.index_select(0, toks);                            // (n*R, E) bf16
  at::Tensor dWx = at::empty({H4, E + H}, f32);
  dWx.narrow(1, 0, E).copy_(at::mm(dG2.t(), x_in, at::kFloat));
  if (n_steps > 1) {
    at::Tensor hprev = h_all.narrow(0, 0, n_steps - 1).reshape({(n_steps - 1) * R, H});
    dWx.narrow(1, E, H).copy_(at::mm(dG2.narrow(0, R, (n_steps - 1) * R).t(), hprev, at::kFloat));
  } else {
    dWx.narrow(1, E, H).zero_();
  }
  at::Tensor dX = at::mm(dG2, wx.narrow(1, 0, E), at::kFloat);        // (n*R, E)
  at::Tensor dvg = dG_all.sum(0, false, at::kFloat);                   // (R, 4H), sum over time
  return {dWx, dWlog, dblog, dX, dvg};
}

// On-GPU CIDEr-D scores of N hypotheses.
at::Tensor cider_score(at::Tensor hyps, at::Tensor hyp_video, std::map<std::string, at::Tensor> t,
                       double log_ref_len, int64_t use_eos) {
  check_cuda(hyps, "hyps");
  check_cuda(hyp_video, "hyp_video");
  TORCH_CHECK(hyps.scalar_type() == at::kLong && hyp_video.scalar_type() == at::kLong,
              "int64 inputs");
  const int64_t N = hyps.size(0), T = hyps.size(1);
  TORCH_CHECK(T <= 63, "hypotheses longer than 63 tokens are not supported");
  at::Tensor out = at::empty({N}, hyps.options().dtype(at::kFloat));
  launch_cider_d(hyps.data_ptr<int64_t>(), (int)T, hyp_video.data_ptr<int64_t>(), (int)N,
                 t["ht_keys"].data_ptr<int64_t>(), t["ht_vals"].data_ptr<float>(),
                 (uint32_t)t["ht_keys"].numel(), t["vid_ref_off"].data_ptr<int32_t>(),
                 t["ref_ng_off"].data_ptr<int32_t>(), t["ref_norm"].data_ptr<float>(),
                 t["ref_len"].data_ptr<int32_t>(), t["ng_key"].data_ptr<int64_t>(),
                 t["ng_val"].data_ptr<float>(), (float)log_ref_len, (int)use_eos, out.data_ptr<float>(),
                 cur_stream());
  return out;
}

at::Tensor flat_adam_step(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v,
                          at::Tensor partials, at::Tensor scal, at::Tensor skip, double lr,
                          double b1, double b2, double eps, double clip, double bc1, double bc2) {
  check_cuda(p, "p");
  TORCH_CHECK(partials.numel() >= 1024 && scal.numel() >= 2, "workspace too small");
  launch_flat_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                   v.data_ptr<float>(), p.numel(), partials.data_ptr<float>(),
                   skip.data_ptr<bool>(), scal.data_ptr<float>(), (float)lr, (float)b1,
                   (float)b2, (float)eps, (float)clip, (float)bc1, (float)bc2, cur_stream());
  return scal.narrow(0, 0, 1).squeeze(0);
}

}  // namespace cst
