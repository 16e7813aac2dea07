// Python bindings of the native extension cst_captioning_amd._C.
#include <torch/extension.h>

#include "host/cider_host.h"
#include "launchers.h"

namespace cst {
std::vector<at::Tensor> decoder_forward(at::Tensor wx, at::Tensor emb, at::Tensor ptab,
                                        at::Tensor whh, at::Tensor wlog,
                                        at::Tensor blog, at::Tensor vgate, int64_t vgate_div,
                                        at::Tensor labels, at::Tensor bos, int64_t R, int64_t T,
                                        std::vector<int64_t> modes, double ss_prob,
                                        double drop_p, double temperature, at::Tensor rng,
                                        bool save, bool want_xe, bool use_counts,
                                        bool use_unfinished, std::vector<at::Tensor> att,
                                        int64_t cell, std::vector<at::Tensor> state0,
                                        std::vector<at::Tensor> up, bool store_exp,
                                        bool xe_rows);
void set_grad_events(bool on);
void grad_event_wait(int64_t k, int64_t stream);
void grad_event_record(int64_t k, int64_t stream);
int64_t grad_event_count(int64_t k);
void set_poll_bound(int64_t n);
void set_bwd_loop(int64_t mode);
void set_att_fuse(bool on);
double lstm_bwd_loop_bench(int64_t R, int64_t H, int64_t T, int64_t iters, at::Tensor phases,
                           int64_t dbg);
int64_t device_errors(int64_t dev_index);
void reset_device_errors(int64_t dev_index);
void gemm_bf16_tuned(at::Tensor out, at::Tensor a, bool ta, at::Tensor b, bool tb,
                     int64_t n_cand);
void gemm_bf16_tuned_batched(at::Tensor out, at::Tensor a, bool ta, at::Tensor b, bool tb,
                             int64_t n_cand);
std::vector<double> gemm_tuned_timings(at::Tensor out, at::Tensor a, bool ta, at::Tensor b,
                                       bool tb);
std::vector<std::vector<double>> gemm_tuned_choices();
std::vector<at::Tensor> decoder_backward(at::Tensor wx, at::Tensor wlog, at::Tensor emb,
                                         at::Tensor lse, at::Tensor logits16,
                                         at::Tensor hdrop_all, at::Tensor gates_all,
                                         at::Tensor c_all, at::Tensor h_all, at::Tensor seq,
                                         at::Tensor labels, at::Tensor toks, at::Tensor dg_sel,
                                         at::Tensor dg_xe, double drop_p, at::Tensor rng,
                                         at::Tensor out_wlog, at::Tensor out_blog,
                                         int64_t comm_stream, std::vector<at::Tensor> att,
                                         at::Tensor out_emb, at::Tensor ds_bias, int64_t cell,
                                         std::vector<at::Tensor> state0,
                                         std::vector<at::Tensor> up, at::Tensor blog,
                                         at::Tensor fix_total, int64_t vgate_div,
                                         at::Tensor xw, std::vector<at::Tensor> vg_bwd,
                                         int64_t vg_nf, double vg_p, int64_t x_wait,
                                         bool exp_zero_off);
std::vector<at::Tensor> beam_search(at::Tensor wx, at::Tensor ptab, at::Tensor whh,
                                    at::Tensor wlog, at::Tensor blog, at::Tensor vgate,
                                    int64_t K, int64_t T, int64_t bos_index,
                                    std::vector<at::Tensor> att, int64_t cell,
                                    std::vector<at::Tensor> state0, std::vector<at::Tensor> up);
double vgrad_colsum_bench(at::Tensor E, at::Tensor alpha, int64_t V, int64_t iters);
double token_sort_bench(at::Tensor toks, int64_t V, int64_t iters);
double att_bench(at::Tensor gv, at::Tensor P, at::Tensor q, at::Tensor wa, at::Tensor ba,
                 int64_t R, int64_t which, int64_t iters);
std::vector<at::Tensor> token_sort(at::Tensor toks, int64_t V);
at::Tensor token_group_sum(at::Tensor x, at::Tensor toks, int64_t V);
std::vector<at::Tensor> cst_loss_forward(at::Tensor seq, at::Tensor lp, at::Tensor scores,
                                         at::Tensor bref, int64_t S, int64_t k);
std::vector<at::Tensor> scst_loss_forward(at::Tensor seq, at::Tensor lp, at::Tensor sample,
                                          at::Tensor greedy);
std::vector<at::Tensor> xe_loss_forward(at::Tensor labels, at::Tensor lp, int64_t off);
at::Tensor xe_loss_backward(at::Tensor cnt, at::Tensor out, at::Tensor dloss, int64_t T);
at::Tensor scst_loss_backward(at::Tensor seq, at::Tensor reward, at::Tensor out,
                              at::Tensor dloss);
at::Tensor featpool_forward(std::vector<at::Tensor> xs, std::vector<at::Tensor> ws,
                            std::vector<at::Tensor> bs, double drop_p, at::Tensor rng);
std::vector<at::Tensor> featpool_backward(at::Tensor dout, at::Tensor out,
                                          std::vector<at::Tensor> xs,
                                          std::vector<at::Tensor> ws, double drop_p,
                                          std::vector<at::Tensor> outs);
std::vector<at::Tensor> att_mfma_fwd(at::Tensor h, at::Tensor wq, at::Tensor P, at::Tensor wa,
                                     at::Tensor ba, at::Tensor gv,
                                     int64_t whole);
std::vector<at::Tensor> decode_step_test(at::Tensor hd, at::Tensor h, at::Tensor wlog,
                                         at::Tensor blog, at::Tensor whh, at::Tensor vgate,
                                         int64_t vdiv, at::Tensor tgt, at::Tensor eoff,
                                         int64_t save, int64_t mode, int64_t step, at::Tensor rng,
                                         at::Tensor ptab, at::Tensor c_prev, double drop_p,
                                         int64_t cell, int64_t eos, at::Tensor unfinished,
                                         double ss_prob);
std::vector<at::Tensor> vocab_select(at::Tensor hd, at::Tensor wlog, at::Tensor blog,
                                     at::Tensor rng, int64_t mode, double temperature,
                                     int64_t step);
double vocab_fwd_bench(at::Tensor hd, at::Tensor wlog, at::Tensor blog, at::Tensor tgt,
                       int64_t flags, bool save, int64_t iters, int64_t variant);
at::Tensor cider_score(at::Tensor hyps, at::Tensor hyp_video, std::map<std::string, at::Tensor> t,
                       double log_ref_len, int64_t use_eos);
at::Tensor flat_adam_step(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v,
                          at::Tensor partials, at::Tensor scal, at::Tensor skip, at::Tensor hyper,
                          double b1, double b2, double eps, double clip, double gscale,
                          int64_t phase, at::Tensor shadow_meta,
                          std::vector<at::Tensor> shadow_dst);
void refresh_shadows(at::Tensor p, at::Tensor shadow_meta, std::vector<at::Tensor> shadow_dst);
void set_stamp_base(int64_t base);
void stamp_buffer(at::Tensor buf);
void stamp_now(int64_t slot);
void busy_copy(at::Tensor buf, int64_t blocks, double us, int64_t stream);
int64_t wall_clock_khz();
void vocab_x(at::Tensor logits16, at::Tensor wlog, at::Tensor out);
at::Tensor att_mfma_phases(at::Tensor gv, at::Tensor P, at::Tensor wa, at::Tensor ba, int64_t R);
at::Tensor wgrad_tn(at::Tensor A, at::Tensor B, int64_t M, int64_t N, int64_t K);
std::vector<at::Tensor> wgrad_tn_colsum(at::Tensor A, at::Tensor B, at::Tensor al, int64_t M,
                                        int64_t N, int64_t K);

template <class T>
static at::Tensor to_tensor(const std::vector<T>& v, at::ScalarType st) {
  at::Tensor t = at::empty({(int64_t)v.size()}, at::TensorOptions().dtype(st));
  if (!v.empty()) std::memcpy(t.data_ptr(), v.data(), v.size() * sizeof(T));
  return t;
}

static std::map<std::string, at::Tensor> cider_build_tables(at::Tensor labels, at::Tensor start,
                                                            at::Tensor end, at::Tensor df_keys,
                                                            at::Tensor df_vals,
                                                            double log_ref_len, int64_t use_eos) {
  TORCH_CHECK(!labels.is_cuda(), "host builder takes CPU tensors");
  labels = labels.contiguous().to(at::kLong);
  start = start.contiguous().to(at::kLong);
  end = end.contiguous().to(at::kLong);
  df_keys = df_keys.contiguous().to(at::kLong);
  df_vals = df_vals.contiguous().to(at::kFloat);
  CiderTables t = build_cider_tables(labels.data_ptr<int64_t>(), (int)labels.size(0),
                                     (int)labels.size(1), start.data_ptr<int64_t>(),
                                     end.data_ptr<int64_t>(), (int)start.numel(),
                                     df_keys.data_ptr<int64_t>(), df_vals.data_ptr<float>(),
                                     (int)df_keys.numel(), log_ref_len, (int)use_eos);
  return {{"ht_keys", to_tensor(t.ht_keys, at::kLong)},
          {"ht_vals", to_tensor(t.ht_vals, at::kFloat)},
          {"vid_ref_off", to_tensor(t.vid_ref_off, at::kInt)},
          {"ref_ng_off", to_tensor(t.ref_ng_off, at::kInt)},
          {"ref_norm", to_tensor(t.ref_norm, at::kFloat)},
          {"ref_len", to_tensor(t.ref_len, at::kInt)},
          {"ng_key", to_tensor(t.ng_key, at::kLong)},
          {"ng_val", to_tensor(t.ng_val, at::kFloat)}};
}

static at::Tensor cider_score_cpu(at::Tensor hyps, at::Tensor hyp_video,
                                  std::map<std::string, at::Tensor> t, double log_ref_len,
                                  int64_t use_eos) {
  hyps = hyps.contiguous().to(at::kLong);
  hyp_video = hyp_video.contiguous().to(at::kLong);
  CiderTablesView v{(uint32_t)t["ht_keys"].numel(), t["ht_keys"].data_ptr<int64_t>(),
                    t["ht_vals"].data_ptr<float>(), t["vid_ref_off"].data_ptr<int32_t>(),
                    t["ref_ng_off"].data_ptr<int32_t>(), t["ref_norm"].data_ptr<float>(),
                    t["ref_len"].data_ptr<int32_t>(), t["ng_key"].data_ptr<int64_t>(),
                    t["ng_val"].data_ptr<float>()};
  at::Tensor out = at::empty({hyps.size(0)}, at::TensorOptions().dtype(at::kFloat));
  cider_score_host(hyps.data_ptr<int64_t>(), (int)hyps.size(0), (int)hyps.size(1),
                   hyp_video.data_ptr<int64_t>(), v, log_ref_len, (int)use_eos,
                   out.data_ptr<float>());
  return out;
}
}  // namespace cst

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "cst_captioning_amd native extension: gfx950 HIP kernels + C++ decoder executor";
  m.def("decoder_forward", &cst::decoder_forward);
  m.def("decoder_backward", &cst::decoder_backward, py::arg("wx"), py::arg("wlog"), py::arg("emb"),
        py::arg("lse"), py::arg("logits16"), py::arg("hdrop_all"), py::arg("gates_all"),
        py::arg("c_all"), py::arg("h_all"), py::arg("seq"), py::arg("labels"), py::arg("toks"),
        py::arg("dg_sel"), py::arg("dg_xe"), py::arg("drop_p"), py::arg("rng"),
        py::arg("out_wlog"), py::arg("out_blog"), py::arg("comm_stream"), py::arg("att"),
        py::arg("out_emb"), py::arg("ds_bias"), py::arg("cell"), py::arg("state0"), py::arg("up"),
        py::arg("blog"), py::arg("fix_total"), py::arg("vgate_div"), py::arg("xw"),
        py::arg("vg_bwd"), py::arg("vg_nf"), py::arg("vg_p"), py::arg("x_wait") = 0,
        py::arg("exp_zero_off") = false);
  m.def("cider_build_tables", &cst::cider_build_tables);
  m.def("cider_score", &cst::cider_score);
  m.def("cider_score_cpu", &cst::cider_score_cpu);
  m.def("flat_adam_step", &cst::flat_adam_step);
  m.def("refresh_shadows", &cst::refresh_shadows);
  m.def("vocab_fwd_bench", &cst::vocab_fwd_bench);
  m.def("vgrad_colsum_bench", &cst::vgrad_colsum_bench);
  m.def("token_sort_bench", &cst::token_sort_bench);
  m.def("att_bench", &cst::att_bench);
  m.def("token_sort", &cst::token_sort);
  m.def("token_group_sum", &cst::token_group_sum);
  m.def("vocab_select", &cst::vocab_select);
  m.def("decode_step_test", &cst::decode_step_test);
  m.def("gemm_bf16_tuned", &cst::gemm_bf16_tuned, py::arg("out"), py::arg("a"), py::arg("ta"),
        py::arg("b"), py::arg("tb"), py::arg("n_cand") = 24);
  m.def("gemm_bf16_tuned_batched", &cst::gemm_bf16_tuned_batched, py::arg("out"), py::arg("a"),
        py::arg("ta"), py::arg("b"), py::arg("tb"), py::arg("n_cand") = 24);
  m.def("gemm_tuned_timings", &cst::gemm_tuned_timings);
  m.def("gemm_tuned_choices", &cst::gemm_tuned_choices);
  m.def("set_grad_events", &cst::set_grad_events);
  m.def("grad_event_wait", &cst::grad_event_wait);
  m.def("grad_event_record", &cst::grad_event_record);
  m.def("grad_event_count", &cst::grad_event_count);
  m.def("set_poll_bound", &cst::set_poll_bound,
        "polls of a bounded cross-workgroup wait before it gives up (tests: 0)");
  m.def("set_bwd_loop", &cst::set_bwd_loop,
        "reverse LSTM loop: 1 one persistent launch, row-read form (default); 2 persistent, "
        "K-split team GEMM; 0 one launch per step");
  m.def("lstm_bwd_loop_bench", &cst::lstm_bwd_loop_bench, py::arg("R"), py::arg("H"), py::arg("T"),
        py::arg("iters"), py::arg("phases"), py::arg("dbg") = 0,
        "persistent reverse loop alone on random operands: us per launch (+ phase stamps)");
  m.def("set_att_fuse", &cst::set_att_fuse,
        "attention backward fused into the reverse step (true, default) or a launch per step");
  m.def("device_errors", &cst::device_errors,
        "failed cross-workgroup hand-offs counted on the device (synchronous read)");
  m.def("reset_device_errors", &cst::reset_device_errors);
  m.def("att_mfma_fwd", &cst::att_mfma_fwd, py::arg("h"), py::arg("wq"), py::arg("P"),
        py::arg("wa"), py::arg("ba"), py::arg("gv"), py::arg("whole") = -1);
  m.def("beam_search", &cst::beam_search);
  m.def("featpool_forward", &cst::featpool_forward);
  m.def("scst_loss_forward", &cst::scst_loss_forward);
  m.def("cst_loss_forward", &cst::cst_loss_forward);
  m.def("scst_loss_backward", &cst::scst_loss_backward);
  m.def("xe_loss_forward", &cst::xe_loss_forward);
  m.def("xe_loss_backward", &cst::xe_loss_backward);
  m.def("featpool_backward", &cst::featpool_backward);
  m.def("set_stamp_base", &cst::set_stamp_base);
  m.def("stamp_buffer", &cst::stamp_buffer);
  m.def("stamp_now", &cst::stamp_now);
  m.def("busy_copy", &cst::busy_copy,
        "stand-in for a collective's kernel: copying workgroups for a given time");
  m.def("wall_clock_khz", &cst::wall_clock_khz);
  m.def("vocab_x", &cst::vocab_x);
  m.def("att_mfma_phases", &cst::att_mfma_phases);
  m.def("wgrad_tn", &cst::wgrad_tn);
  m.def("wgrad_tn_colsum", &cst::wgrad_tn_colsum);
}
