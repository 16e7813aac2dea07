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
//                   backward needs (the exp store E = exp(logit - previous
//                   LSE) in bf16, dropped h, gates, c, [x;h]).
// decoder_backward: batched vocab-head backward without forming dS (two
//                   hipBLASLt GEMMs over all T*R rows of E at once, row scales
//                   and one-hot terms in kernels/vocab_grad.hip), then the
//                   reverse LSTM recurrence (one fused kernel per step), then
//                   the weight-gradient GEMMs (input-token ones over per-token
//                   sums, V rows instead of T*R).
#include <torch/extension.h>
#include <array>
#include <cstdlib>
#include <cstring>
#include <map>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include "launchers.h"

namespace cst {

static hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// Device timeline stamps (kernels/stamp.hip): the caller picks the base slot
// of the next decoder_forward / decoder_backward call (sample and greedy
// decodes of one step use different bases); -1 = no stamps from the executor.
static int g_stamp_base = -1;
void set_stamp_base(int64_t base) { g_stamp_base = (int)base; }
static void stamp(int rel, hipStream_t s) {
  if (g_stamp_base >= 0) launch_stamp(g_stamp_base + rel, s);
}
void stamp_buffer(at::Tensor buf) {
  if (!buf.defined() || buf.numel() == 0) {
    set_stamp_buffer(nullptr, 0);
    return;
  }
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kLong && buf.is_contiguous(),
              "stamp buffer must be a contiguous int64 GPU tensor");
  set_stamp_buffer(buf.data_ptr<int64_t>(), (int)buf.numel());
}
void stamp_now(int64_t slot) { launch_stamp((int)slot, cur_stream()); }

void gemm_bf16_tuned(at::Tensor out, at::Tensor a, bool ta, at::Tensor b, bool tb,
                     int64_t n_cand);
void gemm_bf16_tuned_batched(at::Tensor out, at::Tensor a, bool ta, at::Tensor b, bool tb,
                             int64_t n_cand);

// X = E W of a training forward's exp store (n, R, ldl) bf16 -> out (n, R, H)
// fp32, on the current stream (engine.launch_x; the same GEMM as the
// backward's dHd chunks), through hipBLASLt's measured algorithm choice
// (host/blaslt_tuned.cpp: the heuristic's 32 candidates timed once on an idle
// device, or pinned by CSTCAP_BLASLT_ALGO): interleaved A/B 3.503-3.505 vs
// 3.562-3.574 ms per step against PyTorch's first choice, profiles/r4.
// (A 3-way split-K batch measured slower: 3.74 vs 3.67-3.73 ms per step,
// profiles/r3/ab_xsplitk.txt; the round-4 hand-written persistent GEMM was
// correct but slower in the step, 3.80 vs 3.68 ms, and was removed.)
void vocab_x(at::Tensor logits16, at::Tensor wlog, at::Tensor out) {
  TORCH_CHECK(logits16.is_cuda() && logits16.scalar_type() == at::kBFloat16 &&
                  logits16.dim() == 3 && logits16.is_contiguous(),
              "vocab_x: exp store must be a contiguous bf16 (n, R, ldl) GPU tensor");
  const int64_t NR = logits16.size(0) * logits16.size(1), V = wlog.size(0), H = wlog.size(1);
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == at::kFloat && out.numel() == NR * H &&
                  logits16.size(2) >= V,
              "vocab_x: out must be a contiguous fp32 (n, R, H) tensor");
  const int64_t ldl = logits16.size(2);
  gemm_bf16_tuned(out.view({NR, H}), logits16.view({NR, ldl}).narrow(1, 0, V), false, wlog, false,
                  32);
}
int64_t wall_clock_khz() {
  int dev = 0, khz = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  return khz;
}

template <class T>
static T* ptr_or_null(const at::Tensor& t) {
  return t.defined() && t.numel() > 0 ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}

static void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
// stand-in for a collective's kernel on `stream` (0: the current stream):
// `blocks` copying workgroups for `us` microseconds over `buf` (fp32 scratch)
void busy_copy(at::Tensor buf, int64_t blocks, double us, int64_t stream) {
  check_cuda(buf, "buf");
  TORCH_CHECK(buf.scalar_type() == at::kFloat && buf.is_contiguous(), "busy_copy: fp32 scratch");
  launch_busy_copy(buf.data_ptr<float>(), buf.numel(), (int)blocks, us,
                   stream != 0 ? reinterpret_cast<hipStream_t>(stream) : cur_stream());
}

// rng: int32[2] device tensor {dropout seed, sampling seed} (or undefined /
// empty: seeds 0).  Kernels read it from device memory, so a captured HIP
// graph draws fresh masks and samples on every replay.
static const uint32_t* rng_ptr(const at::Tensor& rng) {
  if (!rng.defined() || rng.numel() == 0) return nullptr;
  TORCH_CHECK(rng.is_cuda() && rng.scalar_type() == at::kInt && rng.numel() >= 2 &&
                  rng.is_contiguous(),
              "rng must be a contiguous int32[2] GPU tensor");
  return reinterpret_cast<const uint32_t*>(rng.data_ptr());
}

// Events and side streams are created once per device and reused: nothing
// is created or destroyed while a HIP graph is being captured.
constexpr int MAX_DHD_CHUNKS = 32;  // per-chunk events of the vocab-head dHd GEMM
constexpr int XE_MAX_STEPS = 64;  // XE all rows: decode steps per forward
struct DeviceAux {
  std::vector<hipEvent_t> ev;
  c10::hip::HIPStream side[2];
  hipEvent_t grad_ev[3];  // data parallelism: gradient groups final (set_grad_events)
  hipEvent_t fwd_ev[2];   // decoder_forward: step 0's exp-store conversion fork / join
};
static DeviceAux& device_aux(int dev_index) {
  static std::map<int, DeviceAux*> aux;
  auto it = aux.find(dev_index);
  if (it == aux.end()) {
    auto* a = new DeviceAux{{}, {c10::hip::getStreamFromPool(false, dev_index),
                                 c10::hip::getStreamFromPool(false, dev_index)}};
    a->ev.resize(7 + MAX_DHD_CHUNKS);  // (the last: decoder_backward's pre-X point)
    for (auto& e : a->ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    for (auto& e : a->grad_ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    for (auto& e : a->fwd_ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    it = aux.emplace(dev_index, a).first;
  }
  return *it->second;
}

// Device error word (one int32 per device, zero until a kernel reports a
// failed cross-workgroup hand-off): a bounded flag poll that runs out of polls
// (lstm.hip att_fuse_wait) adds 1 instead of silently reading operands that
// may not be written yet.  The trainer reads it at log time and raises; the
// bench reports it.  set_poll_bound(0) forces every such wait to give up
// (tests of the counter).
static int g_poll_bound = 1 << 20;
static int* device_err_word(int dev_index) {
  static std::map<int, int*> words;
  auto it = words.find(dev_index);
  if (it == words.end()) {
    int* p = nullptr;
    c10::hip::HIPGuard guard(dev_index);
    TORCH_CHECK(hipMalloc(&p, sizeof(int)) == hipSuccess, "device error word: hipMalloc");
    TORCH_CHECK(hipMemset(p, 0, sizeof(int)) == hipSuccess, "device error word: hipMemset");
    it = words.emplace(dev_index, p).first;
  }
  return it->second;
}
// persistent reverse loop on (default; CSTCAP_BWD_LOOP=0 or set_bwd_loop(false):
// one launch per step)
// (CSTCAP_BWD_LOOP=1: the persistent form whose workgroups read their rows'
// whole dG_{t+1} -- the default; 2: the K-split form that exchanges fp32
// partials instead, measured slower: 361.8 vs 331.6 us per loop alone,
// 3.359-3.371 vs 3.338-3.345 ms per step, profiles/r6/README_r6.md)
static int g_bwd_loop = [] {
  const char* e = getenv("CSTCAP_BWD_LOOP");
  return e == nullptr ? 1 : atoi(e);
}();
void set_bwd_loop(int64_t mode) { g_bwd_loop = (int)mode; }
// fused attention backward (lstm.hip att_bwd_fused_wg, the fp16 scorer values
// of the forward) on; off: the separate att_bwd_mfma launch per step, which
// recomputes tanh(P + q) in fp32 (tests of the fp16 encoding)
static bool g_att_fuse = true;
void set_att_fuse(bool on) { g_att_fuse = on; }
// exchange slabs of the K-split persistent loop, per device (grown on demand
// outside graph capture)
static float* loop_xb(int dev_index, int64_t floats) {
  static std::map<int, std::pair<float*, int64_t>> bufs;
  auto it = bufs.find(dev_index);
  if (it != bufs.end() && it->second.second >= floats) return it->second.first;
  c10::hip::HIPGuard guard(dev_index);
  if (it != bufs.end()) {
    (void)hipDeviceSynchronize();
    (void)hipFree(it->second.first);
    bufs.erase(it);
  }
  float* p = nullptr;
  TORCH_CHECK(hipMalloc(&p, sizeof(float) * floats) == hipSuccess, "loop exchange slabs: hipMalloc");
  bufs.emplace(dev_index, std::make_pair(p, floats));
  return p;
}
void set_poll_bound(int64_t n) { g_poll_bound = (int)std::max<int64_t>(0, n); }
// team counters of the persistent reverse loop (lstm_loop.hip), per device;
// the launcher zeroes the used prefix before every launch
static int* loop_counters(int dev_index, int ints) {
  static std::map<int, std::pair<int*, int>> bufs;
  auto it = bufs.find(dev_index);
  if (it == bufs.end() || it->second.second < ints) {
    TORCH_CHECK(it == bufs.end(), "persistent reverse loop: counter block too small");
    int* p = nullptr;
    c10::hip::HIPGuard guard(dev_index);
    const int n = std::max(ints, 4096);
    TORCH_CHECK(hipMalloc(&p, sizeof(int) * n) == hipSuccess, "loop counters: hipMalloc");
    TORCH_CHECK(hipMemset(p, 0, sizeof(int) * n) == hipSuccess, "loop counters: hipMemset");
    it = bufs.emplace(dev_index, std::make_pair(p, n)).first;
  }
  return it->second.first;
}
int64_t device_errors(int64_t dev_index) {
  int* p = device_err_word((int)dev_index);
  int v = 0;
  c10::hip::HIPGuard guard((int)dev_index);
  TORCH_CHECK(hipMemcpy(&v, p, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess,
              "device error word: read");
  return v;
}
void reset_device_errors(int64_t dev_index) {
  int* p = device_err_word((int)dev_index);
  c10::hip::HIPGuard guard((int)dev_index);
  TORCH_CHECK(hipMemset(p, 0, sizeof(int)) == hipSuccess, "device error word: reset");
}

// Data parallelism, communication overlapped with the backward: with
// set_grad_events(true) decoder_backward records grad_ev[0] once the vocab
// head's gradients (logit W, b) are final (side stream, after dW_logit, which
// then runs under the reverse loop) and grad_ev[1] once the embedding
// gradient is (main stream, after its GEMM).  Inside a graph capture they are
// event-record NODES of the captured graph (record_grad_event), so after each replay
// the trainer's comm stream waits on them (grad_event_wait) and all-reduces
// those bucket slices while the rest of the replayed backward still runs --
// eager RCCL between replays, no collective inside the graph.
static bool g_grad_events_on = false;
void set_grad_events(bool on) { g_grad_events_on = on; }
// host-side count of record calls per group (inline records and captured
// record nodes): the trainer checks that a step (or the capture of one)
// recorded both events before its comm stream relies on them -- a wait on an
// event this step never recorded would order nothing
static int64_t g_grad_ev_count[3] = {0, 0, 0};
int64_t grad_event_count(int64_t k) {
  TORCH_CHECK(k >= 0 && k < 3, "grad_event_count: group 0, 1 or 2");
  return g_grad_ev_count[k];
}
static void record_grad_event(hipEvent_t ev, hipStream_t s, int k) {
  g_grad_ev_count[k]++;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  unsigned long long id = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(s, &cs, &id, &graph, &deps, &nd);
  TORCH_CHECK(e == hipSuccess, "grad event: capture info: ", hipGetErrorString(e));
  if (cs != hipStreamCaptureStatusActive) {
    e = hipEventRecord(ev, s);
    TORCH_CHECK(e == hipSuccess, "grad event: record: ", hipGetErrorString(e));
    return;
  }
  // an event-record node of the graph being captured, after the stream's
  // current dependencies; the stream's later work then follows the node
  // (hipEventRecordWithFlags(hipEventRecordExternal) failed with "invalid
  // argument" inside a capture on this ROCm)
  hipGraphNode_t node = nullptr;
  e = hipGraphAddEventRecordNode(&node, graph, deps, nd, ev);
  TORCH_CHECK(e == hipSuccess, "grad event: record node: ", hipGetErrorString(e));
  e = hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
  TORCH_CHECK(e == hipSuccess, "grad event: capture dependencies: ", hipGetErrorString(e));
}
void grad_event_record(int64_t k, int64_t stream) {
  TORCH_CHECK(k >= 0 && k < 3, "grad_event_record: group 0, 1 or 2");
  int dev = 0;
  (void)hipGetDevice(&dev);
  record_grad_event(device_aux(dev).grad_ev[k], reinterpret_cast<hipStream_t>(stream), (int)k);
}
void grad_event_wait(int64_t k, int64_t stream) {
  TORCH_CHECK(k >= 0 && k < 3, "grad_event_wait: group 0, 1 or 2");
  int dev = 0;
  (void)hipGetDevice(&dev);
  (void)hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), device_aux(dev).grad_ev[k], 0);
}

// Read-only zeros of at least n elements (initial decoder states): one
// persistent buffer per (device, dtype), so a decode does not launch a fill
// kernel per call.  Grown only outside graph capture; replaced buffers stay
// alive (a captured graph may still read them).
static at::Tensor zeros_view(const at::Device& dev, int64_t n, at::ScalarType dtype) {
  static std::map<std::pair<int, int>, std::vector<at::Tensor>> bufs;
  auto& v = bufs[std::make_pair((int)dev.index(), (int)dtype)];
  if (v.empty() || v.back().numel() < n) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(cur_stream(), &cs);
    auto opts = at::TensorOptions().dtype(dtype).device(dev);
    if (cs != hipStreamCaptureStatusNone) return at::zeros({n}, opts);
    v.push_back(at::zeros({std::max<int64_t>(n, 1 << 20)}, opts));
  }
  return v.back().narrow(0, 0, n);
}

// modes[t] = token-selection mode for token t+1 (see SelModeHost)
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
                                        bool xe_rows) {
  check_cuda(wx, "wx");
  TORCH_CHECK(cell >= 0 && cell <= 2, "cell: 0 lstm, 1 gru, 2 rnn (tanh)");  // CellType (common.h)
  check_cuda(emb, "emb");
  check_cuda(wlog, "wlog");
  check_cuda(blog, "blog");
  // temporal attention (num_chunks > 1): att = {Gv (Bv, C, 4H) f32 packed gates,
  // P (Bv, C, A) f32, W_q (A, H) bf16, w_a (A) f32, b_a (1) f32}; vgate unused.
  // MANet (modal attention over the C modality blocks): w_a (C, A), b_a (C)
  const bool has_att = !att.empty();
  if (!has_att) check_cuda(vgate, "vgate");
  TORCH_CHECK(wx.scalar_type() == at::kBFloat16 && emb.scalar_type() == at::kBFloat16 &&
                  wlog.scalar_type() == at::kBFloat16,
              "decoder weights must be bf16");
  if (!has_att) TORCH_CHECK(vgate.scalar_type() == at::kFloat, "vgate must be fp32");
  check_cuda(ptab, "ptab");
  check_cuda(whh, "whh");
  TORCH_CHECK(ptab.scalar_type() == at::kHalf && ptab.size(0) == emb.size(0) &&
                  ptab.size(1) == wx.size(0), "ptab must be fp16 (V, 4H)");
  const uint16_t* PTAB = reinterpret_cast<const uint16_t*>(ptab.data_ptr());
  TORCH_CHECK(whh.scalar_type() == at::kBFloat16 && whh.size(0) >= wx.size(0) &&
                  whh.size(1) * 4 == wx.size(0), "whh must be bf16 (4H[+A], H)");
  const int64_t H4 = wx.size(0), H = H4 / 4, E = emb.size(1), V = wlog.size(0);
  TORCH_CHECK(wx.size(1) == E + H, "wx must be (4H, E+H)");
  TORCH_CHECK(E % 64 == 0 && H % 64 == 0, "E and H must be multiples of 64");
  TORCH_CHECK(wlog.size(1) == H && blog.numel() == V, "logit weight shape");
  if (!has_att)
    TORCH_CHECK(vgate.size(1) == H4 && vgate.size(0) * vgate_div >= R, "vgate shape");
  at::Tensor a_gv, a_pre, a_wq, a_wa, a_ba;
  int64_t Bv = 0, C = 0, A = 0;
  int per_frame = 0;
  if (has_att) {
    TORCH_CHECK(att.size() == 5, "att = {Gv, P, W_q, w_a, b_a}");
    a_gv = att[0], a_pre = att[1], a_wq = att[2], a_wa = att[3], a_ba = att[4];
    for (auto* t : {&a_gv, &a_pre, &a_wq, &a_wa, &a_ba}) check_cuda(*t, "attention operand");
    Bv = a_gv.size(0), C = a_gv.size(1), A = a_pre.size(2);
    TORCH_CHECK(a_gv.scalar_type() == at::kFloat && a_gv.dim() == 3 && a_gv.size(2) == H4,
                "Gv must be fp32 (Bv, C, 4H)");
    TORCH_CHECK(a_pre.scalar_type() == at::kFloat && a_pre.dim() == 3 && a_pre.size(0) == Bv &&
                    a_pre.size(1) == C, "P must be fp32 (Bv, C, A)");
    TORCH_CHECK(A % 64 == 0 && C >= 1 && C <= 32, "attention: A % 64 == 0 and C <= 32");
    TORCH_CHECK(a_wq.scalar_type() == at::kBFloat16 && a_wq.size(0) == A && a_wq.size(1) == H,
                "W_q must be bf16 (A, H)");
    TORCH_CHECK(whh.size(0) == H4 + A, "with attention whh must be [W_hh; W_q] (4H + A, H)");
    TORCH_CHECK(a_wa.scalar_type() == at::kFloat && a_ba.scalar_type() == at::kFloat &&
                    ((a_wa.numel() == A && a_ba.numel() == 1) ||
                     (C > 1 && C <= 8 && a_wa.numel() == C * A && a_ba.numel() == C)),
                "w_a (A) / b_a (1), or per frame (C, A) / (C), fp32");
    TORCH_CHECK(Bv * vgate_div == R, "attention needs R == videos x rows per video");
    per_frame = a_wa.numel() == C * A && C > 1 ? 1 : 0;
  }
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

  // (every entry is written by the combine of its step: no fill kernels)
  at::Tensor seq = at::empty({R, T - 1}, i64);
  at::Tensor g_sel = at::empty({R, T - 1}, f32);
  at::Tensor g_xe = want_xe ? at::empty({R, T}, f32) : at::Tensor();
  at::Tensor lse = at::empty({n_steps, R}, f32);
  at::Tensor part =
      at::empty({(int64_t)vocab_part_slots((int)V) * R * vocab_partial_bytes() / 4}, f32);
  // the end-of-sequence flags of every step (zero-filled)
  const int64_t n_cnt = (T + 1) * combine_count_ints_per_step();
  at::Tensor counts = at::zeros({n_cnt}, at::TensorOptions().dtype(at::kInt).device(dev));
  at::Tensor unfinished =
      use_unfinished ? at::ones({R}, at::TensorOptions().dtype(at::kByte).device(dev))
                     : at::Tensor();
  // saved rows padded to 128 bytes (whole cache lines per row)
  const int64_t ldl = (V + 63) / 64 * 64;
  // Stacked layers (num_layers > 1): layer 0 is the fused pipeline below;
  // layer l >= 1 runs after it in every step: x_l = dropout(h_{l-1}) W_ih_l^T
  // (hipBLASLt, fp32) enters the step kernel as its per-row input term, the
  // kernel adds h_l W_hh_l^T and applies the cell.  Dropout between layers
  // (nn.LSTM's inter-layer dropout) and before the vocab projection share the
  // counter hash, keyed by step + 65536 * (layers above).
  TORCH_CHECK(up.size() % 2 == 0, "up = {[W_ih | W_hh] (4H, 2H), W_hh (4H, H)} per upper layer");
  const int64_t NL = 1 + (int64_t)up.size() / 2;
  if (NL > 1) TORCH_CHECK(!has_att && state0.empty(), "stacked layers: no attention / initial state");
  for (int64_t l = 1; l < NL; ++l) {
    const at::Tensor &wu = up[2 * (l - 1)], &wh = up[2 * (l - 1) + 1];
    check_cuda(wu, "upper-layer weights");
    check_cuda(wh, "upper-layer W_hh");
    TORCH_CHECK(wu.scalar_type() == at::kBFloat16 && wu.is_contiguous() && wu.size(0) == H4 &&
                    wu.size(1) == 2 * H && wh.scalar_type() == at::kBFloat16 &&
                    wh.is_contiguous() && wh.size(0) == H4 && wh.size(1) == H,
                "upper layer: [W_ih | W_hh] bf16 (4H, 2H) and W_hh bf16 (4H, H)");
  }
  auto key = [&](int64_t l, int64_t t) -> int { return (int)(t + 65536 * (NL - 1 - l)); };

  // Per-layer buffers: h_t / c_t / gates_t saved per step in training (else
  // ping-pong), hd_t = dropout(h_t) (the next layer's input; the top layer's
  // is the vocab input)
  at::Tensor logits16;
  std::vector<at::Tensor> Hs(NL), Cs(NL), Gs(NL), HDs(NL);
  std::vector<std::array<at::Tensor, 2>> hpp(NL), cpp(NL);
  // saved vocab rows: fp16 logits, or (store_exp) bf16 E = exp(x - lse of the
  // previous step) for the dS-free backward (kernels/vocab_grad.hip)
  if (save)
    logits16 = at::empty({n_steps, R, ldl}, at::TensorOptions()
                                                .dtype(store_exp ? at::kBFloat16 : at::kHalf)
                                                .device(dev));
  for (int64_t l = 0; l < NL; ++l) {
    if (save) {
      Hs[l] = at::empty({n_steps, R, H}, bf);
      Cs[l] = at::empty({n_steps, R, H}, f32);
      Gs[l] = at::empty({n_steps, R, H4}, bf);
      HDs[l] = at::empty({n_steps, R, H}, bf);
    } else {
      hpp[l] = {at::empty({R, H}, bf), at::empty({R, H}, bf)};
      cpp[l] = {at::empty({R, H}, f32), at::empty({R, H}, f32)};
      if (drop_p > 0) HDs[l] = at::empty({R, H}, bf);
    }
  }
  auto h_tensor = [&](int64_t l, int64_t t) -> at::Tensor {
    return save ? Hs[l][t] : hpp[l][t & 1];
  };
  auto h_buf = [&](int64_t l, int64_t t) -> uint16_t* {
    return reinterpret_cast<uint16_t*>(h_tensor(l, t).data_ptr());
  };
  auto c_buf = [&](int64_t l, int64_t t) -> float* {
    return save ? Cs[l][t].data_ptr<float>() : cpp[l][t & 1].data_ptr<float>();
  };
  auto hd_buf = [&](int64_t l, int64_t t) -> uint16_t* {
    if (!HDs[l].defined()) return nullptr;
    return reinterpret_cast<uint16_t*>((save ? HDs[l][t] : HDs[l]).data_ptr());
  };
  auto out_tensor = [&](int64_t l, int64_t t) -> at::Tensor {  // layer l's output fed upward
    return HDs[l].defined() ? (save ? HDs[l][t] : HDs[l]) : h_tensor(l, t);
  };
  auto gates_buf = [&](int64_t l, int64_t t) -> uint16_t* {
    return save ? reinterpret_cast<uint16_t*>(Gs[l][t].data_ptr()) : nullptr;
  };

  const uint32_t* RNG = rng_ptr(rng);
  const float inv_temp = (float)(1.0 / temperature);
  const uint16_t* W = reinterpret_cast<const uint16_t*>(wlog.data_ptr());
  const uint16_t* WHH = reinterpret_cast<const uint16_t*>(whh.data_ptr());
  const int64_t* LAB = have_labels ? labels.data_ptr<int64_t>() : nullptr;

  // initial state (model_type 'standard': the state after the video step;
  // otherwise zero): state0 = {h0 bf16 (R, H), c0 fp32 (R, H)}
  at::Tensor h0, c0;
  if (!state0.empty()) {
    TORCH_CHECK(state0.size() == 2 && !has_att, "state0 = {h0, c0}, without attention");
    h0 = state0[0], c0 = state0[1];
    check_cuda(h0, "h0");
    check_cuda(c0, "c0");
    TORCH_CHECK(h0.scalar_type() == at::kBFloat16 && h0.is_contiguous() && h0.size(0) == R &&
                    h0.size(1) == H && c0.scalar_type() == at::kFloat && c0.is_contiguous() &&
                    c0.size(0) == R && c0.size(1) == H,
                "h0 bf16 / c0 fp32, contiguous (R, H)");
  } else {
    h0 = zeros_view(dev, R * H, at::kBFloat16).view({R, H});
    c0 = zeros_view(dev, R * H, at::kFloat).view({R, H});
  }
  // pre-activations of the next step (the decode launch's recurrent tiles ->
  // the combine's cell epilogue) in fp16: half the bytes of the combine's
  // largest operand; fp32 where the VALU attention adds its video term into
  // them in place (attention without the MFMA path)
  static const bool pre16_env = [] {
    const char* e = getenv("CSTCAP_PRE16");
    return e == nullptr || atoi(e) != 0;
  }();
  // CSTCAP_GREEDY_ATT_MFMA=1: a forward that saves nothing (the SCST greedy
  // baseline, one row per video) takes the MFMA attention too.  Opt-in: its
  // A / 64 workgroups per video (512 per greedy step at the att8 shape, each
  // computing 32-row tiles for one row) slow the concurrent sampled rollout
  // more than the VALU scorer + query GEMM they replace (att8 4.730 / 4.771
  // vs 4.607 / 4.602 ms, interleaved on one box, profiles/r6/s2/).
  static const bool fwd1_env = [] {
    const char* e = getenv("CSTCAP_GREEDY_ATT_MFMA");
    return e != nullptr && atoi(e) != 0;
  }();
  const bool att_mfma =
      has_att && (save || !fwd1_env
                      ? att_mfma_ok((int)vgate_div, (int)C, (int)A, (int)H, per_frame)
                      : att_mfma_fwd_ok((int)vgate_div, (int)C, (int)A, (int)H, per_frame));
  const bool pre16 = pre16_env && !(has_att && !att_mfma);
  at::Tensor pre = n_steps > 1 ? at::empty({R, H4}, f32.dtype(pre16 ? at::kHalf : at::kFloat))
                               : at::Tensor();
  at::Tensor xin = NL > 1 ? at::empty({R, H4}, f32) : at::Tensor();

  // layer l >= 1 at step t (its zero initial state is h0 / c0's zeros)
  auto upper_step = [&](int64_t l, int64_t t) {
    const at::Tensor& wu = up[2 * (l - 1)];
    at::mm_out(xin, out_tensor(l - 1, t), wu.narrow(1, 0, H).t(), at::kFloat);
    launch_lstm_step_fwd(nullptr, 0, nullptr,
                         t > 0 ? h_buf(l, t - 1) : reinterpret_cast<uint16_t*>(h0.data_ptr()),
                         t > 0 ? c_buf(l, t - 1) : c0.data_ptr<float>(), xin.data_ptr<float>(), 1,
                         (int)R, (int)H,
                         reinterpret_cast<const uint16_t*>(up[2 * (l - 1) + 1].data_ptr()),
                         h_buf(l, t), c_buf(l, t), hd_buf(l, t), (int)H, (float)drop_p, RNG,
                         key(l, t), gates_buf(l, t), st, nullptr, (int)cell);
  };

  // Attention of step t: query q_t = W_q h_{t-1} (hipBLASLt, fp32 out; q_0 = 0),
  // then the attention kernel writes the per-row video gate term vg_rows.
  at::Tensor vg_rows, q_all, alpha_all, q_tmp;
  if (has_att) {
    vg_rows = at::empty({R, H4}, f32);
    if (save) {
      q_all = at::empty({n_steps, R, A}, f32);  // q_0 = 0 is never read
      alpha_all = at::empty({n_steps, R, C}, f32);
    } else {
      q_tmp = at::empty({R, A}, f32);
    }
  }
  auto run_att = [&](int64_t t) {
    const float* qp = nullptr;
    if (t > 0) {
      at::Tensor qo = save ? q_all[t] : q_tmp;
      at::mm_out(qo, h_tensor(0, t - 1), a_wq.t(), at::kFloat);
      qp = qo.data_ptr<float>();
    }
    launch_att_fwd(a_gv.data_ptr<float>(), a_pre.data_ptr<float>(), qp, nullptr,
                   a_wa.data_ptr<float>(), a_ba.data_ptr<float>(), (int)Bv, (int)vgate_div,
                   (int)C, (int)A, (int)H4, vg_rows.data_ptr<float>(),
                   save ? alpha_all[t].data_ptr<float>() : nullptr, st, 0, per_frame);
  };
  const float* VG = has_att ? vg_rows.data_ptr<float>() : vgate.data_ptr<float>();
  const int VDIV = has_att ? 1 : (int)vgate_div;
  // MFMA attention path (kernels/att_mfma.h): from step 1 on, the attention of
  // step t+1 runs as extra workgroups of step t's decode launch (it needs only
  // h_t) and writes bf16 per-row video gates that the combine's cell epilogue
  // adds; no attention launch between the decode launch and the combine.
  // Step 0 (q = 0) and other shapes use the attention kernels of attention.hip.
  const int CPAD = C <= 8 ? 8 : 16;
  at::Tensor gv16, vg16, att_ep, att_cnt, u_all;
  if (att_mfma) {
    // training: the scorer values tanh(P + q) of steps >= 1 (fp16), read by
    // the fused attention backward (lstm.hip att_bwd_fused_wg)
    if (save) u_all = at::empty({n_steps, R, C, A}, f32.dtype(at::kHalf));
    gv16 = at::zeros({Bv, H4, CPAD}, bf);  // frame-minor, frames zero-padded
    gv16.narrow(2, 0, C).copy_(a_gv.transpose(1, 2));
    vg16 = at::empty({R, H4}, bf);
    att_ep = at::empty({Bv, A / 64, 32, CPAD}, f32);
    att_cnt = at::zeros({Bv}, at::TensorOptions().dtype(at::kInt).device(dev));
  }

  // XE all rows (xe_rows: a teacher-forced training forward).  Every input
  // token is a label, known before the vocabulary projection of the previous
  // step, so the cell needs no combine: ONE launch per step runs the
  // vocabulary tiles of step t (E = exp(x), offset 0 -- the backward's
  // VGradRows::zero_off -- and the per-tile partials) together with the WHOLE
  // LSTM step t+1 (lstm_gemm.h lstm_cell_block: recurrent GEMM + table row +
  // cell); ONE combine over all rows after the chain gives every step's LSE
  // and target log-prob: the per-step combine (~12 us with its cell epilogue)
  // leaves the chain.  (Per-step combines on a side stream contended with the
  // chain: XE 3.279 / 3.308 vs 3.213 / 3.258 ms per step, profiles/r6/s2/.)  seq = labels[:, 1:T], exactly as the
  // per-step combine picks them (a step after which every row emitted EOS only
  // forces tokens the labels already hold as 0).
  if (xe_rows) {
    TORCH_CHECK(save && store_exp && want_xe && have_labels && NL == 1 && !has_att &&
                    state0.empty() && n_steps == T && n_steps <= XE_MAX_STEPS,
                "xe_rows: a saved, exp-store teacher-forced forward of a one-layer decoder "
                "without attention / initial state, <= 64 steps");
    for (int64_t t = 0; t + 1 < T; ++t)
      TORCH_CHECK(modes[t] == SEL_GT_H, "xe_rows: teacher forcing at every step");
    const int n_vt = vocab_num_tiles((int)V);
    const int64_t pstep = (int64_t)n_vt * R * vocab_partial_bytes();  // partial bytes per step
    at::Tensor part_all = at::empty({n_steps * pstep / 4}, f32);
    at::Tensor tgt_all = labels.narrow(1, 1, n_steps).t().contiguous();  // (n_steps, R)
    at::Tensor gx = at::empty({n_steps, R}, f32);
    stamp(STAMP_FWD_BEGIN, st);
    launch_lstm_step_fwd(LAB, L, PTAB, nullptr, nullptr, VG, VDIV, (int)R, (int)H, WHH,
                         h_buf(0, 0), c_buf(0, 0), hd_buf(0, 0), (int)H, (float)drop_p, RNG,
                         key(0, 0), gates_buf(0, 0), st, nullptr, (int)cell);
    stamp(STAMP_FWD_STEP0, st);
    for (int64_t t = 0; t < n_steps; ++t) {
      const bool next = t + 1 < n_steps;
      XeCell xc{};
      if (next)
        xc = XeCell{LAB + (t + 1), L, PTAB, c_buf(0, t), h_buf(0, t + 1), c_buf(0, t + 1),
                    hd_buf(0, t + 1), gates_buf(0, t + 1), (float)drop_p, key(0, t + 1),
                    (int)cell};
      char* pt = reinterpret_cast<char*>(part_all.data_ptr()) + t * pstep;
      launch_vocab_lstm_xe(hd_buf(0, t), (int)R, (int)H, W, blog.data_ptr<float>(), (int)V,
                           reinterpret_cast<uint16_t*>(logits16[t].data_ptr()), ldl, pt,
                           tgt_all.data_ptr<int64_t>() + t * R, RNG, h_buf(0, t), WHH, VG, VDIV,
                           next ? &xc : nullptr, st);
    }
    // every step's LSE and target log-probs: one combine over all rows (the
    // per-step partial blocks), after the chain
    launch_vocab_combine(part_all.data_ptr(), n_vt, (int)(n_steps * R), lse.data_ptr<float>(),
                         nullptr, 0, nullptr, 0, gx.data_ptr<float>(), 1, nullptr, 0, SEL_GT_H,
                         0.f, RNG, 0, nullptr, 0, nullptr, st, nullptr, (int)R);
    at::Tensor gxt = gx.t();  // (R, T)
    g_xe.copy_(gxt);
    g_sel.copy_(gxt.narrow(1, 0, T - 1));
    seq.copy_(labels.narrow(1, 1, T - 1));
    stamp(STAMP_FWD_END, st);
    return {seq, g_sel, g_xe, lse, logits16, HDs[0], Gs[0], Cs[0], Hs[0]};
  }

  // step 0: fused cell step from (h_{-1}, c_{-1}) = (h0, c0)
  stamp(STAMP_FWD_BEGIN, st);
  if (has_att) run_att(0);
  // (zero initial state: null h / c, the kernel skips the recurrent GEMM)
  launch_lstm_step_fwd(have_labels ? LAB : bos.data_ptr<int64_t>(), have_labels ? L : 1,
                       PTAB,
                       state0.empty() ? nullptr : reinterpret_cast<uint16_t*>(h0.data_ptr()),
                       state0.empty() ? nullptr : c0.data_ptr<float>(), VG, VDIV, (int)R, (int)H, WHH, h_buf(0, 0),
                       c_buf(0, 0), hd_buf(0, 0), (int)H, (float)drop_p, RNG, key(0, 0),
                       gates_buf(0, 0), st, nullptr, (int)cell);
  for (int64_t l = 1; l < NL; ++l) upper_step(l, 0);
  // Steps t >= 0: ONE launch runs the vocab projection of step t together with
  // the recurrent GEMM of step t+1 (pre = h_t W_hh^T + vgate, layer 0), then
  // the combine picks token t+1 and applies step t+1's cell epilogue (pre +
  // P[token]); the upper layers of step t+1 follow.
  bool conv_join = false;
  for (int64_t t = 0; t < n_steps; ++t) {
    const bool next = t + 1 < n_steps;
    uint16_t* hd = hd_buf(NL - 1, t);
    const uint16_t* vin = hd ? hd : h_buf(NL - 1, t);
    const bool choose = t < T - 1;
    const int mode = choose ? (int)modes[t] : SEL_GT_H;
    const int do_sample = choose && (mode == SEL_SAMPLE_H || mode == SEL_SS_H);
    const bool exp_t = save && store_exp && t > 0;  // step 0: fp16, converted below
    const int vflags = do_sample | ((choose && mode == SEL_GREEDY_H) ? 2 : 0) | (exp_t ? 16 : 0);
    const int64_t* tgt = (have_labels && t + 1 < L) ? LAB + (t + 1) : nullptr;
    // attention: the same launch also projects q_{t+1} = h_t W_q^T (extra
    // W_q tiles of the recurrent GEMM, no vgate add); the attention kernel then
    // adds each row's video term into pre before the combine's cell epilogue
    at::Tensor q_next;
    if (has_att && next) q_next = save ? q_all[t + 1] : q_tmp;
    AttMfmaArgs am{};
    if (att_mfma && next)
      am = AttMfmaArgs{h_buf(0, t), WHH + H4 * H, a_pre.data_ptr<float>(), a_wa.data_ptr<float>(),
                       a_ba.data_ptr<float>(), reinterpret_cast<const uint16_t*>(gv16.data_ptr()),
                       (int)H, (int)A, (int)C, CPAD, (int)H4, (int)vgate_div, (int)Bv,
                       reinterpret_cast<uint16_t*>(vg16.data_ptr()),
                       save ? alpha_all[t + 1].data_ptr<float>() : nullptr,
                       save ? q_next.data_ptr<float>() : nullptr, att_ep.data_ptr<float>(),
                       att_cnt.data_ptr<int>(),
                       save ? reinterpret_cast<uint16_t*>(u_all[t + 1].data_ptr()) : nullptr};
    if (att_mfma && next) am.whole = att_mfma_whole_default((int)C, (int)H);
    const bool q_tiles = has_att && !att_mfma;  // W_q tiles in the recurrent GEMM
    const int n_vt = launch_vocab_lstm_fwd(
        vin, (int)H, (int)R, (int)H, W, blog.data_ptr<float>(), (int)V,
        save ? reinterpret_cast<uint16_t*>(logits16[t].data_ptr()) : nullptr, ldl, part.data_ptr(),
        tgt, L, vflags, inv_temp, RNG, (int)t, h_buf(0, t), WHH, has_att ? nullptr : VG, VDIV,
        next ? reinterpret_cast<float*>(pre.data_ptr()) : nullptr, st, q_tiles ? (int)A : 0,
        q_tiles && next ? q_next.data_ptr<float>() : nullptr,
        exp_t ? lse[t - 1].data_ptr<float>() : nullptr, att_mfma && next ? &am : nullptr,
        pre16 ? 1 : 0);
    if (q_tiles && next)
      launch_att_fwd(a_gv.data_ptr<float>(), a_pre.data_ptr<float>(), q_next.data_ptr<float>(),
                     nullptr, a_wa.data_ptr<float>(), a_ba.data_ptr<float>(), (int)Bv,
                     (int)vgate_div, (int)C, (int)A, (int)H4, pre.data_ptr<float>(),
                     save ? alpha_all[t + 1].data_ptr<float>() : nullptr, st, /*accumulate=*/1,
                     per_frame);
    CellLaunch cl{};
    if (next) {
      TORCH_CHECK(choose, "internal: a next step needs a chosen token");
      cl = CellLaunch{pre.data_ptr(), PTAB, c_buf(0, t), c_buf(0, t + 1),
                      h_buf(0, t + 1), hd_buf(0, t + 1), (int)H, gates_buf(0, t + 1), (int)H,
                      (float)drop_p, key(0, t + 1), (int)cell,
                      att_mfma ? reinterpret_cast<const uint16_t*>(vg16.data_ptr()) : nullptr,
                      pre16 ? 1 : 0};
    }
    launch_vocab_combine(part.data_ptr(), n_vt, (int)R, lse[t].data_ptr<float>(),
                           choose ? seq.data_ptr<int64_t>() + t : nullptr, T - 1,
                           choose ? g_sel.data_ptr<float>() + t : nullptr, T - 1,
                           want_xe ? g_xe.data_ptr<float>() + t : nullptr, T, tgt, L, mode,
                           (float)ss_prob, RNG, (int)t,
                           use_counts ? counts.data_ptr<int>() : nullptr, (int)(t + 1),
                           use_unfinished ? unfinished.data_ptr<uint8_t>() : nullptr, st,
                           next ? &cl : nullptr);
    if (save && store_exp && t == 0) {
      // only the backward reads step 0's exp store: the conversion runs on a
      // side stream, off the decode chain, joined after the loop
      DeviceAux& aux = device_aux((int)dev.index());
      const hipStream_t cs = aux.side[1].stream();
      (void)hipEventRecord(aux.fwd_ev[0], st);
      (void)hipStreamWaitEvent(cs, aux.fwd_ev[0], 0);
      launch_vocab_exp_convert(reinterpret_cast<uint16_t*>(logits16[0].data_ptr()), ldl, (int)V,
                               (int)R, lse[0].data_ptr<float>(), cs);
      (void)hipEventRecord(aux.fwd_ev[1], cs);
      conv_join = true;
    }
    if (next)
      for (int64_t l = 1; l < NL; ++l) upper_step(l, t + 1);
    if (t == 0) stamp(STAMP_FWD_STEP0, st);
  }
  if (conv_join) (void)hipStreamWaitEvent(st, device_aux((int)dev.index()).fwd_ev[1], 0);
  stamp(STAMP_FWD_END, st);
  // saved: {logits16, hd of the top layer (vocab input), layer 0's gates, c, h}
  // (+ {alpha_all, q_all, u_all}) (+ {h, c, gates of layer l, hd of layer l-1} per l >= 1)
  std::vector<at::Tensor> out = {seq, g_sel, want_xe ? g_xe : at::Tensor(), lse};
  if (save) {
    out.push_back(logits16);
    out.push_back(HDs[NL - 1]);
    out.push_back(Gs[0]);
    out.push_back(Cs[0]);
    out.push_back(Hs[0]);
    if (has_att) {
      out.push_back(alpha_all);
      out.push_back(q_all);
      out.push_back(u_all.defined() ? u_all : at::empty({0}, f32.dtype(at::kHalf)));
    }
    for (int64_t l = 1; l < NL; ++l) {
      out.push_back(Hs[l]);
      out.push_back(Cs[l]);
      out.push_back(Gs[l]);
      out.push_back(HDs[l - 1]);
    }
  }
  return out;
}

// Returns {dWx_packed (4H, E+H), dWlog (V, H), dblog (V), d_emb (V, E), d_vgate (R / vgate_div, 4H)}
// (+ {dGv (Bv, C, 4H), dP (Bv, C, A), dw_a (A), db_a (1), dW_q (A, H)} with attention,
// att = {Gv, P, W_q bf16, w_a, alpha_all (n, R, C), q_all (n, R, A)}; dvg_rows empty)
// (+ {dh0 (R, H) through W_hh, dc0 (R, H) the state carry} with an initial
// state, state0 = {h0, c0} of the forward)
// (+ {dW_up_l (4H, 2H) packed [W_ih | W_hh]} per upper layer; up = {[W_ih |
// W_hh] bf16, h_all, c_all, gates_all of layer l, hd_all of layer l-1} each).
// toks: (n_steps*R) input token of every (step, row), step-major.
//
// Schedule (streams):
//   side 0 : row weights alpha and the one-hot terms folded into E (dS =
//            diag(alpha) E'), X = E' W_logit (one BLAS GEMM over all T*R
//            rows), then (under the loop) the scaled rows alpha Hd;
//   main   : the input-token counting sort (under the side stream's GEMM),
//            then waits for X and runs the reverse LSTM loop (one fused
//            kernel per step: recurrent GEMM + cell backward; dHd = alpha X
//            row-scaled as the step loads it), then the per-token
//            gate-gradient sums, the embedding / input-weight gradient GEMMs
//            over them and the batched recurrent-weight GEMMs;
//   side 0 : dW_logit = E'^T (alpha Hd) and the bias column sums -- after
//            the loop on one GPU, concurrently with the loop under data
//            parallelism so the vocab head's all-reduce (comm_stream waits
//            on it) hides under the loop.
std::vector<at::Tensor> featpool_backward(at::Tensor dout, at::Tensor out,
                                          std::vector<at::Tensor> xs,
                                          std::vector<at::Tensor> ws, double drop_p,
                                          std::vector<at::Tensor> outs);

// vg_bwd (concat model, data parallelism with direct gradient slots): the
// video-gate / FeatPool backward and the packed -> PyTorch row order of the
// LSTM weight gradients done HERE instead of after the call, so W_ih's and
// the FeatPool parameters' gradients are final shortly after the reverse loop
// (a third early all-reduce slice, grad event 2):
//   {dst_ie, dst_hh (int64 row maps), W_ih slot (4H x (E + Fv)), W_hh slot
//    (4H x H), W_ih (fp32 parameter), fc (FeatPool output, B x Fv),
//    FeatPool weight slots x vg_nf, bias slots x vg_nf, inputs x vg_nf,
//    weights x vg_nf}; vg_p the FeatPool dropout.
// C = A^T B over the first K rows of the bf16 row-major operands A (K x >= M)
// and B (K x >= N) through the hand-written split-K kernel (kernels/wgrad.hip):
// rows [0, M0) of C into C0 (row stride ldc0), rows [M0, M) into C1.  Returns
// false (nothing launched) when the shapes do not fit the kernel.
// al / db (optional, N = 512): also db[m] = sum_k al[k] A[k][m] (fused column
// sums of the A tiles in LDS)
static bool wgrad_tn_into(const at::Tensor& A, int64_t lda, const at::Tensor& B, int64_t ldb,
                          int64_t M, int64_t N, int64_t K, float* C0, int64_t ldc0, int64_t M0,
                          float* C1, int64_t ldc1, hipStream_t st, const float* al = nullptr,
                          float* db = nullptr) {
  if (A.scalar_type() != at::kBFloat16 || B.scalar_type() != at::kBFloat16 ||
      !wgrad_tn_ok(M, N, K, lda, ldb, A.data_ptr(), B.data_ptr()) || (db != nullptr && N != 512))
    return false;
  const int S = wgrad_tn_splits(M, N, K);
  at::Tensor ws, ws_db;
  if (S > 1) ws = at::empty({S, M, N}, A.options().dtype(at::kFloat));
  if (S > 1 && db != nullptr) ws_db = at::empty({S, M}, A.options().dtype(at::kFloat));
  WgradArgs g{reinterpret_cast<const uint16_t*>(A.data_ptr()), lda,
              reinterpret_cast<const uint16_t*>(B.data_ptr()), ldb, (int)M, (int)N, (int)K, S, 0,
              S > 1 ? ws.data_ptr<float>() : nullptr, C0, ldc0, (int)M0, C1, ldc1,
              db != nullptr ? al : nullptr, db, ws_db.defined() ? ws_db.data_ptr<float>() : nullptr};
  launch_wgrad_tn(g, st);
  return true;
}

// microbenchmark of the persistent reverse loop alone (random operands of the
// given shape): mean us per launch over `iters` launches; `phases` (int64,
// grid x T x 4, nullable-empty) receives the last launch's per-step stamps
// (step start, team wait done, operands + GEMM done, step published)
double lstm_bwd_loop_bench(int64_t R, int64_t H, int64_t T, int64_t iters, at::Tensor phases,
                           int64_t dbg) {
  TORCH_CHECK(lstm_bwd_loop_ok((int)R, (int)H, (int)T), "lstm_bwd_loop_bench: unsupported shape");
  auto dev = at::Device(at::kCUDA, at::hip::getCurrentHIPStream().device_index());
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
  auto b16 = at::TensorOptions().dtype(at::kBFloat16).device(dev);
  at::Tensor dG = at::empty({T, R, 4 * H}, b16);
  at::Tensor whhT = (at::randn({H, 4 * H}, f32) * 0.05).to(at::kBFloat16);
  at::Tensor dh = at::randn({T, R, H}, f32) * 0.01;
  at::Tensor gates = at::rand({T, R, 4 * H}, f32).to(at::kBFloat16);
  at::Tensor c_all = at::randn({T, R, H}, f32);
  at::Tensor dc = at::empty({R, H}, f32);
  at::Tensor rng = at::zeros({2}, at::TensorOptions().dtype(at::kInt).device(dev));
  BwdLoopArgs la{};
  la.dG = reinterpret_cast<uint16_t*>(dG.data_ptr());
  la.whhT = reinterpret_cast<const uint16_t*>(whhT.data_ptr());
  la.dh = dh.data_ptr<float>();
  la.gates = reinterpret_cast<const uint16_t*>(gates.data_ptr());
  la.c_all = c_all.data_ptr<float>();
  la.dc_out = dc.data_ptr<float>();
  la.R = (int)R;
  la.H = (int)H;
  la.T = (int)T;
  la.drop_p = 0.5f;
  la.rng = reinterpret_cast<const uint32_t*>(rng.data_ptr());
  la.cnt = loop_counters(dev.index(), lstm_bwd_loop_counter_ints((int)R, (int)H));
  la.err = device_err_word(dev.index());
  la.poll_bound = g_poll_bound;
  la.dbg = (int)dbg;
  la.form = dbg >= 8 ? 0 : 1;  // (dbg 8: the K-split form; 0-7: the row-read form's variants)
  if (dbg >= 8) la.dbg = 0;
  if (la.form == 0) la.xb = loop_xb(dev.index(), lstm_bwd_loop_xb_floats((int)R, (int)H));
  hipStream_t st = cur_stream();
  for (int i = 0; i < 3; ++i) launch_lstm_bwd_loop(la, st);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, st);
  for (int64_t i = 0; i < iters; ++i) launch_lstm_bwd_loop(la, st);
  (void)hipEventRecord(e1, st);
  if (phases.defined() && phases.numel() > 0) {
    TORCH_CHECK(phases.scalar_type() == at::kLong && phases.is_cuda() && phases.is_contiguous(),
                "phases: int64 GPU tensor");
    la.phases = phases.data_ptr<int64_t>();
    launch_lstm_bwd_loop(la, st);
  }
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamSynchronize(st);
  return ms * 1e3 / std::max<int64_t>(iters, 1);
}

// test entry: C (M x N) fp32 = A[:K]^T B[:K]
at::Tensor wgrad_tn(at::Tensor A, at::Tensor B, int64_t M, int64_t N, int64_t K) {
  check_cuda(A, "A");
  check_cuda(B, "B");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1 &&
                  A.size(0) >= K && B.size(0) >= K && A.size(1) >= M && B.size(1) >= N,
              "wgrad_tn: operand shapes");
  at::Tensor C = at::empty({M, N}, A.options().dtype(at::kFloat));
  TORCH_CHECK(wgrad_tn_into(A, A.stride(0), B, B.stride(0), M, N, K, C.data_ptr<float>(), N, M,
                            nullptr, 0, cur_stream()),
              "wgrad_tn: shapes not supported (N a multiple of 128, 16-byte rows)");
  return C;
}

// test entry of the fused form: {C (M x N), db (M)} with db[m] = sum_k al[k] A[k][m]
std::vector<at::Tensor> wgrad_tn_colsum(at::Tensor A, at::Tensor B, at::Tensor al, int64_t M,
                                        int64_t N, int64_t K) {
  check_cuda(A, "A");
  check_cuda(B, "B");
  check_cuda(al, "al");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1 &&
                  A.size(0) >= K && B.size(0) >= K && A.size(1) >= M && B.size(1) >= N &&
                  al.scalar_type() == at::kFloat && al.is_contiguous() && al.numel() >= K,
              "wgrad_tn_colsum: operand shapes");
  at::Tensor C = at::empty({M, N}, A.options().dtype(at::kFloat));
  at::Tensor db = at::empty({M}, A.options().dtype(at::kFloat));
  TORCH_CHECK(wgrad_tn_into(A, A.stride(0), B, B.stride(0), M, N, K, C.data_ptr<float>(), N, M,
                            nullptr, 0, cur_stream(), al.data_ptr<float>(), db.data_ptr<float>()),
              "wgrad_tn_colsum: shapes not supported (N = 512, 16-byte rows)");
  return {C, db};
}

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
                                         bool exp_zero_off) {
  const int64_t n_steps = logits16.size(0), R = logits16.size(1), ldl = logits16.size(2);
  const int64_t H4 = wx.size(0), H = H4 / 4, E = wx.size(1) - H, V = wlog.size(0);
  const int64_t T_sel = seq.size(1);
  hipStream_t st = cur_stream();
  auto dev = wx.device();
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
  auto i32 = at::TensorOptions().dtype(at::kInt).device(dev);
  const bool has_sel = dg_sel.defined() && dg_sel.numel() > 0;
  const bool has_xe = dg_xe.defined() && dg_xe.numel() > 0;
  if (has_sel) TORCH_CHECK(dg_sel.is_contiguous() && dg_sel.size(1) == T_sel, "dg_sel shape");
  if (has_xe) TORCH_CHECK(dg_xe.is_contiguous() && labels.defined(), "dg_xe needs labels");
  TORCH_CHECK(toks.numel() == n_steps * R, "toks must hold one token per (step, row)");
  const uint32_t* RNG = rng_ptr(rng);
  const bool has_att = !att.empty();
  at::Tensor a_gv, a_pre, a_wq, a_wa, a_alpha, a_q, a_u;
  int64_t Bv = 0, C = 0, A = 0, vdiv = 1;
  if (has_att) {
    TORCH_CHECK(att.size() == 6 || att.size() == 7,
                "att = {Gv, P, W_q, w_a, alpha_all, q_all[, u_all]}");
    a_gv = att[0], a_pre = att[1], a_wq = att[2], a_wa = att[3], a_alpha = att[4], a_q = att[5];
    if (att.size() == 7 && att[6].numel() > 0) a_u = att[6];
    Bv = a_gv.size(0), C = a_gv.size(1), A = a_pre.size(2);
    vdiv = R / Bv;
    TORCH_CHECK(Bv * vdiv == R && a_alpha.size(0) == n_steps && a_alpha.size(2) == C &&
                    a_q.size(2) == A && a_wq.size(0) == A && a_wq.size(1) == H,
                "attention operand shapes");
    TORCH_CHECK(a_wa.numel() == A || (C > 1 && a_wa.numel() == C * A), "w_a shape");
  }
  const int per_frame = has_att && C > 1 && a_wa.numel() == C * A ? 1 : 0;
  const int64_t NWA = per_frame ? C : 1;  // scorer-weight rows
  // dG rows: 4H gate gradients (+ A columns of dq with attention)
  const int64_t KD = H4 + A;
  TORCH_CHECK(up.size() % 5 == 0, "up = {W, h_all, c_all, gates_all, hd_in} per upper layer");
  const int64_t NL = 1 + (int64_t)up.size() / 5;
  if (NL > 1) TORCH_CHECK(!has_att && state0.empty(), "stacked layers: no attention / initial state");
  auto upw = [&](int64_t l, int k) -> const at::Tensor& { return up[5 * (l - 1) + k]; };
  for (int64_t l = 1; l < NL; ++l)
    TORCH_CHECK(upw(l, 0).size(0) == H4 && upw(l, 0).size(1) == 2 * H &&
                    upw(l, 1).size(0) == n_steps && upw(l, 2).size(0) == n_steps &&
                    upw(l, 3).size(0) == n_steps && upw(l, 4).size(0) == n_steps,
                "upper-layer operand shapes");
  auto key = [&](int64_t l, int64_t t) -> int { return (int)(t + 65536 * (NL - 1 - l)); };
  const bool has_s0 = !state0.empty();
  if (has_s0)
    TORCH_CHECK(state0.size() == 2 && !has_att && state0[0].size(0) == R &&
                    state0[0].scalar_type() == at::kBFloat16 && state0[1].size(0) == R &&
                    state0[1].scalar_type() == at::kFloat,
                "state0 = {h0 bf16, c0 fp32} (R, H)");
  TORCH_CHECK(V < 65536, "vocab: token sort supports V < 65536");
  const int64_t NR = n_steps * R;
  DeviceAux& aux = device_aux((int)dev.index());
  hipEvent_t ev_ready = aux.ev[0], ev_done = aux.ev[2], ev_tok = aux.ev[3];
  c10::hip::HIPStream side = aux.side[0], side2 = aux.side[1];
  // dHd = alpha X, X = E' W, is computed in chunks of steps in reverse time
  // order on the side stream, one event per chunk: reverse step t waits only
  // for the chunk that holds its rows, so the loop starts after the first
  // (smallest) chunk instead of after the whole 35,840-row GEMM, and the rest
  // of the GEMM runs under the loop
  std::vector<std::array<int64_t, 2>> dhd_chunks;  // [t0, t1)
  // X = E W computed right after the rollout (engine.launch_x, vocab_x): no
  // GEMM here, the loop waits only for the row weights
  const bool have_x = xw.defined() && xw.numel() > 0;
  if (have_x)
    TORCH_CHECK(xw.is_cuda() && xw.scalar_type() == at::kFloat && xw.is_contiguous() &&
                    xw.numel() == NR * H && !(ds_bias.defined() && ds_bias.numel() > 0),
                "xw must be the forward's fp32 (n_steps, R, H) X = E W (exp store only)");
  if (have_x) {
    dhd_chunks.push_back({0, n_steps});
  } else {
    int64_t t1 = n_steps;
    const int64_t k_first = 2, k_rest = 4;  // steps per chunk
    while (t1 > 0) {
      const int64_t k = dhd_chunks.empty() ? k_first : k_rest;
      const int64_t t0 = std::max<int64_t>(0, t1 - k);
      dhd_chunks.push_back({t0, t1});
      t1 = t0;
    }
    TORCH_CHECK((int)dhd_chunks.size() <= MAX_DHD_CHUNKS, "too many decode steps for the dHd chunks");
  }

  // The whole reverse recurrence as ONE persistent launch (lstm_loop.hip):
  // one-layer decoders without attention / initial state whose shape fits
  // (headline: 256 workgroups, one per CU, all resident: the side stream's
  // vocab-head weight gradients start after it).  CSTCAP_BWD_LOOP=0 keeps the
  // launch per step.
  const bool persistent = g_bwd_loop != 0 && NL == 1 && !has_att && !has_s0 &&
                          lstm_bwd_loop_ok((int)R, (int)H, (int)n_steps);
  // dW_logit after the persistent loop starts once the main stream's token
  // sums are enqueued (1; 0: right after the loop, 2: after the d_emb GEMM):
  // its long-running GEMM workgroups no longer hold every CU while the
  // latency-bound post-loop chain waits for slots.  Interleaved on one box:
  // 3.210-3.218 (1) / 3.232-3.237 (2) vs 3.292-3.295 ms (0) per headline
  // step, XE 3.32-3.34 vs 3.39-3.40 (profiles/r6/README_r6.md)
  static const int dw_late = [] {
    const char* e = getenv("CSTCAP_DW_LATE");
    return e != nullptr ? atoi(e) : 1;
  }();
  // 1-2. vocab head on the side stream.  Exp store (training): alpha and the
  // one-hot terms folded into E, X = E' W (dHd = alpha X, scaled by the
  // loop), the alpha-scaled Hd rows for dW; kernels/vocab_grad.hip.  Dense
  // dS given by the caller (full log-prob API, fp16-logits buffer rewritten
  // as bf16 dS): dHd = dS W.
  const bool ds_ready = ds_bias.defined() && ds_bias.numel() > 0;
  if (ds_ready) {
    TORCH_CHECK(ds_bias.is_cuda() && ds_bias.scalar_type() == at::kFloat && ds_bias.numel() == V,
                "ds_bias must be fp32 (V)");
  } else {
    TORCH_CHECK(logits16.scalar_type() == at::kBFloat16,
                "decoder_backward: the saved rows must be the exp store (forward store_exp) "
                "unless a dense dS is given");
  }
  at::Tensor buf = logits16.scalar_type() == at::kBFloat16 ? logits16 : logits16.view(at::kBFloat16);
  at::Tensor Ev = buf.view({NR, ldl}).narrow(1, 0, V);  // E (or dense dS), K = V columns
  at::Tensor hd2 = hdrop_all.view({NR, H});
  at::Tensor dHd = have_x ? xw.view({NR, H}) : at::empty({NR, H}, f32);
  // the row's one-hot weights / tokens for the loop (forward X only)
  at::Tensor oh_a, oh_ys, oh_b, oh_yx;
  if (have_x) {
    oh_a = at::empty({NR}, f32);
    oh_ys = at::empty({NR}, i32);
    if (has_xe) {
      oh_b = at::empty({NR}, f32);
      oh_yx = at::empty({NR}, i32);
    }
  }
  const bool early = out_wlog.defined() && out_wlog.numel() > 0;
  if (early) {
    TORCH_CHECK(out_wlog.scalar_type() == at::kFloat && out_wlog.is_contiguous() &&
                    out_wlog.size(0) == V && out_wlog.size(1) == H,
                "out_wlog must be a contiguous fp32 (V, H) tensor");
    TORCH_CHECK(out_blog.scalar_type() == at::kFloat && out_blog.numel() == V, "out_blog shape");
  }
  at::Tensor dWlog = early ? out_wlog : at::empty({V, H}, f32);
  at::Tensor dblog = early ? out_blog.view({V}) : at::empty({V}, f32);
  at::Tensor alpha, hs, cs_part;
  // (the bias gradient as two extra bf16 columns (alpha hi / lo) of the dW
  // GEMM instead of the column sums measured slower: the N = 528 GEMM took
  // ~100 us longer, profiles/r3/ab_dbdw.txt)
  // dW GEMM over augmented rows [alpha Hd | alpha_hi | alpha_lo | 0 ...]
  // (bf16, H + dw_pad columns): the same pass over E' also yields the bias
  // gradient (columns H, H + 1 of the product), instead of a separate
  // column-sum pass over the 753 MB exp store.  CSTCAP_DW_AUG=0: the separate
  // column sums (vgrad_colsum).
  static const bool dw_tuned_env = [] {
    const char* e = getenv("CSTCAP_DW_TUNED");
    return e != nullptr && e[0] == '1';
  }();
  // CSTCAP_DW_AUG unset: the augmented rows with the persistent loop only
  // (dW after the loop); with the per-step loop the dW GEMM runs UNDER the
  // loop, where its 16 extra columns contend with the latency-bound step
  // kernels and the column sums' 210 long workgroups leave them CU slots
  static const int dw_aug_env = [] {
    const char* e = getenv("CSTCAP_DW_AUG");
    return e == nullptr || e[0] == 0 ? -1 : atoi(e);
  }();
  static const bool dw_wgrad_env = [] {
    const char* e = getenv("CSTCAP_DW_WGRAD");
    return e != nullptr && atoi(e) != 0;
  }();
  const bool dw_aug = !ds_ready && !dw_wgrad_env && (dw_aug_env < 0 ? persistent : dw_aug_env != 0);
  // (the augmented rows padded to H + 64 columns: hipBLASLt's pick for the
  // split-K batch runs 443 us at N = 576 against 479 at N = 528 and 537 at
  // N = 512, isolated timings, profiles/r6/README_r6.md; CSTCAP_DW_PAD)
  static const int64_t dw_pad = [] {
    const char* e = getenv("CSTCAP_DW_PAD");
    const int64_t v = e != nullptr ? atoll(e) : 64;
    return v >= 16 && v <= 512 && v % 8 == 0 ? v : 64;
  }();
  const int64_t ldhs = dw_aug ? H + dw_pad : H;
  if (!ds_ready) {
    alpha = at::empty({NR}, f32);
    hs = at::empty({NR, ldhs}, wx.options());
    if (!dw_aug) cs_part = at::empty({vgrad_colsum_blocks(NR), V}, f32);
  }
  auto launch_colsum = [&](hipStream_t s) {
    launch_vgrad_colsum(reinterpret_cast<const uint16_t*>(buf.data_ptr()), ldl, (int)V, NR,
                        alpha.data_ptr<float>(), cs_part.data_ptr<float>(),
                        dblog.data_ptr<float>(), s);
  };
  // 3. dW_logit and the bias gradient: exp store: dW = E'^T (alpha Hd), db =
  // sum_r alpha_r E'_r; dense dS: dW = dS^T Hd, db = ds_bias.  Neither needs
  // the reverse loop.  One GPU: after the loop, concurrent with the input-token
  // gradients (3.864-3.872 ms per step vs 3.961 before the loop, 3.889
  // concurrent with it, 3.946 GEMM before / column sums during it;
  // profiles/r2/ab_vh_sched.txt).  Data parallelism runs them concurrently
  // with the loop, so the vocab head's all-reduce hides under it.
  const bool early_comm = early && comm_stream != 0;
  // (data parallelism: dW_logit right after the persistent loop, so the vocab
  // head's all-reduce starts ~270 us before the backward ends and hides under
  // the post-loop chain -- test_gpu_dist.py; late, it would start at the end)
  const int dw_late_at = early_comm || (g_grad_events_on && early) ? 0 : dw_late;
  // DP overlap (set_grad_events): vocab head / embedding gradients final events
  const bool grad_ev = g_grad_events_on && early;
  // dW_logit and the bias column sums run on the side stream under the
  // latency-bound reverse loop (data parallelism: the vocab head's all-reduce
  // starts there too).  Round 4: with the bias column sums in fewer
  // workgroups (vocab_grad.hip) this beats the sums-under-the-loop /
  // dW-after-it schedule on one GPU too: interleaved A/B 3.591-3.604 vs
  // 3.628-3.682 ms per step (profiles/r4/README_r4.md).
  // dW = E'^T (alpha Hd): M = V, N = H, K = NR.  As one GEMM the 256 x 256
  // tiles put only (V / 256) x (H / 256) = 82 workgroups on the 256 CUs; a
  // split-K batch over groups of decode steps multiplies the tiles in flight,
  // the partial products summed afterwards (4 groups: 3.745-3.774 vs
  // 3.792-3.831 ms per step for one GEMM, 7 groups 3.862-3.873,
  // profiles/r3/ab_sched.txt).  The groups split the rows, not the steps:
  // tied to the step count, the 29 steps of an XE step ran one K = 37k GEMM
  // (712 vs 461 us, profiles/r6/steps_xe3.txt)
  const int64_t dw_split = NR % 4 == 0 ? 4 : (NR % 2 == 0 ? 2 : 1);
  // CSTCAP_DW_WGRAD=1: dW_logit AND the bias column sums in one hand-written
  // split-K MFMA kernel instead (kernels/wgrad.hip: M = V with a ragged last
  // tile, the sums from the E' tiles already in LDS): one pass over the exp
  // store too, but 737 us at the headline shape against 392 + 209 us for the
  // vendor batch + the column sums (profiles/r6/README_r6.md)
  bool dw_fused = false;
  auto dw_gemm = [&]() {  // (current stream: side)
    const at::Tensor& rhs = ds_ready ? hd2 : hs;
    if (dw_aug) {
      // split-K batch over the augmented rows; the partial products summed
      // into the dW slot and the bias gradient (hi + lo columns).  (One GEMM
      // over all rows with the measured hipBLASLt choice: 3.439-3.451 vs
      // 3.330-3.343 ms per step, profiles/r6/README_r6.md)
      const int64_t kr = NR / dw_split;
      at::Tensor p;  // (split, V, ldhs)
      if (dw_tuned_env) {
        // the batch with the measured hipBLASLt choice (gemm_bf16_tuned_batched)
        p = at::empty({dw_split, V, ldhs}, f32);
        gemm_bf16_tuned_batched(
            p, buf.view({NR, ldl}).as_strided({dw_split, kr, V}, {kr * ldl, ldl, 1}), true,
            hs.view({dw_split, kr, ldhs}), false, 24);
      } else {
        at::Tensor a = buf.view({NR, ldl}).as_strided({dw_split, V, kr}, {kr * ldl, 1, ldl});
        p = at::bmm(a, hs.view({dw_split, kr, ldhs}), at::kFloat);
      }
      at::sum_out(dWlog, p.narrow(2, 0, H), 0);
      at::sum_out(dblog, p.narrow(2, H, 2), at::IntArrayRef({0, 2}));
      dw_fused = true;
      return;
    }
    if (!ds_ready && dw_wgrad_env &&
        wgrad_tn_into(buf.view({NR, ldl}), ldl, hs, H, V, H, NR, dWlog.data_ptr<float>(), H, V,
                      nullptr, 0, side.stream(), alpha.data_ptr<float>(), dblog.data_ptr<float>())) {
      dw_fused = true;
      return;
    }
    // (hipBLASLt's measured choice as one GEMM: 3.683-3.731 vs 3.628-3.682 ms
    // per step, the round-4 hand-written GEMM 3.746-3.795: the split-K batch)
    if (dw_split == 1) {
      at::mm_out(dWlog, Ev.t(), rhs, at::kFloat);
      return;
    }
    const int64_t kr = NR / dw_split;
    at::Tensor a = buf.view({NR, ldl}).as_strided({dw_split, V, kr}, {kr * ldl, 1, ldl});
    at::sum_out(dWlog, at::bmm(a, rhs.view({dw_split, kr, H}), at::kFloat), 0);
  };
  auto db_sums = [&](hipStream_t s) {  // (current stream: s)
    if (ds_ready)
      dblog.copy_(ds_bias);
    else if (!dw_fused)
      launch_colsum(s);
  };
  auto dw_done = [&]() {
    (void)hipEventRecord(ev_done, side.stream());
    if (grad_ev) record_grad_event(aux.grad_ev[0], side.stream(), 0);
    if (early_comm) (void)hipStreamWaitEvent(reinterpret_cast<hipStream_t>(comm_stream), ev_done, 0);
  };
  // alpha, one-hot terms folded into E (dS = diag(alpha) E'); exp-store range
  // guard: rows whose LSE jumped by > 60 since the previous step are listed
  // and recomputed exactly (vocab_grad.hip vgrad_fix)
  // (only the row counter fix[0] needs zeroing: the list entries are written
  // by vgrad_onehot before vgrad_fix reads them)
  at::Tensor fix = !ds_ready && blog.defined() && blog.numel() == V ? at::empty({1 + NR}, i32)
                                                                     : at::Tensor();
  auto onehot_pass = [&](hipStream_t s) {
    const bool guard = fix.defined();
    VGradRows va{(int)R, (int)n_steps, (int)T_sel, (int)H, (int)V, lse.data_ptr<float>(),
                 has_sel ? seq.data_ptr<int64_t>() : nullptr,
                 has_sel ? dg_sel.data_ptr<float>() : nullptr,
                 has_xe ? labels.data_ptr<int64_t>() + 1 : nullptr,
                 has_xe ? labels.size(1) : 0, has_xe ? dg_xe.data_ptr<float>() : nullptr,
                 has_xe ? dg_xe.size(1) : 0, guard ? fix.data_ptr<int>() : nullptr,
                 ptr_or_null<float>(oh_a), ptr_or_null<int>(oh_ys), ptr_or_null<float>(oh_b),
                 ptr_or_null<int>(oh_yx), have_x ? dHd.data_ptr<float>() : nullptr,
                 exp_zero_off ? 1 : 0};
    launch_vgrad_onehot(va, reinterpret_cast<uint16_t*>(buf.data_ptr()), ldl,
                        alpha.data_ptr<float>(), s);
    if (guard) {
      TORCH_CHECK(blog.is_cuda() && blog.scalar_type() == at::kFloat && blog.is_contiguous(),
                  "blog must be a contiguous fp32 GPU tensor");
      TORCH_CHECK(!fix_total.defined() || fix_total.numel() == 0 ||
                      (fix_total.is_cuda() && fix_total.scalar_type() == at::kInt),
                  "fix_total must be an int32 GPU tensor");
      launch_vgrad_fix(va, reinterpret_cast<const uint16_t*>(hd2.data_ptr()),
                       reinterpret_cast<const uint16_t*>(wlog.data_ptr()), blog.data_ptr<float>(),
                       reinterpret_cast<uint16_t*>(buf.data_ptr()), ldl, alpha.data_ptr<float>(),
                       ptr_or_null<int>(fix_total), s);
    }
    stamp(STAMP_BWD_ONEHOT, s);
  };
  // the vocab head's weight gradients (current stream: side)
  bool rows_early = false;  // the scaled Hd rows already formed (persistent loop)
  auto side_dw = [&]() {
    if (!ds_ready && !rows_early)
      launch_vgrad_rows(alpha.data_ptr<float>(), NR, (int)H,
                        reinterpret_cast<const uint16_t*>(hd2.data_ptr()), nullptr,
                        reinterpret_cast<uint16_t*>(hs.data_ptr()), side.stream(), (int)ldhs);
    stamp(STAMP_BWD_DHD, side.stream());
    dw_gemm();
    stamp(STAMP_BWD_DW, side.stream());
    db_sums(side.stream());
    dw_done();
  };
  // X-independent preparation of the loop first, then the wait for X
  // (x_wait: the event engine.launch_x recorded after X = E W): the counter
  // resets, the dc zeros, the W_hh^T copy and the token sort run under the X
  // GEMM instead of between it and the loop (they sat on the critical path
  // after X, profiles/r6/steps_scst*.txt)
  if (fix.defined()) (void)hipMemsetAsync(fix.data_ptr(), 0, sizeof(int), st);
  at::Tensor dG_all = at::empty({n_steps, R, KD}, wx.options());
  at::Tensor dc = at::zeros({R, H}, f32);
  // W_hh^T (H, 4H): K-contiguous B operand of the fused step kernel; with
  // attention [W_hh^T | W_q^T] (H, 4H + A), so the step GEMM over
  // [dG_{t+1} | dq_{t+1}] also adds dq_{t+1} W_q (q_{t+1} = W_q h_t) into dh_t
  at::Tensor whhT = has_att ? at::cat({wx.narrow(1, E, H).t(), a_wq.t()}, 1).contiguous()
                            : wx.narrow(1, E, H).t().contiguous();
  // token-only operands of the embedding / input-weight gradients: rows
  // grouped by input token (counting sort), per-token sum scratch
  const bool emb_direct = out_emb.defined() && out_emb.numel() > 0;
  if (emb_direct)
    TORCH_CHECK(out_emb.is_contiguous() && out_emb.scalar_type() == at::kFloat &&
                    out_emb.size(0) == V && out_emb.size(1) == E,
                "out_emb must be a contiguous fp32 (V, E) tensor");
  at::Tensor d_emb = emb_direct ? out_emb : at::empty({V, E}, f32);
  at::Tensor sort_ws = at::empty({2 * V + 1}, i32);
  at::Tensor stok = at::empty({NR}, i32), srow = at::empty({NR}, i32);
  at::Tensor S_tok = at::empty({V, H4}, wx.options());  // per-token gate-gradient sums
  at::Tensor S32 = at::empty({V, H4}, f32);  // rows of long groups only (token_long_zero)
  // on the second side stream, off the critical path (needed after the loop)
  hipEvent_t ev_pre = aux.ev[6 + MAX_DHD_CHUNKS];
  (void)hipEventRecord(ev_pre, st);
  (void)hipStreamWaitEvent(side2.stream(), ev_pre, 0);
  launch_token_sort(toks.data_ptr<int64_t>(), (int)NR, (int)V, sort_ws.data_ptr<int>(),
                    stok.data_ptr<int>(), srow.data_ptr<int>(), side2.stream());
  launch_token_long_zero(sort_ws.data_ptr<int>(), (int)V, (int)H4, S32.data_ptr<float>(),
                         side2.stream());
  (void)hipEventRecord(ev_tok, side2.stream());
  if (x_wait != 0) (void)hipStreamWaitEvent(st, reinterpret_cast<hipEvent_t>(x_wait), 0);
  stamp(STAMP_BWD_BEGIN, st);
  // Forward X: the loop's first operands are the row weights of this pass and
  // X itself, so the pass runs on the main stream -- no hop to the side stream
  // and back before the loop; the side stream's dW work waits for it.
  // (3.416-3.427 vs 3.429-3.431 ms per step with the pass on the side stream,
  // interleaved on one box, profiles/r5/tail/ab_ohm_*.json)
  const bool oh_main = have_x && !ds_ready;
  if (oh_main) {
    onehot_pass(st);
    stamp(STAMP_BWD_DHD0, st);
    dhd_chunks.clear();  // (X is final: the loop waits for no chunk)
  }
  (void)hipEventRecord(ev_ready, st);
  // (the side stream's dW work held back until the first 1 / 2 reverse steps
  // are enqueued, so they do not share the CUs with the GEMM's first wave,
  // measured slower: 3.462-3.489 ms per step, profiles/r5/tail/ab_ohm_d*.json)
  (void)hipStreamWaitEvent(side.stream(), ev_ready, 0);
  {
    c10::hip::HIPStreamGuard guard(side);
    if (!ds_ready && !oh_main) onehot_pass(side.stream());
    // X = E' W, chunk by chunk; the reverse loop reads alpha X (row scales at
    // load), and the scaled Hd rows of the dW GEMM are formed under it
    for (size_t ci = 0; ci < dhd_chunks.size(); ++ci) {
      const int64_t r0 = dhd_chunks[ci][0] * R, nr = (dhd_chunks[ci][1] - dhd_chunks[ci][0]) * R;
      at::Tensor dst = dHd.narrow(0, r0, nr);
      if (!have_x) at::mm_out(dst, Ev.narrow(0, r0, nr), wlog, at::kFloat);
      (void)hipEventRecord(aux.ev[6 + ci], side.stream());
      if (ci == 0) stamp(STAMP_BWD_DHD0, side.stream());
    }
    if (!persistent) {
      side_dw();
    } else if (!ds_ready) {
      // the dW GEMM's scaled Hd rows need only alpha: formed now, next to the
      // fold on the main stream, instead of between the loop and the GEMM
      launch_vgrad_rows(alpha.data_ptr<float>(), NR, (int)H,
                        reinterpret_cast<const uint16_t*>(hd2.data_ptr()), nullptr,
                        reinterpret_cast<uint16_t*>(hs.data_ptr()), side.stream(), (int)ldhs);
      rows_early = true;
    }
  }
  // 4. reverse LSTM loop on the main stream
  // (the loop operands filled on the second side stream concurrently with
  // the one-hot pass measured slower: att8 4.487-4.516 vs 4.379-4.417 ms,
  // headline 3.424-3.514 vs 3.337-3.339, profiles/r5/tail/ab_prep*.json)
  at::Tensor dpre_part, dwa_part, dba_part;
  // MFMA attention path backward: dalpha partials from the step kernel's
  // epilogue (lstm.hip) + att_bwd_mfma (attention.hip); else att_bwd
  const int CPAD = C <= 8 ? 8 : 16;
  const bool att_mfma = has_att &&
                        att_mfma_ok((int)vdiv, (int)C, (int)A, (int)H, per_frame) &&
                        att_bwd_epi_ok((int)vdiv, (int)C, (int)H) && (KD / 64) % 2 == 0;
  at::Tensor gvb16, dal_part, att_flags;
  AttBwdEpi abe{};
  // the attention backward of step t + 1 runs as extra workgroups of step t's
  // launch (lstm.hip att_bwd_fused_wg) instead of a launch of its own between
  // the two reverse steps; the dalpha partials alternate between two buffers
  // (att8: 4.717 / 4.728 vs 4.884 / 4.939 ms per step unfused, interleaved on
  // one box, profiles/r5/README_r5.md)
  const bool att_fuse = g_att_fuse && att_mfma && n_steps > 1 && a_u.defined() &&
                        a_u.scalar_type() == at::kHalf && a_u.size(0) == n_steps &&
                        a_u.size(1) == R && a_u.size(2) == C && a_u.size(3) == A &&
                        att_bwd_fuse_ok((int)vdiv, (int)C, (int)A, (int)H, (int)Bv, (int)R);
  if (att_mfma) {
    // gate tables with the 4 packed gates of a unit innermost: (Bv, H, CP, 4)
    gvb16 = at::zeros({Bv, H, CPAD, 4}, wx.options());
    gvb16.narrow(2, 0, C).copy_(a_gv.view({Bv, C, H, 4}).permute({0, 2, 1, 3}));
    dal_part = at::empty({2, H / 64, R, CPAD}, f32);
    if (att_fuse) att_flags = at::zeros({n_steps, Bv}, i32);
    abe = AttBwdEpi{reinterpret_cast<const uint16_t*>(gvb16.data_ptr()), (int)vdiv, (int)C, CPAD,
                    dal_part.data_ptr<float>()};
    dpre_part = at::zeros({Bv, C, A}, f32);
    dwa_part = at::zeros({Bv, A}, f32);
    dba_part = at::zeros({Bv, 1}, f32);
  } else if (has_att) {
    const int64_t nwg = Bv * att_groups((int)vdiv);
    dpre_part = at::zeros({nwg, C, A}, f32);
    dwa_part = at::zeros({nwg, NWA * A}, f32);
    dba_part = at::zeros({nwg, NWA}, f32);
  }
  // upper layers: W_hh_l^T (K-contiguous B operands), gate gradients, carries
  std::vector<at::Tensor> whhT_up(NL), dG_up(NL), dc_up(NL);
  at::Tensor dX_up = NL > 1 ? at::empty({R, H}, f32) : at::Tensor();
  for (int64_t l = 1; l < NL; ++l) {
    whhT_up[l] = upw(l, 0).narrow(1, H, H).t().contiguous();
    dG_up[l] = at::empty({n_steps, R, H4}, wx.options());
    dc_up[l] = at::zeros({R, H}, f32);
  }
  // the vocab head's gradient rows enter the loop as X = E' W with the row
  // scales alpha applied at load (exp store); a dense dS gives dHd directly
  auto dh_scale_t = [&](int64_t t) -> const float* {
    return ds_ready ? nullptr : alpha.data_ptr<float>() + t * R;
  };
  // forward X: the one-hot rows of the top layer's h gradient (see DhOneHot)
  auto dh_onehot_t = [&](int64_t t) -> DhOneHot {
    if (!have_x) return DhOneHot{};
    return DhOneHot{reinterpret_cast<const uint16_t*>(wlog.data_ptr()),
                    oh_a.data_ptr<float>() + t * R, oh_ys.data_ptr<int>() + t * R,
                    has_xe ? oh_b.data_ptr<float>() + t * R : nullptr,
                    has_xe ? oh_yx.data_ptr<int>() + t * R : nullptr};
  };
  if (persistent) {
    // every dHd chunk first (forward X: none), then the loop
    for (size_t ci = 0; ci < dhd_chunks.size(); ++ci)
      (void)hipStreamWaitEvent(st, aux.ev[6 + ci], 0);
    BwdLoopArgs la{};
    la.dG = reinterpret_cast<uint16_t*>(dG_all.data_ptr());
    la.whhT = reinterpret_cast<const uint16_t*>(whhT.data_ptr());
    la.dh = dHd.data_ptr<float>();
    la.scale = ds_ready ? nullptr : alpha.data_ptr<float>();
    if (have_x) {
      la.oh_W = reinterpret_cast<const uint16_t*>(wlog.data_ptr());
      la.oh_a = oh_a.data_ptr<float>();
      la.oh_ys = oh_ys.data_ptr<int>();
      if (has_xe) {
        la.oh_b = oh_b.data_ptr<float>();
        la.oh_yx = oh_yx.data_ptr<int>();
      }
    }
    la.gates = reinterpret_cast<const uint16_t*>(gates_all.data_ptr());
    la.c_all = c_all.data_ptr<float>();
    la.dc_out = dc.data_ptr<float>();
    la.R = (int)R;
    la.H = (int)H;
    la.T = (int)n_steps;
    la.cell = (int)cell;
    la.drop_p = (float)drop_p;
    la.rng = RNG;
    la.cnt = loop_counters((int)dev.index(), lstm_bwd_loop_counter_ints((int)R, (int)H));
    la.err = device_err_word((int)dev.index());
    la.poll_bound = g_poll_bound;
    la.form = g_bwd_loop == 2 ? 0 : 1;
    if (la.form == 0) la.xb = loop_xb((int)dev.index(), lstm_bwd_loop_xb_floats((int)R, (int)H));
    TORCH_CHECK(gates_all.is_contiguous() && c_all.is_contiguous() && dG_all.is_contiguous() &&
                    dHd.is_contiguous() && gates_all.size(0) >= n_steps && c_all.size(0) >= n_steps,
                "persistent reverse loop: operand layout");
    launch_lstm_bwd_loop(la, st);
    stamp(STAMP_BWD_LOOP0, st);
    // the vocab head's weight gradients after the loop (every CU is the
    // loop's until it ends), concurrently with the post-loop chain below
    // (CSTCAP_DW_LATE=1 / 2: started after the token sums / the d_emb GEMM
    // of that chain instead)
    if (dw_late_at == 0) {
      (void)hipEventRecord(aux.ev[4], st);
      (void)hipStreamWaitEvent(side.stream(), aux.ev[4], 0);
      c10::hip::HIPStreamGuard guard(side);
      side_dw();
    }
  }
  auto late_dw = [&](int at) {
    if (!persistent || dw_late_at != at) return;
    (void)hipEventRecord(aux.ev[4], st);
    (void)hipStreamWaitEvent(side.stream(), aux.ev[4], 0);
    c10::hip::HIPStreamGuard guard(side);
    side_dw();
  };
  size_t next_chunk = 0;
  for (int64_t t = persistent ? -1 : n_steps - 1; t >= 0; --t) {
    if (next_chunk < dhd_chunks.size() && t == dhd_chunks[next_chunk][1] - 1)
      (void)hipStreamWaitEvent(st, aux.ev[6 + next_chunk++], 0);  // dHd rows of this chunk
    const DhOneHot oh_t = dh_onehot_t(t);
    // top layer first: its h gradient comes from the vocab head (dHd, with the
    // vocab dropout mask); layer l < top gets dG_{l+1, t} W_ih_{l+1} through
    // the inter-layer dropout mask of layer l's output
    for (int64_t l = NL - 1; l >= 1; --l) {
      const float* dh_in = dHd.data_ptr<float>() + t * R * H;
      const float* dh_sc = dh_scale_t(t);
      const DhOneHot* ohp = &oh_t;
      if (l < NL - 1) {
        at::mm_out(dX_up, dG_up[l + 1][t], upw(l + 1, 0).narrow(1, 0, H), at::kFloat);
        dh_in = dX_up.data_ptr<float>();
        dh_sc = nullptr;
        ohp = nullptr;
      }
      launch_lstm_step_bwd(
          t + 1 < n_steps ? reinterpret_cast<const uint16_t*>(dG_up[l][t + 1].data_ptr()) : nullptr,
          reinterpret_cast<const uint16_t*>(whhT_up[l].data_ptr()), dh_in,
          dc_up[l].data_ptr<float>(), reinterpret_cast<const uint16_t*>(upw(l, 3)[t].data_ptr()),
          upw(l, 2)[t].data_ptr<float>(), t > 0 ? upw(l, 2)[t - 1].data_ptr<float>() : nullptr,
          (int)R, (int)H, (float)drop_p, RNG, key(l, t),
          reinterpret_cast<uint16_t*>(dG_up[l][t].data_ptr()), (int)H4, st, (int)cell, dh_sc,
          nullptr, ohp);
    }
    const float* dh0_in = dHd.data_ptr<float>() + t * R * H;
    const float* dh0_sc = dh_scale_t(t);
    if (NL > 1) {
      at::mm_out(dX_up, dG_up[1][t], upw(1, 0).narrow(1, 0, H), at::kFloat);
      dh0_in = dX_up.data_ptr<float>();
      dh0_sc = nullptr;
    }
    if (att_mfma) {
      abe.dal_part = dal_part[t & 1].data_ptr<float>();
      abe.flags = nullptr;
      if (att_fuse && t + 1 < n_steps) {  // + step t + 1's attention backward
        abe.flags = att_flags[t + 1].data_ptr<int>();
        abe.dal_next = dal_part[(t + 1) & 1].data_ptr<float>();
        abe.alpha = a_alpha[t + 1].data_ptr<float>();
        abe.u = reinterpret_cast<const uint16_t*>(a_u[t + 1].data_ptr());
        abe.wa = a_wa.data_ptr<float>();
        abe.Bv = (int)Bv;
        abe.A = (int)A;
        abe.G4 = (int)H4;
        abe.dP_acc = dpre_part.data_ptr<float>();
        abe.dwa_part = dwa_part.data_ptr<float>();
        abe.dba_part = dba_part.data_ptr<float>();
        abe.poll_bound = g_poll_bound;
        abe.poll_err = device_err_word((int)dev.index());
      }
    }
    launch_lstm_step_bwd(
        t + 1 < n_steps ? reinterpret_cast<const uint16_t*>(dG_all[t + 1].data_ptr()) : nullptr,
        reinterpret_cast<const uint16_t*>(whhT.data_ptr()), dh0_in, dc.data_ptr<float>(),
        reinterpret_cast<const uint16_t*>(gates_all[t].data_ptr()), c_all[t].data_ptr<float>(),
        t > 0 ? c_all[t - 1].data_ptr<float>() : (has_s0 ? state0[1].data_ptr<float>() : nullptr),
        (int)R, (int)H, (float)drop_p, RNG, key(0, t),
        reinterpret_cast<uint16_t*>(dG_all[t].data_ptr()), (int)KD, st, (int)cell, dh0_sc,
        att_mfma ? &abe : nullptr, NL == 1 ? &oh_t : nullptr);
    if (att_fuse) {
      // (step t's attention backward: in step t - 1's launch, or after the loop)
    } else if (att_mfma)
      launch_att_bwd_mfma(dal_part[t & 1].data_ptr<float>(), (int)(H / 64), (int)R,
                          a_alpha[t].data_ptr<float>(), t > 0 ? a_q[t].data_ptr<float>() : nullptr,
                          a_pre.data_ptr<float>(), a_wa.data_ptr<float>(), (int)Bv, (int)vdiv,
                          (int)C, CPAD, (int)A, (int)H4,
                          reinterpret_cast<uint16_t*>(dG_all[t].data_ptr()), (int)KD, t > 0 ? 1 : 0,
                          dpre_part.data_ptr<float>(), dwa_part.data_ptr<float>(),
                          dba_part.data_ptr<float>(), st);
    else if (has_att)  // dq_t (bf16, columns [4H, 4H+A) of dG_t) + dP / dw_a / db_a partials
      launch_att_bwd(reinterpret_cast<uint16_t*>(dG_all[t].data_ptr()), (int)KD,
                     a_gv.data_ptr<float>(), a_pre.data_ptr<float>(),
                     t > 0 ? a_q[t].data_ptr<float>() : nullptr, a_alpha[t].data_ptr<float>(),
                     a_wa.data_ptr<float>(), (int)Bv, (int)vdiv, (int)C, (int)A, (int)H4,
                     t > 0 ? 1 : 0, dpre_part.data_ptr<float>(), dwa_part.data_ptr<float>(),
                     dba_part.data_ptr<float>(), st, per_frame);
    if (t == n_steps - 1) stamp(STAMP_BWD_LOOP0, st);
  }
  if (att_fuse)
    launch_att_bwd_mfma(dal_part[0].data_ptr<float>(), (int)(H / 64), (int)R,
                        a_alpha[0].data_ptr<float>(), nullptr, a_pre.data_ptr<float>(),
                        a_wa.data_ptr<float>(), (int)Bv, (int)vdiv, (int)C, CPAD, (int)A, (int)H4,
                        reinterpret_cast<uint16_t*>(dG_all[0].data_ptr()), (int)KD, 0,
                        dpre_part.data_ptr<float>(), dwa_part.data_ptr<float>(),
                        dba_part.data_ptr<float>(), st);
  stamp(STAMP_BWD_LOOP, st);
  // attention: the per-frame gate-table gradient dGv needs only the finished
  // dG rows; it runs on the second side stream under the post-loop chain
  // below (joined before the results are returned).  (Its tensors live at
  // function scope: allocated on the main stream, which waits for them.)
  at::Tensor dgv_part, dGv_side;
  if (has_att && C <= 8) {
    dgv_part = at::empty({att_dgv_chunks((int)n_steps), Bv, C, H4}, f32);
    dGv_side = at::empty({Bv, C, H4}, f32);
    (void)hipEventRecord(aux.ev[1], st);
    (void)hipStreamWaitEvent(side2.stream(), aux.ev[1], 0);
    launch_att_dgv(reinterpret_cast<const uint16_t*>(dG_all.data_ptr()), (int)KD,
                   a_alpha.data_ptr<float>(), (int)n_steps, (int)R, (int)Bv, (int)vdiv, (int)C,
                   (int)H4, dgv_part.data_ptr<float>(), side2.stream());
    {
      c10::hip::HIPStreamGuard guard(side2);
      at::sum_out(dGv_side, dgv_part, 0);
    }
    (void)hipEventRecord(aux.ev[5], side2.stream());
  }
  at::Tensor dvg;
  const bool vg_direct = !has_att && !vg_bwd.empty();
  if (vg_direct)
    TORCH_CHECK(vg_nf >= 1 && (int64_t)vg_bwd.size() == 6 + 4 * vg_nf && NL == 1 && !has_s0,
                "vg_bwd = {dst_ie, dst_hh, W_ih slot, W_hh slot, packed W_iv shadow, fc, FeatPool slots, "
                "inputs, weights}");
  std::vector<at::Tensor> vg_keep;  // (side-stream temporaries, released after the join)
  if (!has_att) {
    TORCH_CHECK(vgate_div >= 1 && R % vgate_div == 0, "vgate_div must divide the rows");
    dvg = at::empty({R / vgate_div, H4}, f32);
    // (Bv, 4H): sum over time and over the rows of each video in one pass
    // (kernels/embed_grad.hip), streaming the finished dG rows on the second
    // side stream under the post-loop GEMM chain (joined before returning)
    (void)hipEventRecord(aux.ev[1], st);
    (void)hipStreamWaitEvent(side2.stream(), aux.ev[1], 0);
    launch_video_gate_grad(reinterpret_cast<const uint16_t*>(dG_all.data_ptr()), KD,
                           (int)n_steps, (int)R, (int)vgate_div, (int)H4, dvg.data_ptr<float>(),
                           side2.stream());
    if (vg_direct) {
      // video-gate and FeatPool backward on the same stream (ops/featpool.py
      // _FeatPoolVgateFn does this after the call otherwise): dfc = dvg W_iv,
      // dW_iv = dvg^T fc into W_ih's slot, FeatPool gradients into theirs
      c10::hip::HIPStreamGuard guard(side2);
      // dfc = dvg W_iv (packed gate order on both sides: vg_bwd[4] is the
      // engine's packed bf16 W_iv shadow, zero rows in unused slots) and
      // dW_iv = dvg^T fc (PyTorch gate order, into the slot's column range):
      // bf16 operands, fp32 accumulation and output, the measured hipBLASLt
      // choices.  As fp32 at::mm, dfc ran as an MT32x16 fp32 kernel: 79 us
      // alone and 380-575 us next to the dW_logit GEMM after the persistent
      // loop (profiles/r6/steps_xe*.txt)
      TORCH_CHECK(vg_bwd[4].scalar_type() == at::kBFloat16 && vg_bwd[4].size(0) == H4,
                  "vg_bwd[4]: the packed bf16 (4H, Fv) W_iv shadow");
      const int64_t Fv = vg_bwd[4].size(1);
      at::Tensor dvg_p16 = dvg.to(at::kBFloat16);
      at::Tensor dvg16 = dvg_p16.index_select(1, vg_bwd[0]);  // PyTorch gate order
      at::Tensor dvg_u = dvg16;
      at::Tensor dfc = at::empty({dvg.size(0), Fv}, f32);
      at::Tensor wiv16 = vg_bwd[4];
      at::Tensor fc16 = vg_bwd[5].to(at::kBFloat16);
      gemm_bf16_tuned(dfc, dvg_p16, false, wiv16, false, 24);
      at::Tensor wiv_slot = vg_bwd[2].narrow(1, E, Fv);
      gemm_bf16_tuned(wiv_slot, dvg16, true, fc16, false, 24);
      std::vector<at::Tensor> outs(vg_bwd.begin() + 6, vg_bwd.begin() + 6 + 2 * vg_nf);
      std::vector<at::Tensor> xs(vg_bwd.begin() + 6 + 2 * vg_nf, vg_bwd.begin() + 6 + 3 * vg_nf);
      std::vector<at::Tensor> wsv(vg_bwd.begin() + 6 + 3 * vg_nf, vg_bwd.begin() + 6 + 4 * vg_nf);
      (void)featpool_backward(dfc, vg_bwd[5], xs, wsv, vg_p, outs);
      vg_keep = {dvg_u, dfc, dvg16, dvg_p16, fc16};
    }
    (void)hipEventRecord(aux.ev[5], side2.stream());
  }
  at::Tensor dGx = dG_all.view({NR, KD});  // [dG | dq] rows
  at::Tensor dG2 = dGx.narrow(1, 0, H4);
  // 6. weight gradients dWx = dG^T [x ; h_prev].  The K = steps*rows
  //    reductions run as batched GEMMs over groups of steps (many more output
  //    tiles in flight than one K = 35k GEMM), summed afterwards.
  at::Tensor dWx = at::empty({H4, E + H}, f32);
  at::Tensor dWq = has_att ? at::empty({A, H}, f32) : at::Tensor();
  auto grouped_wgrad = [&](at::Tensor a_rows, at::Tensor b_rows, int64_t nsteps) {
    int64_t G = 1;  // steps per group: largest divisor <= 7
    for (int64_t g = 7; g >= 1; --g)
      if (nsteps % g == 0) { G = g; break; }
    const int64_t nc = nsteps / G;
    at::Tensor a = a_rows.view({nc, G * R, a_rows.size(1)}).transpose(1, 2);
    at::Tensor b = b_rows.reshape({nc, G * R, b_rows.size(1)});
    return at::bmm(a, b, at::kFloat).sum(0);
  };
  // recurrent columns dW_hh = sum_t dG_t^T h_{t-1} (+ dG_0^T h0 with an
  // initial state); with attention the extra rows of [dG | dq]^T h_prev are dW_q
  auto whh_grad = [&](hipStream_t ws) {  // (current stream: ws)
    if (n_steps > 1 && h_all.is_contiguous() &&
        wgrad_tn_into(dGx.narrow(0, R, (n_steps - 1) * R), KD, h_all, H, KD, H,
                      (n_steps - 1) * R, dWx.data_ptr<float>() + E, E + H, H4,
                      has_att ? dWq.data_ptr<float>() : nullptr, H, ws)) {
      // (hand-written split-K MFMA kernel, kernels/wgrad.hip: rows [0, 4H) of
      // [dG | dq]^T h_prev into dW_hh's columns of dWx, the dq rows into dW_q)
    } else if (n_steps > 1) {
      at::Tensor wh;
      wh = grouped_wgrad(dGx.narrow(0, R, (n_steps - 1) * R),
                         h_all.narrow(0, 0, n_steps - 1).reshape({(n_steps - 1) * R, H}),
                         n_steps - 1);
      dWx.narrow(1, E, H).copy_(wh.narrow(0, 0, H4));
      if (has_att) dWq.copy_(wh.narrow(0, H4, A));
    } else {
      dWx.narrow(1, E, H).zero_();
      if (has_att) dWq.zero_();
    }
    if (has_s0) dWx.narrow(1, E, H).add_(at::mm(dG2.narrow(0, 0, R).t(), state0[0], at::kFloat));
  };
  // The recurrent-weight gradient (hand-written split-K GEMM, kernels/wgrad.hip)
  // on the first side stream, idle after dW_logit + the bias sums, concurrent
  // with the input-token chain below: interleaved on one box 3.351-3.386 vs
  // 3.362-3.402 ms per step after that chain on the main stream
  // (profiles/r5/tail/ab_ws_*.json; with the round-4 vendor GEMMs the same
  // move measured slower)
  {
    (void)hipEventRecord(aux.ev[4], st);  // the loop's dG rows
    (void)hipStreamWaitEvent(side.stream(), aux.ev[4], 0);
    c10::hip::HIPStreamGuard guard(side);
    whh_grad(side.stream());
    if (vg_direct) vg_bwd[3].copy_(dWx.narrow(1, E, H).index_select(0, vg_bwd[1]));
    (void)hipEventRecord(ev_done, side.stream());  // (joined below)
  }

  // 5. input-token gradients through the per-token sums S[v] = sum of the dG
  //    rows whose input token is v (bf16, V x 4H): embedding gradient S W_ie,
  //    input-weight gradient S^T emb -- GEMMs over V rows instead of n*R
  (void)hipStreamWaitEvent(st, ev_tok, 0);  // the token sort (second side stream)
  launch_token_group_sum(reinterpret_cast<const uint16_t*>(dG_all.data_ptr()), (int)H4, KD,
                         stok.data_ptr<int>(), srow.data_ptr<int>(), (int)NR,
                         sort_ws.data_ptr<int>(), (int)V,
                         reinterpret_cast<uint16_t*>(S_tok.data_ptr()), S32.data_ptr<float>(), st);
  stamp(STAMP_BWD_TOKSUM, st);
  late_dw(1);
  // d_emb = S W_ie (M = V, N = E, K = 4H): the measured hipBLASLt choice
  // (host/blaslt_tuned.cpp) -- PyTorch's heuristic pick ran it at 0.17 PF/s
  // (130 us, profiles/r5/final5/steps_final5.txt).  CSTCAP_DEMB_TUNED=0: at::mm.
  static const bool demb_tuned = [] {
    const char* e = getenv("CSTCAP_DEMB_TUNED");
    return e == nullptr || atoi(e) != 0;
  }();
  if (demb_tuned && d_emb.is_contiguous() && d_emb.scalar_type() == at::kFloat &&
      S_tok.is_contiguous() && wx.stride(1) == 1)
    gemm_bf16_tuned(d_emb, S_tok, false, wx.narrow(1, 0, E), false, 24);
  else
    at::mm_out(d_emb, S_tok, wx.narrow(1, 0, E), at::kFloat);
  if (grad_ev && emb_direct) record_grad_event(aux.grad_ev[1], st, 1);
  late_dw(2);
  // (dW_ie on the second side stream, concurrent with the embedding GEMM:
  // 3.355-3.361 vs 3.342-3.356 ms per step, profiles/r5/tail/ab_wie_*.json)
  // input columns dW_ie = S^T emb: M = 4H, N = E, K = V.  One GEMM puts only
  // (4H / 64) x (E / 64) tiles on the chip with a 10.5k-long K (164 us, ~134
  // TFLOP/s at V = 10,509); a split-K batch over the largest divisor of V up to
  // 8 multiplies the tiles in flight, the partial products summed afterwards
  // (49 us + a ~20 us sum, profiles/r2/kernel_summary_r2_v19.txt).
  {
    int64_t nk = 1;
    for (int64_t g = 8; g >= 2; --g)
      if (V % g == 0 && V / g >= 512) { nk = g; break; }
    at::Tensor dWie = dWx.narrow(1, 0, E);
    if (emb.dim() == 2 && emb.stride(1) == 1 && S_tok.is_contiguous() &&
        wgrad_tn_into(S_tok, H4, emb, emb.stride(0), H4, E, V, dWie.data_ptr<float>(), E + H, H4,
                      nullptr, 0, st)) {
      // (hand-written split-K MFMA kernel, kernels/wgrad.hip)
    } else if (nk > 1 && emb.is_contiguous())
      at::sum_out(dWie,
                  at::bmm(S_tok.view({nk, V / nk, H4}).transpose(1, 2), emb.view({nk, V / nk, E}),
                          at::kFloat),
                  0);
    else
      dWie.copy_(at::mm(S_tok.t(), emb, at::kFloat));
  }
  stamp(STAMP_BWD_TOKGEMM, st);
  if (vg_direct) {
    // W_ih's token columns (packed -> PyTorch rows) and, from the second side
    // stream, its video columns and the FeatPool gradients: slice 2 is final
    vg_bwd[2].narrow(1, 0, E).copy_(dWx.narrow(1, 0, E).index_select(0, vg_bwd[0]));
    (void)hipStreamWaitEvent(st, aux.ev[5], 0);
    if (grad_ev) record_grad_event(aux.grad_ev[2], st, 2);
  }
  at::Tensor dh0;
  if (has_s0)  // step 0's recurrent input h0: dh0 = dG_0 W_hh
    dh0 = at::mm(dG2.narrow(0, 0, R), wx.narrow(1, E, H), at::kFloat);
  std::vector<at::Tensor> res;
  if (!has_att) {
    (void)hipStreamWaitEvent(st, aux.ev[5], 0);  // dvg (second side stream, above)
  } else {
    // dGv[b, c] = sum_{t, rows of b} alpha[t, r, c] dG_t[r] (kernels/attention.hip:
    // one pass over the bf16 dG rows, partials per step chunk)
    at::Tensor dGv;
    if (C <= 8) {  // (computed on the side stream after the loop)
      (void)hipStreamWaitEvent(st, aux.ev[5], 0);
      dGv = dGv_side;
    } else {  // one batched GEMM per (step, video), K = rows per video
      at::Tensor al = a_alpha.to(at::kBFloat16).view({n_steps * Bv, vdiv, C}).transpose(1, 2);
      at::Tensor dgv = dG_all.view({n_steps * Bv, vdiv, KD}).narrow(2, 0, H4);
      dGv = at::bmm(al, dgv, at::kFloat).view({n_steps, Bv, C, H4}).sum(0);
    }
    if (att_mfma) {
      res = {dGv, dpre_part, dwa_part.sum(0).view_as(a_wa), dba_part.sum(0).view({1}), dWq};
    } else {
      const int64_t ng = att_groups((int)vdiv);
      res = {dGv, dpre_part.view({Bv, ng, C, A}).sum(1), dwa_part.sum(0).view_as(a_wa),
             dba_part.sum(0).view({NWA}), dWq};
    }
  }
  stamp(STAMP_BWD_END, st);
  // (The bias column sums at the end of the main chain, which ends ~0.3 ms
  // before the side stream's in step_timeline_r2_v20.txt, measured slower:
  // 3.86-3.88 vs 3.76-3.86 ms, they contend with the dW_logit GEMM;
  // profiles/r2/ab_colsum_main.txt.)
  // join the side stream (dW_logit): every tensor it touched was allocated
  // on the main stream and is released after this point
  (void)hipStreamWaitEvent(st, ev_done, 0);
  std::vector<at::Tensor> out = {dWx, dWlog, dblog, d_emb, dvg};
  out.insert(out.end(), res.begin(), res.end());
  if (has_s0) {
    out.push_back(dh0);
    out.push_back(dc);  // carry into step -1 (LSTM: dc0; GRU / RNN: direct dh0 term)
  }
  for (int64_t l = 1; l < NL; ++l) {  // dW_l = dG_l^T [hd_{l-1, t} | h_{l, t-1}]
    at::Tensor dWu = at::empty({H4, 2 * H}, f32);
    at::Tensor dGl = dG_up[l].view({NR, H4});
    dWu.narrow(1, 0, H).copy_(grouped_wgrad(dGl, upw(l, 4).reshape({NR, H}), n_steps));
    if (n_steps > 1)
      dWu.narrow(1, H, H).copy_(grouped_wgrad(
          dGl.narrow(0, R, (n_steps - 1) * R),
          upw(l, 1).narrow(0, 0, n_steps - 1).reshape({(n_steps - 1) * R, H}), n_steps - 1));
    else
      dWu.narrow(1, H, H).zero_();
    out.push_back(dWu);
  }
  return out;
}

// FeatPool (csrc/kernels/featpool.hip): xs[f] (rows, d_f), ws[f] (H, d_f),
// bs[f] (H), all fp32 contiguous GPU tensors; returns the concatenated
// (rows, F*H) output after ReLU and dropout (mask from rng slot 0).
static FeatPoolArgs featpool_args(const std::vector<at::Tensor>& xs,
                                  const std::vector<at::Tensor>& ws,
                                  const std::vector<at::Tensor>& bs) {
  TORCH_CHECK(!xs.empty() && xs.size() <= FEATPOOL_MAX_F && ws.size() == xs.size() &&
                  (bs.empty() || bs.size() == xs.size()),
              "featpool: 1..", FEATPOOL_MAX_F, " modalities, one weight (and bias) each");
  FeatPoolArgs a{};
  a.nf = (int)xs.size();
  a.rows = (int)xs[0].size(0);
  a.H = (int)ws[0].size(0);
  TORCH_CHECK(a.H % 64 == 0, "featpool: output size must be a multiple of 64");
  for (int f = 0; f < a.nf; ++f) {
    const at::Tensor &x = xs[f], &w = ws[f];
    // x may be a column slice of a wider row (the loader gathers every
    // modality in one pass): unit column stride, 16-byte-aligned rows
    TORCH_CHECK(x.is_cuda(), "featpool x must be a GPU tensor");
    check_cuda(w, "featpool w");
    TORCH_CHECK(x.scalar_type() == at::kFloat && w.scalar_type() == at::kFloat && x.dim() == 2 &&
                    w.dim() == 2 && x.size(0) == a.rows && w.size(0) == a.H &&
                    x.size(1) == w.size(1) && x.size(1) % 4 == 0 &&
                    (x.size(1) == 1 || x.stride(1) == 1) && x.stride(0) % 4 == 0 &&
                    x.stride(0) >= x.size(1) &&
                    reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
                "featpool: fp32 x (rows, d) with unit column stride and 16-byte-aligned rows, "
                "w (H, d), d % 4 == 0");
    a.s[f].x = x.data_ptr<float>();
    a.s[f].w = w.data_ptr<float>();
    if (!bs.empty()) {
      check_cuda(bs[f], "featpool b");
      TORCH_CHECK(bs[f].scalar_type() == at::kFloat && bs[f].numel() == a.H, "featpool: bias (H)");
      a.s[f].b = bs[f].data_ptr<float>();
    }
    a.s[f].d = (int)x.size(1);
    a.s[f].ld = (int)x.stride(0);
  }
  featpool_layout(a);
  return a;
}

at::Tensor featpool_forward(std::vector<at::Tensor> xs, std::vector<at::Tensor> ws,
                            std::vector<at::Tensor> bs, double drop_p, at::Tensor rng) {
  TORCH_CHECK(bs.size() == xs.size(), "featpool: one bias per modality");
  FeatPoolArgs a = featpool_args(xs, ws, bs);
  auto f32 = xs[0].options();
  at::Tensor wsp = at::empty({(int64_t)a.fwd_blocks * 64 * 64}, f32);
  at::Tensor out = at::empty({a.rows, (int64_t)a.nf * a.H}, f32);
  launch_featpool_fwd(a, wsp.data_ptr<float>(), out.data_ptr<float>(), (float)drop_p,
                      rng_ptr(rng), cur_stream());
  return out;
}

// -> {dW_0 .. dW_{F-1}, db_0 .. db_{F-1}} given dL/d(out) and the forward's out;
// written into `outs` (2F contiguous fp32 tensors, e.g. gradient-bucket
// slots) when given
std::vector<at::Tensor> featpool_backward(at::Tensor dout, at::Tensor out,
                                          std::vector<at::Tensor> xs,
                                          std::vector<at::Tensor> ws, double drop_p,
                                          std::vector<at::Tensor> outs) {
  FeatPoolArgs a = featpool_args(xs, ws, {});
  check_cuda(dout, "featpool dout");
  check_cuda(out, "featpool out");
  TORCH_CHECK(dout.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat &&
                  dout.numel() == (int64_t)a.rows * a.nf * a.H && out.numel() == dout.numel(),
              "featpool: dout / out (rows, F*H) fp32");
  std::vector<at::Tensor> res;
  FeatPoolGrads g{};
  if (!outs.empty()) {
    TORCH_CHECK((int)outs.size() == 2 * a.nf, "featpool: outs = {dW_f} + {db_f}");
    for (int f = 0; f < a.nf; ++f) {
      TORCH_CHECK(outs[f].is_cuda() && outs[f].is_contiguous() &&
                      outs[f].scalar_type() == at::kFloat && outs[f].numel() == ws[f].numel() &&
                      outs[a.nf + f].is_cuda() && outs[a.nf + f].is_contiguous() &&
                      outs[a.nf + f].scalar_type() == at::kFloat && outs[a.nf + f].numel() == a.H,
                  "featpool: output slots must be contiguous fp32 (H, d) / (H)");
    }
    res = outs;
  } else {
    for (int f = 0; f < a.nf; ++f) res.push_back(at::empty_like(ws[f]));
    for (int f = 0; f < a.nf; ++f) res.push_back(at::empty({a.H}, ws[f].options()));
  }
  for (int f = 0; f < a.nf; ++f) {
    g.dw[f] = res[f].data_ptr<float>();
    g.db[f] = res[a.nf + f].data_ptr<float>();
  }
  launch_featpool_bwd(a, dout.data_ptr<float>(), out.data_ptr<float>(), (float)drop_p, g,
                      cur_stream());
  return res;
}

// SCST loss (csrc/kernels/loss.hip): seq (R, T) int64, lp (R, T) fp32,
// sample (R), greedy (R or R / gdiv) fp32 -> {loss (0-dim), out = [loss, m, b,
// sum mask], reward (R)}
std::vector<at::Tensor> scst_loss_forward(at::Tensor seq, at::Tensor lp, at::Tensor sample,
                                          at::Tensor greedy) {
  for (auto* t : {&seq, &lp, &sample, &greedy}) check_cuda(*t, "scst_loss operand");
  const int64_t R = seq.size(0), T = seq.size(1);
  TORCH_CHECK(seq.scalar_type() == at::kLong && lp.scalar_type() == at::kFloat &&
                  lp.size(0) == R && lp.size(1) == T && sample.scalar_type() == at::kFloat &&
                  sample.numel() == R && greedy.scalar_type() == at::kFloat &&
                  greedy.numel() > 0 && R % greedy.numel() == 0,
              "scst_loss: seq / lp (R, T), sample (R), greedy (R or R / rows per video)");
  auto f32 = lp.options();
  at::Tensor out = at::empty({4}, f32), reward = at::empty({R}, f32), loss = at::empty({}, f32);
  at::Tensor ws = at::zeros({scst_loss_ws_ints((int)R)}, f32.dtype(at::kInt));
  launch_scst_loss_fwd(seq.data_ptr<int64_t>(), lp.data_ptr<float>(), (int)R, (int)T,
                       sample.data_ptr<float>(), greedy.data_ptr<float>(),
                       (int)(R / greedy.numel()), reward.data_ptr<float>(), out.data_ptr<float>(),
                       loss.data_ptr<float>(), ws.data_ptr<int>(), CstBase{nullptr, 0, 0},
                       cur_stream());
  return {loss, out, reward};
}

// CST loss (the same launch, consensus baseline): scores (R) fp32 of the
// rewarded rows, S rows per video (R % S == 0, S <= 64); bref: (R) GT
// consensus scores (scb_baseline 1) or empty (scb_baseline 2: the scores
// themselves); k = scb_captions (0: reward = score) -> {loss, out, reward}
std::vector<at::Tensor> cst_loss_forward(at::Tensor seq, at::Tensor lp, at::Tensor scores,
                                         at::Tensor bref, int64_t S, int64_t k) {
  for (auto* t : {&seq, &lp, &scores}) check_cuda(*t, "cst_loss operand");
  const int64_t R = seq.size(0), T = seq.size(1);
  const bool has_ref = bref.defined() && bref.numel() > 0;
  TORCH_CHECK(seq.scalar_type() == at::kLong && lp.scalar_type() == at::kFloat &&
                  lp.size(0) == R && lp.size(1) == T && scores.scalar_type() == at::kFloat &&
                  scores.numel() == R && S >= 1 && S <= 64 && R % S == 0 && k >= 0 && k <= S,
              "cst_loss: seq / lp (R, T), scores (R), 1 <= S <= 64 dividing R, 0 <= k <= S");
  if (has_ref) {
    check_cuda(bref, "cst_loss bref");
    TORCH_CHECK(bref.scalar_type() == at::kFloat && bref.numel() == R, "cst_loss: bref (R) fp32");
  }
  auto f32 = lp.options();
  at::Tensor out = at::empty({4}, f32), reward = at::empty({R}, f32), loss = at::empty({}, f32);
  at::Tensor ws = at::zeros({scst_loss_ws_ints((int)R)}, f32.dtype(at::kInt));
  launch_scst_loss_fwd(seq.data_ptr<int64_t>(), lp.data_ptr<float>(), (int)R, (int)T,
                       scores.data_ptr<float>(), scores.data_ptr<float>(), 1,
                       reward.data_ptr<float>(), out.data_ptr<float>(), loss.data_ptr<float>(),
                       ws.data_ptr<int>(),
                       CstBase{has_ref ? bref.data_ptr<float>() : nullptr, (int)S, (int)k},
                       cur_stream());
  return {loss, out, reward};
}

at::Tensor scst_loss_backward(at::Tensor seq, at::Tensor reward, at::Tensor out,
                              at::Tensor dloss) {
  for (auto* t : {&seq, &reward, &out, &dloss}) check_cuda(*t, "scst_loss operand");
  TORCH_CHECK(dloss.scalar_type() == at::kFloat && dloss.numel() == 1, "dloss: fp32 scalar");
  const int64_t R = seq.size(0), T = seq.size(1);
  at::Tensor dlp = at::empty({R, T}, reward.options());
  launch_scst_loss_bwd(seq.data_ptr<int64_t>(), reward.data_ptr<float>(), out.data_ptr<float>(),
                       dloss.data_ptr<float>(), (int)R, (int)T, dlp.data_ptr<float>(),
                       cur_stream());
  return dlp;
}

// XE loss (csrc/kernels/loss.hip): labels (R, L) int64 -- the full label
// rows the loader's masks come from --, lp (R, T) fp32 gathered GT log-probs
// of columns off .. off + T - 1 -> {loss (0-dim), out = [loss, sum mask], cnt
// (R) counted positions per row}
std::vector<at::Tensor> xe_loss_forward(at::Tensor labels, at::Tensor lp, int64_t off) {
  check_cuda(labels, "xe_loss labels");
  check_cuda(lp, "xe_loss lp");
  const int64_t R = labels.size(0), L = labels.size(1), T = lp.size(1);
  TORCH_CHECK(labels.scalar_type() == at::kLong && lp.scalar_type() == at::kFloat &&
                  labels.dim() == 2 && lp.dim() == 2 && lp.size(0) == R && off >= 0 &&
                  off + T <= L,
              "xe_loss: labels (R, L) int64, lp (R, T) fp32 with off + T <= L");
  auto f32 = lp.options();
  at::Tensor out = at::empty({2}, f32), cnt = at::empty({R}, f32), loss = at::empty({}, f32);
  at::Tensor ws = at::zeros({scst_loss_ws_ints((int)R)}, f32.dtype(at::kInt));
  launch_xe_loss_fwd(labels.data_ptr<int64_t>(), (int)L, (int)off, lp.data_ptr<float>(), (int)R,
                     (int)T, cnt.data_ptr<float>(), out.data_ptr<float>(), loss.data_ptr<float>(),
                     ws.data_ptr<int>(), cur_stream());
  return {loss, out, cnt};
}

at::Tensor xe_loss_backward(at::Tensor cnt, at::Tensor out, at::Tensor dloss, int64_t T) {
  for (auto* t : {&cnt, &out, &dloss}) check_cuda(*t, "xe_loss operand");
  TORCH_CHECK(dloss.scalar_type() == at::kFloat && dloss.numel() == 1 &&
                  cnt.scalar_type() == at::kFloat && out.numel() == 2,
              "xe_loss_backward: fp32 cnt (R), out (2), dloss scalar");
  const int64_t R = cnt.size(0);
  at::Tensor dlp = at::empty({R, T}, cnt.options());
  launch_xe_loss_bwd(cnt.data_ptr<float>(), out.data_ptr<float>(), dloss.data_ptr<float>(), (int)R,
                     (int)T, dlp.data_ptr<float>(), cur_stream());
  return dlp;
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

// Shadow-copy segments from Python: meta = int64 CPU (n, 8) rows {off, n,
// kind, cols, H, E, ld2, slots}; dsts = 2 tensors per row (dst, dst2; undefined or
// empty when unused).
static ShadowSegs make_shadow_segs(const at::Tensor& meta, const std::vector<at::Tensor>& dsts) {
  ShadowSegs ss{};
  if (!meta.defined() || meta.numel() == 0) return ss;
  TORCH_CHECK(!meta.is_cuda() && meta.scalar_type() == at::kLong && meta.dim() == 2 &&
                  meta.size(1) == 8 && meta.size(0) <= SHADOW_MAX_SEGS,
              "shadow meta must be an int64 CPU (n <= ", SHADOW_MAX_SEGS, ", 8) tensor");
  TORCH_CHECK((int64_t)dsts.size() == 2 * meta.size(0), "two destination tensors per segment");
  auto m = meta.accessor<int64_t, 2>();
  ss.n = (int)meta.size(0);
  for (int k = 0; k < ss.n; ++k) {
    ShadowSeg& g = ss.s[k];
    g.off = m[k][0], g.n = m[k][1], g.kind = (int)m[k][2], g.cols = (int)m[k][3];
    g.H = (int)m[k][4], g.E = (int)m[k][5], g.ld2 = (int)m[k][6], g.slots = (int)m[k][7];
    const at::Tensor& d = dsts[2 * k];
    const at::Tensor& d2 = dsts[2 * k + 1];
    TORCH_CHECK(d.is_cuda() && d.scalar_type() == at::kBFloat16, "shadow dst must be bf16 GPU");
    g.dst = reinterpret_cast<uint16_t*>(d.data_ptr());
    g.dst2 = d2.defined() && d2.numel() ? reinterpret_cast<uint16_t*>(d2.data_ptr()) : nullptr;
    if (g.kind == SHADOW_PLAIN) {
      TORCH_CHECK(d.numel() >= g.n, "plain shadow too small");
    } else {
      const int64_t rows = g.cols > 0 ? g.n / g.cols : 0;
      const int64_t gates = g.H > 0 ? rows / g.H : 0;
      TORCH_CHECK(g.H > 0 && g.cols > 0 && g.n % g.cols == 0 && rows % g.H == 0 &&
                      (gates == 1 || gates == 3 || gates == 4) &&
                      d.numel() >= 4 * (int64_t)g.H * (g.E + g.H),
                  "gate-weight shadow segment shape");
      for (int q = 0; q < gates; ++q)
        for (int q2 = 0; q2 < q; ++q2)
          TORCH_CHECK(((g.slots >> (2 * q)) & 3) != ((g.slots >> (2 * q2)) & 3),
                      "gate slot map must be injective");
      if (g.kind == SHADOW_GATES_HH)
        TORCH_CHECK(g.dst2 != nullptr && g.cols == g.H && d2.numel() >= 4 * (int64_t)g.H * g.ld2,
                    "W_hh shadow needs its packed copy");
      if (g.kind == SHADOW_GATES_IH && g.dst2 != nullptr)
        TORCH_CHECK(g.cols > g.E && g.ld2 >= g.cols - g.E && d2.numel() >= 4 * (int64_t)g.H * g.ld2,
                    "W_ih video-column shadow shape");
    }
  }
  return ss;
}

// hyper (device fp32): [lr, step before, skipped, step after] (kernels/adam.hip).
// phase: 0 = both passes; 1 = sum of squares only (the caller all-reduces the
// partials of a sharded update before phase 2); 2 = update only.
at::Tensor flat_adam_step(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v,
                          at::Tensor partials, at::Tensor scal, at::Tensor skip, at::Tensor hyper,
                          double b1, double b2, double eps, double clip, double gscale,
                          int64_t phase, at::Tensor shadow_meta,
                          std::vector<at::Tensor> shadow_dst) {
  check_cuda(p, "p");
  for (auto* t : {&g, &m, &v}) {
    check_cuda(*t, "adam operand");
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == p.numel(), "adam operand shape");
  }
  TORCH_CHECK(partials.numel() >= 1024 && scal.numel() >= 2, "workspace too small");
  TORCH_CHECK(hyper.is_cuda() && hyper.scalar_type() == at::kFloat && hyper.numel() >= 4,
              "hyper must be fp32 [lr, step, skipped, step after] on the GPU");
  TORCH_CHECK(phase >= 0 && phase <= 2, "phase: 0 both, 1 sumsq, 2 update");
  const ShadowSegs ss = make_shadow_segs(shadow_meta, shadow_dst);
  for (int k = 0; k < ss.n; ++k)
    TORCH_CHECK(ss.s[k].off >= 0 && ss.s[k].off + ss.s[k].n <= p.numel(), "shadow range");
  launch_flat_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                   v.data_ptr<float>(), p.numel(), partials.data_ptr<float>(),
                   skip.data_ptr<bool>(), scal.data_ptr<float>(), hyper.data_ptr<float>(),
                   (float)b1, (float)b2, (float)eps, (float)clip, (float)gscale, (int)phase, ss,
                   cur_stream());
  return scal.narrow(0, 0, 1).squeeze(0);
}

void refresh_shadows(at::Tensor p, at::Tensor shadow_meta, std::vector<at::Tensor> shadow_dst) {
  check_cuda(p, "p");
  const ShadowSegs ss = make_shadow_segs(shadow_meta, shadow_dst);
  for (int k = 0; k < ss.n; ++k)
    TORCH_CHECK(ss.s[k].off >= 0 && ss.s[k].off + ss.s[k].n <= p.numel(), "shadow range");
  launch_shadow_refresh(p.data_ptr<float>(), ss, cur_stream());
}

// Batched beam search (reference sample_beam, model.py:369-512) for B videos
// x K beams, entirely on the GPU: per step one LSTM launch (h/c of each row's
// parent beam via row_map), one vocab launch (fp32 logits + LSE partials),
// the LSE combine, a top-K launch and one beam-step launch.  Returns
// {best_seq (B, T) int64, best_logprobs (B, T) fp32}, T = seq_length,
// padded with zeros like the reference.
std::vector<at::Tensor> beam_search(at::Tensor wx, at::Tensor ptab, at::Tensor whh,
                                    at::Tensor wlog, at::Tensor blog, at::Tensor vgate,
                                    int64_t K, int64_t T, int64_t bos_index,
                                    std::vector<at::Tensor> att, int64_t cell,
                                    std::vector<at::Tensor> state0, std::vector<at::Tensor> up) {
  check_cuda(wx, "wx");
  check_cuda(vgate, "vgate");
  TORCH_CHECK(K >= 1 && K <= 16, "beam_size must be in [1, 16]");
  const int64_t H4 = wx.size(0), H = H4 / 4, V = wlog.size(0), B = vgate.size(0), R = B * K;
  TORCH_CHECK(K <= V, "beam_size > vocab_size");
  // temporal attention: att = {Gv, P, W_q, w_a, b_a} as in decoder_forward; the
  // query of a beam row comes from its parent's h (q rows gathered by parent)
  const bool has_att = !att.empty();
  int64_t C = 0, A = 0;
  at::Tensor vg_rows, qb;
  if (has_att) {
    TORCH_CHECK(att.size() == 5 && att[0].size(0) == B && att[0].size(2) == H4,
                "att = {Gv (B, C, 4H), P, W_q, w_a, b_a}");
    C = att[0].size(1), A = att[1].size(2);
    TORCH_CHECK(A % 64 == 0 && C >= 1 && C <= 32 &&
                    att[2].size(0) == A && att[2].size(1) == H, "attention shapes");
    TORCH_CHECK(att[3].numel() == A || (C > 1 && C <= 8 && att[3].numel() == C * A &&
                                        att[4].numel() == C), "w_a / b_a shapes");
  }
  const int per_frame = has_att && C > 1 && att[3].numel() == C * A ? 1 : 0;
  auto dev = wx.device();
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
  auto i64 = at::TensorOptions().dtype(at::kLong).device(dev);
  auto i32 = at::TensorOptions().dtype(at::kInt).device(dev);
  hipStream_t st = cur_stream();
  const int64_t ldl = (V + 7) / 8 * 8;
  const int n_vt = vocab_num_tiles((int)V);
  // K <= 8: the vocab launch keeps each tile's K best logits per row (VF_TOPK)
  // and the top-K merges n_vt * K candidates -- no R x V fp32 logits
  const bool tile_topk = K <= 8;
  at::Tensor logits = tile_topk ? at::empty({(int64_t)n_vt * R * K * 2}, f32) : at::empty({R, ldl}, f32);
  at::Tensor lse = at::empty({R}, f32);
  at::Tensor part = at::empty({(int64_t)n_vt * R * vocab_partial_bytes() / 4}, f32);
  at::Tensor top_v = at::empty({R, K}, f32);
  at::Tensor top_i = at::empty({R, K}, i32);
  at::Tensor beam_sum = at::zeros({R}, f32);
  at::Tensor seq_hist = at::zeros({2, R, T}, i64);
  at::Tensor lp_hist = at::zeros({2, R, T}, f32);
  at::Tensor best_ppl = at::full({B}, INFINITY, f32);
  at::Tensor best_seq = at::zeros({B, T}, i64);
  at::Tensor best_lp = at::zeros({B, T}, f32);
  at::Tensor tok = at::full({R}, bos_index, i64);
  at::Tensor parent = at::empty({R}, i32);
  // stacked layers: up = {[W_ih | W_hh] (4H, 2H), W_hh (4H, H)} per upper layer
  TORCH_CHECK(up.size() % 2 == 0, "up = {[W_ih | W_hh], W_hh} per upper layer");
  const int64_t NL = 1 + (int64_t)up.size() / 2;
  if (NL > 1) TORCH_CHECK(!has_att && state0.empty(), "stacked layers: no attention / initial state");
  std::vector<std::array<at::Tensor, 2>> hl(NL), cl(NL);
  for (int64_t l = 0; l < NL; ++l) {
    hl[l] = {at::zeros({R, H}, wx.options()), at::empty({R, H}, wx.options())};
    cl[l] = {at::zeros({R, H}, f32), at::empty({R, H}, f32)};
  }
  at::Tensor xin = NL > 1 ? at::empty({R, H4}, f32) : at::Tensor();
  at::Tensor* h = hl[0].data();
  at::Tensor* c = cl[0].data();
  if (!state0.empty()) {  // per-video initial state {h0 (B, H), c0 (B, H)}, one copy per beam
    TORCH_CHECK(state0.size() == 2 && !has_att && state0[0].size(0) == B &&
                    state0[1].size(0) == B && state0[0].size(1) == H && state0[1].size(1) == H,
                "state0 = {h0, c0} (B, H), without attention");
    h[0].copy_(state0[0].repeat_interleave(K, 0));
    c[0].copy_(state0[1].repeat_interleave(K, 0));
  }
  const uint16_t* W = reinterpret_cast<const uint16_t*>(wlog.data_ptr());
  const uint16_t* WHH = reinterpret_cast<const uint16_t*>(whh.data_ptr());
  // (MFMA attention for the beam rows -- parent-gathered query input, the
  // decode launch's attention workgroups on their own -- measured slower,
  // 26.0k vs 29.6k videos/s at att8 beam 5, profiles/r4/README_r4.md)
  if (has_att) {
    vg_rows = at::empty({R, H4}, f32);
    qb = at::empty({R, A}, f32);
  }
  // Fused form (one layer, no attention, K <= 8): per decode step TWO launches
  // -- the vocab launch (tile top-K candidates + partials) carrying the NEXT
  // step's recurrent GEMM pre = h W_hh^T + video gates for every current row,
  // then beam_fused_step_kernel (LSE, candidate top-K, selection / fork /
  // harvest, and the cell of the new beams from their parents' pre and c) --
  // instead of five (vocab, combine, top-K merge, beam step, LSTM step).
  // With temporal attention (MFMA shape) the vocab launch also carries the
  // attention workgroups: every current row's next video gates (bf16) from
  // its own h_t, which the fused step adds for the parent like pre.
  const bool att_fused = has_att && !per_frame && att_mfma_ok((int)K, (int)C, (int)A, (int)H, 0);
  if (tile_topk && NL == 1 && (!has_att || att_fused)) {
    at::Tensor pre = at::empty({R, H4}, f32);
    const float* VG = has_att ? nullptr : vgate.data_ptr<float>();
    at::Tensor gv16, vg16, att_ep, att_cnt;
    const int CPAD = C <= 8 ? 8 : 16;
    if (has_att) {
      gv16 = at::zeros({B, H4, CPAD}, wx.options());  // frame-minor, frames zero-padded
      gv16.narrow(2, 0, C).copy_(att[0].transpose(1, 2));
      vg16 = at::empty({R, H4}, wx.options());
      att_ep = at::empty({B, A / 64, 32, CPAD}, f32);
      att_cnt = at::zeros({B}, at::TensorOptions().dtype(at::kInt).device(wx.device()));
      // step 0 (q = 0): the VALU scorer's fp32 video gates of every row
      launch_att_fwd(att[0].data_ptr<float>(), att[1].data_ptr<float>(), nullptr, nullptr,
                     att[3].data_ptr<float>(), att[4].data_ptr<float>(), (int)B, (int)K, (int)C,
                     (int)A, (int)H4, vg_rows.data_ptr<float>(), nullptr, st, 0, per_frame);
    }
    // step 0: every row's cell from the initial state and BOS
    launch_lstm_step_fwd(tok.data_ptr<int64_t>(), 1, reinterpret_cast<const uint16_t*>(ptab.data_ptr()),
                         reinterpret_cast<const uint16_t*>(h[0].data_ptr()), c[0].data_ptr<float>(),
                         has_att ? vg_rows.data_ptr<float>() : VG, has_att ? 1 : (int)K, (int)R,
                         (int)H, WHH,
                         reinterpret_cast<uint16_t*>(h[1].data_ptr()), c[1].data_ptr<float>(),
                         nullptr, (int)H, 0.f, nullptr, 0, nullptr, st, nullptr, (int)cell);
    for (int64_t t = 1; t < T - 1; ++t) {
      // vocab projection of h_t (rows = beams of step t) + pre_{t+1} of every row
      const at::Tensor& ht = h[t & 1];
      const bool next = t < T - 2;
      AttMfmaArgs am{};
      if (has_att && next)
        am = AttMfmaArgs{reinterpret_cast<const uint16_t*>(ht.data_ptr()),
                         reinterpret_cast<const uint16_t*>(att[2].data_ptr()),
                         att[1].data_ptr<float>(), att[3].data_ptr<float>(),
                         att[4].data_ptr<float>(), reinterpret_cast<const uint16_t*>(gv16.data_ptr()),
                         (int)H, (int)A, (int)C, CPAD, (int)H4, (int)K, (int)B,
                         reinterpret_cast<uint16_t*>(vg16.data_ptr()), nullptr, nullptr,
                         att_ep.data_ptr<float>(), att_cnt.data_ptr<int>()};
      if (has_att && next) am.whole = att_mfma_whole_default((int)C, (int)H);
      (void)launch_vocab_lstm_fwd(reinterpret_cast<const uint16_t*>(ht.data_ptr()), (int)H, (int)R,
                                  (int)H, W, blog.data_ptr<float>(), (int)V,
                                  reinterpret_cast<uint16_t*>(logits.data_ptr()), ldl,
                                  part.data_ptr(), nullptr, 0, VF_TOPK_H | ((int)K << 8), 1.f,
                                  nullptr, (int)t, reinterpret_cast<const uint16_t*>(ht.data_ptr()),
                                  WHH, VG, (int)K, next ? pre.data_ptr<float>() : nullptr, st, 0,
                                  nullptr, nullptr, has_att && next ? &am : nullptr);
      BeamFusedArgs ba{reinterpret_cast<const VocabPartial*>(part.data_ptr()),
                       reinterpret_cast<const float2*>(logits.data_ptr()), n_vt, (int)R, (int)K,
                       (int)B, (int)T, beam_sum.data_ptr<float>(), seq_hist.data_ptr<int64_t>(),
                       lp_hist.data_ptr<float>(), best_ppl.data_ptr<float>(),
                       best_seq.data_ptr<int64_t>(), best_lp.data_ptr<float>(),
                       tok.data_ptr<int64_t>(), next ? pre.data_ptr<float>() : nullptr,
                       reinterpret_cast<const uint16_t*>(ptab.data_ptr()), c[t & 1].data_ptr<float>(),
                       c[(t + 1) & 1].data_ptr<float>(),
                       reinterpret_cast<uint16_t*>(h[(t + 1) & 1].data_ptr()), (int)H, (int)cell,
                       has_att && next ? reinterpret_cast<const uint16_t*>(vg16.data_ptr())
                                       : nullptr};
      launch_beam_fused_step(ba, (int)t, st);
    }
    return {best_seq, best_lp};
  }
  for (int64_t t = 0; t < T - 1; ++t) {
    if (t >= 1) {
      if (tile_topk)
        launch_beam_topk_cand(logits.data_ptr(), n_vt, (int)R, (int)K, lse.data_ptr<float>(),
                              top_v.data_ptr<float>(), top_i.data_ptr<int>(), st);
      else
        launch_beam_topk(logits.data_ptr<float>(), ldl, (int)V, (int)R, (int)K,
                         lse.data_ptr<float>(), top_v.data_ptr<float>(), top_i.data_ptr<int>(),
                         st);
      launch_beam_step(top_v.data_ptr<float>(), top_i.data_ptr<int>(), (int)B, (int)K, (int)T,
                       (int)t, beam_sum.data_ptr<float>(), seq_hist.data_ptr<int64_t>(),
                       lp_hist.data_ptr<float>(), best_ppl.data_ptr<float>(),
                       best_seq.data_ptr<int64_t>(), best_lp.data_ptr<float>(),
                       tok.data_ptr<int64_t>(), parent.data_ptr<int>(), st);
      if (t == T - 2) break;  // the reference's last LSTM step feeds nothing
    }
    const at::Tensor& hp = h[t & 1];
    const at::Tensor& cp = c[t & 1];
    at::Tensor& ho = h[(t + 1) & 1];
    at::Tensor& co = c[(t + 1) & 1];
    if (has_att) {
      if (t >= 1) at::mm_out(qb, hp, att[2].t(), at::kFloat);
      launch_att_fwd(att[0].data_ptr<float>(), att[1].data_ptr<float>(),
                     t >= 1 ? qb.data_ptr<float>() : nullptr, t >= 1 ? parent.data_ptr<int>() : nullptr,
                     att[3].data_ptr<float>(), att[4].data_ptr<float>(), (int)B, (int)K, (int)C,
                     (int)A, (int)H4, vg_rows.data_ptr<float>(), nullptr, st, 0, per_frame);
    }
    launch_lstm_step_fwd(tok.data_ptr<int64_t>(), 1, reinterpret_cast<const uint16_t*>(ptab.data_ptr()),
                         reinterpret_cast<const uint16_t*>(hp.data_ptr()), cp.data_ptr<float>(),
                         has_att ? vg_rows.data_ptr<float>() : vgate.data_ptr<float>(),
                         has_att ? 1 : (int)K, (int)R, (int)H, WHH,
                         reinterpret_cast<uint16_t*>(ho.data_ptr()), co.data_ptr<float>(), nullptr,
                         (int)H, 0.f, nullptr, (int)t, nullptr, st,
                         t >= 1 ? parent.data_ptr<int>() : nullptr, (int)cell);
    for (int64_t l = 1; l < NL; ++l) {  // upper layers: their state follows the parent beam too
      at::mm_out(xin, hl[l - 1][(t + 1) & 1], up[2 * (l - 1)].narrow(1, 0, H).t(), at::kFloat);
      launch_lstm_step_fwd(nullptr, 0, nullptr,
                           reinterpret_cast<const uint16_t*>(hl[l][t & 1].data_ptr()),
                           cl[l][t & 1].data_ptr<float>(), xin.data_ptr<float>(), 1, (int)R,
                           (int)H, reinterpret_cast<const uint16_t*>(up[2 * (l - 1) + 1].data_ptr()),
                           reinterpret_cast<uint16_t*>(hl[l][(t + 1) & 1].data_ptr()),
                           cl[l][(t + 1) & 1].data_ptr<float>(), nullptr, (int)H, 0.f, nullptr,
                           (int)t, nullptr, st, t >= 1 ? parent.data_ptr<int>() : nullptr,
                           (int)cell);
    }
    const at::Tensor& htop = hl[NL - 1][(t + 1) & 1];
    launch_vocab_fwd(reinterpret_cast<const uint16_t*>(htop.data_ptr()), (int)H, (int)R, (int)H, W,
                     blog.data_ptr<float>(), (int)V,
                     reinterpret_cast<uint16_t*>(logits.data_ptr()), ldl, part.data_ptr(),
                     nullptr, 0, tile_topk ? (VF_TOPK_H | ((int)K << 8)) : /*fp32 logits*/ 8, 1.f,
                     nullptr, (int)t, st);
    launch_vocab_combine(part.data_ptr(), n_vt, (int)R, lse.data_ptr<float>(), nullptr, 0,
                         nullptr, 0, nullptr, 0, nullptr, 0, SEL_GT_H, 0.f, nullptr, (int)t, nullptr,
                         0, nullptr, st);
  }
  return {best_seq, best_lp};
}

// Microbenchmarks of single kernels (scripts/microbench_kernels.py): mean
// microseconds per launch over `iters` back-to-back launches, HIP events.
template <class F>
static double time_launches(F&& launch, int64_t iters, hipStream_t st) {
  launch(0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < iters; ++i) launch(i);
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return 1000.0 * ms / (double)iters;
}

double vocab_fwd_bench(at::Tensor hd, at::Tensor wlog, at::Tensor blog, at::Tensor tgt,
                       int64_t flags, bool save, int64_t iters, int64_t variant) {
  const int64_t R = hd.size(0), H = hd.size(1), V = wlog.size(0);
  TORCH_CHECK(H % 64 == 0 && wlog.size(1) == H && blog.numel() == V, "shapes");
  auto dev = hd.device();
  const int64_t ldl = (V + 7) / 8 * 8;
  at::Tensor logits = save ? at::empty({R, ldl}, hd.options().dtype(at::kHalf)) : at::Tensor();
  const int n_vt = vocab_num_tiles((int)V);
  at::Tensor part = at::empty({(int64_t)n_vt * R * vocab_partial_bytes() / 4},
                              at::TensorOptions().dtype(at::kFloat).device(dev));
  at::Tensor rng = at::full({2}, 1234, at::TensorOptions().dtype(at::kInt).device(dev));
  const int64_t* tg = tgt.defined() && tgt.numel() ? tgt.data_ptr<int64_t>() : nullptr;
  hipStream_t st = cur_stream();
  return time_launches(
      [&](int i) {
        launch_vocab_fwd_variant((int)variant, reinterpret_cast<const uint16_t*>(hd.data_ptr()),
                                 (int)H, (int)R, (int)H,
                                 reinterpret_cast<const uint16_t*>(wlog.data_ptr()),
                                 blog.data_ptr<float>(), (int)V,
                                 save ? reinterpret_cast<uint16_t*>(logits.data_ptr()) : nullptr,
                                 ldl, part.data_ptr(), tg, 1, (int)flags, 1.f, rng_ptr(rng), i, st);
      },
      iters, st);
}

// bias-gradient column sums over the exp store: E (n, R, ldl) bf16, alpha (n*R)
double vgrad_colsum_bench(at::Tensor E, at::Tensor alpha, int64_t V, int64_t iters) {
  check_cuda(E, "E");
  const int64_t NR = E.size(0) * E.size(1), ldl = E.size(2);
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(E.device());
  at::Tensor part = at::empty({vgrad_colsum_blocks(NR), V}, f32), db = at::empty({V}, f32);
  hipStream_t st = cur_stream();
  return time_launches(
      [&](int) {
        launch_vgrad_colsum(reinterpret_cast<const uint16_t*>(E.data_ptr()), ldl, (int)V, NR,
                            alpha.data_ptr<float>(), part.data_ptr<float>(), db.data_ptr<float>(),
                            st);
      },
      iters, st);
}

// Phase stamps of one launch of the MFMA attention workgroups (microbenchmark,
// scripts/microbench_att.py): (Bv * A / 64, 8) int64 wall-clock ticks, phases
// 0 start, 1 operands in LDS, 2 query MFMA, 3 scores, 4 ticket, and for the
// video's last workgroup 5 slot sums, 7 softmax, 6 end (-1 where not reached).
at::Tensor att_mfma_phases(at::Tensor gv, at::Tensor P, at::Tensor wa, at::Tensor ba, int64_t R) {
  check_cuda(gv, "gv");
  const int64_t Bv = gv.size(0), C = gv.size(1), H4 = gv.size(2), A = P.size(2), H = H4 / 4;
  const int vdiv = (int)(R / Bv), CP = C <= 8 ? 8 : 16;
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(gv.device());
  auto bf = gv.options().dtype(at::kBFloat16);
  at::Tensor h = (at::rand({R, H}, f32) * 2 - 1).to(at::kBFloat16);
  at::Tensor wq = (at::randn({A, H}, f32) * 0.05).to(at::kBFloat16);
  at::Tensor gv16 = at::zeros({Bv, H4, CP}, bf), vg = at::empty({R, H4}, bf);
  gv16.narrow(2, 0, C).copy_(gv.transpose(1, 2));
  at::Tensor alpha = at::empty({R, C}, f32), qo = at::empty({R, A}, f32);
  at::Tensor ep = at::empty({Bv, A / 64, 32, CP}, f32);
  at::Tensor cnt = at::zeros({Bv}, f32.dtype(at::kInt));
  at::Tensor dbg = at::full({Bv * (A / 64), 8}, -1, f32.dtype(at::kLong));
  AttMfmaArgs am{reinterpret_cast<const uint16_t*>(h.data_ptr()),
                 reinterpret_cast<const uint16_t*>(wq.data_ptr()), P.data_ptr<float>(),
                 wa.data_ptr<float>(), ba.data_ptr<float>(),
                 reinterpret_cast<const uint16_t*>(gv16.data_ptr()), (int)H, (int)A, (int)C, CP,
                 (int)H4, vdiv, (int)Bv, reinterpret_cast<uint16_t*>(vg.data_ptr()),
                 alpha.data_ptr<float>(), qo.data_ptr<float>(), ep.data_ptr<float>(),
                 cnt.data_ptr<int>(), nullptr, nullptr};
  hipStream_t st = cur_stream();
  launch_att_mfma_fwd(am, st);  // warm-up
  (void)hipStreamSynchronize(st);
  am.dbg = dbg.data_ptr<int64_t>();
  launch_att_mfma_fwd(am, st);
  (void)hipStreamSynchronize(st);
  return dbg;
}

// temporal attention kernels alone (one decode / reverse step): Gv (Bv, C, 4H)
// fp32, P (Bv, C, A), q (R, A), w_a (A), b_a (1); which = 0: forward
// (accumulating into pre), 1: backward (dG rows (R, 4H + A) bf16, dq written)
double att_bench(at::Tensor gv, at::Tensor P, at::Tensor q, at::Tensor wa, at::Tensor ba,
                 int64_t R, int64_t which, int64_t iters) {
  check_cuda(gv, "gv");
  const int64_t Bv = gv.size(0), C = gv.size(1), H4 = gv.size(2), A = P.size(2);
  TORCH_CHECK(R % Bv == 0 && q.size(0) == R && q.size(1) == A, "att_bench shapes");
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(gv.device());
  const int vdiv = (int)(R / Bv);
  at::Tensor pre = at::zeros({R, H4}, f32), alpha = at::full({R, C}, 1.f / C, f32);
  at::Tensor dG = at::zeros({R, H4 + A}, gv.options().dtype(at::kBFloat16));
  const int rpw_b = which == 4 ? 2 : ATT_BWD_RPW;  // 1: backward, 4: backward at 2 rows
  const int64_t nwg = Bv * att_groups(vdiv, rpw_b);
  at::Tensor dpp = at::zeros({nwg, C, A}, f32), dwp = at::zeros({nwg, A}, f32),
             dbp = at::zeros({nwg, 1}, f32);
  hipStream_t st = cur_stream();
  const int64_t H = H4 / 4;
  if (which == 5 || which == 6) {  // MFMA path: att_mfma forward workgroups / att_bwd_mfma
    auto bf = gv.options().dtype(at::kBFloat16);
    const int CP = C <= 8 ? 8 : 16;
    at::Tensor h = (at::rand({R, H}, f32) * 2 - 1).to(at::kBFloat16);
    at::Tensor wq = (at::randn({A, H}, f32) * 0.05).to(at::kBFloat16);
    at::Tensor gv16 = at::zeros({Bv, H4, CP}, bf), vg = at::empty({R, H4}, bf);
    gv16.narrow(2, 0, C).copy_(gv.transpose(1, 2));
    at::Tensor qo = at::empty({R, A}, f32), dal = at::randn({H / 64, R, CP}, f32);
    at::Tensor dP = at::zeros({Bv, C, A}, f32), dwa = at::zeros({Bv, A}, f32),
               dba = at::zeros({Bv, 1}, f32);
    at::Tensor ep = at::empty({Bv, A / 64, 32, CP}, f32);
    at::Tensor cnt = at::zeros({Bv}, f32.dtype(at::kInt));
    AttMfmaArgs am{reinterpret_cast<const uint16_t*>(h.data_ptr()),
                   reinterpret_cast<const uint16_t*>(wq.data_ptr()), P.data_ptr<float>(),
                   wa.data_ptr<float>(), ba.data_ptr<float>(),
                   reinterpret_cast<const uint16_t*>(gv16.data_ptr()), (int)H, (int)A, (int)C, CP,
                   (int)H4, vdiv, (int)Bv, reinterpret_cast<uint16_t*>(vg.data_ptr()),
                   alpha.data_ptr<float>(), qo.data_ptr<float>(), ep.data_ptr<float>(),
                   cnt.data_ptr<int>()};
    return time_launches(
        [&](int) {
          if (which == 5)
            launch_att_mfma_fwd(am, st);
          else
            launch_att_bwd_mfma(dal.data_ptr<float>(), (int)(H / 64), (int)R,
                                alpha.data_ptr<float>(), q.data_ptr<float>(), P.data_ptr<float>(),
                                wa.data_ptr<float>(), (int)Bv, vdiv, (int)C, CP, (int)A, (int)H4,
                                reinterpret_cast<uint16_t*>(dG.data_ptr()), (int)(H4 + A), 1,
                                dP.data_ptr<float>(), dwa.data_ptr<float>(),
                                dba.data_ptr<float>(), st);
        },
        iters, st);
  }
  return time_launches(
      [&](int) {
        if (which != 1 && which != 4)  // forward at 4 (0), 2 (2) or 1 (3) rows per workgroup
          launch_att_fwd(gv.data_ptr<float>(), P.data_ptr<float>(), q.data_ptr<float>(), nullptr,
                         wa.data_ptr<float>(), ba.data_ptr<float>(), (int)Bv, vdiv, (int)C, (int)A,
                         (int)H4, pre.data_ptr<float>(), alpha.data_ptr<float>(), st, 1, 0,
                         which == 2 ? 2 : which == 3 ? 1 : 4);
        else
          launch_att_bwd(reinterpret_cast<uint16_t*>(dG.data_ptr()), (int)(H4 + A),
                         gv.data_ptr<float>(), P.data_ptr<float>(), q.data_ptr<float>(),
                         alpha.data_ptr<float>(), wa.data_ptr<float>(), (int)Bv, vdiv, (int)C,
                         (int)A, (int)H4, 1, dpp.data_ptr<float>(), dwp.data_ptr<float>(),
                         dbp.data_ptr<float>(), st, 0, rpw_b);
      },
      iters, st);
}

// counting sort of n token ids < V (the embedding-gradient grouping)
double token_sort_bench(at::Tensor toks, int64_t V, int64_t iters) {
  check_cuda(toks, "toks");
  const int64_t N = toks.numel();
  auto i32 = at::TensorOptions().dtype(at::kInt).device(toks.device());
  at::Tensor ws = at::empty({2 * V + 1}, i32), stok = at::empty({N}, i32), srow = at::empty({N}, i32);
  hipStream_t st = cur_stream();
  return time_launches(
      [&](int) {
        launch_token_sort(toks.data_ptr<int64_t>(), (int)N, (int)V, ws.data_ptr<int>(),
                          stok.data_ptr<int>(), srow.data_ptr<int>(), st);
      },
      iters, st);
}

// the vocab projection + sampler/argmax + combine alone (tests of the exact
// two-level sampler): rows hd (R, H) bf16 -> {token (R) int64, lse (R)}.
// mode: SEL_SAMPLE_H (1) or SEL_GREEDY_H (2).
// MFMA temporal-attention workgroups as a launch of their own (tests /
// microbenchmarks of kernels/att_mfma.h): h (R, H) bf16, wq (A, H) bf16,
// P (Bv, C, A), wa (A), ba (1) fp32, gv (Bv, C, 4H) fp32 ->
// {vg (R, 4H) bf16, alpha (R, C), q (R, A)}
std::vector<at::Tensor> att_mfma_fwd(at::Tensor h, at::Tensor wq, at::Tensor P, at::Tensor wa,
                                     at::Tensor ba, at::Tensor gv, int64_t whole) {
  for (auto* t : {&h, &wq, &P, &wa, &ba, &gv}) check_cuda(*t, "att_mfma operand");
  TORCH_CHECK(h.scalar_type() == at::kBFloat16 && wq.scalar_type() == at::kBFloat16 &&
                  P.scalar_type() == at::kFloat && wa.scalar_type() == at::kFloat &&
                  ba.scalar_type() == at::kFloat && gv.scalar_type() == at::kFloat,
              "att_mfma: h / wq bf16, P / wa / ba / gv fp32");
  const int64_t R = h.size(0), H = h.size(1), A = wq.size(0), Bv = P.size(0), C = P.size(1);
  TORCH_CHECK(wq.size(1) == H && P.size(2) == A && wa.numel() == A && ba.numel() == 1 &&
                  gv.size(0) == Bv && gv.size(1) == C && gv.size(2) == 4 * H && R % Bv == 0,
              "att_mfma: operand shapes");
  const int vdiv = (int)(R / Bv), CP = C <= 8 ? 8 : 16;
  TORCH_CHECK(att_mfma_fwd_ok(vdiv, (int)C, (int)A, (int)H, 0), "att_mfma: unsupported shape");
  at::Tensor gv16 = at::zeros({Bv, 4 * H, CP}, h.options());
  gv16.narrow(2, 0, C).copy_(gv.transpose(1, 2));
  at::Tensor vg = at::empty({R, 4 * H}, h.options());
  at::Tensor alpha = at::empty({R, C}, P.options()), q = at::empty({R, A}, P.options());
  at::Tensor ep = at::empty({Bv, A / 64, 32, CP}, P.options());
  at::Tensor cnt = at::zeros({Bv}, P.options().dtype(at::kInt));
  AttMfmaArgs a{reinterpret_cast<const uint16_t*>(h.data_ptr()),
                reinterpret_cast<const uint16_t*>(wq.data_ptr()), P.data_ptr<float>(),
                wa.data_ptr<float>(), ba.data_ptr<float>(),
                reinterpret_cast<const uint16_t*>(gv16.data_ptr()), (int)H, (int)A, (int)C, CP,
                (int)(4 * H), vdiv, (int)Bv, reinterpret_cast<uint16_t*>(vg.data_ptr()),
                alpha.data_ptr<float>(), q.data_ptr<float>(), ep.data_ptr<float>(),
                cnt.data_ptr<int>()};
  a.whole = whole < 0 ? att_mfma_whole_default((int)C, (int)H) : (whole != 0 ? 1 : 0);
  launch_att_mfma_fwd(a, cur_stream());
  return {vg, alpha, q};
}

std::vector<at::Tensor> vocab_select(at::Tensor hd, at::Tensor wlog, at::Tensor blog,
                                     at::Tensor rng, int64_t mode, double temperature,
                                     int64_t step) {
  check_cuda(hd, "hd");
  check_cuda(wlog, "wlog");
  TORCH_CHECK(hd.scalar_type() == at::kBFloat16 && wlog.scalar_type() == at::kBFloat16 &&
                  blog.scalar_type() == at::kFloat, "bf16 hd / W, fp32 bias");
  TORCH_CHECK(mode == SEL_SAMPLE_H || mode == SEL_GREEDY_H, "mode: 1 sample, 2 greedy");
  const int64_t R = hd.size(0), H = hd.size(1), V = wlog.size(0);
  TORCH_CHECK(H % 64 == 0 && wlog.size(1) == H && blog.numel() == V, "shapes");
  auto dev = hd.device();
  const int n_vt = vocab_num_tiles((int)V);
  at::Tensor part = at::empty({(int64_t)n_vt * R * vocab_partial_bytes() / 4},
                              at::TensorOptions().dtype(at::kFloat).device(dev));
  at::Tensor tok = at::zeros({R, 1}, at::TensorOptions().dtype(at::kLong).device(dev));
  at::Tensor lse = at::empty({R}, at::TensorOptions().dtype(at::kFloat).device(dev));
  hipStream_t st = cur_stream();
  launch_vocab_fwd(reinterpret_cast<const uint16_t*>(hd.data_ptr()), (int)H, (int)R, (int)H,
                   reinterpret_cast<const uint16_t*>(wlog.data_ptr()), blog.data_ptr<float>(),
                   (int)V, nullptr, 0, part.data_ptr(), nullptr, 0, mode == SEL_SAMPLE_H ? 1 : 2,
                   (float)(1.0 / temperature), rng_ptr(rng), (int)step, st);
  launch_vocab_combine(part.data_ptr(), n_vt, (int)R, lse.data_ptr<float>(),
                       tok.data_ptr<int64_t>(), 1, nullptr, 0, nullptr, 0, nullptr, 0, (int)mode,
                       0.f, rng_ptr(rng), (int)step, nullptr, 0, nullptr, st);
  return {tok.view({R}), lse};
}

// One decode step for tests: the decode launch + vocab_combine_kernel.  save: 0 none, 1 fp16 logits, 2 exp store
// (eoff given).  Cell (ptab defined): the next step's cell from c_prev and
// the chosen tokens (dropout drop_p, step key `step + 1`).  eos: 0 no
// end-of-sequence rules; 1 / 2 the all-rows-ended counter with a live / dead
// previous step; unfinished (R) uint8 nullable: the per-row mask, updated in
// place.  Returns {lse, tok, g_sel, g_xe, saved rows (R, ldl), pre (R, 4H),
// n_parts, h, c, h_drop, gates, counts}.
std::vector<at::Tensor> decode_step_test(at::Tensor hd, at::Tensor h, at::Tensor wlog,
                                         at::Tensor blog, at::Tensor whh, at::Tensor vgate,
                                         int64_t vdiv, at::Tensor tgt, at::Tensor eoff,
                                         int64_t save, int64_t mode, int64_t step, at::Tensor rng,
                                         at::Tensor ptab, at::Tensor c_prev, double drop_p,
                                         int64_t cell, int64_t eos, at::Tensor unfinished,
                                         double ss_prob) {
  check_cuda(hd, "hd");
  check_cuda(wlog, "wlog");
  const int64_t R = hd.size(0), H = hd.size(1), V = wlog.size(0);
  TORCH_CHECK(hd.scalar_type() == at::kBFloat16 && wlog.scalar_type() == at::kBFloat16 &&
                  hd.is_contiguous() && wlog.is_contiguous() && wlog.size(1) == H &&
                  blog.scalar_type() == at::kFloat && blog.numel() == V, "hd / wlog / blog");
  const bool lstm = whh.defined() && whh.numel() > 0;
  if (lstm)
    TORCH_CHECK(h.scalar_type() == at::kBFloat16 && h.is_contiguous() && h.sizes() == hd.sizes() &&
                    whh.scalar_type() == at::kBFloat16 && whh.is_contiguous() &&
                    whh.size(0) == 4 * H && whh.size(1) == H, "h / whh");
  const bool has_vg = vgate.defined() && vgate.numel() > 0;
  if (has_vg)
    TORCH_CHECK(vgate.scalar_type() == at::kFloat && vgate.is_contiguous() &&
                    vgate.size(0) * vdiv == R && vgate.size(1) == 4 * H, "vgate (R / vdiv, 4H)");
  const bool has_tgt = tgt.defined() && tgt.numel() > 0;
  if (has_tgt) TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.numel() == R, "tgt (R) int64");
  if (save == 2)
    TORCH_CHECK(eoff.defined() && eoff.scalar_type() == at::kFloat && eoff.numel() == R, "eoff (R)");
  const bool do_cell = ptab.defined() && ptab.numel() > 0;
  if (do_cell) {
    TORCH_CHECK(lstm, "the cell needs the recurrent part");
    check_cuda(ptab, "ptab");
    check_cuda(c_prev, "c_prev");
    TORCH_CHECK(ptab.scalar_type() == at::kHalf && ptab.size(0) == V && ptab.size(1) == 4 * H &&
                    c_prev.scalar_type() == at::kFloat && c_prev.numel() == R * H,
                "ptab (V, 4H) fp16 / c_prev (R, H) fp32");
  }
  const bool has_unf = unfinished.defined() && unfinished.numel() > 0;
  if (has_unf)
    TORCH_CHECK(unfinished.is_cuda() && unfinished.scalar_type() == at::kByte &&
                    unfinished.numel() == R, "unfinished (R) uint8");
  auto dev = hd.device();
  auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
  auto bf = at::TensorOptions().dtype(at::kBFloat16).device(dev);
  const int64_t ldl = (V + 63) / 64 * 64;
  at::Tensor part = at::empty({(int64_t)vocab_part_slots((int)V) * R * vocab_partial_bytes() / 4}, f32);
  at::Tensor saved = save ? at::zeros({R, ldl}, at::TensorOptions()
                                                    .dtype(save == 2 ? at::kBFloat16 : at::kHalf)
                                                    .device(dev))
                          : at::Tensor();
  at::Tensor pre = lstm ? at::zeros({R, 4 * H}, f32) : at::Tensor();
  at::Tensor lse = at::empty({R}, f32), gsel = at::zeros({R}, f32), gxe = at::zeros({R}, f32);
  at::Tensor tok = at::zeros({R}, at::TensorOptions().dtype(at::kLong).device(dev));
  at::Tensor h_out, c_out, hdrop, gates;
  if (do_cell) {
    h_out = at::zeros({R, H}, bf);
    c_out = at::zeros({R, H}, f32);
    hdrop = at::zeros({R, H}, bf);
    gates = at::zeros({R, 4 * H}, bf);
  }
  // counts: steps 0..2 of the end-of-sequence flags; this step is count step 2
  const int cps = combine_count_ints_per_step();
  at::Tensor counts = at::zeros({3 * cps}, at::TensorOptions().dtype(at::kInt).device(dev));
  if (eos == 1) counts.narrow(0, cps, 1).fill_(1);  // a live row at the previous step
  int* CNT = eos ? counts.data_ptr<int>() : nullptr;
  hipStream_t st = cur_stream();
  const int flags = (mode == SEL_SAMPLE_H || mode == SEL_SS_H ? 1 : 0) |
                    (mode == SEL_GREEDY_H ? 2 : 0) | (save == 2 ? 16 : 0);
  const int64_t* TG = has_tgt ? tgt.data_ptr<int64_t>() : nullptr;
  uint8_t* UNF = has_unf ? unfinished.data_ptr<uint8_t>() : nullptr;
  const int n = launch_vocab_lstm_fwd(
      reinterpret_cast<const uint16_t*>(hd.data_ptr()), (int)H, (int)R, (int)H,
      reinterpret_cast<const uint16_t*>(wlog.data_ptr()), blog.data_ptr<float>(), (int)V,
      save ? reinterpret_cast<uint16_t*>(saved.data_ptr()) : nullptr, ldl, part.data_ptr(), TG, 1,
      flags, 1.f, rng_ptr(rng), (int)step,
      lstm ? reinterpret_cast<const uint16_t*>(h.data_ptr()) : nullptr,
      lstm ? reinterpret_cast<const uint16_t*>(whh.data_ptr()) : nullptr,
      has_vg ? vgate.data_ptr<float>() : nullptr, (int)vdiv, lstm ? pre.data_ptr<float>() : nullptr,
      st, 0, nullptr, save == 2 ? eoff.data_ptr<float>() : nullptr, nullptr);
  CellLaunch cl{};
  if (do_cell)
    cl = CellLaunch{pre.data_ptr<float>(), reinterpret_cast<const uint16_t*>(ptab.data_ptr()),
                    c_prev.data_ptr<float>(), c_out.data_ptr<float>(),
                    reinterpret_cast<uint16_t*>(h_out.data_ptr()),
                    reinterpret_cast<uint16_t*>(hdrop.data_ptr()), (int)H,
                    reinterpret_cast<uint16_t*>(gates.data_ptr()), (int)H, (float)drop_p,
                    (int)step + 1, (int)cell, nullptr, 0};
  launch_vocab_combine(part.data_ptr(), n, (int)R, lse.data_ptr<float>(), tok.data_ptr<int64_t>(),
                       1, gsel.data_ptr<float>(), 1, has_tgt ? gxe.data_ptr<float>() : nullptr, 1,
                       TG, 1, (int)mode, (float)ss_prob, rng_ptr(rng), (int)step, CNT, 2, UNF, st,
                       do_cell ? &cl : nullptr);
  return {lse, tok, gsel, gxe, saved, pre, at::full({1}, n, at::TensorOptions().dtype(at::kLong)),
          h_out, c_out, hdrop, gates, counts};
}

// the counting sort itself, for tests: returns {stok, srow} (int32)
std::vector<at::Tensor> token_sort(at::Tensor toks, int64_t V) {
  check_cuda(toks, "toks");
  TORCH_CHECK(toks.scalar_type() == at::kLong, "int64 token ids");
  const int64_t N = toks.numel();
  auto i32 = at::TensorOptions().dtype(at::kInt).device(toks.device());
  at::Tensor ws = at::empty({2 * V + 1}, i32), stok = at::empty({N}, i32), srow = at::empty({N}, i32);
  launch_token_sort(toks.data_ptr<int64_t>(), (int)N, (int)V, ws.data_ptr<int>(),
                    stok.data_ptr<int>(), srow.data_ptr<int>(), cur_stream());
  return {stok, srow};
}

// per-token row sums for tests: x (N, C) bf16, toks (N) int64 -> S (V, C) bf16
at::Tensor token_group_sum(at::Tensor x, at::Tensor toks, int64_t V) {
  check_cuda(x, "x");
  check_cuda(toks, "toks");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1, "x: (N, C) bf16");
  TORCH_CHECK(toks.scalar_type() == at::kLong && toks.numel() == x.size(0), "toks: (N) int64");
  const int64_t N = toks.numel(), C = x.size(1);
  auto i32 = at::TensorOptions().dtype(at::kInt).device(toks.device());
  at::Tensor ws = at::empty({2 * V + 1}, i32), stok = at::empty({N}, i32), srow = at::empty({N}, i32);
  at::Tensor S = at::empty({V, C}, x.options());
  at::Tensor S32 = at::empty({V, C}, x.options().dtype(at::kFloat));
  hipStream_t st = cur_stream();
  launch_token_sort(toks.data_ptr<int64_t>(), (int)N, (int)V, ws.data_ptr<int>(),
                    stok.data_ptr<int>(), srow.data_ptr<int>(), st);
  launch_token_long_zero(ws.data_ptr<int>(), (int)V, (int)C, S32.data_ptr<float>(), st);
  launch_token_group_sum(reinterpret_cast<const uint16_t*>(x.data_ptr()), (int)C, x.stride(0),
                         stok.data_ptr<int>(), srow.data_ptr<int>(), (int)N, ws.data_ptr<int>(),
                         (int)V, reinterpret_cast<uint16_t*>(S.data_ptr()), S32.data_ptr<float>(),
                         st);
  return S;
}

}  // namespace cst
