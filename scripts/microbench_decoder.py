"""Micro-benchmark of the fused decoder forward in isolation (one call =
T decode steps), per token-selection mode / save option.  Run under
rocprofv3 --kernel-trace to split per-kernel time."""
import sys, time, json
import torch
sys.path.insert(0, '.')
from cst_captioning_amd import _ext

C = _ext.ops()
dev = 'cuda'
R, H, E, V, L = 1280, 512, 512, 10509, 30
T = L - 1
torch.manual_seed(0)
wx = (torch.randn(4 * H, E + H, device=dev) * 0.05).bfloat16()
emb = (torch.rand(V, E, device=dev) * 0.2 - 0.1).bfloat16()
wlog = (torch.rand(V, H, device=dev) * 0.2 - 0.1).bfloat16()
blog = torch.zeros(V, device=dev)
vg = torch.randn(64, 4 * H, device=dev) * 0.1
labels = torch.randint(3, V, (R, L), device=dev)
labels[:, 0] = 1
bos = torch.ones(R, dtype=torch.long, device=dev)
whh = wx[:, E:].contiguous()
ptab = torch.mm(emb, wx[:, :E].t(), out_dtype=torch.float32)
res = {}
import os
variants = [int(x) for x in os.environ.get('VARIANTS', '4').split(',')]
lvariants = [int(x) for x in os.environ.get('LSTM_VARIANTS', '0').split(',')]
for var, lvar in [(a, b) for a in variants for b in lvariants]:
  C.set_vocab_variant(var)
  C.set_lstm_fwd_variant(lvar)
  for name, modes, save, drop in [('greedy_nosave', [2] * (T - 1), False, 0.0),
                                ('sample_nosave', [1] * (T - 1), False, 0.0),
                                ('sample_save_drop', [1] * (T - 1), True, 0.5),
                                ('gt_save_drop', [0] * (T - 1), True, 0.5)]:
    args = lambda: C.decoder_forward(wx, emb, ptab, whh, wlog, blog, vg, 20, labels, bos, R, T, modes, 0.0,
                                     drop, 1.0, 7, save, False, True, False)
    for _ in range(3):
        args()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        args()
    torch.cuda.synchronize()
    res['v%d_l%d_%s' % (var, lvar, name)] = round((time.perf_counter() - t0) / 10 * 1e3, 3)
print(json.dumps(res))
