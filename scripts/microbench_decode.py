"""Decode-launch diagnostics at the headline shape (R = 1,280, V = 10,509,
H = 512): HIP-event time of the 128 x 64-tile launch (variant 0) and the
256 x 256-tile launch (variant 9) for the sampled step with the exp store,
and the big launch's per-workgroup phase stamps (main loop, first-half
statistics, rest): median / max over workgroups, and the spread of start
times.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cst_captioning_amd import _ext

C = _ext.ops()


def main():
    torch.manual_seed(0)
    dev = 'cuda'
    V, H, R = 10509, 512, 1280
    W = (torch.randn(V, H, device=dev) * 0.05).bfloat16()
    b = torch.randn(V, device=dev) * 0.1
    hd = torch.randn(R, H, device=dev).bfloat16()
    none = torch.empty(0, dtype=torch.long, device=dev)
    res = {}
    for var in (0, 9):
        for name, flags, save in (('mainloop', 4, False), ('stats', 0, False),
                                  ('sample', 1, False), ('sample_exp', 17, True)):
            res['v%d_%s' % (var, name)] = round(C.vocab_fwd_bench(hd, W, b, none, flags, save, 50,
                                                                 var), 2)
    khz = C.wall_clock_khz() or 100000
    n_wg = ((V + 255) // 256) * ((R + 255) // 256)
    dbg = torch.zeros(4 * n_wg, dtype=torch.int64, device=dev)
    for flags, save, tag in ((17, True, 'sample_exp'), (4, False, 'mainloop')):
        C.big_debug_buffer(dbg)
        C.vocab_fwd_bench(hd, W, b, none, flags, save, 1, 9)
        torch.cuda.synchronize()
        C.big_debug_buffer(torch.empty(0, dtype=torch.int64, device=dev))
        t = dbg.view(n_wg, 4).double().cpu() * (1e3 / khz)  # us
        t0 = t[:, 0].min()
        ph = {'start': t[:, 0] - t0, 'main': t[:, 1] - t[:, 0], 'end': t[:, 3] - t0}
        if flags != 4:
            ph['stats0'] = t[:, 2] - t[:, 1]
            ph['rest'] = t[:, 3] - t[:, 2]
        for k, v in ph.items():
            res['phase_%s_%s_med' % (tag, k)] = round(float(v.median()), 2)
            res['phase_%s_%s_max' % (tag, k)] = round(float(v.max()), 2)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
