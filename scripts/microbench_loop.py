"""Persistent reverse LSTM loop alone (csrc/kernels/lstm_loop.hip, random
operands, headline shape by default; DBG variants 1 plain B loads, 2 no B
loads, 4 plain dG stores -- timing only): us per launch and the per-step phase
breakdown from the kernel's wall-clock stamps (100 MHz), averaged over
workgroups and steps.  Usage: microbench_loop.py [R H T iters [DBG]]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cst_captioning_amd import _ext


def main():
    R, H, T, iters = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (1280, 512, 29, 20)))
    dbg = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    ops = _ext.ops()
    nwg = 8 * (H // 64) * (((R + 7) // 8 + 47) // 48)
    ph = torch.zeros(nwg, T, 4, dtype=torch.int64, device='cuda')
    us = ops.lstm_bwd_loop_bench(R, H, T, iters, ph, dbg)
    p = ph.double() / 100.0  # us
    t0 = p[:, 0, 0].min()
    step = p[:, 1:, 0] - p[:, :-1, 0]        # step start to next step start
    wait = p[:, 1:, 1] - p[:, 1:, 0]         # team wait (steps with a GEMM)
    gemm = p[:, 1:, 2] - p[:, 1:, 1]         # B loads + MFMA + reduction store + operand drain
    epi = p[:, :, 3] - p[:, :, 2]            # cell backward + stores + drain
    res = {'R': R, 'H': H, 'T': T, 'dbg': dbg, 'us_per_launch': round(us, 2), 'us_per_step': round(us / T, 2),
           'step_us_mean': round(step.mean().item(), 2),
           'wait_us_mean': round(wait.mean().item(), 2), 'wait_us_max': round(wait.max().item(), 2),
           'gemm_us_mean': round(gemm.mean().item(), 2), 'gemm_us_max': round(gemm.max().item(), 2),
           'epi_us_mean': round(epi.mean().item(), 2), 'epi_us_max': round(epi.max().item(), 2),
           'first_start_spread_us': round((p[:, 0, 0].max() - t0).item(), 2),
           'last_end_us': round((p[:, -1, 3].max() - t0).item(), 2),
           'device_errors': int(ops.device_errors(0))}
    print(json.dumps(res))


if __name__ == '__main__':
    main()
