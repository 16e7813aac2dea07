"""The hand-written persistent NT GEMM (csrc/kernels/gemm_sk.hip) against a
plain PyTorch fp64/fp32 reference: exact on small-integer operands (every
partial sum is exact in fp32), so a wrong tile, K range, slab piece or
fragment map shows as a mismatch, not as rounding; shapes cover phase 1 only,
phase 2 only (every tile split over many workgroups) and both, and the
headline X = E W shape through engine.vocab_x."""
import pytest
import torch

from cst_captioning_amd import _ext

pytestmark = pytest.mark.gpu


def _ops():
    return _ext.ops()


def _int_operands(M, N, K, ld_pad=0, seed=0):
    g = torch.Generator(device='cuda').manual_seed(seed)
    a = torch.randint(-2, 3, (M, K + ld_pad), generator=g, device='cuda').bfloat16()
    b = torch.randint(-2, 3, (N, K + ld_pad), generator=g, device='cuda').bfloat16()
    return a[:, :K], b[:, :K]


@pytest.mark.parametrize('variant', [0, 1])
@pytest.mark.parametrize('M,N,K', [
    (256 * 10, 512, 64 * 20),      # 20 (or 40) tiles < CUs: phase 2 only, many pieces per tile
    (256 * 140, 512, 64 * 24),     # headline rows: phase 1 + a 24-tile remainder
    (256 * 4, 256, 64 * 3),        # fewer K-iterations than workgroups: one-iteration pieces
    (256 * 300, 256, 64 * 5),      # > 1 phase-1 round
    (256 * 9 + 13, 512, 64 * 7),   # edge M tile (rows past M dropped)
])
def test_gemm_nt_sk_exact_on_integers(M, N, K, variant):
    ops = _ops()
    if not ops.gemm_nt_sk_ok(M, N, K, variant):
        pytest.skip('shape not tiled by this variant')
    a, b = _int_operands(M, N, K, ld_pad=64 if K % 128 else 0)
    out = torch.full((M, N), float('nan'), device='cuda')
    ops.gemm_nt_sk(out, a, b, variant)
    ref = (a.double() @ b.double().t()).float()
    bad = (out != ref)
    assert not bad.any(), (variant, bad.sum().item(), bad.nonzero()[:8].tolist())
    # run-to-run identical (the remainder tiles' pieces are summed in piece order)
    out2 = torch.empty_like(out)
    ops.gemm_nt_sk(out2, a, b, variant)
    assert torch.equal(out, out2)


@pytest.mark.parametrize('variant', [0, 1])
@pytest.mark.parametrize('M,N,K,ldm', [
    (10509, 512, 64 * 40, 10560),  # dW_logit's M (edge tile), short K: phase 2
    (256 * 3, 256, 64 * 9, 256 * 3),
    (1000, 512, 64 * 300, 1024),   # long K split over many workgroups
])
def test_gemm_tn_sk_exact_on_integers(M, N, K, ldm, variant):
    """out = a^T b with a (K x M, row stride ldm) and b (K x N): the
    transposed-read (ds_read_b64_tr_b16) operand path."""
    ops = _ops()
    if not ops.gemm_nt_sk_ok(M, N, K, variant):
        pytest.skip('shape not tiled by this variant')
    g = torch.Generator(device='cuda').manual_seed(1)
    a = torch.randint(-2, 3, (K, ldm), generator=g, device='cuda').bfloat16()[:, :M]
    b = torch.randint(-2, 3, (K, N), generator=g, device='cuda').bfloat16()
    out = torch.full((M, N), float('nan'), device='cuda')
    ops.gemm_tn_sk(out, a, b, variant)
    ref = (a.double().t() @ b.double()).float()
    bad = (out != ref)
    assert not bad.any(), (variant, bad.sum().item(), bad.nonzero()[:8].tolist())


def test_gemm_sk_refuses_untiled_shapes():
    ops = _ops()
    a = torch.zeros(100, 60, device='cuda', dtype=torch.bfloat16)
    b = torch.zeros(256, 60, device='cuda', dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.gemm_nt_sk(torch.empty(100, 256, device='cuda'), a, b, 0)


def test_transpose_pad():
    ops = _ops()
    w = torch.randn(1000, 96, device='cuda').bfloat16()
    t = ops.transpose_pad_bf16(w, 1024)
    assert t.shape == (96, 1024)
    assert torch.equal(t[:, :1000], w.t())
    assert (t[:, 1000:] == 0).all()


@pytest.mark.parametrize('variant', [0, 1])
def test_vocab_x_sk_matches_fp32_at_headline_shape(variant, monkeypatch):
    """X = E W at the headline shape (28 x 1280 rows, V = 10,509 padded to
    10,560, H = 512) through the hand-written GEMM vs fp32 PyTorch on the same
    bf16 operands; the exp store's pad columns are zero as the vocab kernel
    writes them."""
    ops = _ops()
    n, R, V, H = 28, 1280, 10509, 512
    ldl = (V + 63) // 64 * 64
    torch.manual_seed(0)
    E = torch.zeros(n, R, ldl, device='cuda', dtype=torch.bfloat16)
    E[:, :, :V] = (torch.rand(n, R, V, device='cuda') * 2e-3).bfloat16()
    W = (torch.randn(V, H, device='cuda') * 0.05).bfloat16()
    out = torch.empty(n * R, H, device='cuda')
    a = E.view(n * R, ldl)
    ops.gemm_nt_sk(out, a, ops.transpose_pad_bf16(W, ldl), variant)
    ref = a[:, :V].float() @ W.float()
    err = (out - ref).norm() / ref.norm()
    assert err < 1e-5, err.item()
    # dW_logit = E^T Hs at the same shape (TN path, M = V edge tile)
    Hs = (torch.randn(n * R, H, device='cuda') * 0.1).bfloat16()
    dW = torch.empty(V, H, device='cuda')
    ops.gemm_tn_sk(dW, a[:, :V], Hs, variant)
    ref = a[:, :V].float().t() @ Hs.float()
    err = (dW - ref).norm() / ref.norm()
    assert err < 1e-5, err.item()
