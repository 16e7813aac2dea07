"""The weight-gradient GEMM of the decoder backward (``csrc/kernels/wgrad.hip``:
C = A^T B over K-major bf16 operands, LDS-DMA staging, transposed LDS reads,
split-K with a fixed-order reduce) against a plain PyTorch fp32 reference of
the same product, at the shapes the engine uses (dW_hh: K = 27 x 1280 rows of
[dG | dq] and h_prev; dW_ie: K = V = 10,509 token rows, not a multiple of the
64-row K-tile) and small ragged ones."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _ops():
    from cst_captioning_amd import _ext
    assert _ext.available(), 'native extension must be built for GPU tests'
    return _ext.ops()


def _check(M, N, K, lda=None, ldb=None, rows_extra=0, seed=0):
    g = torch.Generator(device='cpu').manual_seed(seed)
    lda, ldb = lda or M, ldb or N
    A = (torch.randn(K + rows_extra, lda, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    B = (torch.randn(K + rows_extra, ldb, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    if rows_extra:  # rows past K must not contribute (NaN there would show)
        A[K:] = float('nan')
        B[K:] = float('nan')
    C = _ops().wgrad_tn(A, B, M, N, K)
    torch.cuda.synchronize()
    ref = A[:K, :M].float().t() @ B[:K, :N].float()
    err = ((C - ref).norm() / ref.norm()).item()
    assert torch.isfinite(C).all()
    assert err < 1e-5, (M, N, K, err)
    # deterministic: the split-K partials are summed in a fixed order
    C2 = _ops().wgrad_tn(A, B, M, N, K)
    assert torch.equal(C, C2)


@pytest.mark.parametrize('M,N,K', [(128, 128, 64), (128, 128, 100), (256, 128, 1000),
                                   (128, 256, 4097), (512, 384, 3000)])
def test_wgrad_small_shapes(M, N, K):
    _check(M, N, K)


def test_wgrad_rows_past_k_and_strides():
    _check(256, 128, 777, lda=264, ldb=136, rows_extra=13)


def test_wgrad_headline_whh_shape():
    # [dG | dq]^T h_prev of the att8 step: M = 4H + A, K = 27 steps x 1280 rows
    _check(2048 + 512, 512, 27 * 1280, seed=1)


def test_wgrad_headline_token_shape():
    # S^T emb: K = V = 10,509 per-token rows
    _check(2048, 512, 10509, seed=2)


def _check_colsum(M, K, lda, seed=0, nan_pad=True):
    """dW_logit form: M = V columns of the exp store (row stride lda >= M, the
    last 128-column tile ragged), N = H = 512, plus the fused weighted column
    sums db = A^T al (the bias gradient)."""
    g = torch.Generator(device='cpu').manual_seed(seed)
    N = 512
    A = torch.rand(K, lda, generator=g).to(torch.bfloat16).to(DEV)
    if nan_pad and lda > M:  # the row padding past V must not reach any output
        A[:, M:] = float('nan')
    B = (torch.randn(K, N, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    al = (torch.randn(K, generator=g) * 1e-2).to(DEV)
    C, db = _ops().wgrad_tn_colsum(A, B, al, M, N, K)
    torch.cuda.synchronize()
    ref = A[:, :M].float().t() @ B.float()
    ref_db = A[:, :M].float().t() @ al
    assert torch.isfinite(C).all() and torch.isfinite(db).all()
    assert ((C - ref).norm() / ref.norm()).item() < 1e-5
    assert ((db - ref_db).norm() / ref_db.norm()).item() < 1e-5
    C2, db2 = _ops().wgrad_tn_colsum(A, B, al, M, N, K)
    assert torch.equal(C, C2) and torch.equal(db, db2)


@pytest.mark.parametrize('M,K,lda', [(300, 1000, 320), (128, 64, 128), (1299, 5 * 130, 1344)])
def test_wgrad_ragged_m_with_column_sums(M, K, lda):
    _check_colsum(M, K, lda)


def test_wgrad_headline_dw_logit_with_bias_sums():
    # dW_logit = E'^T (alpha Hd) and db = E'^T alpha: M = V = 10,509 (ldl =
    # 10,560), K = 28 x 1280 rollout rows
    _check_colsum(10509, 28 * 1280, 10560, seed=3, nan_pad=False)
