"""Host-side work split of the persistent GEMM (csrc/kernels/gemm_sk.hip,
gemm_sk_plan): whole tiles first, the remainder's K-iterations split over
min(G, I) workgroups.  Checked against a plain-Python model of the split:
every K-iteration of a remainder tile is owned by exactly one workgroup,
every workgroup of phase 2 gets at least one iteration, and the slab
workspace covers the largest number of pieces of any tile.  (CPU only: the
plan is host code; the kernel itself is tested in test_gpu_gemm_sk.py.)"""
import pytest

from cst_captioning_amd import _ext


def _model(M, N, K, G, BN):
    tiles = ((M + 255) // 256) * (N // BN)
    full, rem = divmod(tiles, G)
    nk = K // 64
    if rem == 0:
        return rem, 0
    I = rem * nk
    G2 = min(G, I)
    lo = [b * I // G2 for b in range(G2 + 1)]
    assert all(lo[b] < lo[b + 1] for b in range(G2))  # >= 1 iteration each
    owner = [None] * I
    for b in range(G2):
        for x in range(lo[b], lo[b + 1]):
            assert owner[x] is None
            owner[x] = b
    assert None not in owner
    pmax = max(len({owner[x] for x in range(q * nk, (q + 1) * nk)}) for q in range(rem))
    return rem, rem * pmax * 256 * BN


@pytest.mark.parametrize('M,N,K,G,variant', [
    (35840, 512, 10560, 256, 0),   # headline X = E W
    (10509, 512, 35840, 256, 0),   # headline dW_logit (edge M tile)
    (35840, 512, 10560, 256, 1),
    (2560, 512, 1280, 256, 0),     # phase 2 only
    (1024, 256, 192, 256, 0),      # fewer iterations than workgroups
    (76800, 256, 320, 256, 1),     # several phase-1 rounds
    (10509, 512, 35840, 128, 0),   # reduced grid
])
def test_gemm_sk_plan_matches_model(M, N, K, G, variant):
    ops = _ext.ops()
    BN = 128 if variant == 1 else 256
    assert tuple(ops.gemm_sk_plan(M, N, K, G, variant)) == _model(M, N, K, G, BN)
