"""CPU checks of the host-side weight packers of the dedicated MI355X kernels:
each packed buffer is decoded back through the kernel's documented fragment
map (lane -> row / k) and must reproduce the original weights.  The GPU tests
check the kernels themselves against fp32 references."""
import torch

from jax_raft_amd.ops import native as nat


def _frag(lane, j):
    """mfma_f32_16x16x32_bf16 A-operand map: lane l holds A[row l & 15][k 8 (l >> 4) + j]."""
    return lane & 15, 8 * (lane >> 4) + j


def test_pack_conv1x1_decodes_to_weights():
    K, N, kpad = 324, 256, 352
    w = torch.randn(1, 1, K, N)
    pk = nat.pack_conv1x1(w, kpad).float().reshape(N // 64, kpad // 32, 4, 64, 8)
    wb = w.reshape(K, N).to(torch.bfloat16).float()
    for g, ks, t, lane, j in [(0, 0, 0, 0, 0), (3, 10, 3, 63, 7), (1, 5, 2, 17, 3), (2, 10, 1, 40, 4)]:
        r, kk = _frag(lane, j)
        k = 32 * ks + kk
        co = 64 * g + 16 * (r >> 2) + 4 * t + (r & 3)
        want = wb[k, co] if k < K else 0.0
        assert pk[g, ks, t, lane, j].item() == want
    # every weight appears exactly once
    assert torch.allclose(pk.sum(), wb.sum(), rtol=1e-3, atol=1e-2)


def test_pack_taps_decodes_to_weights():
    K = 256
    w = torch.randn(3, 3, K, 2)
    pk = nat.pack_taps(w).float().reshape(K // 32, 2, 64, 8)
    taps = w.reshape(9, K, 2).permute(1, 0, 2).reshape(K, 18).to(torch.bfloat16).float()
    for ks in range(K // 32):
        for t in range(2):
            for lane in range(64):
                r, kk = _frag(lane, 0)
                o = 16 * t + r
                got = pk[ks, t, lane, :]
                want = taps[32 * ks + kk:32 * ks + kk + 8, o] if o < 18 else torch.zeros(8)
                assert torch.equal(got, want), (ks, t, lane)


def test_pack_convex_head_decodes_to_weights():
    w = torch.randn(1, 1, 256, 576)
    b = torch.randn(576)
    pk, bias = nat.pack_convex_head(w, b)
    pk = pk.float().reshape(8, 9, 4, 64, 8)      # [k-step][tap][sub-pixel group][lane][8]
    wb = w.reshape(256, 576).to(torch.bfloat16).float()
    for ks, k, g, lane, j in [(0, 0, 0, 0, 0), (7, 8, 3, 63, 7), (3, 4, 1, 22, 5)]:
        r, kk = _frag(lane, j)
        assert pk[ks, k, g, lane, j].item() == wb[32 * ks + kk, 64 * k + 16 * g + r].item()
    assert torch.equal(bias, b)


def test_pack_taps_epi_decodes_to_weights():
    w = torch.randn(3, 3, 256, 2)
    pk = nat.pack_taps_epi(w).float()              # [group 4][kstep 2][tile 2][lane 64][8]
    wt = w.reshape(9, 256, 2).permute(0, 2, 1).reshape(18, 256).to(torch.bfloat16).float()
    for g, s, t, lane, j in [(0, 0, 0, 0, 0), (3, 1, 0, 63, 7), (2, 0, 1, 16, 3), (1, 1, 1, 1, 5), (0, 1, 0, 47, 2)]:
        o = 16 * t + (lane & 15)
        c = 64 * g + 16 * (lane >> 4) + 8 * s + j
        want = wt[o, c].item() if o < 18 else 0.0
        assert pk[g, s, t, lane, j].item() == want
    # every (o < 18, c) weight appears exactly once
    assert torch.allclose(pk.sum(), wt.sum(), rtol=1e-3, atol=1e-2)
