"""Deferred grouped launches (deferred.py -> cmx_gemm_grouped / cmx_reduce_grouped) against a
plain PyTorch fp32 reference.

A batch of weight-gradient problems of the step's shapes (stage-1 64 x 64 over 38400 tokens,
fc1 / fc2, a conv wgrad with 9C columns, a strided column slice of a shared gradient as in
FRM's spatial 1x1, the decoder's linear_fuse) is queued, flushed as ONE GEMM launch + ONE
reduce launch, and compared with dz^T x in fp32.  Tolerance 2e-3 relative (bf16 operands,
fp32 accumulation in a different order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_grouped_wgrads_and_bias(dev, dt):
    from rgbx_semantic_segmentation_amd import deferred
    torch.manual_seed(0)
    shapes = [(2, 38400, 64, 64, True), (2, 38400, 256, 64, True), (2, 38400, 64, 256, True),
              (2, 4800, 128, 576, True), (2, 600, 512, 2048, True), (1, 38400, 512, 2048, False),
              (2, 1200, 320, 320, True), (2, 600, 40, 512, True)]
    jobs = []
    for G, M, N, k, has_b in shapes:
        dz = torch.randn(G, M, N, device=dev).to(dt)
        x = torch.randn(G, M, k, device=dev).to(dt)
        Wg = torch.full((G, N, k), float("nan"), device=dev)
        bg = torch.full((G, N), float("nan"), device=dev) if has_b else None
        queued = deferred.wgrad(dz, x, Wg, bg)
        assert queued, (G, M, N, k)
        jobs.append((dz, x, Wg, bg))
    # a strided column slice of one gradient (FRM: gW0[:, :C] and gW0[:, C:])
    M, N, C = 19200, 64, 64
    dzs = torch.randn(1, M, N, device=dev).to(dt)
    xa, xb = torch.randn(1, M, C, device=dev).to(dt), torch.randn(1, M, C, device=dev).to(dt)
    W2 = torch.full((1, N, 2 * C), float("nan"), device=dev)
    b2 = torch.full((1, N), float("nan"), device=dev)
    assert deferred.wgrad(dzs, xa, W2[:, :, :C], b2) and deferred.wgrad(dzs, xb, W2[:, :, C:])
    assert deferred.pending()
    deferred.flush()
    torch.cuda.synchronize()
    assert not deferred.pending()
    for dz, x, Wg, bg in jobs:
        ref = torch.bmm(dz.float().transpose(1, 2), x.float())
        assert rel(Wg, ref) < 2e-3, (dz.shape, x.shape, rel(Wg, ref))
        if bg is not None:
            assert rel(bg, dz.float().sum(1)) < 2e-3
    ref = torch.cat([dzs.float()[0].t() @ xa.float()[0], dzs.float()[0].t() @ xb.float()[0]], 1)
    assert rel(W2[0], ref) < 2e-3
    assert rel(b2[0], dzs.float()[0].sum(0)) < 2e-3


def test_grouped_reduce_split_destinations(dev):
    """LayerNorm-style [dgamma | dbeta] rows and DWConv-style [9 taps | bias] rows."""
    from rgbx_semantic_segmentation_amd import deferred
    torch.manual_seed(1)
    G, nb, C = 2, 128, 320
    ws = torch.randn(G, nb, 2 * C, device=dev)
    gg, bb = torch.empty(G, C, device=dev), torch.empty(G, C, device=dev)
    deferred.reduce(ws, gg, bb, G, nb, nb * 2 * C, 2 * C, 1, 2 * C, C, C, 0, C, 0)
    P, Cd = 37, 256
    wd = torch.randn(G, P, Cd * 10, device=dev)
    dw, db = torch.zeros(G, Cd, 9, device=dev), torch.ones(G, Cd, device=dev)
    deferred.reduce(wd, dw, db, G, P, P * Cd * 10, Cd * 10, Cd, 10, 9, Cd * 9, 9, Cd, 1, accumulate=True)
    deferred.flush()
    torch.cuda.synchronize()
    s = ws.sum(1)
    assert rel(gg, s[:, :C]) < 1e-5 and rel(bb, s[:, C:]) < 1e-5
    t = wd.sum(1).view(G, Cd, 10)
    assert rel(dw, t[..., :9]) < 1e-5 and rel(db, 1 + t[..., 9]) < 1e-5


def test_grouped_flush_in_graph_capture(dev):
    """The flush of a captured backward replays correctly (pinned tables kept alive)."""
    from rgbx_semantic_segmentation_amd import deferred
    torch.manual_seed(2)
    dz = torch.randn(2, 9600, 128, device=dev).bfloat16()
    x = torch.randn(2, 9600, 512, device=dev).bfloat16()
    Wg = torch.zeros(2, 128, 512, device=dev)
    bg = torch.zeros(2, 128, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        deferred.wgrad(dz, x, Wg, bg)
        deferred.flush()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        deferred.wgrad(dz, x, Wg, bg)
        deferred.flush()
    Wg.zero_(); bg.zero_()
    dz.mul_(2)
    g.replay()
    torch.cuda.synchronize()
    ref = torch.bmm(dz.float().transpose(1, 2), x.float())
    assert rel(Wg, ref) < 2e-3 and rel(bg, dz.float().sum(1)) < 2e-3
