"""The data-parallel step on the GPU at world size 1 over RCCL (backend "nccl"): the full
CMX-B0 model with SyncBatchNorm in the decoder (train.py:64-65, MLPDecoder.py:51-55), the
parameter broadcast, BucketedGradSync (segment all-reduces on a side stream, overlapped with
the backward; fp32 and bf16 payloads) and HIP-graph capture of the whole step, as bench.py
runs it for N > 1.  At world size 1 every collective is an identity, so the DP step must
equal the plain step (BatchNorm2d, no process group) to rounding.

8-GPU runs are the driver's; this exercises every line of the N > 1 path that one GPU can."""
import gc
import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _model(dev, norm, state=None):
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    torch.manual_seed(0)
    m = EncoderDecoder(dict(backbone="mit_b0", num_classes=9, compute_dtype="bfloat16", decoder_embed_dim=256),
                       norm_layer=norm).to(dev)
    if state is not None:
        m.load_state_dict(state)
    return m


def _run(model, opt, batch, captured_steps=2, pre_step=None):
    """bench.py's sequence: 2 eager steps, a side-stream warm-up, capture, replays."""
    rgb, x, lab = batch

    def step():
        loss = model(rgb, x, lab)
        loss.backward()
        if pre_step is not None:
            pre_step()
        opt.step()
        return loss

    for _ in range(2):
        step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    gc.collect()                       # no pinned-host frees of earlier tests inside the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        step()
    for _ in range(captured_steps):
        graph.replay()
    torch.cuda.synchronize()
    return model.store.flat.clone()


@pytest.mark.parametrize("payload", ["fp32", "bf16"])
def test_dp_world1_graph_step_equals_plain_step(dev, payload):
    from rgbx_semantic_segmentation_amd import dist as cdist
    from rgbx_semantic_segmentation_amd.optim import FusedAdamW
    from rgbx_semantic_segmentation_amd.data import make_batch
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(29650 + (os.getpid() % 300))
    batch = tuple(t.to(dev) for t in make_batch(2, 96, 128, 9, seed=5))
    plain = _model(dev, torch.nn.BatchNorm2d)
    state = {k: v.detach().cpu().clone() for k, v in plain.state_dict().items()}
    plain.train()
    # no DropPath / Dropout2d randomness: the same keep masks on both sides
    flags = torch.ones(sum(plain.backbone.depths), 2, 4)
    flags[1, 0, 1] = 0.0
    d2 = torch.ones(2, 256)
    d2[0, :7] = 0.0
    flags, d2 = flags.to(dev), d2.to(dev)            # device-resident: no H2D copy inside the capture
    plain.forced_masks = {"droppath": flags, "dropout2d": d2}
    p0 = plain.store.flat.clone()
    # the bf16 payload at world size 1 delivers float(bf16(g)) (a one-rank reduce-scatter and
    # all-gather are copies): the plain reference rounds its gradients the same way
    g = plain.store.grad
    rounding = (lambda: g.copy_(g.to(torch.bfloat16).float())) if payload == "bf16" else None
    ref = _run(plain, FusedAdamW(plain), batch, pre_step=rounding)

    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        group = dist.group.WORLD
        dp = _model(dev, torch.nn.SyncBatchNorm, state)
        dp.process_group = group
        cdist.broadcast_parameters(dp, group)
        sync = cdist.BucketedGradSync(dp.store, group, payload=payload, chunk_mb=8)
        dp.backbone.grad_sync = sync
        dp.train()
        dp.forced_masks = {"droppath": flags, "dropout2d": d2}
        got = _run(dp, FusedAdamW(dp, grad_sync=sync), batch)
        assert sync.launched == set() and not sync.works          # every segment joined by the optimizer
    finally:
        dist.destroy_process_group()
    d = (got - ref).abs().max().item()
    rel = ((got - ref).norm() / (ref - p0).norm()).item()
    print(f"payload {payload}: after 5 steps max |param diff| {d:.3e}, |diff| / |distance travelled| {rel:.3e}")
    # SyncBN finalizes from all-reduced fp64 sums (separate launch) where BatchNorm2d folds them
    # in one kernel; AdamW's ~lr * sign(g) updates turn a rounding-level gradient difference
    # of an element near 0 into a full step for that element: compare the trajectories in norm
    assert rel < 1e-3, (rel, d)


def test_bf16_payload_casts_against_cpu(dev):
    """The two kernels of the bf16 gradient exchange (dist.BucketedGradSync._reduce_bf16): the
    fp32 -> bf16 payload cast (round to nearest even) and the bf16 -> fp32 copy of the gathered
    sums, bit for bit against torch's CPU casts, over magnitudes 1e-6 .. 1e3."""
    from rgbx_semantic_segmentation_amd import _lib
    n = 8 * 1237
    g = torch.Generator().manual_seed(3)
    src = (torch.randn(n, generator=g) * torch.logspace(-6, 3, n)).float()
    send = torch.empty(n, dtype=torch.bfloat16, device=dev)
    s_dev = src.to(dev)
    _lib.call("cmx_cast_f32_bf16", _lib.ptr(s_dev), _lib.ptr(send), n, _lib.stream())
    assert torch.equal(send.cpu(), src.to(torch.bfloat16))
    back = torch.empty(n, dtype=torch.float32, device=dev)
    _lib.call("cmx_cast_bf16_f32", _lib.ptr(send), _lib.ptr(back), n, _lib.stream())
    assert torch.equal(back.cpu(), src.to(torch.bfloat16).float())
