"""Multi-process (world_size 2, gloo, CPU) tests of the data-parallel host logic:
* the flat-gradient all-reduce + 1/P scale equals DDP's average of per-rank gradients of the
  per-rank mean loss (train.py:141-149);
* SyncBN statistics from all-reduced fp64 sums equal the global-batch statistics.
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rgbx_semantic_segmentation_amd.dist import GradAllReduce, all_reduce_tensor
        from rgbx_semantic_segmentation_amd.functions import sync_bn_sums
        torch.manual_seed(0)
        # a tiny model, per-rank data slices of one global batch
        w = torch.randn(6, 4, dtype=torch.float64)
        X = torch.randn(world * 5, 4, dtype=torch.float64)
        Y = torch.randn(world * 5, 6, dtype=torch.float64)
        xs, ys = X[rank * 5:(rank + 1) * 5], Y[rank * 5:(rank + 1) * 5]
        wr = w.clone().requires_grad_(True)
        ((xs @ wr.t() - ys) ** 2).mean().backward()

        class Store:
            pass
        st = Store()
        st.grad = wr.grad.flatten().clone()
        scale = GradAllReduce(st, None)(st.grad)
        ours = st.grad * scale
        # DDP reference: mean over ranks of per-rank gradients
        ref = torch.zeros_like(w)
        for r in range(world):
            wr2 = w.clone().requires_grad_(True)
            ((X[r * 5:(r + 1) * 5] @ wr2.t() - Y[r * 5:(r + 1) * 5]) ** 2).mean().backward()
            ref += wr2.grad / world
        ok1 = torch.allclose(ours.view_as(w), ref)
        # SyncBN sums
        feats = torch.randn(world * 7, 3, dtype=torch.float64)
        mine = feats[rank * 7:(rank + 1) * 7]
        sums = torch.stack([mine.sum(0), (mine * mine).sum(0)])
        count = sync_bn_sums(sums, 7.0, dist.group.WORLD)
        mean = sums[0] / count
        var = sums[1] / count - mean ** 2
        ok2 = count == world * 7 and torch.allclose(mean, feats.mean(0)) and torch.allclose(var, feats.var(0, unbiased=False))
        loss = all_reduce_tensor(torch.tensor([float(rank)]), world_size=world)
        ok3 = abs(loss.item() - (world - 1) / 2) < 1e-12
        # segment-bucketed overlap: launching segments out of order / in pieces, then waiting,
        # equals one all-reduce of the whole flat buffer
        from rgbx_semantic_segmentation_amd.dist import BucketedGradSync
        st2 = Store()
        st2.grad = torch.arange(23, dtype=torch.float32) * (rank + 1)
        st2.segments = [(0, 0, 9), (1, 9, 16), (2, 16, 23)]
        bs = BucketedGradSync(st2, None)
        bs._launch(1)
        bs._launch(0)
        sc = bs(st2.grad)          # launches the rest, waits
        ok3 = ok3 and sc == 1.0 / world and torch.equal(st2.grad, torch.arange(23, dtype=torch.float32) * sum(
            r + 1 for r in range(world))) and not bs.works
        q.put((rank, bool(ok1), bool(ok2), bool(ok3)))
    finally:
        dist.destroy_process_group()


def test_dp_semantics_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] and r[2] and r[3] for r in res), res


def _worker_store(rank, world, port, payload, q):
    """BucketedGradSync over the real ParamStore layout of CMX-B0 (4 backward segments),
    gradients from the oracle on each rank's slice of one global batch whose slices have
    DIFFERENT numbers of valid (non-ignored) pixels."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.cmx_ref import EncoderDecoder as RefModel, CMXConfig
        from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder, backward_segment
        from rgbx_semantic_segmentation_amd.params import ParamStore
        from rgbx_semantic_segmentation_amd.dist import BucketedGradSync
        torch.manual_seed(0)
        ref = RefModel(CMXConfig(backbone="mit_b0", num_classes=5))
        ref.eval()
        prod = EncoderDecoder(dict(backbone="mit_b0", num_classes=5, decoder_embed_dim=512))
        store = ParamStore(prod, "cpu", torch.float32, segment_of=backward_segment)
        assert len(store.segments) == 4
        g = torch.Generator().manual_seed(1)
        H, W = 32, 48
        rgb = torch.randn(world, 3, H, W, generator=g)
        x = torch.randn(world, 3, H, W, generator=g)
        lab = torch.randint(0, 5, (world, H, W), generator=g)
        for r in range(world):                     # rank r: 40 * (r + 1) rows ignored
            lab[r, :10 * (r + 1)] = 255

        def grads(r):
            ref.zero_grad()
            ref(rgb[r:r + 1], x[r:r + 1], lab[r:r + 1]).backward()
            return {n: p.grad.clone() for n, p in ref.named_parameters()}

        mine = grads(rank)
        for n, p in prod.named_parameters():        # the store's gradient views <- this rank's grads
            p.grad.copy_(mine[n])
        sync = BucketedGradSync(store, None, payload=payload, chunk_mb=0.05)   # many small chunks
        for sid in (2, 0, 3, 1):                     # segments may complete in any order
            sync._launch(sid)
        scale = sync(store.grad)
        per = [grads(r) for r in range(world)]
        ddp = {n: sum(pr[n] for pr in per) / world for n in mine}     # DDP: mean of per-rank means
        ref.zero_grad()
        ref(rgb, x, lab).backward()                  # the global-pixel-mean gradient differs
        worst, worst_glob = 0.0, 0.0
        for n, p in prod.named_parameters():
            got = p.grad * scale
            den = ddp[n].abs().max().clamp_min(1e-12)
            worst = max(worst, ((got - ddp[n]).abs().max() / den).item())
            worst_glob = max(worst_glob, ((ref.get_parameter(n).grad - ddp[n]).abs().max() / den).item())
        tol = 1e-6 if payload == "fp32" else 4e-3           # bf16: ONE rounding of the fp32 sum (<= 2^-8 rel.)
        q.put((rank, worst <= tol, worst_glob > 1e-3, worst, worst_glob))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("payload", ["fp32", "bf16"])
def test_bucketed_grad_sync_paramstore_unequal_pixels_gloo_world2(payload):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 500) + (0 if payload == "fp32" else 1)
    procs = [ctx.Process(target=_worker_store, args=(r, 2, port, payload, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] and r[2] for r in res), res


def test_chunk_is_16B_aligned_for_fractional_mb(monkeypatch):
    """A fractional CMX_DP_CHUNK_MB must not misalign later chunks for the 16-B vector cast /
    shard-sum kernels: the chunk is a multiple of 64 elements."""
    from rgbx_semantic_segmentation_amd import dist as cdist

    class _Store:
        segments = [(0, 0, 1 << 20)]
    monkeypatch.setattr(cdist.BucketedGradSync, "_world", lambda self: 2)
    for mb, payload in ((0.05, "bf16"), (0.05, "fp32"), (0.3, "bf16"), (25, "fp32")):
        s = cdist.BucketedGradSync(_Store(), None, payload=payload, chunk_mb=mb)
        assert s.chunk % 64 == 0, (mb, payload, s.chunk)


def _worker_buffers(rank, world, port, q):
    """DDP's per-forward buffer broadcast (broadcast_buffers=True, train.py:145-146) on the
    flat BatchNorm buffer: after a local training step every rank's running statistics
    differ; the broadcast at the next forward makes them rank 0's, through the module views."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rgbx_semantic_segmentation_amd.dist import broadcast_buffers, flatten_bn_buffers
        torch.manual_seed(1)
        m = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 1), torch.nn.BatchNorm2d(4), torch.nn.ReLU(),
                                torch.nn.BatchNorm2d(4))
        flat = flatten_bn_buffers(m)
        ok = flat is not None and flat.numel() == 16 and m[1].running_mean.data_ptr() == flat.data_ptr()
        torch.manual_seed(100 + rank)               # a per-rank batch: local statistics drift apart
        m.train()
        m(torch.randn(2, 3, 5, 5))
        mine = flat.clone()
        allv = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(allv, mine)
        ok = ok and not torch.equal(allv[0], allv[1])
        # a subgroup without global rank 0 (world 3, group {1, 2}): the source is the group's
        # first member, global rank 1 (every rank creates the group; only members broadcast)
        sub = dist.new_group([1, 2]) if world >= 3 else None
        if sub is not None and rank in (1, 2):
            mine_sub = flat.clone()
            broadcast_buffers(flat, sub)
            ok = ok and torch.equal(flat, allv[1]) and (rank == 1 or not torch.equal(mine_sub, flat))
            flat.copy_(mine_sub)
        dist.barrier()
        broadcast_buffers(flat)
        ok = ok and torch.equal(flat, allv[0]) and torch.equal(m[3].running_var, allv[0][12:16])
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_bn_buffer_broadcast_gloo_world3_subgroup():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker_buffers, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] for r in res), res


def test_model_bn_buffers_are_one_flat_tensor():
    """EncoderDecoder's BatchNorm running statistics (FFM channel-embed BNs + the decoder's
    linear_fuse BN) flatten into one tensor with the state_dict keys / shapes unchanged."""
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    from rgbx_semantic_segmentation_amd.dist import flatten_bn_buffers
    m = EncoderDecoder(dict(backbone="mit_b0", num_classes=9, decoder_embed_dim=256))
    before = {k: v.clone() for k, v in m.state_dict().items() if "running" in k}
    flat = flatten_bn_buffers(m)
    after = {k: v for k, v in m.state_dict().items() if "running" in k}
    assert set(before) == set(after) and len(before) >= 4
    assert flat.numel() == sum(v.numel() for v in before.values())
    for k in before:
        assert torch.equal(before[k], after[k])
    flat.fill_(3.0)
    assert all(float(v.min()) == 3.0 for k, v in m.state_dict().items() if "running" in k)
