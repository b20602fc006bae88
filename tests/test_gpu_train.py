"""train.py drop-in loop on the HIP path: runs, loss is finite and falls, checkpoints resume."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def test_train_loop_and_resume(dev, tmp_path, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    import train
    base = ["--backbone", "mit_b0", "--num-classes", "9", "--height", "96", "--width", "128", "--batch-size", "2",
            "--niters-per-epoch", "4", "--warm-up-epoch", "0", "--lr", "1e-4", "--compute-dtype", "float32",
            "--checkpoint-dir", str(tmp_path)]
    l1 = train.main(base + ["--nepochs", "1"])
    assert l1 == l1 and l1 > 0
    ck = tmp_path / "epoch-1.pth"
    assert ck.exists()
    sd = torch.load(ck, weights_only=True)
    assert sd["epoch"] == 1 and sd["iteration"] == 3
    assert len(sd["optimizer"]["state"]) == len(sd["optimizer"]["param_groups"][0]["params"]) + \
        len(sd["optimizer"]["param_groups"][1]["params"])
    # resume: epoch 2 runs from the restored weights / moments; the same 4 samples again -> lower loss
    # (lr 1e-4: at 1e-3 AdamW overshoots on these random labels and epoch 2 rises even uninterrupted)
    l2 = train.main(base + ["--nepochs", "2", "-c", str(ck)])
    assert l2 < l1, (l1, l2)


@pytest.mark.gpu
def test_segment_allreduce_sees_final_gradients(dev):
    """The overlapped gradient exchange (dist.BucketedGradSync) must reduce each segment only
    after every gradient in it is final.  World-size-1 rehearsal: the "all-reduce" doubles its
    segment on the side stream; any gradient written after its segment was launched stays
    undoubled and shows up against 2x the gradients of a plain backward."""
    from rgbx_semantic_segmentation_amd.dist import BucketedGradSync
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder

    class Doubling(BucketedGradSync):
        def _world(self):
            return 1

        def _reduce(self, seg):
            seg.mul_(2.0)

    torch.manual_seed(0)
    model = EncoderDecoder(dict(backbone="mit_b0", num_classes=9, compute_dtype="bfloat16",
                                decoder_embed_dim=256)).to(dev)
    model.eval()                        # deterministic (no DropPath / Dropout2d randomness)
    g = torch.Generator().manual_seed(3)
    rgb = torch.randn(2, 3, 64, 96, generator=g).to(dev)
    x = torch.randn(2, 3, 64, 96, generator=g).to(dev)
    lab = torch.randint(0, 9, (2, 64, 96), generator=g).to(dev)
    assert len(model.store.segments) == 4, model.store.segments
    model(rgb, x, lab).backward()
    torch.cuda.synchronize()
    ref = model.store.grad.clone()
    sync = Doubling(model.store, None)
    model.backbone.grad_sync = sync
    try:
        model(rgb, x, lab).backward()
        assert sync.launched, "no segment was launched during the backward"
        assert sync(model.store.grad) == 1.0
    finally:
        model.backbone.grad_sync = None
    torch.cuda.synchronize()
    bad = (model.store.grad - 2 * ref).abs() > 1e-6 * (1 + ref.abs())
    assert not bad.any(), f"{int(bad.sum())} gradient elements were reduced before they were final"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_graph_replay_matches_eager_backward(dev, dtype):
    """The backward replayed from a HIP graph (grouped weight-gradient launch, FFM side-stream
    fork / join as graph edges) gives the eager backward's gradients bit for bit."""
    from rgbx_semantic_segmentation_amd import deferred
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    torch.manual_seed(0)
    model = EncoderDecoder(dict(backbone="mit_b0", num_classes=9, compute_dtype=dtype,
                                decoder_embed_dim=256)).to(dev)
    model.eval()
    g = torch.Generator().manual_seed(4)
    rgb = torch.randn(2, 3, 64, 96, generator=g).to(dev)
    x = torch.randn(2, 3, 64, 96, generator=g).to(dev)
    lab = torch.randint(0, 9, (2, 64, 96), generator=g).to(dev)
    model(rgb, x, lab).backward()
    torch.cuda.synchronize()
    ref = model.store.grad.clone()
    deferred.reserve()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        model(rgb, x, lab).backward()
    torch.cuda.current_stream().wait_stream(s)
    import gc
    gc.collect()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        model(rgb, x, lab).backward()
    model.store.grad.zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(model.store.grad, ref), float((model.store.grad - ref).abs().max())


@pytest.mark.gpu
def test_grad_scaler_matches_torch_grad_scaler(dev):
    """a15 (train.py:13,56,185-198): the device GradScaler + FusedAdamW against torch's own
    ``torch.amp.GradScaler('cpu')`` stepping ``torch.optim.AdamW(group_weight(...))`` on the
    SAME scaled gradients, over a sequence of clean steps and steps with an inf / nan
    gradient: scale, growth tracker, skipped steps (AdamW's step count) and the parameters after
    every step.  The HIP side never syncs the host inside a step."""
    from oracle.cmx_ref import EncoderDecoder as RefModel, CMXConfig
    from oracle.train_ref import make_optimizer
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    from rgbx_semantic_segmentation_amd.optim import FusedAdamW, GradScaler
    torch.manual_seed(0)
    ccfg = CMXConfig(backbone="mit_b0", num_classes=9)
    ref = RefModel(ccfg)
    mod = EncoderDecoder(dict(backbone="mit_b0", num_classes=9, compute_dtype="float32",
                              decoder_embed_dim=512)).to(dev)
    mod.load_state_dict(ref.state_dict(), strict=True)
    ref.eval()
    mod.eval()
    g = torch.Generator().manual_seed(5)
    rgb = torch.randn(2, 3, 64, 96, generator=g).to(dev)
    x = torch.randn(2, 3, 64, 96, generator=g).to(dev)
    lab = torch.randint(0, 9, (2, 64, 96), generator=g).to(dev)
    opt_t = make_optimizer(ref, ccfg)
    opt = FusedAdamW(mod, lr=ccfg.lr, betas=(0.9, 0.999), weight_decay=ccfg.weight_decay)
    sc_t = torch.amp.GradScaler("cpu", init_scale=2.0 ** 10, growth_interval=2)
    sc = GradScaler(init_scale=2.0 ** 10, growth_interval=2, device=dev)
    gp = dict(mod.named_parameters())
    plan = ["clean", "inf", "clean", "clean", "nan", "clean", "clean"]
    for it, kind in enumerate(plan):
        sc.scale(mod(rgb, x, lab)).backward()
        if kind != "clean":                       # one bad element of one parameter's gradient
            gp["decode_head.linear_pred.weight"].grad.view(-1)[7] = float(kind)
        torch.cuda.synchronize()
        sc_t.scale(torch.ones(()))                # torch's scaler initialises lazily in scale()
        for n, p in ref.named_parameters():       # the SAME scaled gradients on both sides
            p.grad = gp[n].grad.detach().cpu().clone()
        sc_t.step(opt_t)
        sc_t.update()
        sc.step(opt)
        sc.update()
        torch.cuda.synchronize()
        steps_t = {float(st["step"]) for st in opt_t.state.values()} or {0.0}
        assert sc.get_scale() == sc_t.get_scale(), (it, kind, sc.get_scale(), sc_t.get_scale())
        assert int(sc.tracker.item()) == int(sc_t._growth_tracker.item()), (it, kind)
        assert steps_t == {float(opt.step_t.item())}, (it, kind, steps_t, opt.step_t.item())
        worst = 0.0
        for n, p in ref.named_parameters():
            q = gp[n].detach().cpu()
            worst = max(worst, ((q - p.detach()).abs() - 1e-6 * p.detach().abs()).max().item())
        print(f"step {it} ({kind}): scale {sc.get_scale():g}, tracker {int(sc.tracker.item())}, "
              f"adamw steps {opt.step_t.item():g}, max(|dp| - 1e-6|p|) {worst:.2e}")
        assert worst <= 1e-8, (it, kind, worst)
    assert sc.get_scale() == 2.0 ** 10 and float(opt.step_t.item()) == 5.0
