"""Optimizer, loop-trajectory and checkpoint parity of the HIP training step against the CPU
oracle (rows a1, a14, f1 of SURVEY.md §8).

* FusedAdamW (csrc/adamw.hip, one launch over the flat buffer) against
  torch.optim.AdamW(group_weight(model)) fed the SAME gradients, 4 steps with WarmUpPolyLR
  applied after each step (train.py:201-207) and the warm-up crossing steps 0 -> 1 -> 2:
  parameters and both moments after every step.
* 4 steps of train.py's loop body (train mode, injected DropPath / Dropout2d masks) against
  oracle/train_ref.train_steps in fp64: the loss of every step, and the parameter / moment
  trajectories.
* Checkpoints in the reference format (engine.py:84-150: model / optimizer / epoch /
  iteration, optionally with DDP's ``module.`` prefix) written by the oracle's
  torch.optim.AdamW restore into the HIP model + FusedAdamW (Engine.restore_checkpoint), and
  the HIP side's checkpoints load into torch.optim.AdamW; a step after the restore matches.
"""
import copy

import pytest
import torch

from oracle.cmx_ref import EncoderDecoder as RefModel, CMXConfig, DropPath
from oracle.train_ref import WarmUpPolyLR, make_optimizer, train_steps

pytestmark = pytest.mark.gpu

BACKBONE, K, B, H, W = "mit_b0", 9, 2, 128, 160


def _pair(dev, dtype="float32", seed=0):
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    torch.manual_seed(seed)
    ref = RefModel(CMXConfig(backbone=BACKBONE, num_classes=K))
    model = EncoderDecoder(dict(backbone=BACKBONE, num_classes=K, compute_dtype=dtype, decoder_embed_dim=512)).to(dev)
    model.load_state_dict(ref.state_dict(), strict=True)
    return ref, model


def _batch(seed=3):
    from rgbx_semantic_segmentation_amd.data import make_batch
    return make_batch(B, H, W, K, seed=seed)


def _moments(opt_t, ref):
    """{name: (exp_avg, exp_avg_sq, step)} of a torch.optim.AdamW over ``ref``'s parameters."""
    names = {id(p): n for n, p in ref.named_parameters()}
    out = {}
    for grp in opt_t.param_groups:
        for p in grp["params"]:
            st = opt_t.state[p]
            out[names[id(p)]] = (st["exp_avg"], st["exp_avg_sq"], float(st["step"]))
    return out


def _gpu_moments(opt, model):
    sd = opt.state_dict()
    order = opt._order
    names = {id(p): n for n, p in model.named_parameters()}
    return {names[id(p)]: (sd["state"][i]["exp_avg"].cpu(), sd["state"][i]["exp_avg_sq"].cpu(),
                           float(sd["state"][i]["step"])) for i, p in enumerate(order)}


def test_fused_adamw_matches_torch_adamw_on_shared_gradients(dev):
    from rgbx_semantic_segmentation_amd.optim import FusedAdamW
    ref, model = _pair(dev)
    ref.eval()
    model.eval()
    cfg = CMXConfig(backbone=BACKBONE, num_classes=K)
    opt_t = make_optimizer(ref, cfg)                       # group_weight + AdamW(0.9, 0.999), wd 0.01
    opt = FusedAdamW(model, lr=cfg.lr, betas=(0.9, 0.999), weight_decay=cfg.weight_decay)
    pol = WarmUpPolyLR(cfg.lr, cfg.lr_power, 100, 2)
    rgb, x, lab = _batch()
    gp = dict(model.named_parameters())
    for it in range(4):
        model(rgb.to(dev), x.to(dev), lab.to(dev)).backward()
        torch.cuda.synchronize()
        for n, p in ref.named_parameters():                # the SAME gradients on both sides
            p.grad = gp[n].grad.detach().cpu().clone()
        opt_t.step()
        opt.step()
        lr = pol.get_lr(it)                                # the LR lands one step late
        for grp in opt_t.param_groups:
            grp["lr"] = lr
        for grp in opt.param_groups:
            grp["lr"] = lr
        torch.cuda.synchronize()
        mt, mg = _moments(opt_t, ref), _gpu_moments(opt, model)
        worst_p = worst_m = 0.0
        for n, p in ref.named_parameters():
            q = gp[n].detach().cpu()
            dp = ((q - p.detach()).abs() - 1e-6 * p.detach().abs()).max().item()
            worst_p = max(worst_p, dp)
            for a, b in zip(mg[n][:2], mt[n][:2]):
                worst_m = max(worst_m, ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item())
            assert mg[n][2] == mt[n][2] == it + 1
        print(f"step {it}: next lr {lr:.3e}; max(|dp| - 1e-6 |p|) {worst_p:.2e}; moments rel {worst_m:.2e}")
        assert worst_p <= 1e-8, (it, worst_p)
        assert worst_m <= 1e-5, (it, worst_m)


def _inject(model, refs, n_calls, seed=7):
    g = torch.Generator().manual_seed(seed)
    bb = model.backbone
    flags = torch.ones(sum(bb.depths), 2, 2 * B)
    bi, per = 0, []
    for s in range(4):
        for i in range(bb.depths[s]):
            for stream, pre in enumerate(("", "extra_")):
                rblk = getattr(refs[0].backbone, f"{pre}block{s + 1}")[i]
                if isinstance(rblk.drop_path, DropPath):
                    mk = [(torch.rand(B, generator=g) > 0.3).double() for _ in range(2)]
                    per.append((f"{pre}block{s + 1}", i, mk))
                    for br in range(2):
                        flags[bi, br, stream * B:(stream + 1) * B] = mk[br].float()
            bi += 1
    d2 = (torch.rand(B, 512, generator=g) > 0.1).double()
    for r in refs:
        for name, i, mk in per:
            getattr(r.backbone, name)[i].drop_path.masks = [m.clone() for _ in range(n_calls) for m in mk]
        r.decode_head.dropout.mask = d2
    model.forced_masks = {"droppath": flags, "dropout2d": d2.float()}


def test_train_loop_trajectory_vs_oracle(dev):
    """train.py's loop body on both sides for 4 steps, each side computing its own gradients
    (HIP fp32 vs oracle fp64).  AdamW's first steps move every parameter by ~lr * sign(m), so a
    gradient element within rounding of 0 can flip its own update: the trajectory is compared in
    norm, relative to the distance travelled, and the losses step by step."""
    from rgbx_semantic_segmentation_amd.optim import FusedAdamW
    ref, model = _pair(dev)
    ref = ref.double()
    p0 = {n: p.detach().clone() for n, p in ref.named_parameters()}
    cfg = CMXConfig(backbone=BACKBONE, num_classes=K)
    opt_t = make_optimizer(ref, cfg)
    opt = FusedAdamW(model, lr=cfg.lr, betas=(0.9, 0.999), weight_decay=cfg.weight_decay)
    pol = WarmUpPolyLR(cfg.lr, cfg.lr_power, 100, 2)
    ref.train()
    model.train()
    steps = 4
    _inject(model, [ref], n_calls=steps)
    batches = [_batch(seed=3 + i) for i in range(steps)]
    gp = dict(model.named_parameters())
    for it, (rgb, x, lab) in enumerate(batches):
        l_ref = train_steps(ref, opt_t, pol, [(rgb.double(), x.double(), lab)], start_iter=it)[0]
        loss = model(rgb.to(dev), x.to(dev), lab.to(dev))
        l_gpu = loss.item()
        opt.zero_grad()
        loss.backward()
        opt.step()
        for grp in opt.param_groups:
            grp["lr"] = pol.get_lr(it)
        torch.cuda.synchronize()
        assert abs(l_gpu - l_ref) / abs(l_ref) < 1e-4, (it, l_gpu, l_ref)
        num = den = 0.0
        for n, p in ref.named_parameters():
            num += (gp[n].detach().cpu().double() - p.detach()).pow(2).sum().item()
            den += (p.detach() - p0[n]).pow(2).sum().item()
        rel = (num / max(den, 1e-300)) ** 0.5
        mt, mg = _moments(opt_t, ref), _gpu_moments(opt, model)
        mnum = mden = 0.0
        for n in mt:
            mnum += (mg[n][0].double() - mt[n][0]).pow(2).sum().item()
            mden += mt[n][0].pow(2).sum().item()
        mrel = (mnum / max(mden, 1e-300)) ** 0.5
        print(f"step {it}: loss gpu {l_gpu:.6f} oracle {l_ref:.6f}; |p - p_ref| / |p_ref - p0| {rel:.2e}; "
              f"exp_avg rel {mrel:.2e}")
        if den > 0:
            assert rel < 1e-2, (it, rel)
        assert mrel < 1e-3, (it, mrel)


def _ref_checkpoint(tmp_path, prefix=""):
    """Oracle model + torch.optim.AdamW(group_weight) after 2 steps, saved like
    engine.py:84-110 (epoch 3, iteration 5)."""
    torch.manual_seed(5)
    ref = RefModel(CMXConfig(backbone=BACKBONE, num_classes=K))
    ref.eval()
    cfg = CMXConfig(backbone=BACKBONE, num_classes=K)
    opt_t = make_optimizer(ref, cfg)
    pol = WarmUpPolyLR(cfg.lr, cfg.lr_power, 100, 0)
    rgb, x, lab = _batch(seed=9)
    for it in range(2):
        loss = ref(rgb, x, lab)
        opt_t.zero_grad()
        loss.backward()
        opt_t.step()
        for grp in opt_t.param_groups:
            grp["lr"] = pol.get_lr(it)
    path = tmp_path / "epoch-3.pth"
    torch.save({"model": {prefix + k: v for k, v in ref.state_dict().items()}, "optimizer": opt_t.state_dict(),
                "epoch": 3, "iteration": 5}, path)
    return ref, opt_t, path


@pytest.mark.parametrize("prefix", ["", "module."])
def test_restore_reference_checkpoint_then_step(dev, tmp_path, monkeypatch, prefix):
    from rgbx_semantic_segmentation_amd.engine.engine import Engine
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    from rgbx_semantic_segmentation_amd.optim import FusedAdamW
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    ref, opt_t, path = _ref_checkpoint(tmp_path, prefix)
    torch.manual_seed(123)                     # different init: everything must come from the file
    model = EncoderDecoder(dict(backbone=BACKBONE, num_classes=K, compute_dtype="float32",
                                decoder_embed_dim=512)).to(dev)
    model.eval()
    opt = FusedAdamW(model)
    with Engine(argv=["-c", str(path)]) as e:
        e.register_state(model=model, optimizer=opt)
        e.restore_checkpoint()
        assert e.state.epoch == 4 and e.state.iteration == 5
    gp = dict(model.named_parameters())
    for n, p in ref.named_parameters():
        assert torch.equal(gp[n].detach().cpu(), p.detach()), n
    mt, mg = _moments(opt_t, ref), _gpu_moments(opt, model)
    for n in mt:
        assert torch.equal(mg[n][0], mt[n][0]) and torch.equal(mg[n][1], mt[n][1]) and mg[n][2] == mt[n][2] == 2.0
    assert opt.param_groups[0]["lr"] == opt_t.param_groups[0]["lr"]
    # one more step on each side, same batch: the restored state drives the same update
    rgb, x, lab = _batch(seed=10)
    gref = copy.deepcopy(ref).double()
    opt_64 = make_optimizer(gref, CMXConfig(backbone=BACKBONE, num_classes=K))
    opt_64.load_state_dict(opt_t.state_dict())        # same group_weight order: state maps by position
    gref(rgb.double(), x.double(), lab).backward()
    opt_64.step()
    model(rgb.to(dev), x.to(dev), lab.to(dev)).backward()
    opt.step()
    torch.cuda.synchronize()
    num = den = 0.0
    for n, p in gref.named_parameters():
        p_before = dict(ref.named_parameters())[n].detach().double()
        num += (gp[n].detach().cpu().double() - p.detach()).pow(2).sum().item()
        den += (p.detach() - p_before).pow(2).sum().item()
    assert (num / den) ** 0.5 < 1e-2, (num / den) ** 0.5


def test_hip_checkpoint_loads_into_torch_adamw(dev, tmp_path, monkeypatch):
    """The other direction: Engine.save_checkpoint of the HIP model + FusedAdamW is a
    reference checkpoint (torch.optim.AdamW(group_weight(model)) and the oracle model load it)."""
    from rgbx_semantic_segmentation_amd.engine.engine import Engine
    from rgbx_semantic_segmentation_amd.optim import FusedAdamW
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    ref, model = _pair(dev)
    model.eval()
    opt = FusedAdamW(model)
    rgb, x, lab = _batch(seed=4)
    for _ in range(2):
        model(rgb.to(dev), x.to(dev), lab.to(dev)).backward()
        opt.step()
    with Engine(argv=[]) as e:
        e.register_state(model=model, optimizer=opt)
        e.update_iteration(7, 2)
        e.save_and_link_checkpoint(str(tmp_path / "ck"), str(tmp_path / "log"), str(tmp_path / "log_last"))
    sd = torch.load(tmp_path / "ck" / "epoch-7.pth", weights_only=True)
    assert set(sd) == {"model", "optimizer", "epoch", "iteration"}
    ref2 = RefModel(CMXConfig(backbone=BACKBONE, num_classes=K))
    ref2.load_state_dict(sd["model"], strict=True)
    opt_t = make_optimizer(ref2, CMXConfig(backbone=BACKBONE, num_classes=K))
    opt_t.load_state_dict(sd["optimizer"])
    mt, mg = _moments(opt_t, ref2), _gpu_moments(opt, model)
    for n in mt:
        assert torch.equal(mt[n][0], mg[n][0].cpu()) and mt[n][2] == 2.0
    gp = dict(model.named_parameters())
    for n, p in ref2.named_parameters():
        assert torch.equal(p.detach(), gp[n].detach().cpu())

