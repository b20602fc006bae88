"""Model-level parity of the BENCHMARKED bf16 training step at the BASELINE.json configs.

The HIP EncoderDecoder in bf16 (the compute dtype of bench.py) runs one train-mode step with
injected DropPath / Dropout2d masks at the configs' full shapes; the CPU oracle
(oracle/cmx_ref.py) runs the same weights, inputs and masks in fp64.  Compared: train-mode
logits (encode_decode), the loss, EVERY parameter gradient and the BN running statistics.

This is the only end-to-end check of the bf16-only kernels inside a whole step: the
deferred grouped weight-gradient GEMM, the implicit-GEMM patch-embed / SR convolutions, the
LDS-resident SRA attention kernels (Nk = 300 at 480 x 640, the key-chunked ones at
Nk = 1024 for B5) and the DWConv saved-activation backward.

Tolerance (derived, not picked): the same oracle run in fp32 with bf16 STORAGE emulated
(oracle/bf16_emul.py: bf16 GEMM weights, every Linear / Conv / norm input and output and the
gradients crossing them rounded to bf16) gives, per compared tensor, the error e_emu that bf16
storage alone causes against fp64.  The GPU error e_gpu must satisfy e_gpu <= RATIO * e_emu
(RATIO = 4: the emulation rounds at fewer points than the fused kernels, e.g. not the GELU
output or the attention probabilities), with a bounded number of outliers up to
OUTLIER_RATIO * e_emu (ReLU / max-pool decisions flipped by rounding move the few gradients
that sum over such a decision).  e = max|x - x64| / max|x64|.

Reference: models/builder.py:212-253, models/encoders/dual_segformer.py:366-442,
models/net_utils.py, models/decoders/MLPDecoder.py (train.py:185-200 step)."""
import copy
import time

import pytest
import torch

from oracle.cmx_ref import EncoderDecoder as RefModel, CMXConfig, DropPath
from oracle.bf16_emul import emulate_storage

pytestmark = pytest.mark.gpu

RATIO = 4.0
OUTLIER_RATIO = 12.0
# CM-FRM / FFM tensors of the bf16 cases: at most 2x the
# emulated error, outliers up to 4x for at most 8 % of them (11 of 148 at B2 / B4), and every
# yardstick (the error the comparison allows) below YARD_MAX of the tensor's largest gradient, so
# that no check is vacuous.  Two documented adjustments:
#  * ChannelWeights' first Linear (FRMs.s.channel_weights.mlp.0): a hidden unit whose ReLU
#    decision differs between the GPU step and fp64 in some sample (the GPU's post-ReLU activation,
#    recorded by functions.FRM_PROBE, against the sign of the fp64 pre-activation z) -- or between
#    the bf16 emulation and fp64 -- moves its whole gradient row (round 4: stage 2 unit 81 with
#    z = -0.00038, whose fp64 row is exactly zero).  Such a flipped row is excluded from the row
#    comparison when the flip is one rounding can cause: the fp64 |z| of the flipped sample lies
#    within the band bf16 storage puts on the layer's pre-activations (RATIO x the emulation's
#    largest pre-activation error in that sample, and at least 2^-7 of the layer's typical |z|).
#    A flip outside that band is an error and stays in the comparison.  The excluded count is
#    recorded (the round-5 form capped a band guess at 5 % of the rows instead, which rejected
#    the faster stage-3 SRA forward on config 4 for flips that were all inside the band);
#  * SpatialWeights' biases (a sum over all B*H*W pixels with heavy cancellation, e.g. 600 terms
#    at stage 4 whose sum is ~1/9 of the sum of their magnitudes): the yardstick is at least the
#    random-walk size of the bf16-storage emulation's per-pixel term errors,
#    sqrt(sum (dz_emu - dz_64)^2) / max|gradient| (rounding noise adds up like sqrt(N), not like
#    the L1 worst case N), and at least 2^-8 x sqrt(sum dz_64^2) / max|gradient|, the random-walk
#    error of bf16 inputs alone.
# The outlier share of the fusion tensors: measured on config 4 (B4, 148 fusion tensors) with the
# two SRA forward kernels of stage 3, whose summation orders differ and whose errors against fp64
# are equal at that shape (test_sra_fwd_kernel_choice): gpu / emu ratio median 1.29 / 1.23, 5 / 7
# tensors above 2x, none above 2.9x (profiles/r06_parity/).  4 % (5 of 148) sat exactly at the run-
# to-run spread of one kernel; 8 % keeps the 2x body and the 4x ceiling.
RATIO_FUSION = 2.0
OUTLIER_FUSION = 4.0
FUSION_OUTLIER_SHARE = 0.08
ZBAND = 2.0 ** -7
YARD_MAX = 0.25
BF16_EPS = 2.0 ** -8

CONFIGS = {
    # name: (backbone, H, W, batch, classes, dtype)   BASELINE.json configs[0..4] (configs[2] is
    # configs[1] per GPU: its multi-rank path is test_gpu_dist.py / test_dist_gloo.py)
    "config1_b0_240x320_bs1": ("mit_b0", 240, 320, 1, 9, "bfloat16"),
    "config2_b2_480x640_bs2": ("mit_b2", 480, 640, 2, 40, "bfloat16"),
    "config4_b4_480x640_bs4": ("mit_b4", 480, 640, 4, 9, "bfloat16"),
    "config5_b5_1024x1024_bs1": ("mit_b5", 1024, 1024, 1, 19, "bfloat16"),
    # config 5 as BASELINE states it: fp16 storage + dynamic loss scaling (train.py:185-198); the
    # backward runs on the loss times the GradScaler's initial scale, gradients unscaled after
    "config5_b5_1024x1024_bs1_fp16": ("mit_b5", 1024, 1024, 1, 19, "float16"),
    "config1_b0_240x320_bs1_fp16": ("mit_b0", 240, 320, 1, 9, "float16"),
}
LOSS_SCALE = 2.0 ** 16          # torch.cuda.amp.GradScaler's init_scale


def err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _masks(model_gpu, refs, B, n_calls, seed=11):
    """The same DropPath (per block, per branch, per sample) and Dropout2d (per sample,
    channel) keep masks for the GPU model and every oracle model, for ``n_calls`` forwards."""
    g = torch.Generator().manual_seed(seed)
    bb = model_gpu.backbone
    flags = torch.ones(sum(bb.depths), 2, 2 * B)
    bi = 0
    per_ref = []
    for s in range(4):
        for i in range(bb.depths[s]):
            for stream, pre in enumerate(("", "extra_")):
                rblk = getattr(refs[0].backbone, f"{pre}block{s + 1}")[i]
                if isinstance(rblk.drop_path, DropPath):
                    mk = [(torch.rand(B, generator=g) > 0.3).double() for _ in range(2)]
                    per_ref.append((f"{pre}block{s + 1}", i, mk))
                    for br in range(2):
                        flags[bi, br, stream * B:(stream + 1) * B] = mk[br].float()
            bi += 1
    d2 = (torch.rand(B, model_gpu.decode_head.embed_dim, generator=g) > 0.1).double()
    for ref in refs:
        for name, i, mk in per_ref:
            getattr(ref.backbone, name)[i].drop_path.masks = [m.clone() for _ in range(n_calls) for m in mk]
        ref.decode_head.dropout.mask = d2
    model_gpu.forced_masks = {"droppath": flags, "dropout2d": d2.float()}


def _inputs(B, H, W, K, seed=3):
    from rgbx_semantic_segmentation_amd.data import make_batch
    return make_batch(B, H, W, K, seed=seed)


def _record(case, loss, loss64, rows, bad, grad_bad, notes=None):
    """The per-tensor margins on record: {case}.json under $CMX_PARITY_OUT (default
    gpurun_out/parity, copied into profiles/ after a GPU run) with e_gpu, e_emu and their
    ratio for every compared tensor."""
    import json
    import os
    out = os.environ.get("CMX_PARITY_OUT", os.path.join("gpurun_out", "parity"))
    os.makedirs(out, exist_ok=True)
    notes = notes or {}
    tab = [dict({"tensor": n, "e_gpu": e, "e_emu": ee, "ratio": e / max(ee, 1e-30)},
                **({"note": notes[n]} if n in notes else {})) for n, e, ee in rows]
    rs = sorted(t["ratio"] for t in tab)
    with open(os.path.join(out, f"{case}.json"), "w") as f:
        json.dump({"case": case, "ratio_bound": RATIO, "outlier_ratio_bound": OUTLIER_RATIO,
                   "fusion_ratio_bound": RATIO_FUSION, "fusion_outlier_ratio_bound": OUTLIER_FUSION,
                   "fusion_yardstick_max": YARD_MAX,
                   "loss_gpu": loss, "loss_fp64": loss64, "n_tensors": len(tab),
                   "ratio_median": rs[len(rs) // 2], "ratio_max": rs[-1],
                   "n_over_bound": len(bad) + len(grad_bad), "tensors": tab}, f, indent=1)


def _fusion_probes(ref64):
    """fp64 hooks on every CM-FRM: the channel MLP's first-layer pre-activation z (B, 4C) of
    the last forward, and the gradients of the spatial head's two 1x1 conv outputs (their bias
    gradients are the sums of these over the pixels)."""
    probes = {}
    for s, frm in enumerate(ref64.backbone.FRMs):
        if not hasattr(frm, "channel_weights"):
            continue

        def zhook(m, a, o, s=s):
            probes[("z", s)] = o.detach()
        frm.channel_weights.mlp[0].register_forward_hook(zhook)
        for i in (0, 2):
            def ghook(m, a, o, s=s, i=i):
                if o.requires_grad:
                    o.register_hook(lambda g, s=s, i=i: probes.__setitem__((f"dsw{i}", s), g.detach()))
            frm.spatial_weights.mlp[i].register_forward_hook(ghook)
    return probes


def _fusion_adjust(n, gpu_g, emu_g, g64, den, probes, probes_emu=None, relu_gpu=None):
    """(e_gpu, e_emu, note) for the two adjusted CM-FRM cases (see RATIO_FUSION), else None.
    ``relu_gpu``: {stage: GPU post-ReLU channel-MLP hidden activation (B, 4C)}."""
    import re
    m = re.match(r"backbone\.FRMs\.(\d+)\.channel_weights\.mlp\.0\.(weight|bias)$", n)
    if m and ("z", int(m.group(1))) in probes and relu_gpu and int(m.group(1)) in relu_gpu:
        s = int(m.group(1))
        z = probes[("z", s)]
        band = (ZBAND * z.abs().median()).expand_as(z)
        if probes_emu and ("z", s) in probes_emu:     # the pre-activation error bf16 storage allows
            ez = (probes_emu[("z", s)].double() - z).abs().amax(1, keepdim=True)    # per sample, over units
            band = torch.maximum(band, RATIO * ez)
        on64 = z > 0
        flip_gpu = (relu_gpu[s].double().cpu() > 0) != on64                         # (B, 4C)
        flip = flip_gpu
        if probes_emu and ("z", s) in probes_emu:
            flip = flip | ((probes_emu[("z", s)].double() > 0) != on64)
        explained = flip & (z.abs() <= band)
        drop = explained.any(0)                       # rows with a rounding-band flip in some sample
        wild = int((flip & ~explained).any(0).sum())  # flips rounding cannot explain: kept in
        keep = ~drop
        if bool(keep.any()):
            eg = (gpu_g - g64)[keep].abs().max().item() / den
            ee = (emu_g - g64)[keep].abs().max().item() / den
            return eg, ee, (f"{int(drop.sum())} of {z.shape[1]} hidden units excluded: ReLU decision flipped "
                            f"inside the bf16 band ({int(flip_gpu.any(0).sum())} flipped on the GPU); "
                            f"{wild} flips outside the band (kept)")
    m = re.match(r"backbone\.FRMs\.(\d+)\.spatial_weights\.mlp\.(0|2)\.bias$", n)
    if m and (f"dsw{m.group(2)}", int(m.group(1))) in probes:
        key = (f"dsw{m.group(2)}", int(m.group(1)))
        t = probes[key]
        gmax = max(g64.abs().max().item(), 1e-300)
        allow = BF16_EPS * t.pow(2).sum((0, 2, 3)).sqrt().max().item() / gmax
        if probes_emu and key in probes_emu:
            allow = max(allow, (probes_emu[key].double() - t).pow(2).sum((0, 2, 3)).sqrt().max().item() / gmax)
        eg = (gpu_g - g64).abs().max().item() / den
        ee = (emu_g - g64).abs().max().item() / den
        return eg, max(ee, allow), f"random-walk allowance {allow:.3g} (emulated sum error {ee:.3g})"
    return None


def _check(name, e_gpu, e_emu, bad, ratio=RATIO):
    ok = e_gpu <= ratio * e_emu
    if not ok:
        bad.append((round(e_gpu / max(e_emu, 1e-30), 2), e_gpu, e_emu, name))
    return ok


@pytest.mark.timeout(1800)
@pytest.mark.parametrize("case", list(CONFIGS))
def test_bf16_train_step_vs_fp64_oracle(dev, case):
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    backbone, H, W, B, K, dtype = CONFIGS[case]
    h16 = {"bfloat16": torch.bfloat16, "float16": torch.float16}[dtype]
    S = LOSS_SCALE if h16 == torch.float16 else 1.0
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    torch.manual_seed(0)
    ref = RefModel(CMXConfig(backbone=backbone, num_classes=K))
    g = torch.Generator().manual_seed(1)
    for n, b in ref.named_buffers():             # non-trivial BN running statistics
        if n.endswith("running_mean"):
            b.copy_(torch.rand(b.shape, generator=g) * 0.2 - 0.1)
        elif n.endswith("running_var"):
            b.copy_(torch.rand(b.shape, generator=g) + 0.5)
    model = EncoderDecoder(dict(backbone=backbone, num_classes=K, compute_dtype=dtype,
                                decoder_embed_dim=512)).to(dev)
    model.load_state_dict(ref.state_dict(), strict=True)
    emu = emulate_storage(copy.deepcopy(ref), h16)
    ref64 = ref.double()
    probes = _fusion_probes(ref64) if h16 == torch.bfloat16 else {}
    probes_emu = _fusion_probes(emu) if h16 == torch.bfloat16 else {}
    from rgbx_semantic_segmentation_amd import functions as F
    F.FRM_PROBE = {} if h16 == torch.bfloat16 else None
    for m in (ref64, emu, model):
        m.train()
    _masks(model, [ref64, emu], B, n_calls=2)
    rgb, x, lab = _inputs(B, H, W, K)

    t0 = time.time()
    with torch.no_grad():
        lo64 = ref64.encode_decode(rgb.double(), x.double())
        lo_emu = emu.encode_decode(rgb, x)
        lo = model.encode_decode(rgb.to(dev), x.to(dev))
    t_cpu = time.time() - t0
    # fp16: back off from the initial scale like the GradScaler until the scaled backward is
    # finite (the scale a dynamic scaler settles at); the emulated oracle uses the same scale
    bufs = {n: b.detach().clone() for n, b in model.named_buffers()}
    while True:
        with torch.no_grad():                 # a retry starts from the same BN running statistics
            for n, b in model.named_buffers():
                b.copy_(bufs[n])
        loss = model(rgb.to(dev), x.to(dev), lab.to(dev))
        (loss * S).backward()
        torch.cuda.synchronize()
        if S == 1.0 or bool(torch.isfinite(model.store.grad).all()):
            break
        assert S > 1.0, "fp16 backward overflows at every loss scale"
        S *= 0.5
    model.store.grad.div_(S)
    relu_gpu = {}
    if F.FRM_PROBE is not None:
        for s_, frm in enumerate(model.backbone.FRMs):
            w = getattr(getattr(frm, "channel_weights", None), "mlp", [None])[0]
            if w is not None and id(w.weight) in F.FRM_PROBE:
                relu_gpu[s_] = F.FRM_PROBE[id(w.weight)]
        F.FRM_PROBE = None
    t0 = time.time()
    loss64 = ref64(rgb.double(), x.double(), lab)
    loss64.backward()
    loss_emu = emu(rgb, x, lab)
    (loss_emu * S).backward()
    for p in emu.parameters():
        p.grad.div_(S)
    t_cpu += time.time() - t0

    bad, rows = [], []
    e_l, e_le = err(lo, lo64), err(lo_emu, lo64)
    rows.append(("logits", e_l, e_le))
    _check("logits", e_l, e_le, bad)
    el = abs(loss.item() - loss64.item()) / abs(loss64.item())
    ele = abs(loss_emu.item() - loss64.item()) / abs(loss64.item())
    rows.append(("loss", el, ele))
    _check("loss", el, max(ele, 1e-6), bad)

    p64 = dict(ref64.named_parameters())
    pem = dict(emu.named_parameters())
    gmax = max(p.grad.abs().max().item() for p in ref64.parameters())
    grad_bad, fusion_bad, yard_bad, notes = [], [], [], {}
    n_fusion = 0
    for n, p in model.named_parameters():
        g64 = p64[n].grad
        assert g64 is not None and p.grad is not None, n
        den = max(g64.abs().max().item(), 1e-6 * gmax)
        gg = p.grad.detach().double().cpu()
        eg = (gg - g64).abs().max().item() / den
        ee = (pem[n].grad.double() - g64).abs().max().item() / den
        fusion = h16 == torch.bfloat16 and (".FRMs." in n or ".FFMs." in n)
        if fusion:
            adj = _fusion_adjust(n, gg, pem[n].grad.double(), g64, den, probes, probes_emu, relu_gpu)
            if adj is not None:
                eg, ee, notes[n] = adj
            n_fusion += 1
            _check(n, eg, ee, fusion_bad, ratio=RATIO_FUSION)
            if g64.abs().max().item() < 1e-6 * gmax:
                # structurally zero (a bias whose output a BatchNorm re-centres: ChannelEmbed's
                # channel_embed.3 / .4 biases and norm bias through the decoder's linear_fuse BN):
                # relative error is meaningless; held to RATIO_FUSION x the emulation's absolute error
                notes.setdefault(n, "structurally zero gradient (BatchNorm follows)")
            elif ee > YARD_MAX:
                # bf16 storage upstream of the block moves this gradient by more than YARD_MAX in
                # the emulation itself: the end-to-end check cannot bite, so the block's kernels
                # are held to a yardstick < YARD_MAX on identical inputs at this config's stage
                # shapes by tests/test_gpu_fusion_local.py
                yard_bad.append((round(ee, 3), n))
                notes[n] = (notes.get(n, "") + "; " if n in notes else "") + \
                    f"yardstick {ee:.3g} > {YARD_MAX}: bounded locally (tests/test_gpu_fusion_local.py)"
        else:
            _check(n, eg, ee, grad_bad)
        rows.append((n, eg, ee))
    for n, b in model.named_buffers():
        if "running" in n:
            b64 = dict(ref64.named_buffers())[n]
            eb, ebe = err(b, b64), err(dict(emu.named_buffers())[n], b64)
            rows.append((n, eb, ebe))
            _check(n, eb, max(ebe, 1e-7), bad)
    import os
    if os.environ.get("CMX_PARITY_DUMP"):
        # the GPU step's CM-FRM / FFM gradients and loss for an off-box look at where they
        # round (scripts/parity_frm_probe.py reruns the oracle variants on the same seeds)
        import numpy as np
        out = os.environ.get("CMX_PARITY_OUT", os.path.join("gpurun_out", "parity"))
        os.makedirs(out, exist_ok=True)
        keep = {n: p.grad.detach().float().cpu().numpy() for n, p in model.named_parameters()
                if (".FRMs." in "." + n or ".FFMs." in "." + n) and p.grad.numel() <= 3_000_000}
        np.savez_compressed(os.path.join(out, f"{case}_grads.npz"), loss=np.float64(loss.item()), **keep)
    ratios = sorted((e / max(ee, 1e-30), n) for n, e, ee in rows)
    print(f"\n{case}: loss scale {S:g}; cpu oracle {t_cpu:.1f} s; loss gpu {loss.item():.6f} fp64 {loss64.item():.6f}; "
          f"logits e_gpu {e_l:.3e} e_emu {e_le:.3e}; {len(rows)} tensors, gpu/emu error ratio "
          f"median {ratios[len(ratios) // 2][0]:.2f}, max {ratios[-1][0]:.2f} ({ratios[-1][1]})")
    print("worst ratios:", [(round(r, 2), n) for r, n in ratios[-8:]])
    _record(case, loss.item(), loss64.item(), rows, bad, grad_bad + fusion_bad, notes)
    n_allowed = max(2, len(rows) // 100)
    assert not bad, bad
    assert len(grad_bad) <= n_allowed and all(b[0] <= OUTLIER_RATIO for b in grad_bad), grad_bad[:10]
    n_fusion_allowed = max(2, int(FUSION_OUTLIER_SHARE * n_fusion))
    assert len(fusion_bad) <= n_fusion_allowed and all(b[0] <= OUTLIER_FUSION for b in fusion_bad), fusion_bad
    # the delegated tensors (yard_bad) are few and all in the fusion blocks' spatial / channel heads
    assert len(yard_bad) <= max(2, int(0.1 * n_fusion)), f"CM-FRM / FFM yardsticks above {YARD_MAX}: {yard_bad}"
