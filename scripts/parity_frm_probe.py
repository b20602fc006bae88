"""Where does the bf16 GPU step's CM-FRM / FFM gradient error come from?  

Reads the GPU gradients dumped by tests/test_config_parity.py (CMX_PARITY_DUMP=1:
<case>_grads.npz), rebuilds the same oracle (seeds, weights, masks, inputs as the test) in
fp64 and in fp32 with bf16 storage emulated, and reports e_gpu / e_emu per FRM / FFM tensor
for emulation variants that round at additional points the GPU kernels round at:
  base      oracle/bf16_emul.py as the test uses it;
  +sum      the FRM output's gradient (FFM input + next stage input, summed by autograd in
            bf16 on the GPU) and the FFM residual sums rounded to bf16;
  +frmfp32  the FRM channel-MLP / spatial-head tensors NOT rounded (the GPU keeps them fp32).
Usage: python scripts/parity_frm_probe.py gpurun_out/parity/config2_b2_480x640_bs2_grads.npz"""
import copy
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

from oracle.cmx_ref import EncoderDecoder as RefModel, CMXConfig  # noqa: E402
from oracle import bf16_emul  # noqa: E402
import test_config_parity as T  # noqa: E402


def build(case):
    backbone, H, W, B, K, dtype = T.CONFIGS[case]
    torch.manual_seed(0)
    ref = RefModel(CMXConfig(backbone=backbone, num_classes=K))
    g = torch.Generator().manual_seed(1)
    for n, b in ref.named_buffers():
        if n.endswith("running_mean"):
            b.copy_(torch.rand(b.shape, generator=g) * 0.2 - 0.1)
        elif n.endswith("running_var"):
            b.copy_(torch.rand(b.shape, generator=g) + 0.5)
    return ref, (backbone, H, W, B, K)


def grads(model, rgb, x, lab, dtype):
    model.zero_grad()
    model.train()
    with torch.no_grad():
        model.encode_decode(rgb.to(dtype), x.to(dtype))          # the test's first (no-grad) forward
    loss = model(rgb.to(dtype), x.to(dtype), lab)
    loss.backward()
    return {n: p.grad.detach().double() for n, p in model.named_parameters()}


def round_grad_hook(t):
    return t.register_hook(lambda g: g.to(torch.bfloat16).to(g.dtype))


def main(path):
    case = os.path.basename(path).replace("_grads.npz", "")
    gpu = np.load(path)
    ref, (backbone, H, W, B, K) = build(case)
    variants = {}
    ref64 = copy.deepcopy(ref).double()
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    fake = EncoderDecoder(dict(backbone=backbone, num_classes=K, decoder_embed_dim=512))   # masks only (CPU)
    models = {"fp64": ref64}
    models["base"] = bf16_emul.emulate_storage(copy.deepcopy(ref), torch.bfloat16)
    T._masks(fake, list(models.values()), B, n_calls=2)      # (re-drawn identically per call: fixed seed)
    rgb, x, lab = T._inputs(B, H, W, K)
    g64 = grads(ref64, rgb, x, lab, torch.float64)
    variants["base"] = grads(models["base"], rgb, x, lab, torch.float32)
    # the same emulation with other fp32 summation orders (CPU thread counts): how much do these
    # gradients move when only the order of fp32 accumulation changes?
    nt = torch.get_num_threads()
    for t in (1, 3):
        torch.set_num_threads(t)
        em = bf16_emul.emulate_storage(copy.deepcopy(ref), torch.bfloat16)
        T._masks(fake, [em], B, n_calls=2)
        variants[f"threads{t}"] = grads(em, rgb, x, lab, torch.float32)
    torch.set_num_threads(nt)
    names = [n for n in gpu.files if n != "loss"]
    gmax = max(v.abs().max().item() for v in g64.values())
    print(f"{case}: GPU loss {float(gpu['loss']):.6f}")
    print(f"{'tensor':60s} {'e_gpu':>9s} " + " ".join(f"{k:>9s}" for k in variants))
    for n in sorted(names):
        ref_g = g64[n]
        den = max(ref_g.abs().max().item(), 1e-6 * gmax)
        eg = (torch.from_numpy(gpu[n]).double() - ref_g).abs().max().item() / den
        es = [(v[n] - ref_g).abs().max().item() / den for v in variants.values()]
        print(f"{n:60s} {eg:9.3e} " + " ".join(f"{e:9.3e}" for e in es) + f"   ratio {eg / max(es[0], 1e-30):6.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
