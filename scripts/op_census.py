"""Which aten ops run in one eager B2 step (forward+backward+AdamW)? Counts + CUDA time, with
the Python frame that issued them, to find glue copies / adds / fills."""
import os, sys, collections
sys.path.insert(0, os.getcwd())
import torch
from torch.profiler import profile, ProfilerActivity
from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
from rgbx_semantic_segmentation_amd.optim import FusedAdamW
from rgbx_semantic_segmentation_amd.data import make_batch
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = EncoderDecoder(dict(backbone="mit_b2", num_classes=40, compute_dtype="bfloat16", decoder_embed_dim=512)).to(dev)
model.train()
opt = FusedAdamW(model, lr=6e-5, betas=(0.9, 0.999), weight_decay=0.01)
rgb, x, lab = make_batch(2, 480, 640, 40, seed=1, device=dev)
for _ in range(2):
    l = model(rgb, x, lab); l.backward(); opt.step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
    l = model(rgb, x, lab); l.backward(); opt.step()
    torch.cuda.synchronize()
want = ("aten::copy_", "aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::clone", "aten::contiguous",
        "aten::cat", "aten::mul", "aten::sum", "aten::index", "aten::zeros", "aten::to", "aten::_to_copy")
cnt = collections.Counter()
for ev in prof.events():
    if ev.name in want:
        st = [f for f in (ev.stack or []) if "rgbx_semantic" in f or "torch/autograd" in f or "bench" in f]
        key = (ev.name, st[0] if st else "?")
        cnt[key] += 1
for (n, f), c in sorted(cnt.items(), key=lambda kv: -kv[1]):
    print(f"{c:4d} {n:22s} {f}")
