"""Time the fused AdamW launch (cmx_adamw_step) on a B2-sized flat buffer (66.58 M fp32
parameters + bf16 shadow) for several CMX_ADAMW_BLOCKS grid caps and the per-workgroup / per-lane
step scalars (CMX_ADAMW_BS), interleaved in one process
(cmx_tune), HIP events around 20 launches each.  Prints us per launch and TB/s of the 30 B /
parameter algorithmic traffic."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rgbx_semantic_segmentation_amd import kernels as K  # noqa: E402
from rgbx_semantic_segmentation_amd._lib import call, ptr, stream  # noqa: E402

n = 66_580_480
p = torch.randn(n, device="cuda") * 0.02
g = torch.randn(n, device="cuda") * 1e-3
m = torch.zeros(n, device="cuda")
v = torch.zeros(n, device="cuda")
sh = torch.empty(n, dtype=torch.bfloat16, device="cuda")
dec = torch.ones(n // 64, dtype=torch.uint8, device="cuda")
lr = torch.full((1,), 6e-5, device="cuda")
step = torch.zeros(1, device="cuda")


def run():
    call("cmx_adamw_step", ptr(p), ptr(g), ptr(m), ptr(v), ptr(sh), 1, ptr(dec), n, ptr(lr), ptr(step), 0.9, 0.999,
         1e-8, 0.01, 1.0, 0, stream())


for rep in range(2):
    for cap, bs in ((32768, 1), (16384, 1), (0, 1), (0, 0)):
        K.tune("ADAMW_BLOCKS", cap)
        K.tune("ADAMW_BS", bs)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        print(f"rep {rep} ADAMW_BLOCKS={cap:6d} ADAMW_BS={bs}: {us:7.1f} us  {30.0 * n / us / 1e6:5.2f} TB/s")
