"""Per-shape GEMM probe: time chosen step shapes under several launch-policy knob settings
(cmx_tune), beside torch.bmm (hipBLASLt) and a device copy of the same output bytes (the
achievable write + read rate).  Usage (GPU box):
    python scripts/gemm_probe.py [KNOB=v1,v2 ...]"""
from __future__ import annotations

import itertools
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rgbx_semantic_segmentation_amd import kernels as K  # noqa: E402
from scripts.gemm_sweep import timeit  # noqa: E402

SHAPES = [(2, 38400, 256, 64, 0), (2, 38400, 64, 64, 1), (2, 38400, 64, 256, 0), (2, 9600, 128, 128, 1),
          (2, 9600, 512, 128, 0), (2, 2400, 320, 320, 1), (2, 2400, 1280, 320, 0), (2, 600, 512, 512, 1),
          (2, 38400, 64, 256, 1), (2, 38400, 256, 64, 1), (2, 9600, 128, 512, 0), (2, 9600, 512, 128, 1),
          (1, 38400, 512, 64, 0), (2, 2400, 320, 1280, 0)]


def operands(G, M, N, Kd, tB):
    A = torch.randn(G, M, Kd, device="cuda").to(torch.bfloat16)
    B = (torch.randn(G, Kd, N, device="cuda").to(torch.bfloat16).transpose(1, 2) if tB
         else torch.randn(G, N, Kd, device="cuda").to(torch.bfloat16))
    C = torch.empty(G, M, N, device="cuda", dtype=torch.bfloat16)
    return A, B, C


def main():
    arms = [a.split("=") for a in sys.argv[1:]]
    names = [n for n, _ in arms]
    grid = list(itertools.product(*[[int(v) for v in vs.split(",")] for _, vs in arms])) or [()]
    print(f"{'shape':34s} " + " ".join(f"{','.join(map(str, g)) or 'default':>12s}" for g in grid)
          + f" {'torch':>8s} {'copy':>8s} {'MB':>7s}")
    for G, M, N, Kd, tB in SHAPES:
        A, B, C = operands(G, M, N, Kd, tB)
        ts = []
        for g in grid:
            for n, v in zip(names, g):
                K.tune(n, v)
            ts.append(timeit(lambda: K.gemm(A, B, C)))
        tt = timeit(lambda: torch.bmm(A, B.transpose(1, 2)))
        D = torch.empty_like(C)
        tc = timeit(lambda: D.copy_(C))
        mb = (A.numel() + B.numel() + C.numel()) * 2 / 1e6
        print(f"G{G} M{M} N{N} K{Kd} tB{tB}".ljust(34) + " " + " ".join(f"{t:12.2f}" for t in ts)
              + f" {tt:8.2f} {tc:8.2f} {mb:7.1f}")


if __name__ == "__main__":
    main()
