"""Algorithmic work of the CMX training step, counted op by op as the reference executes
it: every Linear, Conv2d (incl. depthwise and the SR
patchify), QK^T, PV, K^T V and Q ctx; no elementwise / norm / softmax / pool / interpolate.
FLOP = 2 * MAC; training = 3 x forward.  Reported roofline fractions use THIS count."""
from __future__ import annotations

from .models.encoders.dual_segformer import MIT_SPECS, NUM_HEADS, SR_RATIOS


def _grid(H, W, k, s, p):
    return (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1


def forward_macs_per_image(backbone="mit_b2", H=480, W=640, K=40, E=512) -> int:
    dims, depths = MIT_SPECS[backbone]["embed_dims"], MIT_SPECS[backbone]["depths"]
    total = 0
    h, w = H, W
    cin = 3
    grids = []
    for s in range(4):
        k, st = (7, 4) if s == 0 else (3, 2)
        h, w = _grid(h, w, k, st, k // 2)
        N, C = h * w, dims[s]
        grids.append((N, C))
        pe = N * C * cin * k * k
        R = SR_RATIOS[s]
        if R > 1:
            hk, wk = _grid(h, w, R, R, 0)
            Nk = hk * wk
        else:
            Nk = N
        blk = N * C * C + 2 * Nk * C * C + 2 * N * Nk * C + N * C * C + 8 * N * C * C + 36 * N * C
        if R > 1:
            blk += Nk * R * R * C * C
        total += 2 * (pe + depths[s] * blk)                    # both modality streams
        d = C // NUM_HEADS[s]
        total += 2 * N * C * C + 2 * N * C + 24 * C * C        # FRM
        total += 17 * N * C * C + 4 * N * C * d + 9 * N * C    # FFM
        cin = C
    N1 = grids[0][0]
    total += sum(N * C * E for N, C in grids) + N1 * 4 * E * E + N1 * E * K
    return total


def train_flops_per_image(**kw) -> float:
    return 6.0 * forward_macs_per_image(**kw)


if __name__ == "__main__":
    m = forward_macs_per_image()
    print(m, train_flops_per_image() / 1e9, "GFLOP/img")
