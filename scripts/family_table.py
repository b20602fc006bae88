"""Per-family roofline table of the CMX-B2 480x640 bs=2 train step:
kernel time and launches per family from a step census (scripts/step_census.py output), the
family's ALGORITHMIC work per step (FLOPs and/or HBM bytes counted from the layer shapes, each
tensor read once and written once at its storage dtype), the achieved rate and its fraction of
the roof (bf16 dense MFMA 2516.6 TFLOP/s, HBM 8 TB/s: /opt/skills/guides/MI355X_MICROARCH.md).

Usage:  python scripts/family_table.py profiles/r03_m_step_census.txt [--md]"""
from __future__ import annotations

import re
import sys

MFMA_TF, HBM_TBS = 2516.6, 8.0
B, G, H, W, K = 2, 2, 480, 640, 40
DIMS, DEPTHS, HEADS, SR = [64, 128, 320, 512], [3, 4, 6, 3], [1, 2, 5, 8], [8, 4, 2, 1]
E = 512                      # decoder embed dim
BF = 2                       # bytes per bf16 element


def grid(h, w, k, s, p):
    return (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1


def stage_shapes():
    out, h, w, cin = [], H, W, 3
    for s in range(4):
        k, st = (7, 4) if s == 0 else (3, 2)
        h, w = grid(h, w, k, st, k // 2)
        hk, wk = grid(h, w, SR[s], SR[s], 0) if SR[s] > 1 else (h, w)
        out.append(dict(N=h * w, C=DIMS[s], Nk=hk * wk, cin=cin, k=k, R=SR[s], d=DIMS[s] // HEADS[s], depth=DEPTHS[s]))
        cin = DIMS[s]
    return out


def work():
    """Per-step algorithmic work by family: {family: (flop, bytes)}."""
    imgs = B * G                              # image-streams per step (both modalities)
    gemm_mac = sra_flop = 0.0
    dw_elems = ln_rows_c = 0.0
    for st in stage_shapes():
        N, C, Nk, R = st["N"], st["C"], st["Nk"], st["R"]
        pe = N * C * st["cin"] * st["k"] ** 2
        blk = N * C * C + 2 * Nk * C * C + N * C * C + 8 * N * C * C + (Nk * R * R * C * C if R > 1 else 0)
        gemm_mac += imgs * (pe + st["depth"] * blk)
        gemm_mac += B * (2 * N * C * C + 24 * C * C + 17 * N * C * C)          # FRM + FFM 1x1s (per image pair)
        sra_flop += imgs * st["depth"] * 4 * N * Nk * C * 3.5                   # fwd + bwd (2.5x fwd)
        dw_elems += imgs * st["depth"] * N * 4 * C
        # norms: norm1, norm2 per block (+ attention norm on Nk rows), patch-embed norm, stage norm
        ln_rows_c += imgs * (st["depth"] * (2 * N + (Nk if R > 1 else 0)) + 2 * N) * C
    N1 = stage_shapes()[0]["N"]
    gemm_mac += B * (sum(s["N"] * s["C"] * E for s in stage_shapes()) + N1 * 4 * E * E + N1 * E * K)
    # forward + dgrad of every GEMM (the weight gradients are the grouped launch's)
    gemm_flop = 2 * 2 * gemm_mac
    wgrad_flop = 2 * gemm_mac
    return {
        "GEMM fwd+dgrad (tile / k-group / split-K)": (gemm_flop, None),
        "grouped wgrad GEMM + grouped reduce": (wgrad_flop, 2.079e9),
        "SRA attention (fwd, dQ, dK/dV, reduce)": (sra_flop, None),
        # fwd: read h, write out + act'(z) = 6 B; bwd: read da, act', h, write dh = 8 B per element
        "DWConv 3x3 + GELU (fwd_save, bwd_saved)": (None, dw_elems * (3 + 4) * BF),
        # fwd: read x, write y (4 B); bwd: read dy (+dy2), x, write dx (+dxs) ~ 5 tensors (10 B)
        "LayerNorm (fwd, bwd)": (None, ln_rows_c * (2 + 5) * BF),
        # 66.58 M params x (p, g, m, v read 16 B + p, m, v write 12 B + 16-bit shadow 2 B)
        "AdamW": (None, 66.58e6 * 30),
    }


FAMILIES = [
    ("grouped wgrad GEMM + grouped reduce", r"gemm_grouped_kernel|reduce_grouped_kernel"),
    ("GEMM fwd+dgrad (tile / k-group / split-K)", r"gemm_bf16_kernel|gemm_stream|gemm_reg|gemm_generic|splitk_reduce"),
    ("SRA attention (fwd, dQ, dK/dV, reduce)", r"sra_"),
    ("DWConv 3x3 + GELU (fwd_save, bwd_saved)", r"dw2_|dw_"),
    ("LayerNorm (fwd, bwd)", r"ln_fwd|ln_bwd|rowln"),
    ("AdamW", r"adamw"),
    ("BatchNorm (stats, fold, apply, bwd)", r"bn_"),
    ("FRM (pool, channel MLP, combine)", r"pool_|linear_fwd|linear_bwd|combine_|frm_|reduce_partials"),
    ("FFM context / cross attention", r"ffm_"),
    ("upsample + CE", r"ce_|upsample"),
    ("bilinear (decoder fuse adjoint)", r"bilinear"),
    ("im2col / col2im", r"im2col|col2im"),
]


def main():
    path = sys.argv[1]
    md = "--md" in sys.argv
    rows = []
    total = launches = 0.0
    head = ""
    for line in open(path):
        if line.startswith("launches/step"):
            head = line.strip()
            continue
        m = re.match(r"\s*(\d+)\s+([\d.]+)\s+([\d.]+)\s+(.*)", line)
        if m:
            rows.append((int(m.group(1)), float(m.group(2)), m.group(4)))
    fam = {name: [0, 0.0] for name, _ in FAMILIES}
    fam["other"] = [0, 0.0]
    for n, us, name in rows:
        total += us
        launches += n
        for fname, rx in FAMILIES:
            if re.search(rx, name):
                fam[fname][0] += n
                fam[fname][1] += us
                break
        else:
            fam["other"][0] += n
            fam["other"][1] += us
    wk = work()
    out = []
    hdr = ["family", "launches", "us/step", "share", "alg. GFLOP", "TFLOP/s", "of MFMA", "alg. GB", "TB/s", "of HBM"]
    out.append(hdr)
    for fname, (n, us) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        if n == 0:
            continue
        flop, byts = wk.get(fname, (None, None))
        row = [fname, str(n), f"{us:.0f}", f"{us / total:.1%}"]
        if flop:
            tf = flop / (us * 1e-6) / 1e12
            row += [f"{flop / 1e9:.1f}", f"{tf:.0f}", f"{tf / MFMA_TF:.1%}"]
        else:
            row += ["-", "-", "-"]
        if byts:
            tb = byts / (us * 1e-6) / 1e12
            row += [f"{byts / 1e9:.2f}", f"{tb:.2f}", f"{tb / HBM_TBS:.1%}"]
        else:
            row += ["-", "-", "-"]
        out.append(row)
    print(f"# {path}: {head}  (kernel time summed {total:.0f} us over {launches:.0f} launches)")
    if md:
        print("| " + " | ".join(out[0]) + " |")
        print("|" + "---|" * len(out[0]))
        for r in out[1:]:
            print("| " + " | ".join(r) + " |")
    else:
        for r in out:
            print(f"{r[0]:44s} " + " ".join(f"{c:>10s}" for c in r[1:]))


if __name__ == "__main__":
    main()
