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
    """Per-step algorithmic work by family: {family: (flop, bytes)}, from the as-executed model
    of rgbx_semantic_segmentation_amd/floor.py (the same count as the bench line's step floor
    and the roofline object: executed FLOPs, e.g. 211.2 GFLOP for the grouped weight gradients
    after the decoder commute)."""
    sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
    from rgbx_semantic_segmentation_amd.floor import step_work
    w = step_work(backbone="mit_b2", H=H, W=W, B=B, K=K, E=E, n_params=66.58e6)
    names = {"gemm": "GEMM fwd+dgrad (tile / streaming / k-group / multi / split-K)", "wgrad": "grouped wgrad GEMM + grouped reduce",
             "sra": "SRA attention (fwd, dQ, dK/dV, reduce)", "dwconv": "DWConv 3x3 + GELU (fwd_save, bwd_saved)",
             "layernorm": "LayerNorm (fwd, bwd)", "adamw": "AdamW", "batchnorm": "BatchNorm (stats, fold, apply, bwd)",
             "frm": "FRM (pool, channel MLP, combine)", "ffm": "FFM context / cross attention",
             "ce": "upsample + CE", "bilinear": "bilinear (decoder fuse adjoint)", "im2col": "im2col / col2im",
             "pe1": "stage-1 patch embed (direct conv fwd, wgrad)"}
    return {names[k]: (v[0] or None, v[1] or None) for k, v in w.items()}


FAMILIES = [
    ("grouped wgrad GEMM + grouped reduce", r"gemm_grouped_kernel|reduce_grouped_kernel"),
    ("Mix-FFN bands", r"mixffn_"),
    ("GEMM fwd+dgrad (tile / streaming / k-group / multi / split-K)", r"gemm_bf16_kernel|gemm_stream|gemm_multi|gemm_generic|splitk_reduce"),
    ("SRA attention (fwd, dQ, dK/dV, reduce)", r"sra_"),
    ("DWConv 3x3 + GELU (fwd_save, bwd_saved)", r"dw2_|dw_"),
    ("LayerNorm (fwd, bwd)", r"ln_fwd|ln_bwd|rowln"),
    ("AdamW", r"adamw"),
    ("BatchNorm (stats, fold, apply, bwd)", r"bn_"),
    ("FRM (pool, channel MLP, combine)", r"pool_|linear_fwd|linear_bwd|combine_|frm_|reduce_partials"),
    ("FFM context / cross attention", r"ffm_"),
    ("upsample + CE", r"ce_|upsample"),
    ("bilinear (decoder fuse adjoint)", r"bilinear|adj3_|up3_"),
    ("im2col / col2im", r"im2col|col2im"),
    ("stage-1 patch embed (direct conv fwd, wgrad)", r"pe1_"),
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
    hdr = ["family", "launches", "us/step", "share", "alg. GFLOP", "TFLOP/s", "of MFMA", "alg. GB", "TB/s", "of HBM",
           "floor us", "x floor"]
    floor_total = 0.0
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
        fl = max((flop or 0) / (MFMA_TF * 1e6), (byts or 0) / (HBM_TBS * 1e6))
        floor_total += fl
        row += [f"{fl:.0f}" if fl else "-", f"{us / fl:.1f}" if fl else "-"]
        out.append(row)
    print(f"# {path}: {head}  (kernel time summed {total:.0f} us over {launches:.0f} launches)")
    wall = float(re.search(r"wall (\d+)", head).group(1)) if re.search(r"wall (\d+)", head) else total
    foot = (f"step floor (sum over families of max(FLOP / {MFMA_TF} TFLOP/s, bytes / {HBM_TBS} TB/s), "
            f"rgbx_semantic_segmentation_amd/floor.py): {floor_total:.0f} us = {floor_total / wall:.3f} of the {wall:.0f} us step")
    if md:
        print("| " + " | ".join(out[0]) + " |")
        print("|" + "---|" * len(out[0]))
        for r in out[1:]:
            print("| " + " | ".join(r) + " |")
        print("\n" + foot)
    else:
        for r in out:
            print(f"{r[0]:44s} " + " ".join(f"{c:>10s}" for c in r[1:]))
        print(foot)


if __name__ == "__main__":
    main()
