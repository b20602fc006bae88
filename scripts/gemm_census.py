"""GEMM census of one CMX training step: every cmx_gemm call (shape, transposes, epilogue),
re-timed standalone on its own operands with HIP events, beside torch.bmm (hipBLASLt) on the
same views.  Usage (GPU box):  python scripts/gemm_census.py [--backbone mit_b2] [--out file]
    [--ab KNOB=v1,v2,...]  time every call under each value of a launch-policy knob (cmx_tune),
                           interleaved call by call, and print per-shape and total deltas"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rgbx_semantic_segmentation_amd import kernels as K  # noqa: E402
from rgbx_semantic_segmentation_amd import functions as F  # noqa: E402


def timeit(fn, iters=20, warm=3):
    """GPU time per call: `iters` calls captured in one HIP graph (no host launch cost)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backbone", default="mit_b2")
    ap.add_argument("--out", default="gpurun_out/gemm_census.json")
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--ab", default="", help="KNOB=v1,v2: interleaved A/B of a cmx_tune knob")
    a = ap.parse_args()
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    from rgbx_semantic_segmentation_amd.data import make_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = EncoderDecoder(dict(backbone=a.backbone, num_classes=40, compute_dtype="bfloat16",
                                decoder_embed_dim=512)).to(dev)
    model.train()
    rgb, x, lab = make_batch(2, 480, 640, 40, seed=1, device=dev)
    calls = []
    orig = K.gemm

    def rec(A, B, C, **kw):
        calls.append((A, B, C, dict(kw)))
        return orig(A, B, C, **kw)

    K.gemm = rec
    loss = model(rgb, x, lab)
    loss.backward()
    torch.cuda.synchronize()
    K.gemm = orig
    if a.ab:
        return ab_census(calls, orig, a.ab)
    rows = []
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for A, B, C, kw in calls:
        G, M, K1 = A.shape
        Kd = K1 + (kw["A2"].shape[2] if kw.get("A2") is not None else 0)
        N = B.shape[1]
        tA = int(A.stride(1) == 1 and A.stride(2) != 1)
        tB = int(B.stride(1) == 1 and B.stride(2) != 1)
        flop = 2.0 * G * M * N * Kd
        t = timeit(lambda: orig(A, B, C, **kw))
        tt = None
        if not a.no_torch and kw.get("A2") is None:
            Bt = B.transpose(1, 2)
            od = {} if C.dtype == A.dtype else {"out_dtype": torch.float32}
            try:
                tt = timeit(lambda: torch.bmm(A, Bt, **od))
            except Exception:
                tt = None
        nbytes = (G * M * Kd + G * N * Kd) * A.element_size() + G * M * N * C.element_size()
        key = f"G{G} M{M} N{N} K{Kd} tA{tA} tB{tB} om{kw.get('out_mode', 0)} db{int(kw.get('dbias') is not None)}"
        r = dict(key=key, us=round(t, 2), tflops=round(flop / t / 1e6, 1), gbs=round(nbytes / t / 1e3, 1),
                 torch_us=round(tt, 2) if tt else None, flop=flop, bytes=nbytes)
        rows.append(r)
        g = agg[(tA, tB)]
        g[0] += 1; g[1] += t; g[2] += flop; g[3] += tt or 0.0
    tot = sum(r["us"] for r in rows)
    tott = sum(r["torch_us"] or 0 for r in rows)
    print(f"{len(rows)} gemm calls, cmx total {tot:.0f} us, torch(bmm) total {tott:.0f} us (where comparable)")
    for (tA, tB), (n, t, f, tt) in sorted(agg.items()):
        print(f"  tA{tA} tB{tB}: {n} calls {t:.0f} us  {f / t / 1e6:.1f} TFLOP/s  (torch {tt:.0f} us)")
    byk = collections.OrderedDict()
    for r in rows:
        k = byk.setdefault(r["key"], [0, 0.0, 0.0, r])
        k[0] += 1; k[1] += r["us"]; k[2] += r["torch_us"] or 0.0
    print(f"  {'shape':48s} {'n':>3} {'total_us':>9} {'us/call':>8} {'TF':>7} {'GB/s':>7} {'torch_us/call':>13}")
    for key, (n, t, tt, r) in sorted(byk.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"  {key:48s} {n:3d} {t:9.1f} {t / n:8.1f} {r['flop'] / (t / n) / 1e6:7.1f} "
              f"{r['bytes'] / (t / n) / 1e3:7.0f} {tt / n:13.1f}")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=0)


def ab_census(calls, orig, spec):
    knob, vals = spec.split("=")
    vals = [int(v) for v in vals.split(",")]
    base = K.tune_get(knob)
    byk = collections.OrderedDict()
    tot = [0.0] * len(vals)
    for A, B, C, kw in calls:
        G, M, K1 = A.shape
        Kd = K1 + (kw["A2"].shape[2] if kw.get("A2") is not None else 0)
        N = B.shape[1]
        tA = int(A.stride(1) == 1 and A.stride(2) != 1)
        tB = int(B.stride(1) == 1 and B.stride(2) != 1)
        key = f"G{G} M{M} N{N} K{Kd} tA{tA} tB{tB} om{kw.get('out_mode', 0)} db{int(kw.get('dbias') is not None)}"
        ts = []
        for rep in range(2):                   # two interleaved rounds, keep the best of each arm
            for i, v in enumerate(vals):
                K.tune(knob, v)
                t = timeit(lambda: orig(A, B, C, **kw))
                if rep == 0:
                    ts.append(t)
                else:
                    ts[i] = min(ts[i], t)
        e = byk.setdefault(key, [0, [0.0] * len(vals)])
        e[0] += 1
        for i, t in enumerate(ts):
            e[1][i] += t
            tot[i] += t
    if base >= 0:
        K.tune(knob, base)
    print(f"{len(calls)} gemm calls, knob {knob}: " + "  ".join(f"{v}: {t:.0f} us" for v, t in zip(vals, tot)))
    print(f"  {'shape':48s} {'n':>3} " + " ".join(f"{str(v):>9}" for v in vals))
    for key, (n, ts) in sorted(byk.items(), key=lambda kv: -max(kv[1][1]) + min(kv[1][1])):
        if max(ts) - min(ts) < 2.0:
            continue
        print(f"  {key:48s} {n:3d} " + " ".join(f"{t:9.1f}" for t in ts))


if __name__ == "__main__":
    main()
