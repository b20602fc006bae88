"""Per-step kernel census from a rocprofv3 kernel trace of bench.py: the launches between two
consecutive step-start markers (one HIP-graph replay = one step; the steady-state step of median
wall time), grouped by kernel family.  The marker is step_masks_kernel, the one launch every step
opens with (drop-path masks); AdamW closes the step only without the per-segment overlap, which
splits it into several launches on a side stream.
Usage: python scripts/step_census.py <run_results.db> [top]"""
import collections
import re
import sqlite3
import sys


def kname(n):
    """Kernel name without its argument list: 'void ' and '(anonymous namespace)::' dropped, then
    everything from the first '(' that opens the PARAMETER list (the anonymous-namespace prefix
    used to be cut at its own '(' and left a blank name)."""
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)


c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = c.execute("select start, end, name from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if kname(r[2]).startswith("step_masks")]
if len(idx) < 3:   # older traces: AdamW (one launch per step) closes the step
    idx = [i + 1 for i, r in enumerate(rows) if kname(r[2]).startswith("adamw")]
# the step whose wall time is the median over the steady-state steps (the first three replays
# and the bench's last, host-drained ones aside): one representative replay, not the tail
def wall(j):
    seg_ = rows[idx[j]:idx[j + 1]]
    return max(r[1] for r in seg_) - seg_[0][0]
walls = [(wall(j), j) for j in range(3, len(idx) - 2)] or [(0, len(idx) - 2)]
pick = sorted(walls)[len(walls) // 2][1]
seg = rows[idx[pick]:idx[pick + 1]]
print(f"launches/step {len(seg)}  wall {(max(r[1] for r in seg) - seg[0][0]) / 1e3:.0f} us  busy {sum(r[1] - r[0] for r in seg) / 1e3:.0f} us"
      f"  (step {pick + 1} of {len(idx) - 1}: median wall of the steady-state steps)")
# idle time between one step's AdamW and the next step's first kernel (the replay boundary), and
# the largest idle gaps inside the step
prev = max(rows[:idx[pick]], key=lambda r: r[1])
print(f"boundary gap {(seg[0][0] - prev[1]) / 1e3:.1f} us after {kname(prev[2])[:40]}; first kernels: "
      + ", ".join(kname(r[2])[:30] for r in seg[:3]))
gaps, end, last = [], seg[0][1], seg[0]
for r in seg[1:]:
    s_, e_, n_ = r
    if s_ > end:
        gaps.append(((s_ - end) / 1e3, kname(n_)[:60], (end - seg[0][0]) / 1e3, kname(last[2])[:60]))
    if e_ > end:
        end, last = e_, r
print(f"idle inside the step {sum(g[0] for g in gaps):.0f} us over {len(gaps)} gaps; largest: "
      + "; ".join(f"{g:.1f} us before {n}" for g, n, _, _ in sorted(gaps, reverse=True)[:6]))
# every gap over 20 us with the kernel that ended last before it, where it sits in the step, and
# the launches around it in start order (which stream feeds which is not in the trace)
for g, n, at, prev_ in sorted(gaps, reverse=True):
    if g <= 20:
        break
    print(f"  gap {g:.1f} us at {at:.0f} us into the step: after {prev_} -> before {n}")
    t0 = seg[0][0] + at * 1e3
    near = [r for r in seg if t0 - 60e3 <= r[1] <= t0 + g * 1e3 + 30e3 or t0 - 60e3 <= r[0] <= t0 + g * 1e3 + 30e3]
    for r in near[:14]:
        print(f"      {(r[0] - seg[0][0]) / 1e3:8.1f} .. {(r[1] - seg[0][0]) / 1e3:8.1f}  {kname(r[2])[:70]}")
cat = collections.defaultdict(lambda: [0, 0.0])
for s, e, n in seg:
    k = kname(n)
    cat[k][0] += 1
    cat[k][1] += (e - s) / 1e3
for k, (n, t) in sorted(cat.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{n:5d} {t:8.1f} {t / n:7.2f}  {k[:100]}")

# kernel families of the step (DESIGN.md per-family table)
FAMILIES = [
    ("grouped wgrad + reduce (deferred weight gradients)", r"^(gemmk::)?gemm_grouped|^reduce_grouped"),
    ("GEMM (MFMA: linear / conv / decoder / attention projections)", r"^(gemmk::)?(gemm_|splitk_reduce)"),
    ("SRA attention (MFMA)", r"^sra_"),
    ("depthwise 3x3 conv + GELU (MixFFN)", r"^dw2_|^dw_"),
    ("Mix-FFN bands (fc1+DW+GELU, fc2 dgrad+DW bwd)", r"^mixffn_"),
    ("LayerNorm", r"^ln_"),
    ("BatchNorm", r"^bn_"),
    ("FRM (CM-FRM)", r"^pool_|^linear_|^combine_|^ifrm"),
    ("FFM (cross attention contexts)", r"^ffm_"),
    ("CE loss + upsample", r"^ce_|^upsample_ce"),
    ("bilinear / col2im / im2col / patch", r"^bilinear|^adj3_|^up3_|^col2im|^im2col|^patch"),
    ("optimizer (AdamW, non-finite check, step)", r"^adamw|^nonfinite|^step_"),
    ("elementwise / casts / partial sums", r"^act_|^residual|^scale_|^cast_|^reduce_partials|^partials|^colsum|^mul2"),
    ("torch / runtime", r"^at::|^__amd|^void at::"),
]
fam = collections.defaultdict(lambda: [0, 0.0])
for k, (n, t) in cat.items():
    name = next((f for f, rx in FAMILIES if re.search(rx, k)), "other")
    fam[name][0] += n
    fam[name][1] += t
busy = sum(t for _, t in fam.values())
print(f"\nfamily                                                       launches      us   share")
for f, (n, t) in sorted(fam.items(), key=lambda x: -x[1][1]):
    print(f"{f:60s} {n:8d} {t:8.1f} {100 * t / busy:6.1f}%")
