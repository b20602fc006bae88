"""Deferred weight-gradient work of the backward pass, issued as grouped launches.

In the reference every ``nn.Linear`` / ``nn.Conv2d`` / ``nn.LayerNorm`` backward computes its
weight gradient right away (autograd, ``train.py:192``) and DDP's reducer picks the gradients
up as they complete (``train.py:145-146``).  Nothing on the backward's critical path reads a
weight gradient, though: only the optimizer (and the gradient all-reduce) does.  On MI355X
the per-layer weight-gradient GEMMs, their split-K combines and the LayerNorm / DWConv
partial-sum reductions were ~550 small launches per CMX-B2 step, each a few microseconds of
mostly idle chip.  Here they are queued while the backward runs and issued as

  * ONE grouped GEMM launch (``cmx_gemm_grouped``): every queued weight-gradient problem of
    the segment, each with its own tile shape and split, in one grid;
  * ONE grouped reduce launch (``cmx_reduce_grouped``): the split-K slabs of those problems
    plus the queued LayerNorm dgamma/dbeta and DWConv dW/db partials;

when the segment's backward is done (``flush()``; ``arm()`` queues a flush at the end of
the backward pass as an autograd-engine callback).  Queued operands stay alive until the
flush, which costs HBM (the saved activations and upstream gradients of a segment), not
time -- 288 GB per GPU leaves room for it.

Records are packed on the host by the library (``cmx_*_pack``) into pinned memory and copied
to the device on the launch stream (``cmx_upload``).  Inside a HIP-graph capture the pinned
table must outlive the graph (every replay re-reads it): it is kept for the process lifetime.
Outside a capture it is released once an event recorded after the copy has completed.

``CMX_DEFER=0`` runs every weight gradient immediately instead (A/B switch for measurements).
"""
from __future__ import annotations

import collections
import ctypes
import os

import torch

from . import _lib
from ._lib import LIB, call, query, ptr, stream

ENABLED = os.environ.get("CMX_DEFER", "1") == "1"

_GREC = query("cmx_gemm_group_record_size")
_RREC = query("cmx_reduce_record_size")


class _Queue:
    def __init__(self):
        self.gemms = []        # argument tuples of cmx_gemm_group_pack (minus rec / ws / splitk / blk0)
        self.convs = []        # argument tuples of cmx_gemm_group_pack_conv_wgrad (one per tap)
        self.reds = []         # argument tuples of cmx_reduce_pack (minus rec / blk0)
        self.keep = []         # tensors the queued work reads or writes
        self.streams = {}      # streams the queued operands were produced on (FFM's side stream)
        self.dtype = 0         # operand dtype code of the queued GEMMs (1 bf16, 2 fp16; 0 = none yet)
        self.post = []         # callables run right after the next flush (deferred.after)
        self.armed = False


def _note_stream():
    st = torch.cuda.current_stream()
    _q.streams[st.cuda_stream] = st


_q = _Queue()
# observer(dev_table, nrec, blocks, problems, keep) is called after each grouped GEMM launch
# (bench.py's roofline re-times that launch standalone); None in normal operation
observer = None
_graph_tables = []             # pinned tables referenced by captured graphs (never freed)
_inflight = collections.deque()   # (event, pinned table) of eager uploads


def pending() -> bool:
    return bool(_q.gemms or _q.convs or _q.reds)


def arm() -> None:
    """Flush at the end of the running backward pass (idempotent per pass).  Outside a
    backward pass (direct callers, tests) the caller flushes explicitly."""
    if not _q.armed and torch._C._current_autograd_node() is not None:
        _q.armed = True
        torch.autograd.Variable._execution_engine.queue_callback(flush)


_H16 = {torch.bfloat16: 1, torch.float16: 2}


def _h16_code(*ts) -> int:
    """1 (bf16) / 2 (fp16) when every operand has that 16-bit dtype and matches the queue's
    GEMMs, else 0 (not eligible: the caller runs the problem now)."""
    code = _H16.get(ts[0].dtype, 0)
    if code == 0 or any(t.dtype != ts[0].dtype for t in ts) or (_q.dtype and _q.dtype != code):
        return 0
    return code


def _operand(t: torch.Tensor):
    if t.stride(2) == 1:
        return 0, t.stride(1), t.stride(0)
    if t.stride(1) == 1:
        return 1, t.stride(2), t.stride(0)
    return None


def wgrad(dz: torch.Tensor, x: torch.Tensor, Wg: torch.Tensor, bg: torch.Tensor | None = None) -> bool:
    """Queue Wg (fp32 (G, N, k) view) = dz^T x and bg (G, N) = column sums of dz, with
    dz (G, M, N), x (G, M, k) bf16 / fp16.  Returns False (nothing queued) when the problem is
    not eligible for the grouped 16-bit path; the caller then runs it immediately."""
    if not ENABLED or not dz.is_cuda:
        return False
    code = _h16_code(dz, x)
    if not code:
        return False
    if not _free:
        reserve()
    A, B = dz.transpose(1, 2), x.transpose(1, 2)           # (G, N, M), (G, k, M)
    G, N, M = A.shape
    k = B.shape[1]
    if Wg.shape != (G, N, k) or Wg.dtype != torch.float32 or Wg.stride(2) != 1:
        return False
    oa, ob = _operand(A), _operand(B)
    if oa is None or ob is None or oa[0] != 1 or ob[0] != 1:
        return False
    if bg is not None and (bg.dtype != torch.float32 or bg.shape[-1] != N or bg.stride(-1) != 1):
        return False
    Nk = k + (1 if bg is not None else 0)
    sdb = (bg.stride(0) if bg.dim() == 2 else 0) if bg is not None else 0
    args = (A, B, Wg, bg, G, N, Nk, M, oa[1], ob[1], Wg.stride(1), oa[2], ob[2], Wg.stride(0), sdb)
    # validate now (shape / alignment / 31-bit extents) so a refusal falls back immediately
    rec = (ctypes.c_uint8 * _GREC)()
    st = LIB.cmx_gemm_group_pack(ctypes.addressof(rec), ptr(A), ptr(B), ptr(Wg), ptr(bg), 1, G, N, Nk, M,
                                 oa[1], ob[1], Wg.stride(1), oa[2], ob[2], Wg.stride(0), sdb, 1, 1, 1,
                                 int(bg is not None), 1, 0)
    if st <= 0:
        return False
    _q.gemms.append(args)
    _q.dtype = code
    _q.keep.extend((dz, x))
    _note_stream()
    arm()
    return True


def after(fn) -> None:
    """Run ``fn`` on the flushing stream right after the next flush, which forms every weight
    gradient queued so far (the decoder fold's chain rule reads its queued dM_i products);
    with nothing queued, now."""
    if pending():
        _q.post.append(fn)
        arm()
    else:
        fn()


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, Wg: torch.Tensor, bg, geom) -> bool:
    """Queue the weight gradient of an NHWC convolution without im2col: one grouped-GEMM
    record per tap, its B operand gathered from x at that tap (cmx_gemm_group_pack_conv_wgrad).
    dy (G, NIg*Ho*Wo, N), x (G*NIg, H, W, C) bf16 / fp16, Wg fp32 (G, N, KH*KW*C), bg (G, N) or None;
    geom = (G, NIg, H, W, C, KH, KW, stride, pad, Ho, Wo).  False: not eligible, run the
    im2col path instead."""
    if not ENABLED:
        return False
    code = _h16_code(dy, x)
    if not code:
        return False
    G, NIg, H, W, C, KH, KW, st, pad, Ho, Wo = geom
    N = dy.shape[-1]
    if not (dy.is_contiguous() and x.is_contiguous() and Wg.stride(2) == 1 and Wg.shape[-1] == KH * KW * C):
        return False
    if C % 8 or N % 8 or (NIg * Ho * Wo) % 8:
        return False
    if not _free:
        reserve()
    sdy, sx = dy.stride(0), NIg * H * W * C
    sdb = (bg.stride(0) if bg.dim() == 2 else 0) if bg is not None else 0
    for tap in range(KH * KW):
        b = bg if tap == 0 else None
        _q.convs.append((dy, x, Wg, b, G, NIg, H, W, C, KH, KW, st, pad, Ho, Wo, N, tap, sdy, sx, Wg.stride(0), sdb))
    _q.dtype = code
    _q.keep.extend((dy, x))
    _note_stream()
    arm()
    return True


def reduce(src: torch.Tensor, dst: torch.Tensor, dst2: torch.Tensor | None, G: int, nblk: int, sg: int, sb: int,
           rows: int, cols: int, csplit: int, dg: int, ldd: int, dg2: int = 0, ldd2: int = 0,
           accumulate: bool = False) -> None:
    """Queue dst/dst2 (+)= sum over nblk partial rows of src (see cmx_reduce_pack)."""
    if not _free:
        reserve()
    _q.reds.append((src.data_ptr(), dst.data_ptr(), ptr(dst2), G, nblk, sg, sb, rows, cols, csplit, dg, ldd, dg2,
                    ldd2, int(accumulate)))
    _q.keep.append(src)
    _note_stream()
    arm()


# one pinned record table: 1 MiB (> 4000 grouped-GEMM records).  The B5 1024^2 step packs
# 284 KB of records into one flush; a 256 KB table made its HIP-graph capture fail and the
# bench fell back to eager launches (78 ms/step instead of ~30)
_TABLE_BYTES = 1024 * 1024
_free = []                        # pinned tables ready for reuse


def reserve(n: int = 16) -> None:
    """Pre-allocate pinned record tables.  Pinned allocation is not permitted while a stream
    is capturing, so a HIP-graph capture draws on this pool (EncoderDecoder.cuda() and every
    eager flush top it up)."""
    if torch.cuda.is_current_stream_capturing():
        return
    _drain()
    while len(_free) < n:
        _free.append(torch.empty(_TABLE_BYTES, dtype=torch.uint8, pin_memory=True))


def _drain() -> None:
    if torch.cuda.is_current_stream_capturing():      # event queries are not permitted then
        return
    while _inflight and _inflight[0][0].query():
        _free.append(_inflight.popleft()[1])


def _table(nbytes: int) -> torch.Tensor:
    if nbytes > _TABLE_BYTES:
        if torch.cuda.is_current_stream_capturing():
            raise _lib.CMXError(f"deferred: record table of {nbytes} B exceeds the pinned table size inside a capture")
        return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    _drain()
    if not _free:
        if torch.cuda.is_current_stream_capturing():
            raise _lib.CMXError("deferred: pinned table pool exhausted inside a HIP-graph capture; "
                                "call deferred.reserve(n) before capturing")
        reserve(4)
    return _free.pop()


def _upload(table: torch.Tensor, nbytes: int, device) -> torch.Tensor:
    dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
    call("cmx_upload", dev.data_ptr(), table.data_ptr(), nbytes, stream())
    if torch.cuda.is_current_stream_capturing():
        _graph_tables.append(table)          # every replay re-reads it
    else:
        ev = torch.cuda.Event()
        ev.record()
        _inflight.append((ev, table))
    return dev


def flush(max_blocks: int = 0) -> None:
    """Issue the queued weight-gradient GEMMs (one launch) and reductions (one launch) on the
    current stream.  max_blocks > 0 caps the GEMM launch's grid (a multiple of 8: each
    workgroup walks several tiles), for a flush issued beside the backward on a side stream."""
    _q.armed = False
    if _q.gemms or _q.convs or _q.reds:
        _issue(max_blocks)
    post, _q.post = _q.post, []
    for fn in post:
        fn()


def _issue(max_blocks: int = 0) -> None:
    q = _q
    gemms, convs, reds, keep, dcode = q.gemms, q.convs, list(q.reds), q.keep, q.dtype
    producers = q.streams
    q.gemms, q.convs, q.reds, q.keep, q.streams, q.dtype = [], [], [], [], {}, 0
    device = keep[0].device
    cur = torch.cuda.current_stream()
    for sid, st in producers.items():      # operands made on another stream: order after them
        if sid != cur.cuda_stream:
            cur.wait_stream(st)
            for t in keep:
                t.record_stream(cur)
    # the grouped-GEMM records and the reduce records share ONE pinned table and ONE upload
    gtab = None
    if gemms or convs:
        # one record per problem: (G, M, N incl. bias column, K, has_bias) drives split and slabs
        dims = [(a[4], a[5], a[6], a[7], a[3] is not None) for a in gemms]
        for c in convs:
            G, NIg, H, W, C, KH, KW, st, pad, Ho, Wo, N = c[4:16]
            dims.append((G, N, C + (1 if c[3] is not None else 0), NIg * Ho * Wo, c[3] is not None))
        splits = [query("cmx_gemm_grouped_splitk", G, M, N, K, int(hb)) for (G, M, N, K, hb) in dims]
        sizes = [query("cmx_gemm_workspace", G, M, N, s) if s > 1 else 0 for (G, M, N, K, hb), s in zip(dims, splits)]
        arena = torch.empty(max(1, sum((z + 255) // 256 * 64 for z in sizes)), dtype=torch.float32, device=device)
        nrec = len(dims)
        gbytes = (nrec * _GREC + 255) // 256 * 256
        # the reduce records follow the GEMM records: size the table for both (every split-K
        # problem adds at most two reduce records)
        nred_max = len(reds) + 2 * sum(1 for s in splits if s > 1)
        table = _table(gbytes + nred_max * _RREC)
        base = table.data_ptr()
        blk, off = 0, 0
        for i in range(nrec):
            s, sz = splits[i], sizes[i]
            ws = arena.data_ptr() + off if s > 1 else 0
            if i < len(gemms):
                A, B, Wg, bg, G, M, N, K, lda, ldb, ldc, sA, sB, sC, sdb = gemms[i]
                nb = LIB.cmx_gemm_group_pack(base + i * _GREC, ptr(A), ptr(B), ptr(Wg), ptr(bg), ws, G, M, N, K, lda,
                                             ldb, ldc, sA, sB, sC, sdb, 1, 1, 1, int(bg is not None), s, blk)
                dst = Wg.data_ptr()
            else:
                (dy, x, Wg, bg, G, NIg, H, W, C, KH, KW, st, pad, Ho, Wo, Nout, tap, sdy, sx, sC, sdb) = \
                    convs[i - len(gemms)]
                nb = LIB.cmx_gemm_group_pack_conv_wgrad(base + i * _GREC, ptr(dy), ptr(x), ptr(Wg), ptr(bg), ws, G, NIg,
                                                        H, W, C, KH, KW, st, pad, Ho, Wo, Nout, tap, sdy, sx, sC, sdb, s,
                                                        blk)
                M, N, ldc = Nout, C + (1 if bg is not None else 0), KH * KW * C
                dst = Wg.data_ptr() + 4 * tap * C
            if nb <= 0:
                raise _lib.CMXError(f"grouped-GEMM record pack failed ({nb}): {_lib.last_error()}")
            blk += nb
            if s > 1:
                # slabs: (G, s, M, Nr) fp32, Nr = real columns; then the bias-gradient column (G, s, M)
                Nr = N - 1 if bg is not None else N
                reds.append((ws, dst, 0, G, s, s * M * Nr, M * Nr, M, Nr, Nr, sC, ldc, 0, 0, 0))
                if bg is not None:
                    reds.append((ws + 4 * G * s * M * Nr, bg.data_ptr(), 0, G, s, s * M, M, 1, M, M, sdb, M, 0, 0, 0))
                off += (sz + 255) // 256 * 256
        gtab = (table, gbytes, nrec, blk, dims, arena)
    if reds:
        if gtab is None:
            table, gbytes = _table(len(reds) * _RREC), 0
        else:
            table, gbytes = gtab[0], gtab[1]
        base = table.data_ptr() + gbytes
        rblk = 0
        for i, r in enumerate(reds):
            nb = LIB.cmx_reduce_pack(base + i * _RREC, *r, rblk)
            if nb <= 0:
                raise _lib.CMXError(f"cmx_reduce_pack failed ({nb}): {_lib.last_error()}")
            rblk += nb
    if gtab is not None or reds:
        total = gbytes + len(reds) * _RREC
        dev = _upload(table, total, device)
        if gtab is not None:
            _, _, nrec, blk, dims, arena = gtab
            call("cmx_gemm_grouped_capped", dev.data_ptr(), nrec, blk, int(max_blocks) // 8 * 8, dcode, stream())
            keep.append(arena)
            if observer is not None:
                # algorithmic work per problem: (G, M, real N, K) and operand / result bytes
                work = [(G, M, N - (1 if hb else 0), K) for (G, M, N, K, hb) in dims]
                observer(dev, nrec, blk, work, keep, dcode)
        if reds:
            call("cmx_reduce_grouped", dev.data_ptr() + gbytes, len(reds), rblk, stream())
    # the caching allocator may hand the queued buffers out again once this stream has
    # passed the launches above (stream-ordered reuse): dropping `keep` here is safe
    del keep
