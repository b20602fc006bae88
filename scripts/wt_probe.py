"""Write-through probe (scripts/wt_probe.hip): per-kernel device time of writers with plain,
sc1 (write-through) and nt stores, each followed by a reader of the same bytes and a trivial
kernel, timed with HIP events between every launch, median of 30 repetitions.
Usage: python scripts/wt_probe.py"""
import ctypes
import os
import statistics

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libwt_probe.so"))
for f in (lib.wt_write, lib.wt_read, lib.wt_tiny):
    f.restype = ctypes.c_int
lib.wt_write.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p]
lib.wt_read.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
lib.wt_tiny.argtypes = [ctypes.c_void_p, ctypes.c_void_p]

dev = torch.device("cuda", 0)
buf = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
other = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
out = torch.zeros(4, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
names = {0: "plain", 1: "sc1", 2: "nt"}
print(f"{'MB':>6s} {'store':>6s} {'write us':>9s} {'tiny us':>8s} {'read us':>8s} {'tiny us':>8s}")
for mb in (2, 8, 16, 40, 120):
    nbytes = mb << 20
    grid = min(4096, max(256, nbytes // 16 // 256 // 4))
    for mode in (0, 1, 2):
        res = []
        for rep in range(33):
            lib.wt_read(other.data_ptr(), 200 << 20, 2048, out.data_ptr(), st)    # flush the caches between reps
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            ev[0].record()
            lib.wt_write(mode, buf.data_ptr(), nbytes, grid, st)
            ev[1].record()
            lib.wt_tiny(out.data_ptr(), st)
            ev[2].record()
            lib.wt_read(buf.data_ptr(), nbytes, grid, out.data_ptr(), st)
            ev[3].record()
            lib.wt_tiny(out.data_ptr(), st)
            ev[4].record()
            torch.cuda.synchronize()
            if rep >= 3:
                res.append([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(4)])
        med = [statistics.median(r[i] for r in res) for i in range(4)]
        print(f"{mb:6d} {names[mode]:>6s} " + " ".join(f"{v:8.2f}" for v in med), flush=True)
