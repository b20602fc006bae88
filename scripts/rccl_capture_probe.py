"""Which RCCL collectives survive HIP-graph capture at world size 1 (one case per process:
a crash ends only that case).  Usage: python scripts/rccl_capture_probe.py CASE
CASE in {a2a, ag, rs, rs32, ar, bc}_{eager, graph}: all_to_all_single / all_gather (bf16) /
reduce_scatter (bf16, fp32) / all_reduce (fp32, the default gradient payload and SyncBN) /
broadcast (fp32, the per-forward BatchNorm buffer sync).

Teardown: each phase prints a marker and a faulthandler watchdog dumps every
thread's Python stack if a phase blocks for CMX_PROBE_WATCHDOG_S (default 20 s), so a hang names
its frame.  CMX_PROBE_DEL_GRAPH=1 deletes the captured graph (and synchronises) before
destroy_process_group -- the order bench.py / train.py use."""
import faulthandler
import os
import sys

import torch
import torch.distributed as dist


def main(case):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29400 + os.getpid() % 500))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    print(f"torch {torch.__version__} hip {torch.version.hip} rccl {torch.cuda.nccl.version()}", flush=True)
    n = 1 << 16
    fp32 = case.split("_")[0] in ("rs32", "ar", "bc")
    src = torch.randn(n, device=dev).to(torch.float32 if fp32 else torch.bfloat16)
    out = torch.empty_like(src)

    def op():
        kind = case.split("_")[0]
        if kind == "a2a":
            dist.all_to_all_single(out, src)
        elif kind == "ag":
            dist.all_gather_into_tensor(out, src)
        elif kind in ("rs", "rs32"):
            dist.reduce_scatter_tensor(out, src)
        elif kind == "ar":
            out.copy_(src)
            dist.all_reduce(out)
        else:
            out.copy_(src)
            dist.broadcast(out, src=0)

    op()
    torch.cuda.synchronize()
    if case.endswith("graph"):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            op()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        out.zero_()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            op()
        g.replay()
        torch.cuda.synchronize()
    ok = torch.equal(out, src)
    print(f"{case}: {'ok' if ok else 'WRONG'}", flush=True)
    wd = float(os.environ.get("CMX_PROBE_WATCHDOG_S", "20"))
    faulthandler.dump_traceback_later(wd, repeat=True, exit=False)
    if case.endswith("graph") and os.environ.get("CMX_PROBE_DEL_GRAPH") == "1":
        print("teardown: del graph", flush=True)
        del g
        torch.cuda.synchronize()
    print("teardown: destroy_process_group", flush=True)
    dist.destroy_process_group()
    print("teardown: destroyed; exiting", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main(sys.argv[1])
