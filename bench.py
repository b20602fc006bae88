"""Benchmark: CMX-B2 training step, 480x640, bs=2 per GPU, bf16, synthetic NYUv2-shape batch.

One step = forward + per-pixel CE + backward + (N>1: RCCL gradient all-reduce + SyncBN of
the decoder BN) + fused AdamW, i.e. train.py:185-207 for one batch.  The whole step is
captured once into a HIP graph (torch.cuda.CUDAGraph) and replayed; the WarmUpPolyLR
update is written into the optimizer's device LR scalar between replays.

Protocol: 2 eager steps, capture, W warm-up replays, a settle phase (windows of 10 replays
until >= 1 s of device time and two window medians within 2 %, at most 4 s; CMX_BENCH_SETTLE_S
/ _MAX_S), then EXACTLY K timed replays between barrier + synchronize.  The line carries the
per-replay device times (HIP events between replays: min / median / max of warm-up and timed
window, the settle window medians) and the sysfs sclk / mclk / power sampled over the timed
window, so a slow box shows itself in the record.

Usage:  python bench.py [--gpus N --steps K --warmup W]   (N>1: one rank per GPU via
        torch.distributed.run; rank 0 prints ONE JSON line).
"""
from __future__ import annotations

import argparse
import json
import gc
import os
import sys
import time


def _graph_streams_env(argv, env):
    """The HIP graph executor's stream count: 2 (CMX_GRAPH_STREAMS, 0 = the runtime default of 4).
    The replayed step has two concurrent chains (the encoder / decoder and the FFM branch on its
    side stream); with the default four executor streams the main chain's nodes are dealt
    round-robin over several hardware queues and every hand-over is a cross-queue wait (~9 us each
    in the kernel traces).  Measured (DESIGN.md round 5, 3 interleaved pairs): 272.5 vs 269.5
    img/s; the data-parallel step (RCCL segment all-reduces on a third captured stream) rehearsed
    at world size 1 under the same setting (round 6: 246.9 vs 251.0 img/s without the DP path), so
    every rank of an N-GPU run takes it too.  Never more executor streams than the process has
    hardware queues (GPU_MAX_HW_QUEUES): the count is clamped to it.  Set before torch loads the
    HIP runtime (the runtime reads its flags at load)."""
    n = env.get("CMX_GRAPH_STREAMS", "2")
    hwq = env.get("GPU_MAX_HW_QUEUES")
    if "DEBUG_HIP_FORCE_GRAPH_QUEUES" in env:
        n = env["DEBUG_HIP_FORCE_GRAPH_QUEUES"]
        if hwq and int(n) > int(hwq):
            raise SystemExit(f"[bench] DEBUG_HIP_FORCE_GRAPH_QUEUES={n} exceeds GPU_MAX_HW_QUEUES={hwq}: the HIP "
                             f"graph executor would deal the step over more streams than the process has queues")
        return
    if n == "0":
        n = "4"                                  # the runtime's own choice
        if not (hwq and int(hwq) < 4):
            return
    if hwq and int(n) > int(hwq):
        n = hwq
    env["DEBUG_HIP_FORCE_GRAPH_QUEUES"] = n


if __name__ == "__main__":
    _graph_streams_env(sys.argv[1:], os.environ)

import torch  # noqa: E402  (after the HIP runtime flags above)
import torch.distributed as dist  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_BF16_TFLOPS = 2516.6      # 256 CU x 2.4 GHz x 4096 FLOP/clk/CU (dense, MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--backbone", default="mit_b2")
    p.add_argument("--height", type=int, default=480)
    p.add_argument("--width", type=int, default=640)
    p.add_argument("--batch", type=int, default=2, help="per-GPU batch")
    p.add_argument("--classes", type=int, default=40)
    p.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "bf16", "float16", "fp16", "float32"],
                   help="compute dtype; float16 is the reference's AMP step (config 5) and implies --loss-scaling")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--allow-eager", action="store_true",
                   help="fall back to eager launches when the HIP-graph capture fails (default: exit 3)")
    p.add_argument("--loss-scaling", action="store_true",
                   help="config 5's AMP step: dynamic loss scaling (GradScaler) inside the captured step")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dry-run", action="store_true",
                   help="rehearse the rank launch on the CPU (gloo all-reduce), no GPU work")
    p.add_argument("--cpu-steps", type=int, default=3)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="0: every CPU this process may use (affinity, capped by the cgroup CPU quota)")
    return p.parse_args()


def host_cpus():
    """(threads to use, nproc, CPU model).  ``nproc`` is the machine's count; the usable share
    is the affinity mask capped by the cgroup v2 CPU quota (the GPU box grants a share of a
    much larger host: oversubscribing it would understate the CPU baseline)."""
    nproc = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, nproc, model


def cpu_baseline(args):
    """The oracle's restatement of the reference train step on the host cores (fp32), on
    bounded samples: the SAME workload as the GPU line (1 untimed + args.cpu_steps timed
    steps) and config 1 of BASELINE.json (CMX-B0 240x320 bs=1 K=9: 2 untimed + 10 timed)."""
    from oracle.cmx_ref import CMXConfig
    from oracle.train_ref import time_cpu_steps
    from rgbx_semantic_segmentation_amd.data import make_batch
    usable, nproc, model = host_cpus()
    threads = args.cpu_threads or usable
    batch = make_batch(args.batch, args.height, args.width, args.classes, seed=12345)
    cfg = CMXConfig(backbone=args.backbone, num_classes=args.classes)
    sec = time_cpu_steps(cfg, batch, warmup=1, steps=args.cpu_steps, threads=threads)
    b0 = make_batch(1, 240, 320, 9, seed=12345)
    sec0 = time_cpu_steps(CMXConfig(backbone="mit_b0", num_classes=9), b0, warmup=2, steps=10, threads=threads)
    return {"value": round(args.batch / sec, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle/train_ref.py (fp32 PyTorch-CPU restatement of train.py) {args.backbone} "
                      f"{args.height}x{args.width} bs={args.batch} K={args.classes}: 1 warm-up + {args.cpu_steps} "
                      f"timed steps, {sec:.2f} s/step",
            "host": {"nproc": nproc, "threads_used": threads, "cpu_model": model},
            "config1": {"workload": "CMX-B0 train step 240x320 bs=1 K=9 (BASELINE.json configs[0])",
                        "value": round(1.0 / sec0, 4), "unit": "images/s", "sample": f"2 warm-up + 10 timed steps, "
                                                                                     f"{sec0 * 1e3:.1f} ms/step"}}


def device_sysfs(dev_index: int):
    """The amdgpu sysfs directory of the HIP device (matched by PCI domain:bus:device), or None."""
    try:
        p = torch.cuda.get_device_properties(dev_index)
        path = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        return path if os.path.exists(os.path.join(path, "pp_dpm_sclk")) else None
    except Exception:
        return None


def read_clocks(sysfs):
    """Current (sclk MHz, mclk MHz, power W) from amdgpu sysfs; None for what cannot be read."""
    def cur(name):
        try:
            for line in open(os.path.join(sysfs, name)):
                if line.rstrip().endswith("*"):
                    return int(line.split(":")[1].strip().split("M")[0])
        except (OSError, ValueError, IndexError, TypeError):
            pass
        return None

    def power():
        try:
            import glob
            for h in glob.glob(os.path.join(sysfs, "hwmon", "hwmon*")):
                for n in ("power1_average", "power1_input"):
                    f = os.path.join(h, n)
                    if os.path.exists(f):
                        return round(int(open(f).read()) / 1e6, 1)
        except (OSError, ValueError, TypeError):
            pass
        return None
    if sysfs is None:
        return None, None, None
    return cur("pp_dpm_sclk"), cur("pp_dpm_mclk"), power()


class ClockSampler:
    """Samples sclk / mclk / power from sysfs on a host thread while the timed window runs
    (the replays are asynchronous, so the host thread costs the device nothing)."""

    def __init__(self, sysfs, period_s: float = 0.02):
        import threading
        self.sysfs, self.period, self.samples = sysfs, period_s, []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            self.samples.append(read_clocks(self.sysfs))
            self._stop.wait(self.period)

    def __enter__(self):
        if self.sysfs is not None:
            self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._t.is_alive():
            self._t.join()

    def summary(self):
        def stat(i):
            v = sorted(s[i] for s in self.samples if s[i] is not None)
            return None if not v else {"min": v[0], "median": v[len(v) // 2], "max": v[-1]}
        return {"samples": len(self.samples), "sclk_mhz": stat(0), "mclk_mhz": stat(1), "power_w": stat(2)}


def replay_stats(ms):
    v = sorted(ms)
    if not v:
        return None
    return {"n": len(v), "min": round(v[0], 4), "median": round(v[len(v) // 2], 4), "max": round(v[-1], 4)}


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, nproc: int, port: int):
    """The one-process-per-GPU launch of this script (reference: README.md:129,
    engine/engine.py:56): ``python -m torch.distributed.run`` with ``nproc`` ranks on this node,
    rendezvous on 127.0.0.1, the same bench arguments forwarded to every rank."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def check_world(gpus: int, env) -> str:
    """'launch' (spawn the N ranks), 'run' (this process is a rank or the only one) or raise
    SystemExit when ``--gpus`` disagrees with the launcher's WORLD_SIZE."""
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"[bench] --gpus {gpus} but WORLD_SIZE={world}: refusing to report "
                             f"a {world}-rank number as {gpus} GPUs")
        return "run"
    return "launch" if gpus > 1 else "run"


def main():
    args = parse()
    if args.dtype in ("float16", "fp16"):
        args.dtype, args.loss_scaling = "float16", True     # autocast fp16 always runs with a GradScaler
    # --gpus N > 1 without a launcher: start the N ranks as a child process BEFORE this
    # process touches the GPU, wait, forward its output and exit with its code
    if check_world(args.gpus, os.environ) == "launch":
        import subprocess
        cmd = launch_command(sys.argv[1:], args.gpus, free_port())
        print("[bench] " + " ".join(cmd), file=sys.stderr, flush=True)
        sys.exit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        # launcher rehearsal without a GPU: the ranks rendezvous over gloo, rank 0 reports
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            world_seen = int(t.item())
            dist.destroy_process_group()
        else:
            world_seen = 1
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": world_seen}))
        return
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    # CMX_FORCE_DIST=1: take the data-parallel path (RCCL, SyncBN, overlapped gradient
    # all-reduce) even at world size 1 -- a one-GPU rehearsal of the N > 1 code path
    use_dist = world > 1 or os.environ.get("CMX_FORCE_DIST") == "1"
    if use_dist:
        dist.init_process_group("nccl", device_id=dev)
        group = dist.group.WORLD

    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    from rgbx_semantic_segmentation_amd.optim import FusedAdamW
    from rgbx_semantic_segmentation_amd.data import make_batch
    from rgbx_semantic_segmentation_amd.utils.lr_policy import WarmUpPolyLR
    from rgbx_semantic_segmentation_amd.flops import train_flops_per_image
    from rgbx_semantic_segmentation_amd.floor import floor_table
    from rgbx_semantic_segmentation_amd import dist as cdist

    torch.manual_seed(12345)
    cfg = dict(backbone=args.backbone, num_classes=args.classes, compute_dtype=args.dtype, decoder_embed_dim=512)
    norm = torch.nn.SyncBatchNorm if use_dist else torch.nn.BatchNorm2d
    model = EncoderDecoder(cfg, norm_layer=norm).cuda(dev)
    sync = None
    if use_dist:
        model.process_group = group
        cdist.broadcast_parameters(model, group)
        sync = cdist.BucketedGradSync(model.store, group)
        model.backbone.grad_sync = sync        # segment all-reduces overlap the backward
    model.train()
    opt = FusedAdamW(model, lr=6e-5, betas=(0.9, 0.999), weight_decay=0.01, grad_sync=sync)
    niters = 1449 // 8 + 1
    policy = WarmUpPolyLR(6e-5, 0.9, 200 * niters, niters * 10)
    rgb, x, lab = make_batch(args.batch, args.height, args.width, args.classes, seed=12345 + rank, device=dev)

    scaler = None
    if args.loss_scaling:
        from rgbx_semantic_segmentation_amd.optim import GradScaler
        scaler = GradScaler(device=dev)

    # the backward's seed d loss / d loss = 1 as a persistent tensor: loss.backward() would fill a
    # fresh one with a kernel launch inside every step (same value, same semantics)
    seed = torch.ones((), device=dev)

    def step():
        loss = model(rgb, x, lab)
        opt.zero_grad()                 # train.py:188's order (arms the per-segment update overlap)
        if scaler is not None:
            scaler.scale(loss).backward(seed)
            scaler.step(opt)
            scaler.update()
        else:
            loss.backward(seed)
            opt.step()
        return loss

    it = 0

    def set_lr():
        nonlocal it
        lr = policy.get_lr(it)
        for g in opt.param_groups:
            g["lr"] = lr
        it += 1

    # eager warm-up (also primes the caching allocator and hipBLASLt heuristics)
    for _ in range(2):
        step()
        set_lr()
    torch.cuda.synchronize()
    graph = None
    if not args.no_graph:
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            # no garbage collection (and so no pinned-host frees recording events) inside the
            # capture; other threads' HIP calls cannot invalidate it (thread_local mode)
            gc.collect()
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                static_loss = step()
        except Exception as e:  # pragma: no cover - needs a GPU
            # a BASELINE-config line must not silently degrade to eager launches (a 3x slower
            # number): fail unless eager was asked for
            print(f"[bench] HIP graph capture failed: {e!r}", file=sys.stderr)
            if not args.allow_eager:
                raise SystemExit(3)
            graph = None

    def run_one():
        set_lr()
        if graph is not None:
            graph.replay()
        else:
            step()

    def replays(n):
        """n steps with a HIP event between consecutive ones (on the stream the graph replays
        on); returns the per-step device times in ms once the caller has synchronised."""
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        evs[0].record()
        for i in range(n):
            run_one()
            evs[i + 1].record()
        return lambda: [evs[i].elapsed_time(evs[i + 1]) for i in range(n)]

    sysfs = device_sysfs(local)
    clk_idle = read_clocks(sysfs)
    warm_ms = replays(args.warmup)
    torch.cuda.synchronize()
    warm_ms = warm_ms()
    # settle (warm-up bounded by a stabilised replay time): after the W
    # warm-up steps, replay in windows of 10 until >= settle_s of device time has passed and
    # two consecutive window medians agree within 2 % (at most settle_max_s).  Every rank
    # takes the same decision (the replays hold collectives at N > 1).
    settle_s = float(os.environ.get("CMX_BENCH_SETTLE_S", "1.0"))
    settle_max_s = max(settle_s, float(os.environ.get("CMX_BENCH_SETTLE_MAX_S", "4.0")))
    settle_med, settle_n, settle_t = [], 0, 0.0
    while settle_s > 0:
        w = replays(10)
        torch.cuda.synchronize()
        w = sorted(w())
        settle_n, settle_t = settle_n + 10, settle_t + sum(w) / 1e3
        settle_med.append(w[5])
        done = settle_t >= settle_max_s or (settle_t >= settle_s and len(settle_med) >= 2
                                            and abs(settle_med[-1] - settle_med[-2]) <= 0.02 * settle_med[-2])
        if use_dist:
            flag = torch.tensor([0 if done else 1], device=dev, dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            done = int(flag.item()) == 0
        if done:
            break
    # the host's own cost of one replay (enqueue of every node), with the device queue empty:
    # if it approaches the device time per step, the step turns host-bound
    host_enq = []
    for _ in range(3):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        run_one()
        host_enq.append((time.perf_counter() - h0) * 1e3)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    with ClockSampler(sysfs) as clocks:
        t0 = time.perf_counter()
        timed_ms = replays(args.steps)
        t_enq = time.perf_counter() - t0              # host time to enqueue the K replays
        torch.cuda.synchronize()
        if use_dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    timed_ms = timed_ms()
    print(f"[bench] host enqueue {t_enq / args.steps * 1e3:.3f} ms/step of {elapsed / args.steps * 1e3:.3f}",
          file=sys.stderr)
    trace_n = int(os.environ.get("CMX_BENCH_TRACE", "0"))
    if trace_n > 0:
        # diagnostic: the per-replay device-time series of warm-up, timed window and trace_n
        # more replays, with the clocks sampled beside them
        with ClockSampler(sysfs, 0.05) as tclk:
            extra = replays(trace_n)
            torch.cuda.synchronize()
        extra = extra()
        print("[bench-trace] idle clocks " + json.dumps(clk_idle), file=sys.stderr)
        print("[bench-trace] warmup " + json.dumps([round(v, 3) for v in warm_ms]), file=sys.stderr)
        print("[bench-trace] timed " + json.dumps([round(v, 3) for v in timed_ms]), file=sys.stderr)
        for i in range(0, trace_n, 50):
            print(f"[bench-trace] extra[{i}:] " + json.dumps([round(v, 3) for v in extra[i:i + 50]]), file=sys.stderr)
        print("[bench-trace] extra clocks " + json.dumps(tclk.summary()), file=sys.stderr)
        print("[bench-trace] extra clock series " + json.dumps(tclk.samples[::5]), file=sys.stderr)
    if use_dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms = elapsed / args.steps * 1e3
    images = args.batch * world * args.steps
    ips = images / elapsed
    fl_img = train_flops_per_image(backbone=args.backbone, H=args.height, W=args.width, K=args.classes)
    step_frac = (ips / world) * fl_img / (PEAK_BF16_TFLOPS * 1e12)

    # the step's roofline floor: sum over kernel families of max(FLOP / MFMA peak, bytes / HBM)
    # of the work as executed (floor.py); frac = floor / measured per-rank step time
    frows, ftot = floor_table(backbone=args.backbone, H=args.height, W=args.width, B=args.batch, K=args.classes,
                              n_params=float(model.store.flat.numel()))
    step_floor = {"floor_us": round(ftot, 1), "frac": round(ftot / (ms * 1e3), 4),
                  "families_us": {f: round(us, 1) for f, _, _, us, _ in frows}}

    # The bench line's ``roofline`` is the step's dominant kernel FAMILY by device time INSIDE the
    # replayed step: a kernel trace of 10 replays after the timed window,
    # every launch classified by name, the family's summed kernel time per step against its
    # algorithmic work.  Beside it: ``reissue`` (the same family with each launch re-issued in
    # place, warm -- the round-5 figure) and ``second`` (the grouped weight-gradient launch
    # re-launched standalone).  Every rank runs those two eager measurement steps (their SyncBN
    # collectives need all ranks); no optimizer step follows, so the gradient all-reduce hooks
    # are detached first.  They run last: their in-place re-launches leave the activations and
    # BN statistics meaningless.
    from rgbx_semantic_segmentation_amd.roofline import measure_dominant, measure_gemm_family, measure_in_step
    workload = f"CMX-{args.backbone.replace('mit_', '').upper()} train step {args.height}x{args.width} " \
               f"bs={args.batch} K={args.classes}"
    shape = dict(backbone=args.backbone, H=args.height, W=args.width, B=args.batch, K=args.classes)
    # (CMX_BENCH_NO_ROOFLINE=1: skipped, for the PMC / kernel-trace passes, whose per-launch
    # records must be the graph replays' only)
    skip = os.environ.get("CMX_BENCH_NO_ROOFLINE") == "1"
    roof = families = None
    if not skip and graph is not None:
        try:
            roof, families = measure_in_step(run_one, workload, shape, float(model.store.flat.numel()),
                                             step_us=ms * 1e3)
        except Exception as e:  # pragma: no cover - tracer availability is the box's
            print(f"[bench] in-step kernel trace failed: {e!r}", file=sys.stderr)
    model.backbone.grad_sync = None
    reissue = None if skip else measure_gemm_family(model, (rgb, x, lab), workload, shape)
    second = None if skip else measure_dominant(model, (rgb, x, lab), workload)
    if roof is None:
        roof = reissue
    else:
        roof["reissue"] = reissue
    if roof is None:
        roof = second
    elif second is not None:
        roof["second"] = second

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        out = {
            "metric": "train images/sec CMX-B2 480x640 bs=2/GPU at 1/2/4/8 MI355X; % MFMA roofline",
            "value": round(ips, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"bfloat16": "bf16", "bf16": "bf16", "float16": "fp16"}.get(args.dtype, "fp32"),
            "data": "synthetic (seeded uint8 RGB + replicated X plane, ImageNet-normalised; uniform labels "
                    "with one 25x25 ignore block per image; random-init weights)",
            "config": {"workload": workload, "model": f"CMX-{args.backbone}",
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "image": [args.height, args.width], "classes": args.classes,
                       "parallelism": f"dp{world}", "hip_graph": graph is not None,
                       "hip_graph_streams": os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES", "runtime default"),
                       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "runtime default"),
                       "loss_scaling": bool(args.loss_scaling)},
            "step_mfma_roofline": {"train_gflop_per_image": round(fl_img / 1e9, 3),
                                   "achieved_tflops": round((ips / world) * fl_img / 1e12, 2),
                                   "peak_tflops": PEAK_BF16_TFLOPS, "frac": round(step_frac, 5)},
            "step_floor": step_floor,
            "roofline": roof,
            "families_in_step": families,
            "cpu_baseline": cpu,
            "replay_ms": {"warmup": replay_stats(warm_ms), "timed": replay_stats(timed_ms),
                          "settle": {"replays": settle_n, "device_s": round(settle_t, 3),
                                     "window_medians": [round(v, 3) for v in settle_med]},
                          "host_enqueue_idle_queue": sorted(round(v, 3) for v in host_enq)},
            "clocks": {"idle": dict(zip(("sclk_mhz", "mclk_mhz", "power_w"), clk_idle)),
                       "timed": clocks.summary()},
        }
        print(json.dumps(out), flush=True)
    # teardown order: the captured graph holds RCCL work; release it and
    # drain the device before the communicator goes away
    del graph
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
