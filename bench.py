#!/usr/bin/env python3
"""Benchmark: YOLOv11-s training throughput on MI355X (BASELINE.json configs[1] / [2]).

One step = one full training iteration on a synthetic 640x640 batch of 64 images per GPU:
forward (HIP plan) + v8 loss (fused kernels) + backward + RCCL gradient all-reduce (N > 1)
+ clip_grad_norm_(10) + AdamW — exactly train_yolo11_cuda.train_one_epoch's body.

    python bench.py [--gpus N --steps K --warmup W]

N > 1: either launched by torchrun (one process per GPU, RANK / WORLD_SIZE in the environment), or run
directly, in which case this process starts torchrun with N ranks as a child and relays rank 0's line.

Rank 0 prints ONE JSON line.  `roofline` is the dense 3x3 conv family against the 16-bit MFMA peak
(the north star's target: every fwd / dgrad / wgrad launch of a k=3 Conv block bracketed with HIP
events on its launch stream, in a pass that runs all launches on one stream, algorithmic FLOPs
summed / durations summed; in that pass the forward BatchNorm finalize is its own launch, not the conv
launch's tail as in the timed steps); `roofline_families` gives the same for every conv forward, data-gradient,
weight-gradient launch and the BatchNorm passes (HBM); `roofline_probe` is the heaviest single conv
launch; `roofline_step` prices the whole step against the MFMA peak.  `traffic` fields are read from
the committed counter passes (profiles/traffic.json, labelled with their source and commit), not
measured in this run.  `cpu_baseline` times the CPU oracle restatement (test infrastructure, fp32) on
a bounded sample of the same workload on every usable host CPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "yolo-scratch_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "images/sec at 640×640 bs=64/GPU, YOLOv11-s, 1/2/4/8 MI355X; mAP50 parity"
PEAK_BF16_TFLOPS = 2500.0          # dense bf16 MFMA, MI355X_MICROARCH.md chip table
HBM_PEAK_GBS = 8000.0
DP_TRACE_STEPS = 3
PROBE_STEPS = 3


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def traffic_entry(key: str):
    """The committed counter-pass entry for `key` (profiles/traffic.json), with its source labelled
    '<profiles dir> @ <commit>' — the traffic is NOT measured in this run (rocprofv3 counters need their
    own passes, tools/pmc_traffic.py / tools/pmc_layers.py), so the bench says where it comes from."""
    try:
        d = json.loads((ROOT / "profiles" / "traffic.json").read_text())
    except (OSError, ValueError):
        return None
    e = d.get(key)
    if not e:
        return None
    src = e.get("source", "profiles")
    if e.get("commit"):
        src += f" @ {e['commit']}"
    return {"bytes_per_launch": e["bytes_per_launch"], "source": f"profiles/traffic.json ({src})"}


def traffic_for(key: str):
    """HBM bytes per launch of the probe kernel from the committed rocprofv3 counter pass
    (profiles/traffic.json, written by tools/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE per the
    MI355X guide's gfx950 correction), or None when no pass for this probe exists."""
    f = ROOT / "profiles" / "traffic.json"
    try:
        d = json.loads(f.read_text())
    except (OSError, ValueError):
        return None
    e = d.get(key)
    return e["bytes_per_launch"] if e else None


def host_cpus():
    """(threads to use, description) for the CPU baseline: every CPU this process may run on —
    os.cpu_count(), bounded by its affinity mask and its cgroup CPU quota (a GPU box shows the whole
    machine's CPUs but grants a share of them) — plus the CPU model."""
    n = os.cpu_count() or 1
    usable = n
    try:
        usable = min(usable, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = -(-int(q) // int(per))
            usable = min(usable, max(quota, 1))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, {"nproc": n, "cgroup_quota_cpus": quota, "cpu_model": model}


def cpu_baseline(batch: int = 16, imgsz: int = 640, warmup: int = 1, steps: int = 3):
    """Oracle (fp32 CPU restatement of the reference) train step on a bounded sample, on every usable
    host CPU (SURVEY §8(d) CPU-baseline plan: torch.set_num_threads(os.cpu_count()), nproc and the CPU
    model stated)."""
    import torch
    from oracle import model as om
    from oracle import loss as ol
    from datasets.synthetic import synth_batch
    threads, host = host_cpus()
    torch.set_num_threads(threads)
    layers, save, P = om.build(om.load_cfg("s"))
    params = [v.requires_grad_(True) for k, v in P.items()
              if v.is_floating_point() and "running" not in k and not k.endswith("dfl.conv.weight")]
    opt = torch.optim.AdamW(params, lr=1e-3, weight_decay=5e-4)
    times = []
    for i in range(warmup + steps):
        b = synth_batch(batch, imgsz, seed=900 + i)
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        heads = om.forward(P, layers, save, b["img"], training=True)
        loss, _ = ol.v8_loss(heads, b)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 10.0)
        opt.step()
        times.append(time.perf_counter() - t0)
    t = sorted(times[warmup:])[len(times[warmup:]) // 2]
    return {"value": round(batch / t, 3), "unit": "images/sec", "cores": threads, "kind": "port", **host,
            "sample": f"YOLOv11-s {imgsz}x{imgsz} bs={batch} full train step (fwd+loss+bwd+clip+AdamW), "
                      f"oracle fp32 restatement, median of {steps} steps after {warmup} warm-up"}


def dp_overlap_probe(step_parts, dp, dev, first: int, steps: int) -> dict:
    """Per-bucket collective start / end and the backward's end, in ms from the step's start (events on the
    device; the median over `steps` steps), on THIS rank (rank 0's line).  Labelled unmeasured-on-hardware when
    the collectives ran over gloo (a one-GPU rehearsal)."""
    import statistics
    import torch
    import torch.distributed as dist
    recs = []
    dp.set_trace(True)
    try:
        for k in range(steps):
            evs = {}

            def mark(name):
                e = torch.cuda.Event(enable_timing=True)
                e.record(torch.cuda.current_stream(dev))
                evs[name] = e
            step_parts(first + k, mark)
            torch.cuda.synchronize(dev)
            t0 = evs["start"]
            tr = dp.last_trace()
            recs.append({"backward_end": t0.elapsed_time(evs["backward_end"]),
                         "sync_end": t0.elapsed_time(evs["sync_end"]),
                         "buckets": [(r["bucket"], r["bytes"], t0.elapsed_time(r["start"]), t0.elapsed_time(r["end"]))
                                     for r in tr if "start" in r]})
    finally:
        dp.set_trace(False)
    med = lambda xs: round(statistics.median(xs), 3) if xs else None
    nb = min(len(r["buckets"]) for r in recs) if recs else 0
    buckets = []
    for j in range(nb):
        buckets.append({"bucket": recs[0]["buckets"][j][0], "mb": round(recs[0]["buckets"][j][1] / 2 ** 20, 2),
                        "start_ms": med([r["buckets"][j][2] for r in recs]),
                        "end_ms": med([r["buckets"][j][3] for r in recs])})
    bwd = med([r["backward_end"] for r in recs])
    sync_end = med([r["sync_end"] for r in recs])
    coll = sum(b["end_ms"] - b["start_ms"] for b in buckets)
    hidden = sum(max(0.0, min(b["end_ms"], bwd) - b["start_ms"]) for b in buckets) if bwd is not None else 0.0
    backend = dist.get_backend()
    return {"steps": steps, "backend": backend, "buckets": buckets, "backward_end_ms": bwd, "sync_end_ms": sync_end,
            "exposed_ms": round(sync_end - bwd, 3) if bwd is not None else None,
            "collective_ms": round(coll, 3), "collective_before_backward_end_frac": round(hidden / coll, 3) if coll else None,
            "note": ("collectives bracketed by events on the comm stream (each waits for its collective: buckets serialized, "
                     "as one process group's collectives are); times from the step's start on rank 0") +
                    ("" if backend == "nccl" else "; gloo rehearsal, NOT an RCCL / xGMI measurement")}


def needs_launch(gpus: int, env=None) -> bool:
    """True when `--gpus N` (N > 1) was asked for but this process is not a rank of an N-process job: the
    driver's one-GPU command form (`python bench.py --gpus N`) then starts the ranks itself."""
    env = os.environ if env is None else env
    return gpus > 1 and "WORLD_SIZE" not in env and "RANK" not in env


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(gpus: int, argv, port: int):
    """The torchrun command that runs this script as `gpus` ranks on one node (one process per GPU,
    rendezvous on 127.0.0.1), with the caller's own arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def launch(gpus: int, argv) -> int:
    """Parent of an N-rank run: never touches the GPU (the ranks do), starts torchrun as a child process,
    relays its output (rank 0 prints the JSON line) and returns its exit code."""
    import subprocess
    cmd = launch_cmd(gpus, argv, free_port())
    log("launching", " ".join(cmd))
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main():
    # `--gpus N` without a torchrun environment: start the N ranks (before importing anything that could
    # initialise the GPU in this parent process)
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    known, _ = pre.parse_known_args()
    if needs_launch(known.gpus):
        sys.exit(launch(known.gpus, sys.argv[1:]))

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="images per GPU")
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--scale", default="s")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    # N > 1: the DP comm stream and RCCL's own stream join the 4 compute streams (default, 2 DAG, weight
    # gradients); with HIP's default 4 hardware queues they would share queues with compute streams (a
    # collective queued behind weight-gradient kernels).  8 queues, set before HIP initialises, give each
    # stream its own; at N = 1 8 vs 4 queues measured equal (profiles/r04/hw_queues_ab.txt).
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"

    import torch
    import torch.distributed as dist
    from yolomi import dist as ydist
    from models import build_yolo11
    from losses import v8DetectionLoss
    from datasets.synthetic import synth_batch
    from datasets import prepare_batch
    import yaml

    # A/B runs of a library policy in the step: YM_LIB_SET="ym_bn_set_bwd_fold=2 ym_conv_set_pipe=1" calls those
    # process-wide setters (include/yolomi.h) before the model is built; unset in the driver's runs
    if os.environ.get("YM_LIB_SET"):
        from yolomi._lib import lib as _yl0
        for kv in os.environ["YM_LIB_SET"].split():
            name, val = kv.split("=")
            getattr(_yl0(), name)(int(val))

    ctx = ydist.init_from_env()
    rank = ctx.rank if ctx else 0
    world = ctx.world if ctx else 1
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but this job has {world} rank(s) (WORLD_SIZE); "
                         f"run it as `python bench.py --gpus N` or under torchrun with N processes")
    if os.environ.get("YM_BENCH_RANKS_ONLY") == "1":
        # launcher check (tests/test_bench_launch_cpu.py): the job's rank count over a host all-reduce, no GPU
        one = torch.ones(1)
        if ctx:
            dist.all_reduce(one)
        if rank == 0:
            print(json.dumps({"n_gpus": world, "ranks_seen": int(one.item())}), flush=True)
        ydist.shutdown()
        return
    dev = torch.device("cuda", ctx.local_rank if ctx else 0)
    torch.cuda.set_device(dev)
    # every rank answers: the count of ranks that took part in one all-reduce of ones (RCCL, or gloo in a
    # one-GPU rehearsal), reported in the JSON line
    ranks_seen = 1
    if ctx:
        one = torch.ones(1, device=dev)
        dist.all_reduce(one)
        ranks_seen = int(one.item())
        if ranks_seen != world:
            raise SystemExit(f"bench.py: all-reduce saw {ranks_seen} ranks, expected {world}")

    cfg = yaml.safe_load((PKG / "configs" / "yolo11n_crater.yaml").read_text())
    cfg["scale"] = args.scale
    torch.manual_seed(0)
    model = build_yolo11(cfg, ch=1, nc=5).to(dev).train()
    crit = v8DetectionLoss(model, tal_topk=10)
    # the reference's clip_grad_norm_(10) + AdamW(lr 1e-3, wd 5e-4) (train_yolo11_cuda.py:58-62,
    # 440-451) as yolomi.optim.FusedAdamW: the same update in three HIP launches (YM_OPT=torch: PyTorch's
    # fused AdamW + clip_grad_norm_, for A/B runs)
    if os.environ.get("YM_OPT", "fused") == "torch":
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=5e-4, fused=True)
    else:
        from yolomi.optim import FusedAdamW
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=5e-4, max_grad_norm=10.0)
    fuses_clip = getattr(opt, "fuses_clip", False)
    dp = ydist.GradSync(model, ctx) if ctx else None
    if dp:
        dp.broadcast_state()

    # synthetic inputs resident in HBM before the timed region (per-rank seeds)
    n_batches = 4
    batches = []
    for i in range(n_batches):
        b = synth_batch(args.batch, args.imgsz, seed=1000 * rank + i)
        b = prepare_batch(b, dev)                  # the data path's H2D (records max_gt on the host)
        batches.append(b)

    def step_parts(i, mark=None):
        """One training step; mark(name) (optional) is called at its phase boundaries (dp_overlap_probe)."""
        b = batches[i % n_batches]
        opt.zero_grad(set_to_none=True)
        if mark:
            mark("start")
        preds = model(b["img"])
        loss, items = crit(preds, b)
        loss.backward()
        if mark:
            mark("backward_end")
        if dp:
            dp.sync()
        if mark:
            mark("sync_end")
        if not fuses_clip:
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=10.0)
        opt.step()
        return loss

    def step(i):
        return step_parts(i)

    # model setup: the plan's first forward/backward allocate its workspaces (and with YM_GRAPH=1
    # the second captures them as HIP graphs) — done here, untimed, whatever --warmup is
    for i in range(2):
        step(i)
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    plan = model.__dict__["_ym_last_plan"]
    from yolomi.graph import ConvBN
    convs = [op for op in plan.ops if type(op) is ConvBN]
    dom = max(convs, key=lambda op: op.flops())
    plan.probe, plan.probe_events = dom, []
    # position of the probe among a step's implicit-GEMM forward launches (ConvBN: 1, Detect
    # level: 2), for finding it in a rocprofv3 counter pass (tools/pmc_traffic.py)
    fwd_seq = []
    for op in plan.ops:
        if type(op) is ConvBN:
            fwd_seq.append(op)
        elif type(op).__name__ == "HeadLevel":
            fwd_seq += [op, op]
    probe_rank, probe_count = fwd_seq.index(dom), len(fwd_seq)
    probe_key = f"{dom.ci}->{dom.co} k{dom.k} s{dom.s} out {dom.y.H}x{dom.y.W} bs{args.batch}"
    # the probe kernel is timed in the same process right after the timed region, in PROBE_STEPS
    # eager steps (events on the stream the probe conv is launched on; per-kernel events cannot sit
    # inside a replayed HIP graph, YM_GRAPH=1)
    plan.probe = None

    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    for i in range(args.steps):
        loss = step(args.warmup + i)
        marks.append(time.perf_counter())
    torch.cuda.synchronize()
    if os.environ.get("YM_BENCH_STEP_TIMES"):
        # host time at which each step() returned (no sync inside the loop): a host that runs ahead of
        # the GPU returns faster than the GPU step; one blocked every step returns at the GPU's pace
        log("host step returns (ms): " + " ".join(f"{1e3 * (b - a):.1f}" for a, b in zip([t0] + marks, marks)))
    if dp:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dp:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    # N > 1: where the bucket collectives ran against the backward (dp_overlap in the JSON line), over a few extra steps
    # after the timed region with every collective bracketed by events on the comm stream (Buckets.trace); the
    # exposed communication is what the step waits for after the backward's last kernel
    dp_overlap = dp_overlap_probe(step_parts, dp, dev, args.warmup + args.steps, DP_TRACE_STEPS) if dp else None
    # the probe and family passes time the conv kernels' own work: there the forward BatchNorm finalize runs as its
    # own launch (YM_FOLD=0, timed in the 'bn' family) instead of as the conv launch's tail (the timed region above
    # and the driver's step run it folded)
    saved_fold = os.environ.get("YM_FOLD")
    os.environ["YM_FOLD"] = "0"
    plan.probe, plan.probe_events = dom, []
    for i in range(PROBE_STEPS):
        step(args.warmup + args.steps + i)
    torch.cuda.synchronize()
    plan.probe = None
    # kernel families by time: every conv forward / data-gradient / weight-gradient launch and every
    # BatchNorm pass (finalize + apply, reduce + finalize + apply) bracketed with HIP events over
    # PROBE_STEPS steps, run on ONE stream (YM_STREAMS=1, YM_SIDE_STREAM=0) so that each duration is
    # the kernel's own, not stretched by kernels of other streams sharing the CUs
    saved = {k: os.environ.get(k) for k in ("YM_STREAMS", "YM_SIDE_STREAM")}
    os.environ.update(YM_STREAMS="1", YM_SIDE_STREAM="0")
    plan.family_events = {"fwd": [], "dgrad": [], "wgrad": [], "bn": [], "fwd3": [], "dgrad3": [], "wgrad3": []}
    for i in range(PROBE_STEPS):
        step(args.warmup + args.steps + PROBE_STEPS + i)
    torch.cuda.synchronize()
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    fams = {}
    for kind, evs in plan.family_events.items():
        ms = sum(a.elapsed_time(b) for a, b, _ in evs) / PROBE_STEPS
        work = sum(w for _, _, w in evs) / PROBE_STEPS
        fams[kind] = (ms, work, len(evs) // PROBE_STEPS)
    plan.family_events = None
    if saved_fold is None:
        os.environ.pop("YM_FOLD", None)
    else:
        os.environ["YM_FOLD"] = saved_fold
    # host time to enqueue one step (Python + ctypes launches) vs its wall time: a step whose
    # enqueue time approaches its wall time leaves the GPU waiting on the host
    host = []
    for i in range(3):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        step(args.warmup + args.steps + 2 * PROBE_STEPS + i)
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    host_ms = 1e3 * sorted(host)[1]
    lens = [a.elapsed_time(b) for a, b in plan.probe_events]       # ms
    kern_ms = sum(lens) / max(len(lens), 1)

    imgs = args.batch * world * args.steps
    value = imgs / elapsed
    ms_step = 1e3 * elapsed / args.steps
    # algorithmic FLOPs of the training step from the plan: conv fwd + dgrad + wgrad (3x, minus the
    # stem's dgrad) plus attention (fwd 2 bmm, bwd 4 bmm)
    fwd = sum(op.flops() for op in convs)
    stem = [op for op in plan.ops if type(op).__name__ == "StemConvBN"]
    fwd += sum(2 * op.M * op.co * 9 for op in stem)
    heads = [op for op in plan.ops if type(op).__name__ == "HeadLevel"]
    fwd += sum(2 * op.M * (64 + op.nc) * op.xb.c for op in heads)
    attn = [op for op in plan.ops if type(op).__name__ == "AttnCore"]
    att = sum(2 * args.batch * op.heads * op.N * op.N * (op.kd + op.hd) for op in attn)
    train_flop = 3 * fwd - sum(2 * op.M * op.co * 9 for op in stem) + 3 * att
    per_img = train_flop / args.batch
    dom_tf = dom.flops() / (kern_ms * 1e-3) / 1e12 if kern_ms > 0 else 0.0
    # algorithmic HBM bytes of the probe launch: fp16 input view read once, fp16 weights, fp16 z
    # written once (BN partials are negligible); the binding roof is the larger time bound
    alg_bytes = 2 * (args.batch * dom.x.H * dom.x.W * dom.ci + dom.co * dom.ci * dom.k * dom.k + dom.M * dom.co)
    hbm_bound = alg_bytes / (HBM_PEAK_GBS * 1e9) > dom.flops() / (PEAK_BF16_TFLOPS * 1e12)
    dom_gbs = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    if hbm_bound:
        roof = {"bound": "hbm", "achieved": round(dom_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(dom_gbs / HBM_PEAK_GBS, 4)}
    else:
        roof = {"bound": "mfma", "achieved": round(dom_tf, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(dom_tf / PEAK_BF16_TFLOPS, 4)}
    step_tf = value / world * per_img / 1e12
    import ctypes
    from yolomi._lib import lib as _yl
    probe_kernel = {4: "conv_hpipe_kernel", 3: "conv_direct_kernel", 2: "conv_pipe_kernel", 1: "conv_halo_kernel"}.get(
        _yl().ym_conv_algo(ctypes.byref(dom.desc), 0), "conv_gemm_kernel")
    def fam_rate(kind):
        ms, work, _ = fams[kind]
        if ms <= 0:
            return 0.0, 0.0
        if kind == "bn":
            gbs = work / (ms * 1e-3) / 1e9
            return gbs, gbs / HBM_PEAK_GBS
        tf = work / (ms * 1e-3) / 1e12
        return tf, tf / PEAK_BF16_TFLOPS
    # `roofline`: the dense 3x3 conv kernels (every fwd / dgrad / wgrad launch of a k=3 Conv block, the
    # north star's named target) against the 16-bit MFMA peak: algorithmic FLOPs summed over the launches
    # of one step / their summed HIP-event durations (all launches on one stream, PROBE_STEPS steps)
    c3 = [fams[k] for k in ("fwd3", "dgrad3", "wgrad3")]
    c3_ms, c3_flop, c3_n = sum(v[0] for v in c3), sum(v[1] for v in c3), sum(v[2] for v in c3)
    c3_tf = c3_flop / (c3_ms * 1e-3) / 1e12 if c3_ms > 0 else 0.0
    t3 = traffic_entry(f"family conv3x3 bs{args.batch}")
    roof_c3 = {"bound": "mfma", "achieved": round(c3_tf, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
               "frac": round(c3_tf / PEAK_BF16_TFLOPS, 4),
               "traffic": t3["bytes_per_launch"] if t3 else None,
               "traffic_unit": "HBM bytes per training step, summed over the family's launches",
               "traffic_source": t3["source"] if t3 else None,
               "kernel": f"dense 3x3 conv kernels (conv_pipe / conv_hpipe / conv_halo / conv_gemm / conv_direct "
                         f"fwd + dgrad, "
                         f"wgrad3 + split-K reduce): {c3_n} launches per step, {c3_flop / 1e9:.0f} GFLOP algorithmic "
                         f"in {c3_ms:.3f} ms summed launch time (HIP events on the launch stream, all launches on "
                         f"one stream, {PROBE_STEPS} steps, the forward BN finalize as its own launch)",
               "per_direction_frac": {k[:-1]: round(fam_rate(k)[1], 4) for k in ("fwd3", "dgrad3", "wgrad3")}}
    names = {"fwd": "conv forward (pipelined / halo / implicit-GEMM / direct kernels)",
             "dgrad": "conv data gradient (pipelined / halo / implicit-GEMM / direct kernels)",
             "wgrad": "conv weight gradient (wgrad3 / wgrad1 + split-K reduce)",
             "bn": "BatchNorm + SiLU passes (finalize + apply; bwd reduce + finalize + apply)"}
    families = {}
    for k in ("fwd", "dgrad", "wgrad", "bn"):
        ms, work, n = fams[k]
        rate, frac = fam_rate(k)
        t = traffic_entry(f"family {k} bs{args.batch}")
        families[k] = {"bound": "hbm" if k == "bn" else "mfma", "ms_per_step": round(ms, 3), "launch_groups": n,
                       "achieved": round(rate, 2), "unit": "GB/s" if k == "bn" else "TFLOP/s", "frac": round(frac, 4),
                       "work": f"{work / 1e9:.1f} {'GB' if k == 'bn' else 'GFLOP'} algorithmic per step",
                       "traffic": t["bytes_per_launch"] if t else None, "traffic_source": t["source"] if t else None,
                       "kernel": names[k]}
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "ranks_seen": ranks_seen,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16 fwd / bf16 bwd (fp32 accumulate, fp32 loss + optimizer)",
        "data": f"synthetic ({args.imgsz}x{args.imgsz} uniform images, 1-20 log-uniform boxes/img, seeded per rank)",
        "config": {"workload": f"YOLOv11-{args.scale} {args.imgsz}x{args.imgsz} train step "
                               f"(fwd+loss+bwd+allreduce+clip+AdamW)",
                   "global_batch": args.batch * world, "batch_per_gpu": args.batch, "imgsz": args.imgsz,
                   "parallelism": f"dp{world}"},
        "roofline": roof_c3,
        "roofline_families": families,
        "roofline_probe": {**roof, "traffic": traffic_for(probe_key),
                     "kernel": f"{probe_kernel} fwd {dom.m.__class__.__name__} {dom.ci}->{dom.co} "
                               f"k{dom.k} s{dom.s} out {dom.y.H}x{dom.y.W}, {dom.flops() / 1e9:.1f} GFLOP and "
                               f"{alg_bytes / 1e6:.0f} MB algorithmic per launch, {kern_ms:.3f} ms avg over "
                               f"{len(lens)} launches ({dom_tf:.0f} TFLOP/s = {dom_tf / PEAK_BF16_TFLOPS:.3f} of the "
                               f"MFMA peak, {dom_gbs:.0f} GB/s = {dom_gbs / HBM_PEAK_GBS:.3f} of HBM)"},
        "roofline_step": {"bound": "mfma", "achieved": round(step_tf, 2), "peak": PEAK_BF16_TFLOPS,
                          "unit": "TFLOP/s", "frac": round(step_tf / PEAK_BF16_TFLOPS, 4),
                          "train_gflop_per_img": round(per_img / 1e9, 2)},
        "probe": {"key": probe_key, "rank": probe_rank, "count": probe_count},
        "host_enqueue_ms_per_step": round(host_ms, 3),
    }
    if dp_overlap is not None:
        out["dp_overlap"] = dp_overlap
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline()
        except Exception as e:  # pragma: no cover
            out["cpu_baseline"] = {"value": None, "error": str(e)[:200]}
    if rank == 0:
        log(f"loss {float(loss.detach()):.4f}  {value:.1f} img/s  {ms_step:.1f} ms/step (host enqueue {host_ms:.1f} ms)  "
            f"dominant kernel {kern_ms:.3f} ms ({dom_tf:.0f} TFLOP/s)")
        print(json.dumps(out), flush=True)
    ydist.shutdown()


if __name__ == "__main__":
    main()
