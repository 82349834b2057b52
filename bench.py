#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 data-parallel training throughput on MI355X.

BASELINE.json metric: "images/sec (whole node) ResNet-50 synthetic ImageNet at 1/2/4/8 MI355X;
allreduce ms/step". One process per GPU (torchrun for N > 1, RCCL over xGMI); per-GPU batch is
fixed (weak scaling). Each timed step is the complete training step of the framework:
on-device synthetic batch generation (Philox kernel) -> bf16-autocast forward (channels_last)
-> fused log-softmax+NLL -> backward with bucketed gradient all-reduce overlapped on the C++ RCCL
engine's comm stream -> fused multi-tensor SGD-momentum update (fp32 master weights).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--algorithm builtin|ring|direct]
For N > 1 either launch it under torchrun (python -m torch.distributed.run --nnodes=1 --nproc-per-node N
--master-addr 127.0.0.1 --master-port P bench.py --gpus N ...), or run ``python bench.py --gpus N`` as a
plain command: with no WORLD_SIZE in the environment it starts N ranks itself (a torch.distributed.run
child process, started before this process touches the GPU), relays rank 0's JSON line and exits with the
children's status. Asking for more GPUs than the node has is an error, never a silent 1-GPU run.
(Reference launcher: /root/reference/submit.sh:64 ``mpirun -npernode``; rank -> GPU at
/root/reference/src/main.py:329-331.)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time

_ROOT = os.path.dirname(os.path.abspath(__file__))
# MIOpen find results for these conv shapes on gfx950 ship with the repo, so a fresh box skips the
# multi-minute exhaustive search (torch.backends.cudnn.benchmark) and starts from tuned solvers.
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_ROOT, "miopen_db"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, _ROOT)

import distributed_learning_amd as dla  # noqa: E402
from distributed_learning_amd import knobs  # noqa: E402
from distributed_learning_amd.data import SyntheticBatches  # noqa: E402
from distributed_learning_amd.models import get_spec  # noqa: E402
from distributed_learning_amd.ops import nn as dnn  # noqa: E402
from distributed_learning_amd.ops.loss import cross_entropy  # noqa: E402
from distributed_learning_amd.ops.optim import FusedSGD  # noqa: E402
from distributed_learning_amd.parallel import PipelinedFusedDP, make_reducer  # noqa: E402
from distributed_learning_amd.parallel import context as ctxmod  # noqa: E402
from distributed_learning_amd.utils import telemetry  # noqa: E402

# Reference throughput at the same device count (GoogLeNet on P100 + Gloo/IPoIB):
# N=1 the "single"/Ideal run, N>1 the best published real-DP number (PyTorch DDP).
REFERENCE_IMG_S = {1: 317.5, 2: 573.6, 4: 1096.7, 8: 2040.9, 16: 3703.6}
MODEL_NAMES = {"resnet50": "ResNet-50", "resnet18": "ResNet-18", "resnet34": "ResNet-34", "resnet101": "ResNet-101",
               "resnet152": "ResNet-152", "googlenet": "GoogLeNet", "googlenet_noaux": "GoogLeNet"}


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    # 1280 per GPU, sized for the 288 GB of HBM3E (74.5 GB peak): the stage-3/4 layers (M = batch x 14^2 or
    # 7^2 rows) fill the 256 CUs better and per-step fixed costs are amortised: +4.3 % images/s from 512 to
    # 1024 (profiles/r5f/: 512 -> 12,794-12,819, 768 -> 12,994-13,022, 1024 -> 13,347-13,367) and +2.5 % from
    # 1024 to 1280 with the round-3 kernels (profiles/r3/g45_batch_ab.txt: 14,088-14,102 -> 14,444-14,471,
    # same box). The 24-bit pixel-index limit of the stem / fused stem-pool kernels (N * 112^2 < 2^24, checked
    # on the host) caps the batch at 1337; the largest stage-1 activation (2.06 GB) stays under the 2 GiB
    # buffer-descriptor range.
    ap.add_argument("--batch", type=int, default=1280, help="per-GPU batch size")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--algorithm", default="auto",
                    help="native engine all-reduce: auto (N > 1 or --force_comm: every candidate verified and timed "
                         "before warmup, each bucket gets the fastest, parallel/autotune.py; else builtin) or "
                         "[ipc_]builtin|ring|ring_pipe|direct|rsag|central|hier_ring|hier_coll[:channels]")
    # auto: N > 1 derives the cap from the fitted model of the measured best algorithm (autotune);
    # N = 1 uses 8 MiB of bf16 gradients (= 16 MiB of fp32 on the wire): the cost model's cap for
    # ResNet-50 on an 8-GPU node with an assumed builtin bandwidth (parallel/cost_model.py)
    ap.add_argument("--bucket_mb", default="auto")
    ap.add_argument("--transport", default=None, choices=["rccl", "ipc"],
                    help="gradient transport (default rccl; ipc with --same_device): ipc = peer-mapped windows "
                         "with flag barriers (csrc/comm/ipc.h)")
    ap.add_argument("--same_device", type=int, default=0,
                    help="1 = every rank on cuda:0 (N processes sharing one GPU; gloo process group + IPC "
                         "transport, since RCCL refuses that): the real multi-process data path on a one-GPU box")
    ap.add_argument("--check_dir", default=None,
                    help="each rank saves its final parameters / gradients / master weights to DIR/rank<r>.pt")
    ap.add_argument("--fail_rank", type=int, default=-1,
                    help="fault injection: this rank exits (status 17) after the forward of step --fail_step")
    ap.add_argument("--fail_step", type=int, default=1)
    ap.add_argument("--bucket_mb_sweep", default=None,
                    help="comma list of bucket caps (MiB, 0 = per tensor): time K steps at each and report one line "
                         "with the sub-table (the reference's fusion_experiment sweep)")
    ap.add_argument("--phases", type=int, default=0,
                    help="N > 0: after the timed region, N more steps with per-phase device timers; the record gets "
                         "the reference's latency-breakdown columns (get_data ... optimizer_step, batch)")
    ap.add_argument("--phases_csv", default=None, help="also write those rows as a reference-schema times.csv")
    ap.add_argument("--kernels", default=knobs.get("KERNELS"), choices=["torch", "native"])
    ap.add_argument("--precision", default=knobs.get("PRECISION"), choices=["autocast", "bf16", "fp32"],
                    help="bf16: bf16 weights + fp32 master weights in the fused optimizer (no per-step weight casts, "
                         "bf16 gradients on the wire); autocast: fp32 params + bf16 autocast; fp32: the reference's "
                         "precision (fp32 weights and activations; native BN/pool/loss/SGD kernels + fp32 MFMA convs, "
                         "or with --kernels torch the stock NCHW path)")
    ap.add_argument("--conv", default=knobs.get("CONV"), choices=["miopen", "native"],
                    help="1x1 convolutions on the native MFMA GEMMs (with fused BN statistics) or MIOpen")
    ap.add_argument("--graph", default=knobs.get("GRAPH"), choices=["on", "off"],
                    help="capture the whole training step (data, fwd, bwd, collectives, optimizer) in a HIP graph")
    ap.add_argument("--force_comm", type=int, default=0,
                    help="1 = run the multi-rank gradient path (gather -> RCCL all-reduce -> re-point) even at "
                         "one GPU (diagnostic: the per-GPU cost of the N>1 data path without the link time)")
    ap.add_argument("--wgrad_overlap_rows", type=int, default=None,
                    help="weight gradients of convs with at most this many output rows run concurrently with "
                         "their data gradient on a side stream (0 = off; default: ops/conv.py)")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.5)
    ap.add_argument("--dry_run", type=int, default=0,
                    help="1 = launcher/rendezvous check only: ranks join a gloo group on the CPU, meet at a "
                         "barrier and rank 0 prints who joined (no GPU, no model)")
    ap.add_argument("--launch_timeout", type=float, default=3000.0,
                    help="self-launch mode: seconds before the rank processes are killed")
    return ap.parse_args()


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a) -> int:
    """``--gpus N`` without a WORLD_SIZE: start N ranks as a torch.distributed.run child process.

    Runs before anything initialises the GPU in this process (``torch.cuda.device_count()`` does not, on
    this image). The child inherits stdout, so rank 0's JSON line is relayed as is; the return value is the
    launcher's exit status (non-zero if any rank failed), 124 on timeout."""
    if not a.dry_run and not a.same_device:
        ndev = torch.cuda.device_count()
        if a.gpus > ndev:
            print(f"error: --gpus {a.gpus} requested but this node has {ndev} GPU(s); refusing to measure fewer",
                  file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    if a.same_device:
        env["DLA_SAME_DEVICE"] = "1"
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        rc = p.wait(timeout=a.launch_timeout)
    except subprocess.TimeoutExpired:
        print(f"error: ranks did not finish within {a.launch_timeout:.0f} s; killing them", file=sys.stderr, flush=True)
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
        return 124
    if rc != 0:
        print(f"error: rank launcher exited with status {rc}", file=sys.stderr, flush=True)
    return rc


def dry_run(a) -> None:
    """Rendezvous check of the launch path: every rank joins a gloo group and the barrier."""
    import datetime

    dist.init_process_group("gloo", init_method="env://", timeout=datetime.timedelta(seconds=120))
    world, rank = dist.get_world_size(), dist.get_rank()
    joined = [None] * world
    dist.all_gather_object(joined, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", 0)),
                                    "pid": os.getpid()})
    dist.barrier()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "requested": a.gpus, "ranks_joined": joined}), flush=True)
    dist.destroy_process_group()


PHASES = ("get_data", "data2dev", "zero_grad", "forward", "backprop", "sync", "optimizer_step")


def build_dp(model, reducer, cap_mb: float, dev, a, tune, world):
    """Wrap ``model`` for data parallelism at bucket cap ``cap_mb`` (0 = one bucket per tensor, the
    reference's fusion-off mode); per-bucket algorithms from the autotuner; plans / windows reserved."""
    dp = PipelinedFusedDP(model, reducer, int(cap_mb * 1024 * 1024), dev)
    if a.force_comm and world == 1:
        from distributed_learning_amd.parallel.executor import NativeStreamExecutor

        dp.sync.set_executor(NativeStreamExecutor(reducer.engine, reducer.algorithm, passthrough=False))
    if tune is not None:
        per_size = tune.run_buckets([b.flat.numel() for b in dp.sync.buckets])
        dp.sync.executor.per_bucket = {b.index: per_size[b.flat.numel()] for b in dp.sync.buckets}
        dp.sync.regroup()  # fusion-off launch groups never span two algorithms (advisor r5)
    if world > 1 or a.force_comm:
        dp.sync.executor.reserve(dp.sync.buckets)
    return dp


def time_steps(step, a, dev, engine, graphed, backend, warmup=None):
    """W warmup steps (``warmup``: those not already run, default all), then exactly K timed steps between
    barrier + synchronize on both sides; the elapsed time is the MAX over ranks."""
    warmup = a.warmup if warmup is None else warmup
    tele = {"before_warmup": telemetry.sample(dev.index or 0)}
    # one event per step boundary (warmup and timed): the per-step GPU-stream time distribution goes into
    # the record, so a slow first-steps ramp and a uniformly slow box can be told apart
    wev = [torch.cuda.Event(enable_timing=True) for _ in range(warmup + 1)]
    wev[0].record()
    for i in range(warmup):
        step()
        wev[i + 1].record()
    torch.cuda.synchronize()
    engine.consume_comm_ms()
    engine.set_timing(not graphed)
    engine.impl.collective_counts(True)
    tele["before_timed"] = telemetry.sample(dev.index or 0)
    tev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tev[0].record()
    loss = None
    for i in range(a.steps):
        loss = step()
        tev[i + 1].record()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tele["after_timed"] = telemetry.sample(dev.index or 0)
    comm_ms = engine.consume_comm_ms() / max(1, a.steps)
    engine.set_timing(False)
    ncoll, nunits = (int(v) for v in engine.impl.collective_counts(True))
    t = torch.tensor([elapsed, comm_ms], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    step_ms = [tev[i].elapsed_time(tev[i + 1]) for i in range(a.steps)]
    srt = sorted(step_ms)
    return {"elapsed": float(t[0]), "comm_ms": float(t[1]), "loss": loss, "tele": tele,
            # host-side issue counts (engine.cpp collective_counts): member collectives and submission units
            "collectives_per_step": ncoll / max(1, a.steps), "launch_units_per_step": nunits / max(1, a.steps),
            "warm_ms": [round(wev[i].elapsed_time(wev[i + 1]), 2) for i in range(warmup)],
            "step_ms": {"p50": round(srt[len(srt) // 2], 3), "min": round(srt[0], 3), "max": round(srt[-1], 3),
                        "seq": [round(x, 2) for x in step_ms] if a.steps <= 200 else None}}


def measure_backward(data, opt, model, fwd_loss, dev, backend, n: int = 3) -> float:
    """Seconds of one backward (compute stream, HIP events), the least of the last ``n - 1`` of
    ``n`` eager steps (the first pays lazy setup), MAX over ranks. These are real steps."""
    times = []
    for _ in range(n):
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        loss = fwd_loss(x, y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loss.backward()
        e1.record()
        model.sync_gradients()
        opt.step()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e-3)
    t = torch.tensor([min(times[1:] or times)], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def phase_breakdown(parts, n: int, csv_path=None, name="bench"):
    """Per-phase device time (HIP events, no host sync inside the step) over ``n`` steps, in the
    reference's times.csv columns (/root/reference/src/timing.py:28-40, main.py:54-97)."""
    from distributed_learning_amd.timing import EventTimers

    et = EventTimers()
    data, opt, model, fwd_loss = parts
    for i in range(n):
        et.start("batch")
        et.start("get_data")
        x, y = data.next()
        et.end("get_data")
        et.start("data2dev")  # synthetic batches are generated on the device: nothing to copy
        et.end("data2dev")
        et.start("zero_grad")
        opt.zero_grad(set_to_none=True)
        et.end("zero_grad")
        et.start("forward")
        loss = fwd_loss(x, y)
        et.end("forward")
        et.start("backprop")
        loss.backward()
        et.end("backprop")
        et.start("sync")
        model.sync_gradients()
        et.end("sync")
        et.start("optimizer_step")
        opt.step()
        et.end("optimizer_step")
        et.end("batch")
        et.end_experiment(name, {"batch_count": i, "data_len": x.shape[0]})
    torch.cuda.synchronize()
    et._resolve()
    rows = [r for _, r in et.collected]
    mean = {k: round(sum(r[k] for r in rows) / len(rows), 3) for k in PHASES + ("batch",)}
    if csv_path:
        et.writeout(csv_path)
    return mean


def _dual_calls():
    from distributed_learning_amd.ops import conv as nconv

    return {k: nconv.CALLS[k] for k in ("1x1_dual", "1x1_dual_bn")}


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:
            sys.exit(launch_ranks(a))
        os.environ["WORLD_SIZE"] = "1"
        os.environ["RANK"] = "0"
        os.environ["LOCAL_RANK"] = "0"
    if a.dry_run:
        return dry_run(a)
    if a.gpus != int(os.environ["WORLD_SIZE"]):
        print(f"error: --gpus {a.gpus} but WORLD_SIZE {os.environ['WORLD_SIZE']}", file=sys.stderr, flush=True)
        sys.exit(2)
    same = bool(a.same_device) or os.environ.get(knobs.env_name("SAME_DEVICE")) == "1"
    if a.gpus > torch.cuda.device_count() and not same:
        print(f"error: --gpus {a.gpus} but this node has {torch.cuda.device_count()} GPU(s)", file=sys.stderr, flush=True)
        sys.exit(2)
    c = ctxmod.init(backend="gloo" if same else "nccl", same_device=same, transport=a.transport)
    world, rank = c.world_size, c.rank
    dev = c.device
    if knobs.get("COMPUTE_STREAM") == "high":
        # the step's kernels (and, through autograd, its backward) on a high-priority queue: the late 3x3 weight
        # gradients' side stream (normal priority) then fills in behind the critical path instead of sharing it
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    fp32 = a.precision == "fp32"
    bf16 = a.precision == "bf16"
    # fp32 (the reference's precision): with --kernels native the activations stay channels_last and the fused
    # BN/residual/ReLU, pools, global-average pool, cross-entropy and SGD run on the native kernels' fp32 forms,
    # the convolutions on MIOpen (the MFMA conv kernels are bf16); --kernels torch is the stock NCHW path
    fp32_torch = fp32 and a.kernels == "torch"
    # fp32 means fp32: no TF32-style reduced-precision convolutions / matmuls (torch enables them for MIOpen by
    # default), and MIOpen's immediate mode instead of an exhaustive find over every fp32 conv shape
    torch.backends.cudnn.benchmark = not fp32
    if fp32:
        torch.backends.cudnn.allow_tf32 = False
        torch.backends.cuda.matmul.allow_tf32 = False
    dnn.set_backend(a.kernels)
    dnn.set_native_conv(a.conv == "native" and not fp32)
    # fp32 convolutions on the fp32 matrix-core kernels (ops/conv_f32.py) instead of MIOpen
    dnn.set_native_conv_f32(fp32 and a.conv == "native" and a.kernels == "native")
    if a.wgrad_overlap_rows is not None:
        from distributed_learning_amd.ops import conv as nconv

        nconv.WGRAD_OVERLAP_MAX_ROWS = a.wgrad_overlap_rows

    spec = get_spec(a.model)
    torch.manual_seed(1234)
    base = spec.build().to(dev)
    if not fp32_torch:
        base = base.to(memory_format=torch.channels_last)
    if bf16:
        dnn.bf16_weights(base)
    tune = None
    comm_active = world > 1 or bool(a.force_comm)
    base_algo = "builtin" if a.algorithm == "auto" else a.algorithm
    reducer = make_reducer("immediate", base_algo, native=True)
    engine = reducer.engine
    if a.force_comm and world == 1:
        engine.impl.set_force(True)  # the N>1 data path incl. fp32 staging, as a 1-rank collective
        engine.set_accum_fp32(True)
    grad_dtype = torch.bfloat16 if bf16 else torch.float32
    graphed = a.graph == "on"
    if graphed and comm_active and (engine.transport == "ipc" or a.algorithm.startswith("ipc_")):
        # IPC barrier tokens are host-side launch arguments: a replayed graph would pass every barrier at
        # once (engine.cpp allreduce_ipc refuses capture); the IPC transport runs eagerly
        print("error: --graph on cannot capture the IPC transport; use --graph off", file=sys.stderr, flush=True)
        sys.exit(2)
    if a.algorithm == "auto" and comm_active:
        from distributed_learning_amd.parallel import autotune as at

        def probe_engine():
            e = engine.probe_clone(at.PROBE_TIMEOUT_S)
            if a.force_comm and world == 1:
                e.impl.set_force(True)
                e.set_accum_fp32(True)
            return e

        tune = at.Autotune(engine, grad_dtype, at.candidates(world, engine.transport, include_ipc=not graphed),
                           probe_factory=probe_engine)
        tune.run_grid()
        base_algo = tune.best_model()[0]
        reducer.algorithm = base_algo
    # auto cap with a tuned model: provisional 8 MiB, then re-derived from the measured backward below
    cap_from_backward = a.bucket_mb == "auto" and tune is not None
    if a.bucket_mb == "auto":
        a.bucket_mb = 8.0
    a.bucket_mb = float(a.bucket_mb)
    sweep = [float(v) for v in a.bucket_mb_sweep.split(",")] if a.bucket_mb_sweep else None
    model = build_dp(base, reducer, sweep[0] if sweep else a.bucket_mb, dev, a, tune, world)
    opt = FusedSGD(base.parameters(), lr=a.lr, momentum=a.momentum, master_weights=bf16)
    data = SyntheticBatches(a.batch, spec.input_shape, spec.num_classes, dev,
                            dtype=torch.bfloat16 if bf16 else torch.float32,
                            seed=1234, rank=rank, channels_last=not fp32_torch, device_step=a.graph == "on")
    nstep = [0]

    def fwd_loss(x, y):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.precision == "autocast"):
            out = model(x)
            loss = cross_entropy(out, y)
        nstep[0] += 1
        if rank == a.fail_rank and nstep[0] == a.fail_step:
            print(f"rank {rank}: injected failure after the forward of step {nstep[0]}", file=sys.stderr, flush=True)
            os._exit(17)
        return loss

    def step():
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        loss = fwd_loss(x, y)
        loss.backward()
        model.sync_gradients()
        opt.step()
        return loss

    warm_left = a.warmup
    if cap_from_backward and not sweep and a.warmup > 0:
        # the cap balances exposed collective time against the gradient-ready times of THIS step's
        # backward: the first warmup steps measure it (eager, on the provisional buckets, MAX over ranks;
        # they count as warmup steps), then the buckets are rebuilt. With no warmup the cap stays 8 MiB.
        # the first eager step pays lazy setup (plans, first-call kernel setup): at least two calibration
        # steps, the least of the later ones counts; with fewer warmup steps the provisional cap stays
        ncal = min(a.warmup, 3)
        if ncal >= 2:
            warm_left = a.warmup - ncal
            bwd_s = measure_backward(data, opt, model, fwd_loss, dev, c.backend, n=ncal)
            cpu_model = spec.build()
            cap = float(tune.choose_cap(cpu_model, spec.input_shape, bwd_s))
            del cpu_model
            if abs(cap - a.bucket_mb) > 1e-9:
                model.cleanup()
                model = build_dp(base, reducer, cap, dev, a, tune, world)
            a.bucket_mb = cap
    comm_ms_eager = None
    run_step = step
    if graphed:
        from distributed_learning_amd.parallel.graphs import GraphedStep

        # eager steps first: algorithm selection, lazy state, and the comm time of one eager step
        # (event timers are not recorded inside the graph)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        engine.consume_comm_ms()
        engine.set_timing(True)
        step()
        torch.cuda.synchronize()
        engine.set_timing(False)
        comm_ms_eager = engine.consume_comm_ms()
        run_step = GraphedStep(step, warmup=2, device=dev)

    sweep_rows = []
    if sweep:
        for cap in sweep:
            if cap != sweep[0]:
                model.cleanup()
                model = build_dp(base, reducer, cap, dev, a, tune, world)
            gs = model.sync
            gs.hook_s, gs.hook_calls = 0.0, 0
            r = time_steps(step, a, dev, engine, False, c.backend)
            sweep_rows.append({"bucket_mb": cap, "buckets": len(gs.buckets),
                               "ms_per_step": round(r["elapsed"] / a.steps * 1000.0, 3),
                               "img_s": round(a.batch * world * a.steps / r["elapsed"], 2),
                               "allreduce_ms_per_step": round(r["comm_ms"], 3),
                               "hook_calls_per_step": gs.hook_calls / a.steps,
                               "step_ms_p50": r["step_ms"]["p50"]})
        best = min(sweep_rows, key=lambda x: x["ms_per_step"])
        res = r  # telemetry / loss of the last cap's run; the line's value is the best cap's
    gsync = getattr(model, "sync", None)
    if gsync is not None:
        gsync.hook_s, gsync.hook_calls = 0.0, 0
    if not sweep:
        res = time_steps(run_step, a, dev, engine, graphed, c.backend, warmup=warm_left)
    elapsed = res["elapsed"]
    comm_ms = res["comm_ms"] if not graphed else comm_ms_eager
    final_loss = float(res["loss"].detach().float())
    ms = elapsed / a.steps * 1000.0
    img_s = a.batch * world * a.steps / elapsed
    if sweep:  # the line's value is the best cap of the sweep
        ms, img_s = best["ms_per_step"], best["img_s"]
    phases = None
    if a.phases > 0:  # after the timed region: per-phase device times in the reference's CSV columns
        phases = phase_breakdown((data, opt, model, fwd_loss), a.phases,
                                 a.phases_csv if rank == 0 else None, name=f"bench_{a.model}")
    # the reference publishes fp32 GoogLeNet numbers only: a ratio against a different model or
    # a lower precision measures nothing, so vs_baseline is null unless model and precision match
    ref = REFERENCE_IMG_S.get(world) if (a.model.startswith("googlenet") and fp32) else None
    if rank == 0:
        rec = {
            "metric": f"images/sec (whole node) {MODEL_NAMES.get(a.model, a.model)} synthetic ImageNet",
            "value": round(img_s, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / ref, 3) if ref else None,
            "dtype": "fp32" if fp32 else "bf16",
            "data": "synthetic (on-device Philox uniform images, random labels; random-init weights)",
            "config": {
                "model": a.model,
                "global_batch": a.batch * world,
                "per_gpu_batch": a.batch,
                "seq_len": None,
                "image_size": list(spec.input_shape),
                "parallelism": f"dp{world}",
                "allreduce": a.algorithm if tune is None else "auto:" + base_algo,
                "bucket_mb": round(a.bucket_mb, 4),
                "transport": engine.transport,
                "same_device": same,
                "kernels": a.kernels,
                "precision": a.precision,
                "conv1x1": ("native-f32" if dnn.native_conv_f32() else "miopen") if fp32 else a.conv,
                "layout": "nchw" if fp32_torch else "channels_last",
                # 1x1 backward: both gradients in one pass over dY (gemm_dual.hip), the consuming BN's apply
                # fused where served (ops/conv.py DUAL_*); what actually ran this process
                "conv1x1_bwd": None if fp32 else {k: int(v) for k, v in _dual_calls().items()},
                "hip_graph": graphed,
                "optimizer": f"fused SGD momentum={a.momentum}" + (" (fp32 master weights)" if bf16 else " (fp32 weights)"),
                "force_comm": bool(a.force_comm),
            },
            "knobs": knobs.non_default(),
            "allreduce_ms_per_step": round(comm_ms, 3),
            # the rank count RCCL's own communicator reports (ncclCommCount), not WORLD_SIZE; the IPC-only
            # transport has no communicator and reports its window group
            "comm_world": int(engine.impl.rccl_count()) if engine.impl.has_rccl() else int(engine.impl.world()),
            "comm_world_src": "ncclCommCount" if engine.impl.has_rccl() else "ipc window group",
            "collectives_per_step": res["collectives_per_step"],
            "launch_units_per_step": res["launch_units_per_step"],
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2),
            "final_loss": round(final_loss, 4),
            "baseline_ref": {"value": REFERENCE_IMG_S.get(world),
                             "what": "reference best published img/s at this N (GoogLeNet fp32, P100, Gloo); "
                                     "not comparable unless model=googlenet and precision=fp32"},
            "step_ms": res["step_ms"],
            "warmup_step_ms": res["warm_ms"],
            "telemetry": res["tele"],
        }
        if sweep:
            rec["config"]["bucket_mb"] = best["bucket_mb"]
            rec["bucket_sweep"] = sweep_rows
        if phases is not None:
            rec["latency_breakdown_ms"] = phases
        if gsync is not None and comm_active:
            per_tensor = len(gsync.buckets) > 1 and all(len(b.params) == 1 for b in gsync.buckets)
            if per_tensor:  # fusion off: which form ran (the strict one is the reference's semantics)
                rec["fusion_off"] = {"mode": "grouped" if gsync.groups else "strict",
                                     "tensors": len(gsync.buckets), "launch_groups": len(gsync.groups)}
        if tune is not None:
            rec["allreduce_table"] = tune.report()
            rec["autotune_s"] = round(tune.spent_s, 3)
            ex = model.sync.executor
            rec["allreduce_per_bucket"] = [ex.algorithm_for(b) for b in model.sync.buckets]
        if gsync is not None and gsync.hook_calls:
            rec["hook_host_ms_per_step"] = round(gsync.hook_s * 1000.0 / a.steps, 3)
            rec["hook_calls_per_step"] = gsync.hook_calls / a.steps
        print(json.dumps(rec), flush=True)
    prof_out = knobs.get("TORCH_PROF")
    if prof_out and rank == 0:  # diagnostics only, after the timed region: op -> kernel attribution
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
            for _ in range(3):
                step()
            torch.cuda.synchronize()
        with open(prof_out, "w") as f:
            f.write(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=60, max_name_column_width=90))
            f.write("\n\n")
            f.write(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=40,
                                                                max_name_column_width=60, max_src_column_width=400))
            f.write("\n\n")  # the many small ops (memsets, copies) by call count, with their Python stacks
            f.write(prof.key_averages(group_by_stack_n=8).table(sort_by="count", row_limit=60,
                                                                max_name_column_width=60, max_src_column_width=500))
    if a.check_dir:
        os.makedirs(a.check_dir, exist_ok=True)
        names = dict((id(p), n) for n, p in base.named_parameters())
        st = {"params": {}, "grads": {}, "masters": {}}
        for p in base.parameters():
            n = names[id(p)]
            st["params"][n] = p.detach().cpu()
            if p.grad is not None:
                st["grads"][n] = p.grad.detach().cpu()
            m = opt.state.get(p, {}).get("master")
            if m is not None:
                st["masters"][n] = m.detach().cpu()
        torch.cuda.synchronize()
        torch.save(st, os.path.join(a.check_dir, f"rank{rank}.pt"))
    model.cleanup()
    if tune is not None:
        tune.close()
    ctxmod.shutdown()


if __name__ == "__main__":
    main()
