"""In-run all-reduce selection: measure, verify, fit, choose -- before the timed region.

The reference fixed its all-reduce (a Python ring over Gloo, /root/reference/src/allreduce.py:45-98,
used by main_onestep_reduce at /root/reference/src/main.py:208-213) and its 25 MiB fusion size
(config.py:51), picking the size from an offline sweep (fusion_experiment_ourdist,
main.py:287-301). On an xGMI node the right answer depends on constants nobody has
measured here (RCCL's achieved bus bandwidth, per-step launch cost, the IPC pull rate), so the
first multi-GPU run measures them itself:

1. every candidate algorithm is verified on an exactly representable rank-dependent pattern (a
   transport that returns wrong numbers on this node is excluded, not shipped) and timed with the
   engine's comm-stream events on a size grid; every rank measures, the table is the MAX over ranks;
2. ``T(S) = alpha + beta S`` is fitted per algorithm (least squares over the grid) and replaces the
   cost model's inputs (``cost_model.RCCL_GROUP_US`` / ``bus_gbps`` were assumptions);
3. with ``bucket_mb='auto'`` the bucket cap is re-derived from the fitted model of the best
   algorithm (cost_model.choose_bucket_cap: exposed + contended collective time against the model's
   own gradient-ready times);
4. each actual bucket size is measured again for every verified algorithm and gets its fastest one.

All ranks compute the same decision from the gathered table; rank 0's is broadcast anyway so a
floating-point tie can never split the ranks (RCCL requires identical collective sequences).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import knobs
from . import cost_model as cm

MiB = 1024 * 1024
GRID_MIB = (0.25, 1.0, 4.0, 16.0, 64.0)


def candidates(world: int, transport: str, include_ipc: bool = True) -> List[str]:
    """Algorithms worth timing on one node of ``world`` ranks."""
    if transport == "ipc":  # every schedule runs on the windows; the 'builtin' name is the two-shot emulation
        names = ["builtin", "direct", "ring"]
        if world > 2:
            names += [f"ring:{c}" for c in (1, 3) if c < world - 1]
        return names
    names = ["builtin", "rsag", "direct", "ring:1"]
    if world > 2:
        names += [f"ring:{c}" for c in (3, 7) if c <= world - 1]
    if include_ipc and world > 1:
        names += ["ipc_direct", "ipc_builtin"]
    return names


def _pattern(n: int, rank: int, dtype: torch.dtype, device) -> torch.Tensor:
    """(rank + 1) * small integers: exact in bf16 and fp32, so the mean is checkable."""
    i = torch.arange(n, device=device, dtype=torch.int64)
    return (((i % 7) - 3) * (rank + 1)).to(dtype)


def _time_algo(engine, algo: str, n: int, dtype: torch.dtype, reps: int, warmup: int, verify: bool) -> Tuple[float, bool]:
    dev = engine.device
    world, rank = engine.impl.world(), engine.impl.rank()
    ok = True
    if verify:
        buf = _pattern(n, rank, dtype, dev)
        engine.allreduce(buf, algo, True)
        engine.synchronize()
        i = torch.arange(n, device=dev, dtype=torch.int64)
        want = ((i % 7) - 3).double() * (world + 1) / 2.0
        err = float((buf.double() - want).abs().max()) if n else 0.0
        ok = err <= 0.02 * 3 * (world + 1) / 2.0 + 1e-6
    buf = torch.ones(n, dtype=dtype, device=dev)
    for _ in range(warmup):
        engine.allreduce(buf, algo, True)
    engine.synchronize()
    engine.consume_comm_ms()
    engine.set_timing(True)
    for _ in range(reps):
        engine.allreduce(buf, algo, True)
    ms = engine.consume_comm_ms() / max(1, reps)
    engine.set_timing(False)
    return ms, ok


def _gather_max(table: Dict[str, Dict[int, float]], ok: Dict[str, bool], group) -> Tuple[Dict, Dict]:
    world = dist.get_world_size(group)
    objs: List[object] = [None] * world
    dist.all_gather_object(objs, (table, ok), group=group)
    out: Dict[str, Dict[int, float]] = {}
    okk: Dict[str, bool] = {}
    for t, o in objs:
        for a, row in t.items():
            dst = out.setdefault(a, {})
            for s, v in row.items():
                dst[s] = max(dst.get(s, 0.0), v)
        for a, v in o.items():
            okk[a] = okk.get(a, True) and v
    return out, okk


def measure(engine, algos: Sequence[str], sizes: Sequence[int], dtype: torch.dtype, reps: int = 5,
            warmup: int = 2, verify: bool = True, group=None) -> Tuple[Dict[str, Dict[int, float]], Dict[str, bool]]:
    """Collective: algo -> {elements: ms (max over ranks)}, algo -> verified on every rank.

    Algorithms whose setup fails (e.g. peer memory that cannot be mapped) are reported as not ok;
    setup failures are agreed on across ranks before anything is timed, so no rank is left waiting
    in a collective the others skipped."""
    import os

    group = group if group is not None else engine.group
    table: Dict[str, Dict[int, float]] = {}
    ok: Dict[str, bool] = {}
    for a in algos:
        try:
            engine.reserve(a, list(sizes), dtype)
            good = True
        except Exception:  # noqa: BLE001 - a transport this node cannot run is excluded, not fatal
            good = False
        flags: List[object] = [None] * dist.get_world_size(group)
        dist.all_gather_object(flags, good, group=group)
        if not all(flags):
            ok[a] = False
            continue
        row = {}
        good = True
        # an IPC barrier that never completes gives up after DLA_COMM_TIMEOUT_S: short while probing, so a
        # transport that cannot synchronise on this node costs seconds and is excluded (the engine then
        # refuses IPC; RCCL is untouched)
        key = knobs.env_name("COMM_TIMEOUT_S")  # read by the engine at every barrier launch
        old_to = os.environ.get(key)
        if engine.uses_ipc(a) if hasattr(engine, "uses_ipc") else False:
            os.environ[key] = "30"
        try:
            for n in sizes:
                ms, v = _time_algo(engine, a, int(n), dtype, reps, warmup, verify)
                row[int(n)] = ms
                good = good and v
        except Exception:  # noqa: BLE001
            good = False
        finally:
            if old_to is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = old_to
        if good:
            table[a] = row
        ok[a] = good
    return _gather_max(table, ok, group)


def fit(row: Dict[int, float], esz: int) -> cm.CollectiveModel:
    """Least-squares alpha + beta * bytes over the measured points (beta >= 0, alpha >= 0)."""
    xs = [n * esz for n in row]
    ys = [row[n] * 1e-3 for n in row]
    k = len(xs)
    if k == 0:
        return cm.CollectiveModel("none", math.inf, math.inf)
    if k == 1:
        return cm.CollectiveModel("fit", 0.0, ys[0] / max(1, xs[0]))
    mx, my = sum(xs) / k, sum(ys) / k
    sxx = sum((x - mx) ** 2 for x in xs)
    beta = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx if sxx > 0 else 0.0
    beta = max(beta, 0.0)
    alpha = max(my - beta * mx, 0.0)
    return cm.CollectiveModel("fit", alpha, beta)


# a bucket leaves the model-wide default only for an algorithm faster by more than this fraction: at world 1
# (and between near-identical schedules) the per-size timings differ by noise, and a noise winner per bucket
# buys nothing but extra plans (profiles/r4/g03: four 1-rank candidates within 3 % of each other)
SWITCH_MARGIN = 0.05


def choose_per_size(table: Dict[str, Dict[int, float]], ok: Dict[str, bool], sizes: Sequence[int],
                    default: str, margin: float = SWITCH_MARGIN) -> Dict[int, str]:
    out = {}
    for n in sizes:
        best, bt = default, math.inf
        for a, row in table.items():
            if ok.get(a) and int(n) in row and row[int(n)] < bt:
                best, bt = a, row[int(n)]
        dt = table.get(default, {}).get(int(n))
        if ok.get(default) and dt is not None and bt >= dt * (1.0 - margin):
            best = default
        out[int(n)] = best
    return out


def broadcast_decision(obj, group=None):
    box: List[object] = [obj]
    dist.broadcast_object_list(box, src=0, group=group)
    return box[0]


class Autotune:
    """The whole selection for one model (see the module docstring). ``report()`` is what the
    bench record carries."""

    def __init__(self, engine, dtype: torch.dtype, algos: Sequence[str], reps: int = 5, warmup: int = 2):
        self.engine = engine
        self.dtype = dtype
        self.esz = torch.tensor([], dtype=dtype).element_size()
        # what crosses the links: fp32 staging of bf16 buckets at N > 1 (engine accum_fp32)
        self.wire_esz = 4 if (dtype == torch.bfloat16 and engine.impl.accum_fp32()) else self.esz
        self.algos = list(algos)
        self.reps, self.warmup = reps, warmup
        self.grid_table: Dict[str, Dict[int, float]] = {}
        self.ok: Dict[str, bool] = {}
        self.models: Dict[str, cm.CollectiveModel] = {}
        self.bucket_table: Dict[str, Dict[int, float]] = {}
        self.per_size: Dict[int, str] = {}
        self.cap_mib: Optional[float] = None
        self.cap_rows: List[Dict[str, float]] = []

    def run_grid(self) -> None:
        sizes = [int(m * MiB) // self.esz for m in GRID_MIB]
        self.grid_table, self.ok = measure(self.engine, self.algos, sizes, self.dtype, self.reps, self.warmup)
        self.models = {a: fit(row, self.wire_esz) for a, row in self.grid_table.items() if self.ok.get(a)}

    def best_model(self) -> Tuple[str, cm.CollectiveModel]:
        """The verified algorithm with the least time summed over the grid."""
        live = [(sum(self.grid_table[a].values()), a) for a in self.models]
        if not live:
            raise RuntimeError("autotune: no all-reduce algorithm passed verification on every rank")
        a = min(live)[1]
        return a, self.models[a]

    def choose_cap(self, cpu_model, input_shape, backward_s: float) -> float:
        """Bucket cap (MiB of bucket dtype) from the fitted model of the best algorithm."""
        _, model = self.best_model()
        params = list(cpu_model.parameters())
        ready = cm.ready_times_from_flops(cpu_model, input_shape, backward_s)
        cap_wire, self.cap_rows = cm.choose_bucket_cap(params, ready, backward_s, model,
                                                       wire_bytes_per_elem=self.wire_esz)
        # choose_bucket_cap sizes buckets in wire bytes; the bucketizer caps bucket-dtype bytes
        self.cap_mib = broadcast_decision(cap_wire * self.esz / self.wire_esz, self.engine.group)
        return self.cap_mib

    def run_buckets(self, bucket_sizes: Sequence[int]) -> Dict[int, str]:
        sizes = sorted(set(int(s) for s in bucket_sizes))
        live = [a for a in self.algos if self.ok.get(a)]
        self.bucket_table, ok = measure(self.engine, live, sizes, self.dtype, self.reps, self.warmup)
        for a, v in ok.items():
            self.ok[a] = self.ok.get(a, True) and v
        default = self.best_model()[0]
        self.per_size = broadcast_decision(choose_per_size(self.bucket_table, self.ok, sizes, default),
                                           self.engine.group)
        return self.per_size

    def report(self) -> Dict[str, object]:
        def mib(n):
            return round(n * self.esz / MiB, 4)

        return {
            "candidates": self.algos,
            "verified": {a: bool(v) for a, v in self.ok.items()},
            "grid_ms": {a: {str(mib(n)): round(ms, 4) for n, ms in row.items()} for a, row in self.grid_table.items()},
            "fit": {a: {"alpha_us": round(m.alpha_s * 1e6, 2),
                        "algbw_gbps": round(1e-9 / m.beta_s_per_byte, 1) if m.beta_s_per_byte > 0 else None}
                    for a, m in self.models.items()},
            "bucket_ms": {a: {str(mib(n)): round(ms, 4) for n, ms in row.items()} for a, row in self.bucket_table.items()},
            "per_bucket_size": {str(mib(n)): a for n, a in self.per_size.items()},
            "cap_mib": self.cap_mib,
            "size_unit": "MiB of bucket dtype",
        }
