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

Isolation: ``builtin`` is measured first on the training engine; every other candidate runs on a
probe engine with its own communicator and a 30 s deadline (ProbePool). A candidate that hangs,
raises an RCCL async error or returns wrong numbers is excluded on every rank with its reason
(``report()["excluded"]``), the probe communicator is aborted and replaced, and training continues
on what passed -- the first 8-GPU run cannot be lost to one bad schedule.

All ranks compute the same decision from the gathered table; rank 0's is broadcast anyway so a
floating-point tie can never split the ranks (RCCL requires identical collective sequences).
"""
from __future__ import annotations

import math
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

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


def _time_algo(engine, algo: str, n: int, dtype: torch.dtype, reps: int, warmup: int,
               verify: bool) -> Tuple[List[float], bool]:
    """Per-repetition comm-stream ms of one all-reduce of ``n`` elements (each rep timed on its own, so the
    caller sees the spread, not only the mean), and whether the verification pattern came back exact."""
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
    times = []
    for _ in range(reps):
        engine.set_timing(True)
        engine.allreduce(buf, algo, True)
        times.append(engine.consume_comm_ms())
    engine.set_timing(False)
    return times, ok


def _median(v: Sequence[float]) -> float:
    v = sorted(v)
    k = len(v)
    if k == 0:
        return math.inf
    return v[k // 2] if k % 2 else 0.5 * (v[k // 2 - 1] + v[k // 2])


def _spread(v: Sequence[float]) -> float:
    """Median absolute deviation of the repetitions from their median (0 for fewer than 3): unlike a range or
    an inter-quartile range it ignores up to half the reps being outliers (a preempted launch, a late peer)."""
    k = len(v)
    if k < 3:
        return 0.0
    m = _median(v)
    return _median([abs(x - m) for x in v])


def _gather_max(table: Dict[str, Dict[int, float]], ok: Dict[str, bool], group,
                spread: Optional[Dict[str, Dict[int, float]]] = None) -> Tuple[Dict, Dict, Dict]:
    """Per (algorithm, size): the MAX over ranks of every rank's median and of its spread; verified = AND."""
    world = dist.get_world_size(group)
    objs: List[object] = [None] * world
    dist.all_gather_object(objs, (table, ok, spread or {}), group=group)
    out: Dict[str, Dict[int, float]] = {}
    okk: Dict[str, bool] = {}
    spr: Dict[str, Dict[int, float]] = {}
    for t, o, sp in objs:
        for a, row in t.items():
            dst = out.setdefault(a, {})
            for s, v in row.items():
                dst[s] = max(dst.get(s, 0.0), v)
        for a, row in sp.items():
            dst = spr.setdefault(a, {})
            for s, v in row.items():
                dst[s] = max(dst.get(s, 0.0), v)
        for a, v in o.items():
            okk[a] = okk.get(a, True) and v
    return out, okk, spr


class ProbePool:
    """The engine every non-builtin candidate is probed on: a clone of the training engine with its
    own communicator and a short deadline (NativeEngine.probe_clone). A candidate that fails on
    any rank gets the probe discarded (its communicator aborted) on every rank together, and the
    next candidate gets a fresh one -- the training communicator never runs an unverified schedule
    and is never aborted by probing. ``factory`` is collective; ``None`` probes on the engine itself
    (stand-in engines of the CPU tests that have no communicator to lose)."""

    def __init__(self, factory: Optional[Callable[[], object]] = None):
        self.factory = factory
        self.engine = None
        self.created = 0
        self.discarded = 0

    def get(self, fallback):
        if self.factory is None:
            return fallback
        if self.engine is None:
            self.engine = self.factory()
            self.created += 1
        return self.engine

    def discard(self) -> None:
        if self.engine is not None:
            try:
                self.engine.discard()
            except Exception:  # noqa: BLE001 -- an engine already broken is dropped all the same
                pass
            self.engine = None
            self.discarded += 1

    def close(self) -> None:
        if self.engine is not None:
            try:
                self.engine.close()
            except Exception:  # noqa: BLE001
                try:
                    self.engine.discard()
                except Exception:  # noqa: BLE001
                    pass
            self.engine = None


PROBE_TIMEOUT_S = 30.0


def _agree(flag: bool, why: str, group) -> Tuple[bool, str]:
    """Collective AND of ``flag`` with every failing rank's reason."""
    objs: List[object] = [None] * dist.get_world_size(group)
    dist.all_gather_object(objs, (bool(flag), why), group=group)
    bad = [f"rank {r}: {w[:240]}" for r, (f, w) in enumerate(objs) if not f]
    return (not bad), "; ".join(bad)[:1000]


def _runs_on_probe(engine, algo: str, probe: "ProbePool") -> bool:
    """Every candidate but RCCL's own all-reduce runs on the probe engine. On the IPC transport the name
    'builtin' is the IPC two-shot emulation, whose hang would disable the TRAINING engine's windows for good
    (ipc_broken_), so there it is probed too (advisor r5)."""
    if probe.factory is None:
        return False
    if algo != "builtin":
        return True
    uses_ipc = getattr(engine, "uses_ipc", None)
    return bool(uses_ipc(algo)) if uses_ipc is not None else False


def measure(engine, algos: Sequence[str], sizes: Sequence[int], dtype: torch.dtype, reps: int = 11,
            warmup: int = 2, verify: bool = True, group=None, probe: Optional[ProbePool] = None,
            reasons: Optional[Dict[str, str]] = None, spread: Optional[Dict[str, Dict[int, float]]] = None,
            deadline: Optional[float] = None) -> Tuple[Dict[str, Dict[int, float]], Dict[str, bool]]:
    """Collective: algo -> {elements: median ms over ``reps`` (max over ranks)}, algo -> verified on every rank.

    ``builtin`` (RCCL's own all-reduce, what training falls back to) runs on ``engine``; every other
    candidate runs on ``probe``'s engine (see ProbePool). Setup failures are agreed on across ranks
    before anything is timed, and after every size all ranks agree whether the candidate is still
    good, so a failure on one rank stops the candidate on every rank at the same point instead of
    leaving the others waiting in barriers it will never reach. ``reasons`` collects why each
    excluded candidate was excluded; ``spread`` (out) the median absolute deviation of the repetitions.
    ``deadline`` (``time.perf_counter()`` value): a candidate not yet started when any rank is past it is
    skipped on every rank (reason ``budget``); ``builtin`` is never skipped."""
    group = group if group is not None else engine.group
    probe = probe if probe is not None else ProbePool(None)
    reasons = reasons if reasons is not None else {}
    table: Dict[str, Dict[int, float]] = {}
    spr: Dict[str, Dict[int, float]] = {}
    ok: Dict[str, bool] = {}
    for a in algos:
        if deadline is not None and a != "builtin":
            late = time.perf_counter() > deadline
            in_time, _ = _agree(not late, "budget", group)
            if not in_time:
                ok[a], reasons[a] = False, "budget: autotune time budget spent before this candidate"
                continue
        on_probe = _runs_on_probe(engine, a, probe)
        why = ""
        try:
            eng = probe.get(engine) if on_probe else engine
            eng.reserve(a, list(sizes), dtype)
            good = True
        except Exception as e:  # noqa: BLE001 - a transport this node cannot run is excluded, not fatal
            good, why = False, f"setup: {type(e).__name__}: {e}"
        good, why = _agree(good, why, group)
        if not good:
            ok[a], reasons[a] = False, why
            if on_probe:
                probe.discard()
            continue
        row, srow = {}, {}
        for k, n in enumerate(sizes):
            if deadline is not None and a != "builtin" and k > 0:
                in_time, _ = _agree(time.perf_counter() <= deadline, "budget", group)
                if not in_time:
                    good, why = False, f"budget: autotune time budget spent after {k} of {len(sizes)} sizes"
                    break
            v, why = True, ""
            try:
                times, v = _time_algo(eng, a, int(n), dtype, reps, warmup, verify)
                ms = _median(times)
                if not v:
                    why = f"wrong result at {int(n)} elements"
            except Exception as e:  # noqa: BLE001 -- deadline / async error / transport refusal
                v, why, times, ms = False, f"{type(e).__name__}: {e}", [], math.inf
            v, why = _agree(v, why, group)
            if not v:
                good = False
                break
            row[int(n)] = ms
            srow[int(n)] = _spread(times)
        if good:
            table[a] = row
            spr[a] = srow
        else:
            reasons[a] = why
            if on_probe:
                probe.discard()
        ok[a] = good
    out, okk, sp = _gather_max(table, ok, group, spr)
    if spread is not None:
        for a, row in sp.items():
            spread.setdefault(a, {}).update(row)
    return out, okk


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
# ... and by more than this many median absolute deviations of either algorithm's repetitions at that size
SWITCH_SPREADS = 3.0


def choose_per_size(table: Dict[str, Dict[int, float]], ok: Dict[str, bool], sizes: Sequence[int],
                    default: str, margin: float = SWITCH_MARGIN,
                    spread: Optional[Dict[str, Dict[int, float]]] = None,
                    models: Optional[Dict[str, cm.CollectiveModel]] = None, esz: int = 4) -> Dict[int, str]:
    """Per bucket size: the default unless a verified algorithm beats it by more than ``margin`` AND by more
    than SWITCH_SPREADS x the larger inter-rep spread (median absolute deviation) of the two (``spread``), AND -- where both have fitted
    ``models`` -- the two alpha + beta S lines agree it is faster at that size. Two lines cross at most once,
    so an algorithm can only take a contiguous run of sizes; a default inside such a run (its confirmation
    failed) is filled only where the measured median does not contradict it. Net effect: no flip-flopping
    between adjacent sizes on timings that differ by noise (round-5 record: ring 0.131 vs builtin 0.152 ms at
    5.91 MiB, then 0.192 vs 0.149 at 6.11 MiB)."""
    spread = spread or {}
    models = models or {}
    srt = sorted(int(n) for n in sizes)
    out: Dict[int, str] = {}
    for n in srt:
        dt = table.get(default, {}).get(n)
        if not ok.get(default) or dt is None:  # no default at this size: plain fastest verified
            live = [(row[n], a) for a, row in table.items() if ok.get(a) and n in row]
            out[n] = min(live)[1] if live else default
            continue
        best, bt = default, dt
        for a, row in table.items():
            if a == default or not ok.get(a) or n not in row:
                continue
            t = row[n]
            if t >= dt * (1.0 - margin):
                continue
            sp = max(spread.get(a, {}).get(n, 0.0), spread.get(default, {}).get(n, 0.0))
            if dt - t <= SWITCH_SPREADS * sp:
                continue
            if a in models and default in models and models[a].time(n * esz) >= models[default].time(n * esz):
                continue
            if t < bt:
                best, bt = a, t
        out[n] = best
    # contiguity: a default between two sizes won by the same algorithm takes it when its own median agrees
    for i, n in enumerate(srt):
        if out[n] != default:
            continue
        left = next((out[m] for m in reversed(srt[:i]) if out[m] != default), None)
        right = next((out[m] for m in srt[i + 1:] if out[m] != default), None)
        if left is not None and left == right:
            t = table.get(left, {}).get(n)
            if t is not None and t <= table.get(default, {}).get(n, math.inf):
                out[n] = left
    return out


def broadcast_decision(obj, group=None):
    box: List[object] = [obj]
    dist.broadcast_object_list(box, src=0, group=group)
    return box[0]


class Autotune:
    """The whole selection for one model (see the module docstring). ``report()`` is what the
    bench record carries."""

    def __init__(self, engine, dtype: torch.dtype, algos: Sequence[str], reps: int = 11, warmup: int = 2,
                 probe_factory: Optional[Callable[[], object]] = None, budget_s: Optional[float] = None):
        self.engine = engine
        # wall-clock budget of the whole selection (grid + bucket probes + probe communicators): past it, the
        # candidates not yet started are skipped on every rank and listed in ``excluded`` as "budget"
        if budget_s is None:
            from .. import knobs

            budget_s = float(knobs.get("AUTOTUNE_BUDGET_S"))
        self.budget_s = float(budget_s)
        self.t_start = time.perf_counter()
        self.spent_s = 0.0
        self.dtype = dtype
        self.esz = torch.tensor([], dtype=dtype).element_size()
        # what crosses the links: fp32 staging of bf16 buckets at N > 1 (engine accum_fp32)
        self.wire_esz = 4 if (dtype == torch.bfloat16 and engine.impl.accum_fp32()) else self.esz
        # builtin first: RCCL's own all-reduce is measured on the training engine before any custom
        # schedule is probed (on the probe engine), so the fallback is known good whatever follows
        self.algos = sorted(algos, key=lambda a: a != "builtin")
        self.probe = ProbePool(probe_factory)
        self.excluded: Dict[str, str] = {}
        self.reps, self.warmup = reps, warmup
        self.grid_table: Dict[str, Dict[int, float]] = {}
        self.grid_spread: Dict[str, Dict[int, float]] = {}
        self.bucket_spread: Dict[str, Dict[int, float]] = {}
        self.ok: Dict[str, bool] = {}
        self.models: Dict[str, cm.CollectiveModel] = {}
        self.bucket_table: Dict[str, Dict[int, float]] = {}
        self.per_size: Dict[int, str] = {}
        self.cap_mib: Optional[float] = None
        self.cap_rows: List[Dict[str, float]] = []
        self.backward_s: Optional[float] = None

    def run_grid(self) -> None:
        sizes = [int(m * MiB) // self.esz for m in GRID_MIB]
        self.grid_table, self.ok = measure(self.engine, self.algos, sizes, self.dtype, self.reps, self.warmup,
                                           probe=self.probe, reasons=self.excluded, spread=self.grid_spread,
                                           deadline=self.t_start + self.budget_s)
        self.spent_s = time.perf_counter() - self.t_start
        self.models = {a: fit(row, self.wire_esz) for a, row in self.grid_table.items() if self.ok.get(a)}

    def best_model(self) -> Tuple[str, cm.CollectiveModel]:
        """The model-wide default: the verified algorithm with the least time summed over the grid -- but RCCL's
        own ``builtin`` stays the default unless that sum beats it by more than SWITCH_MARGIN, so two
        equivalent schedules cannot trade places from run to run on noise."""
        live = [(sum(self.grid_table[a].values()), a) for a in self.models]
        if not live:
            raise RuntimeError("autotune: no all-reduce algorithm passed verification on every rank")
        t, a = min(live)
        if "builtin" in self.models and a != "builtin":
            tb = sum(self.grid_table["builtin"].values())
            if t >= tb * (1.0 - SWITCH_MARGIN):
                a = "builtin"
        return a, self.models[a]

    def choose_cap(self, cpu_model, input_shape, backward_s: float) -> float:
        """Bucket cap (MiB of bucket dtype) from the fitted model of the best algorithm, against a
        backward of ``backward_s`` seconds (bench.py passes the warmup steps' measured backward,
        MAX over ranks)."""
        self.backward_s = float(backward_s)
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
        self.bucket_table, ok = measure(self.engine, live, sizes, self.dtype, self.reps, self.warmup,
                                        probe=self.probe, reasons=self.excluded, spread=self.bucket_spread,
                                        deadline=self.t_start + self.budget_s)
        for a, v in ok.items():
            self.ok[a] = self.ok.get(a, True) and v
        default = self.best_model()[0]
        pick = choose_per_size(self.bucket_table, self.ok, sizes, default, spread=self.bucket_spread,
                               models=self.models, esz=self.wire_esz)
        self.per_size = broadcast_decision(pick, self.engine.group)
        self.spent_s = time.perf_counter() - self.t_start
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
            "bucket_mad_ms": {a: {str(mib(n)): round(v, 4) for n, v in row.items()}
                              for a, row in self.bucket_spread.items()},
            "reps": self.reps,
            "statistic": "median of reps per rank, max over ranks",
            "per_bucket_size": {str(mib(n)): a for n, a in self.per_size.items()},
            "cap_mib": self.cap_mib,
            "cap_backward_ms": None if self.backward_s is None else round(self.backward_s * 1e3, 3),
            "size_unit": "MiB of bucket dtype",
            "excluded": dict(self.excluded),
            "probe_engines": {"created": self.probe.created, "discarded": self.probe.discarded},
            "autotune_s": round(self.spent_s, 3),
            "budget_s": self.budget_s,
        }

    def close(self) -> None:
        """Release the probe engine (its communicator and windows); the decisions stay."""
        self.probe.close()
