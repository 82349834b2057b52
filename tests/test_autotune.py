"""In-run all-reduce selection (parallel/autotune.py) on Gloo CPU ranks with a stand-in engine.

The stand-in has the NativeEngine surface the autotuner uses (reserve / allreduce / synchronize /
comm-stream timers) over ``dist.all_reduce``; its algorithms differ in a simulated per-call cost
that is rank-dependent (the table must take the MAX over ranks), one of them returns wrong numbers
(verification must exclude it) and one cannot be set up on one rank (setup failures must be agreed
on before anything is timed). Checked: identical decisions on every rank, the per-size choice, the
alpha/beta fit and the cap derivation. The GPU twin is tests/test_gpu_multiproc.py.
"""
import torch
import torch.distributed as dist

from distributed_learning_amd.parallel import autotune as at
import dist_util

COST_US = {"fast_small": (5.0, 0.004), "fast_large": (60.0, 0.0005), "broken": (1.0, 0.0001),
           "unmappable": (1.0, 0.0001)}  # (alpha us, us per KiB)


class _Impl:
    def __init__(self, rank, world):
        self._r, self._w = rank, world

    def world(self):
        return self._w

    def rank(self):
        return self._r

    def accum_fp32(self):
        return True


class FakeEngine:
    def __init__(self, rank, world):
        self.impl = _Impl(rank, world)
        self.group = dist.group.WORLD
        self.device = torch.device("cpu")
        self.transport = "rccl"
        self._t = 0.0
        self._timing = False

    def reserve(self, algo, sizes, dtype):
        if algo == "unmappable" and self.impl.rank() == 1:
            raise RuntimeError("cannot map peer memory")

    def allreduce(self, buf, algo, average=True):
        dist.all_reduce(buf)
        if average:
            buf /= self.impl.world()
        if algo == "broken":
            buf += 1
        a, b = COST_US[algo]
        ms = (a + b * buf.numel() * buf.element_size() / 1024) * 1e-3 * (1 + 0.5 * self.impl.rank())
        if self._timing:
            self._t += ms

    def synchronize(self):
        pass

    def set_timing(self, on):
        self._timing = on

    def consume_comm_ms(self):
        t, self._t = self._t, 0.0
        return t


def _tune(rank, world):
    eng = FakeEngine(rank, world)
    t = at.Autotune(eng, torch.float32, list(COST_US), reps=2, warmup=1)
    at.GRID_MIB = (0.25, 1.0, 4.0)
    t.run_grid()
    small, large = 1024, 16 << 20
    per = t.run_buckets([small, large, small])
    return {"ok": t.ok, "per": per, "best": t.best_model()[0], "report": t.report(),
            "grid": t.grid_table}


def test_autotune_consistent_verified_and_fastest():
    res = dist_util.run(_tune, 2)
    a, b = res
    assert a["per"] == b["per"] and a["best"] == b["best"] and a["ok"] == b["ok"]
    assert a["ok"]["broken"] is False and a["ok"]["unmappable"] is False
    assert a["ok"]["fast_small"] and a["ok"]["fast_large"]
    assert a["per"][1024] == "fast_small"
    assert a["per"][16 << 20] == "fast_large"
    # the table is the max over ranks: rank 1's simulated costs are 1.5x rank 0's
    row = a["grid"]["fast_small"]
    n = min(row)
    alpha, beta = COST_US["fast_small"]
    want = (alpha + beta * n * 4 / 1024) * 1e-3 * 1.5
    assert abs(row[n] - want) / want < 1e-6
    fit = a["report"]["fit"]["fast_large"]
    assert abs(fit["alpha_us"] - 60.0 * 1.5) < 1.0


def test_fit_recovers_alpha_beta():
    row = {n: (10.0 + 2e-6 * n * 4) for n in (1000, 10_000, 100_000)}  # ms
    m = at.fit(row, 4)
    assert abs(m.alpha_s - 10e-3) < 1e-9
    assert abs(m.beta_s_per_byte - 2e-9) < 1e-15


def test_candidates():
    c8 = at.candidates(8, "rccl")
    assert "builtin" in c8 and "ring:7" in c8 and "ipc_direct" in c8
    assert "ring:7" not in at.candidates(4, "rccl")
    assert all(not x.startswith("ipc_") for x in at.candidates(2, "ipc"))


def test_per_size_choice_keeps_default_within_margin():
    ok = {"builtin": True, "ring": True, "direct": True, "bad": False}
    table = {"builtin": {1: 1.00, 2: 1.00, 3: 1.00}, "ring": {1: 0.97, 2: 0.90, 3: 1.02},
             "direct": {1: 0.99, 2: 0.94}, "bad": {1: 0.10, 2: 0.10, 3: 0.10}}
    per = at.choose_per_size(table, ok, [1, 2, 3], "builtin")
    # 3 % faster is noise at the default margin; 10 % faster switches; unverified never wins
    assert per == {1: "builtin", 2: "ring", 3: "builtin"}
    assert at.choose_per_size(table, ok, [1], "builtin", margin=0.0) == {1: "ring"}


# ---- probe isolation ----------------------------------------------------
# A stand-in with the failure modes of a real RCCL engine: a candidate that HANGS (every rank's wait
# hits the probe deadline; engine.cpp wait_stream then aborts that engine's communicator) and one that
# raises an ASYNC ERROR on one rank only (the other rank sits in the collective until its deadline).
# The training engine must never run a non-builtin candidate and must never be aborted; the run has to
# finish on builtin with identical decisions on every rank and both failures named in the report.

ISO_COST = {"builtin": (20.0, 0.002), "hang": (1.0, 0.0001), "async_err": (1.0, 0.0001), "ring": (30.0, 0.003)}


class IsoEngine(FakeEngine):
    def __init__(self, rank, world, role, log):
        super().__init__(rank, world)
        self.role, self.log = role, log
        self.aborted = False
        self.pending = None

    def reserve(self, algo, sizes, dtype):
        pass

    def allreduce(self, buf, algo, average=True):
        assert not self.aborted, "a call on an aborted communicator"
        self.log.append((self.role, algo))
        if algo in ("hang", "async_err"):
            self.pending = algo  # the collective never completes / errors asynchronously
            return
        dist.all_reduce(buf)
        if average:
            buf /= self.impl.world()
        a, b = ISO_COST[algo]
        if self._timing:
            self._t += (a + b * buf.numel() * buf.element_size() / 1024) * 1e-3

    def synchronize(self):
        p, self.pending = self.pending, None
        if p == "hang":
            self.aborted = True
            raise RuntimeError("CommEngine: communication did not complete within 30.000000 s (peer failure?); "
                               "communicators aborted")
        if p == "async_err":
            self.aborted = True
            if self.impl.rank() == 1:
                raise RuntimeError("CommEngine: RCCL async error: unhandled system error (communicators aborted)")
            raise RuntimeError("CommEngine: communication did not complete within 30.000000 s (peer failure?); "
                               "communicators aborted")

    def consume_comm_ms(self):
        self.synchronize()
        return super().consume_comm_ms()

    def discard(self):
        self.aborted = True


def _tune_isolated(rank, world):
    log = []
    train = IsoEngine(rank, world, "train", log)
    probes = []

    def factory():
        e = IsoEngine(rank, world, f"probe{len(probes)}", log)
        probes.append(e)
        return e

    t = at.Autotune(train, torch.float32, ["hang", "ring", "async_err", "builtin"], reps=2, warmup=1,
                    probe_factory=factory)
    at.GRID_MIB = (0.25, 1.0)
    t.run_grid()
    per = t.run_buckets([4096, 1 << 20])
    t.close()
    return {"ok": t.ok, "per": per, "best": t.best_model()[0], "report": t.report(), "log": log,
            "train_aborted": train.aborted, "probes": len(probes)}


def test_autotune_isolates_hanging_and_erroring_candidates():
    a, b = dist_util.run(_tune_isolated, 2)
    assert a["per"] == b["per"] and a["best"] == b["best"] and a["ok"] == b["ok"]
    assert a["ok"] == {"builtin": True, "hang": False, "ring": True, "async_err": False}
    for r in (a, b):
        assert not r["train_aborted"]
        # builtin ran first, on the training engine; nothing else ever touched it
        assert r["log"][0] == ("train", "builtin")
        assert {alg for role, alg in r["log"] if role == "train"} == {"builtin"}
        # the probe that hung and the one that errored were replaced: 3 probe engines in all
        assert r["probes"] == 3 and r["report"]["probe_engines"] == {"created": 3, "discarded": 2}
        ex = r["report"]["excluded"]
        assert set(ex) == {"hang", "async_err"}
        assert "did not complete" in ex["hang"]
        assert "rank 1: RuntimeError: CommEngine: RCCL async error" in ex["async_err"]
    assert a["best"] == "builtin" and set(a["per"].values()) <= {"builtin", "ring"}


# ---- robust per-bucket decisions ---------------------------------------------
# Ground truth: 'builtin' (low alpha, low bandwidth) and 'ring' (high alpha, twice the bandwidth) cross near
# 19.5 MiB; 'twin' costs exactly what builtin costs. Every repetition carries +-5 % seeded jitter (rank-
# dependent) and one rep in 8 a 3x outlier, as comm-stream timings do. Whatever the seed, the decision must be
# the same, twin must never be picked, and along increasing bucket size the choice may change only once.

JIT_COST = {"builtin": (20.0, 0.004), "ring": (60.0, 0.002), "twin": (20.0, 0.004)}  # (alpha us, us per KiB)


class JitterEngine(FakeEngine):
    def __init__(self, rank, world, seed):
        super().__init__(rank, world)
        import random

        self.rng = random.Random(seed * 7919 + rank)

    def allreduce(self, buf, algo, average=True):
        dist.all_reduce(buf)
        if average:
            buf /= self.impl.world()
        a, b = JIT_COST[algo]
        # the buffers are SCALE x smaller than the sizes they stand for (a CPU gloo all-reduce of 256 MiB per rep
        # would dominate the test); the simulated time is that of the full size
        ms = (a + b * SCALE * buf.numel() * buf.element_size() / 1024) * 1e-3
        ms *= 1.0 + self.rng.uniform(-0.05, 0.05)
        if self.rng.random() < 0.125:
            ms *= 3.0
        if self._timing:
            self._t += ms


SIZES_MIB = (0.25, 1.0, 4.0, 5.91, 6.11, 8.0, 16.0, 96.0, 128.0, 256.0)
SCALE = 4096


def _tune_jitter(rank, world, seed):
    eng = JitterEngine(rank, world, seed)
    at.GRID_MIB = tuple(m / SCALE for m in (0.25, 1.0, 4.0, 16.0, 64.0))
    t = at.Autotune(eng, torch.float32, list(JIT_COST))
    t.run_grid()
    sizes = [int(m * (1 << 20) / SCALE) // 4 for m in SIZES_MIB]
    per = t.run_buckets(sizes)
    return [per[n] for n in sizes]


def test_per_bucket_decision_is_stable_under_jitter():
    decisions = [dist_util.run(_tune_jitter, 2, seed) for seed in range(4)]
    for d in decisions:
        assert d[0] == d[1]  # ranks agree
    first = decisions[0][0]
    for d in decisions[1:]:
        assert d[0] == first, (first, d[0])  # identical across seeds
    assert "twin" not in first
    changes = sum(1 for x, y in zip(first, first[1:]) if x != y)
    assert changes <= 1, first
    assert first[:7] == ["builtin"] * 7 and first[-1] == "ring", first


def test_noise_winner_within_spread_is_not_chosen():
    ok = {"builtin": True, "ring": True}
    table = {"builtin": {1: 1.00}, "ring": {1: 0.90}}
    assert at.choose_per_size(table, ok, [1], "builtin") == {1: "ring"}
    spread = {"builtin": {1: 0.05}, "ring": {1: 0.01}}  # 10 % faster, but within 3 x the 5 % spread (MAD)
    assert at.choose_per_size(table, ok, [1], "builtin", spread=spread) == {1: "builtin"}
    # the fitted lines disagree with the measurement: stays on the default
    models = {"builtin": at.cm.CollectiveModel("fit", 0.0, 1e-9), "ring": at.cm.CollectiveModel("fit", 0.0, 2e-9)}
    assert at.choose_per_size(table, ok, [1], "builtin", models=models) == {1: "builtin"}


# ---- time budget -------------------------------------------------------------

class SlowEngine(JitterEngine):
    def reserve(self, algo, sizes, dtype):
        if algo == "twin":
            import time

            time.sleep(1.5)  # a candidate whose setup (e.g. probe communicator, IPC mapping) is slow


def _tune_budget(rank, world):
    eng = SlowEngine(rank, world, 0)
    at.GRID_MIB = tuple(m / SCALE for m in (0.25, 1.0, 4.0))
    t = at.Autotune(eng, torch.float32, ["builtin", "twin", "ring"], reps=3, budget_s=1.0)
    t.run_grid()
    per = t.run_buckets([256, 4096])
    return {"per": per, "report": t.report(), "ok": t.ok}


def test_budget_skips_remaining_candidates_and_finishes_on_builtin():
    a, b = dist_util.run(_tune_budget, 2)
    for r in (a, b):
        ex = r["report"]["excluded"]
        assert set(ex) == {"twin", "ring"}, ex
        assert all(v.startswith("budget") for v in ex.values()), ex
        assert set(r["per"].values()) == {"builtin"}
        assert r["report"]["autotune_s"] >= 1.0 and r["report"]["budget_s"] == 1.0
    assert a["per"] == b["per"]
