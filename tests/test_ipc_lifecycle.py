"""IPC window lifecycle of NativeEngine._map_windows (parallel/engine.py) on Gloo CPU ranks.

Every new window generation is stamped with a random nonce by its owner, and every importer reads
the nonce back through its fresh mapping (CommEngine.ipc_open, csrc/comm/engine.cpp). A mapping that
shows another nonce is a stale view of an earlier window -- the leading candidate for the round-4
two-process failure (profiles/r4/g23): pulls through it read old data and the peer's flag never
advances, so the first barrier times out. These tests drive the host-side agreement with a stand-in
for the native engine: one rank's first mapping is stale -> every rank allocates again together
and the run goes on; a mapping that stays stale -> every rank raises at the same point (nobody is
left waiting in a collective); the nonces handed to ipc_open are exactly the ones each owner stamped.
The GPU twin is ``scripts/ipc_engine_check.py --regrow`` (tests/test_gpu_multiproc.py).
"""
import torch
import torch.distributed as dist

import dist_util
from distributed_learning_amd.parallel.engine import NativeEngine


class _FakeImpl:
    def __init__(self, rank, world, stale_opens):
        self.r, self.w = rank, world
        self.stale_opens = stale_opens  # this rank's first N opens see a stale peer mapping
        self.cap = 0      # committed (verified) window bytes -- what ipc_capacity() reports
        self.pending = 0  # allocated, not yet verified (engine.cpp ipc_alloc -> ipc_open commits it)
        self.allocs = []
        self.opens = 0

    def world(self):
        return self.w

    def ipc_need(self):
        return 1 << 20

    def ipc_capacity(self):
        return self.cap

    def synchronize(self):
        pass

    def ipc_alloc(self, size, nonce):
        assert nonce & 1 and 0 < nonce < 1 << 64
        self.allocs.append(nonce)
        self.pending = size
        return f"handle-{self.r}-{len(self.allocs)}-{nonce}".encode()

    def ipc_open(self, handles, nonces):
        self.opens += 1
        for r, (h, n) in enumerate(zip(handles, nonces)):
            assert h.decode().endswith(f"-{n}"), "ipc_open got a nonce that is not the owner's stamp"
        if self.opens <= self.stale_opens:
            return f"rank {(self.r + 1) % self.w}'s window maps to nonce 0, expected {nonces[(self.r + 1) % self.w]:x}"
        self.cap, self.pending = self.pending, 0
        return ""


def _map(rank, world, stale_on_rank1):
    impl = _FakeImpl(rank, world, stale_on_rank1 if rank == 1 else 0)
    eng = NativeEngine(impl, dist.group.WORLD, torch.device("cpu"), 1, transport="ipc")
    out = {"raised": None}
    try:
        eng._map_windows()
    except RuntimeError as e:
        out["raised"] = str(e)
    out.update(allocs=len(impl.allocs), stale=eng.stale_mappings, opens=impl.opens, cap=impl.ipc_capacity(), rank=rank)
    if out["raised"] is not None:  # a caller that caught the failure reserves again: every rank re-maps
        impl.stale_opens = 0
        before = len(impl.allocs)
        eng._map_windows()
        out["agreed_remap"] = len(impl.allocs) == before + 1 and impl.ipc_capacity() > 0
    # the next growth starts from an agreed state: a forced new generation works on every rank
    if out["raised"] is None:
        impl.stale_opens = 0
        eng.remap_windows()
        out["allocs_after_remap"] = len(impl.allocs)
    return out


def test_stale_mapping_is_retried_on_every_rank():
    res = dist_util.run(_map, 2, 1)
    for r in res:
        assert r["raised"] is None, r
        assert r["allocs"] == 2 and r["stale"] == 1, r  # both ranks re-allocated once, together
        assert r["allocs_after_remap"] == 3, r


def test_persistently_stale_mapping_raises_everywhere():
    res = dist_util.run(_map, 2, 99)
    for r in res:
        assert r["raised"] and "stale" in r["raised"], r
        assert r["allocs"] == NativeEngine.MAP_ATTEMPTS, r
        # advisor r5: a window that was never verified is not reported as capacity, so the next reserve
        # maps again (or refuses) instead of running collectives past the old, smaller mapping
        # rank 0 verified its own mappings; rank 1 never did: rank 1 reports no capacity, and the next
        # _map_windows on both ranks sees the agreed minimum and maps again together
        assert r["cap"] == (0 if r["rank"] == 1 else r["cap"]), r
        assert r["agreed_remap"], r


def test_clean_mapping_maps_once():
    res = dist_util.run(_map, 2, 0)
    for r in res:
        assert r["raised"] is None and r["allocs"] == 1 and r["stale"] == 0, r
