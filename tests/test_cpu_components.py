"""CPU unit tests: timing CSV schema, CLI parity, optimizer and loss reference paths, data, checkpoints."""
import os
import subprocess
import sys

import pytest
import torch

from distributed_learning_amd import timing
from distributed_learning_amd.config import parse_args
from distributed_learning_amd.data import DataPartitioner, SyntheticBatches, TensorDataset
from distributed_learning_amd.ops.loss import cross_entropy
from distributed_learning_amd.ops.optim import FusedSGD
from distributed_learning_amd.utils.env import eval_arg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_times_csv_schema(tmp_path):
    t = timing.Timers()
    for i in range(2):
        for name in ["batch", "get_data"]:
            t.start(name)
        t.end("get_data")
        for name in ["data2dev", "zero_grad", "forward", "backprop", "sync", "optimizer_step"]:
            t.start(name)
            t.end(name)
        t.end("batch")
        t.end_experiment("single", {"batch_count": i, "data_len": 128})
    f = tmp_path / "single_0_0_times.csv"
    t.writeout(str(f))
    lines = f.read_text().splitlines()
    # exact reference header (SURVEY.md Appendix A / measurements/*_times.csv)
    assert lines[0] == ("experiment_name, get_data, data2dev, zero_grad, forward, backprop, sync, "
                        "optimizer_step, batch, batch_count, data_len")
    assert lines[1].startswith("single, ") and lines[1].endswith(", 0, 128")
    assert len(lines) == 3


def test_reference_cli_and_envarg(monkeypatch):
    monkeypatch.setenv("OMPI_COMM_WORLD_SIZE", "4")
    monkeypatch.setenv("OMPI_COMM_WORLD_RANK", "2")
    assert eval_arg("envarg://OMPI_COMM_WORLD_RANK") == "2"
    c = parse_args(["envarg://OMPI_COMM_WORLD_SIZE", "envarg://OMPI_COMM_WORLD_RANK", "4", "16", "10.0.0.1", "ib0",
                    "imagenet", "/data", "0", "--experiment", "experiment2", "--limit_batches", "30",
                    "--random_input", "1"])
    assert (c.size, c.rank, c.node_dev, c.total_dev) == (4, 2, 4, 16)
    assert c.model_name == "imagenet" and c.grouping_size == 25 * 1024 * 1024
    assert c.lr == 0.01 and c.momentum == 0.5 and c.epoch_count == 100
    assert c.devices == ["cpu"] * 4 and c.backend == "gloo"


@pytest.mark.parametrize("kw", [dict(momentum=0.5), dict(momentum=0.9, nesterov=True, weight_decay=1e-4),
                                dict(momentum=0.9, dampening=0.1), dict(momentum=0.0, weight_decay=0.01)])
def test_fused_sgd_reference_path_matches_torch(kw):
    torch.manual_seed(0)
    ps = [torch.randn(17, requires_grad=True), torch.randn(3, 5, requires_grad=True)]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    a = FusedSGD(ps, lr=0.1, **kw)
    b = torch.optim.SGD(qs, lr=0.1, **kw)
    for s in range(3):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad, q.grad = g.clone(), g.clone()
        a.step()
        b.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p, q)


def test_cross_entropy_reference():
    x = torch.randn(6, 10)
    y = torch.randint(0, 10, (6,))
    torch.testing.assert_close(cross_entropy(x, y), torch.nn.functional.cross_entropy(x, y))


def test_partitioner_semantics():
    ds = TensorDataset(torch.arange(1000).float(), torch.zeros(1000))
    p = DataPartitioner(ds, total_dev=4, batch_size=32)
    parts = [set(p.use(i).index.tolist()) for i in range(4)]
    assert all(len(s) == 1000 // 4 // 32 * 32 for s in parts)
    assert not set.intersection(*parts)
    p2 = DataPartitioner(ds, 4, 32)  # same seed -> same partitions on every rank
    assert [set(p2.use(i).index.tolist()) for i in range(4)] == parts


def test_synthetic_cpu():
    s = SyntheticBatches(4, (3, 8, 8), 10, "cpu", rank=1)
    x, y = s.next()
    assert x.shape == (4, 3, 8, 8) and 0 <= float(x.min()) and float(x.max()) < 1
    assert y.dtype == torch.long and int(y.max()) < 10
    x2, _ = SyntheticBatches(4, (3, 8, 8), 10, "cpu", rank=2).next()
    assert not torch.equal(x, x2)  # per-rank streams differ by default


def test_checkpoint_roundtrip(tmp_path):
    from distributed_learning_amd.models import create_network
    from distributed_learning_amd.train import load_checkpoint, save_checkpoint

    m = create_network("basicnet")
    opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.5)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    opt.step()
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, m, opt, 7)
    m2 = create_network("basicnet")
    opt2 = FusedSGD(m2.parameters(), lr=0.1, momentum=0.5)
    assert load_checkpoint(path, m2, opt2) == 7
    for a, b in zip(m.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b)
    assert len(opt2.state) == len(opt.state)


@pytest.mark.slow
def test_main_cli_experiment3_two_workers(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "distributed_learning_amd.main", "1", "0", "2", "2", "127.0.0.1", "lo", "mnist",
           "/nonexistent", "0", "--experiment", "experiment3", "--random_input", "1", "--limit_batches", "3",
           "--batch_size", "8", "--master_port", str(__import__("dist_util").free_port()),
           "--results_root", str(tmp_path), "--job_id", "t"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    folder = tmp_path / "experiment3_2_t"
    for exp in ["warmup", "ddp", "onestep_reduce", "onestep_seq_merge", "onestep_overlap"]:
        assert (folder / f"{exp}_config.txt").exists()
        for w in (0, 1):
            lines = (folder / f"{exp}_0_{w}_loss.txt").read_text().splitlines()
            assert len(lines) == 3 and lines[0].startswith(f"Worker 0:{w} loss for batch 0: ")
            assert (folder / f"{exp}_0_{w}_times.csv").read_text().startswith("experiment_name, get_data")
    # the three own strategies average identically -> identical loss trajectories
    l1 = (folder / "onestep_reduce_0_0_loss.txt").read_text()
    assert l1 == (folder / "onestep_seq_merge_0_0_loss.txt").read_text()


def test_stem_weight_packing_roundtrip_and_fold_equivalence():
    """The folded 4x4 stem conv (space-to-depth input, packed weight) equals the 7x7/s2/p3 conv; the
    gradient unpacking is the exact inverse of the packing (CPU, fp32 math on bf16 values)."""
    import torch.nn.functional as F

    from distributed_learning_amd.ops.conv import stem_pack_weight, stem_unpack_grad

    torch.manual_seed(0)
    w = torch.randn(64, 3, 7, 7).to(torch.bfloat16)
    wp = stem_pack_weight(w)
    assert wp.shape == (64, 256)
    torch.testing.assert_close(stem_unpack_grad(wp), w, rtol=0, atol=0)
    x = torch.randn(2, 3, 14, 10).to(torch.bfloat16).float()
    ref = F.conv2d(x, w.float(), None, 2, 3)
    n, _, h, wd = x.shape
    xs = x.reshape(n, 3, h // 2, 2, wd // 2, 2).permute(0, 2, 4, 3, 5, 1).reshape(n, h // 2, wd // 2, 12)
    xs = F.pad(xs, (0, 4)).permute(0, 3, 1, 2)  # [n, 16, BH, BW]
    w4 = wp.float().reshape(64, 4, 4, 16).permute(0, 3, 1, 2)  # [co, 16, th, tw]
    got = F.conv2d(F.pad(xs, (2, 1, 2, 1)), w4)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
