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


def _cli(tmp_path, sub, *extra, batches=3):
    out = tmp_path / sub
    out.mkdir(exist_ok=True)
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "distributed_learning_amd.main", "1", "0", "1", "1", "127.0.0.1", "lo", "mnist",
           "/nonexistent", "0", "--experiment", "experiment_single", "--random_input", "1", "--limit_batches",
           str(batches), "--batch_size", "8", "--master_port", str(__import__("dist_util").free_port()),
           "--results_root", str(out), "--job_id", "t", *extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(out))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [float(l.rsplit(": ", 1)[1]) for l in (out / "experiment_single_1_t" / "single_0_0_loss.txt").read_text()
            .splitlines()], (out / "experiment_single_1_t" / "single_0_0_loss.txt").read_text().splitlines()


def test_checkpoint_resume_continues_the_run(tmp_path):
    """6 batches in one run == 3 batches + checkpoint + resumed 3 batches (same data stream, same
    numbering, same weights)."""
    full, _ = _cli(tmp_path, "full", batches=6)
    ck = str(tmp_path / "ck.pt")
    first, _ = _cli(tmp_path, "a", "--checkpoint", ck, batches=3)
    second, lines = _cli(tmp_path, "b", "--resume", ck, batches=3)
    assert lines[0].startswith("Worker 0:0 loss for batch 3: ")
    assert first == full[:3]
    assert second == pytest.approx(full[3:], rel=1e-5, abs=1e-6)


def test_synthetic_seek():
    s = SyntheticBatches(4, (3, 8, 8), 10, "cpu")
    batches = [s.next()[0].clone() for _ in range(4)]
    t = SyntheticBatches(4, (3, 8, 8), 10, "cpu")
    t.seek(2)
    assert torch.equal(t.next()[0], batches[2])


# --- offline loaders on tiny fixtures written here (C24) -----------------------------------------
def test_mnist_idx_loader(tmp_path):
    import struct

    from distributed_learning_amd.data import get_partition_loader, load_mnist

    d = tmp_path / "mnist" / "MNIST" / "raw"
    d.mkdir(parents=True)
    imgs = (torch.arange(20 * 28 * 28) % 256).to(torch.uint8).reshape(20, 28, 28)
    labels = (torch.arange(20) % 10).to(torch.uint8)
    with open(d / "train-images-idx3-ubyte", "wb") as f:
        f.write(struct.pack(">IIII", 0x0803, 20, 28, 28) + imgs.numpy().tobytes())
    with open(d / "train-labels-idx1-ubyte", "wb") as f:
        f.write(struct.pack(">II", 0x0801, 20) + labels.numpy().tobytes())
    ds = load_mnist(str(tmp_path))
    assert len(ds) == 20
    x, y = ds[3]
    assert x.shape == (1, 28, 28) and int(y) == 3
    torch.testing.assert_close(x, (imgs[3].float() / 255.0 - 0.1307).unsqueeze(0) / 0.3081)
    # partition semantics (reference data.py:26-68): 2 workers x 2 batches of 4 -> disjoint 8-sample sets
    seen = []
    for w in range(2):
        dl = get_partition_loader(ds, 0, w, 2, 2, batch_size=4, num_workers=0)
        got = [int(v) for xb, yb in dl for v in yb]
        assert len(got) == 8
        seen.append(dl.dataset.index.tolist())
    assert not set(seen[0]) & set(seen[1])


def test_cifar10_binary_loader(tmp_path):
    from distributed_learning_amd.data import load_cifar10

    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rows = []
    for i in range(5):
        rec = torch.zeros(3073, dtype=torch.uint8)
        rec[0] = i % 10
        rec[1:] = (torch.arange(3072) + i) % 256
        rows.append(rec)
    blob = torch.stack(rows).numpy().tobytes()
    for i in range(1, 6):
        (d / f"data_batch_{i}.bin").write_bytes(blob)
    ds = load_cifar10(str(tmp_path))
    assert len(ds) == 25
    x, y = ds[2]
    assert x.shape == (3, 32, 32) and int(y) == 2
    raw = ((torch.arange(3072) + 2) % 256).float().reshape(3, 32, 32) / 255.0
    mean = torch.tensor([0.4914, 0.4822, 0.4465]).view(3, 1, 1)
    std = torch.tensor([0.2470, 0.2435, 0.2616]).view(3, 1, 1)
    torch.testing.assert_close(x, (raw - mean) / std)


def test_imagefolder_loader(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    from distributed_learning_amd.data import ImageFolder, load_dataset

    root = tmp_path / "ImageFolder"
    for ci, c in enumerate(["cat", "dog"]):
        (root / c).mkdir(parents=True)
        for j in range(2):
            img = PIL.new("RGB", (300, 260), color=(40 * ci + j, 100, 200))
            img.save(root / c / f"{j}.png")
    ds = load_dataset("imagenet", str(tmp_path))
    assert isinstance(ds, ImageFolder) and ds.classes == ["cat", "dog"] and len(ds) == 4
    x, y = ds[3]
    assert x.shape == (3, 224, 224) and y == 1
    want = (torch.tensor([41, 100, 200]) / 255.0 - torch.tensor([0.485, 0.456, 0.406])) / torch.tensor(
        [0.229, 0.224, 0.225])
    torch.testing.assert_close(x[:, 100, 100], want.float(), atol=1e-5, rtol=0)


def _mnist_fixture(root, n=40):
    import struct

    d = root / "mnist" / "MNIST" / "raw"
    d.mkdir(parents=True)
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (n, 28, 28), generator=g, dtype=torch.uint8)
    labels = (torch.arange(n) % 10).to(torch.uint8)
    with open(d / "train-images-idx3-ubyte", "wb") as f:
        f.write(struct.pack(">IIII", 0x0803, n, 28, 28) + imgs.numpy().tobytes())
    with open(d / "train-labels-idx1-ubyte", "wb") as f:
        f.write(struct.pack(">II", 0x0801, n) + labels.numpy().tobytes())


def test_epoch_sampler_resume_order():
    """Per-epoch order is a function of (seed, epoch); resuming at global batch k reproduces the
    uninterrupted sequence from k on, across epoch boundaries, without touching skipped samples."""
    from distributed_learning_amd.data import EpochSampler, resume_position

    n, bs = 40, 4
    bpe = n // bs
    s = EpochSampler(n, seed=7)
    full = []
    for e in range(3):
        s.set_epoch(e)
        full += list(s)
    assert sorted(full[:n]) == list(range(n)) and full[:n] != full[n:2 * n]
    for k in (0, 3, 10, 13, 25):
        e0, skip = resume_position(k, bpe)
        got = []
        for e in range(e0, 3):
            s.set_epoch(e, skip * bs if e == e0 else 0)
            got += list(s)
        assert got == full[k * bs:], k


def test_resume_with_real_loader_continues_the_batch_sequence(tmp_path):
    """a resumed run on a real (shuffled) dataset sees exactly the batches an uninterrupted
    run would, including across an epoch boundary (10 batches per epoch, resume at batch 6, run 8)."""
    _mnist_fixture(tmp_path / "data")

    def run(sub, *extra, batches):
        out = tmp_path / sub
        out.mkdir(exist_ok=True)
        env = dict(os.environ, PYTHONPATH=ROOT)
        cmd = [sys.executable, "-m", "distributed_learning_amd.main", "1", "0", "1", "1", "127.0.0.1", "lo", "mnist",
               str(tmp_path / "data"), "0", "--experiment", "main_single", "--limit_batches", str(batches),
               "--batch_size", "4", "--master_port", str(__import__("dist_util").free_port()),
               "--results_root", str(out), "--job_id", "t", *extra]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(out))
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        lines = (out / "main_single_1_t" / "single_0_0_loss.txt").read_text().splitlines()
        return [float(l.rsplit(": ", 1)[1]) for l in lines], lines

    full, _ = run("full", batches=14)
    ck = str(tmp_path / "ck.pt")
    first, _ = run("a", "--checkpoint", ck, batches=6)
    second, lines = run("b", "--resume", ck, batches=8)
    assert lines[0].startswith("Worker 0:0 loss for batch 6: ")
    assert first == full[:6]
    assert second == pytest.approx(full[6:], rel=1e-5, abs=1e-6)


def test_gradsync_steal_mode_unused_params_without_overlap():
    """Steal mode (the native engine's) + no overlap hooks (SeqMergeDist) + parameters marked unused
    (GoogLeNet aux heads) at one rank: flush must not report the unused ones ready a second time
    (round-3 GPU CLI failure in experiment1's seq_merge)."""
    from distributed_learning_amd.parallel.executor import Executor
    from distributed_learning_amd.parallel.grad_sync import GradSync

    class StealExec(Executor):
        supports_steal = True
        passthrough = True

        def __init__(self):
            self.submitted = []

        def submit(self, b):
            self.submitted.append(b.index)

        def finish(self):
            pass

    net = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4), torch.nn.Linear(4, 2))
    ex = StealExec()
    gs = GradSync(net.parameters(), bucket_cap_bytes=64, executor=ex, overlap=False)
    assert gs.grad_mode == "steal"
    for _ in range(2):
        gs.prepare()
        unused = list(net[1].parameters())
        gs.mark_ready(unused)
        net[2](net[0](torch.randn(3, 4))).sum().backward()
        gs.synchronize()
        assert sorted(ex.submitted) == list(range(len(gs.buckets)))
        ex.submitted.clear()


def test_fused_sgd_master_state_survives_checkpoint(tmp_path):
    """bf16 parameters + fp32 masters: a checkpoint round trip keeps the masters and momentum fp32 and
    bit-exact (torch's load_state_dict would cast them to the parameter dtype)."""
    from distributed_learning_amd.ops.optim import FusedSGD

    p = torch.nn.Parameter(torch.randn(33).to(torch.bfloat16))
    opt = FusedSGD([p], lr=0.1, momentum=0.5, master_weights=True)
    p.grad = torch.randn(33).to(torch.bfloat16)
    opt.step()
    torch.save(opt.state_dict(), tmp_path / "o.pt")
    q = torch.nn.Parameter(p.detach().clone())
    opt2 = FusedSGD([q], lr=0.1, momentum=0.5, master_weights=True)
    opt2.load_state_dict(torch.load(tmp_path / "o.pt", weights_only=True))
    for k in ("master", "momentum_buffer"):
        assert opt2.state[q][k].dtype == torch.float32
        assert torch.equal(opt2.state[q][k], opt.state[p][k])
