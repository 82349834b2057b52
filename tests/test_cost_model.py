"""Bucket-size cost model (parallel/cost_model.py): collective-time formulas, the in-order overlap
simulation, and the cap it derives for ResNet-50 / ResNet-152 on an 8-GPU node."""
import pytest
import torch

from distributed_learning_amd.parallel import cost_model as cm


def test_collective_formulas():
    r = cm.ring_model(8, channels=7, link_gbps=153.0, step_alpha_us=10.0)
    assert r.alpha_s == pytest.approx(14 * 10e-6)
    # 2(N-1)/N * S / (C * link): 100 MB over 7 channels of 153 GB/s
    assert r.time(100e6) - r.alpha_s == pytest.approx(2 * 7 / 8 * 100e6 / (7 * 153e9))
    one = cm.ring_model(8, channels=1)
    assert one.beta_s_per_byte == pytest.approx(7 * r.beta_s_per_byte)  # 7 links vs one
    assert cm.ring_model(1).time(1e9) == 0.0 and cm.builtin_model(1).time(1e9) == 0.0
    b = cm.builtin_model(8, bus_gbps=300.0, alpha_us=20.0)
    assert b.time(0) == pytest.approx(20e-6)


def test_exposed_time_in_order_overlap():
    m = cm.CollectiveModel("t", 1.0, 1.0)  # T(S) = 1 + S seconds
    # ready at 0 and 5, sizes 1 and 1 -> finish 2, then max(5, 2) + 2 = 7; backward ends at 6
    exp, tot = cm.exposed_time([1, 1], [0, 5], 6, m)
    assert (exp, tot) == (1, 4)
    # a bucket queued behind a long one waits for it
    exp, tot = cm.exposed_time([10, 1], [0, 1], 20, m)
    assert exp == 0 and tot == 13
    exp, _ = cm.exposed_time([10, 1], [0, 1], 5, m)
    assert exp == 13 - 5


def test_tiny_buckets_pay_latency_huge_buckets_pay_tail():
    params = [torch.zeros(256 * 1024) for _ in range(64)]  # 64 x 1 MiB fp32
    ready = {id(p): (i + 1) / 64 * 0.01 for i, p in enumerate(reversed(params))}  # uniform over 10 ms
    model = cm.CollectiveModel("t", 200e-6, 1 / 50e9)
    cap, rows = cm.choose_bucket_cap(params, ready, 0.01, model, caps_mib=(1, 4, 16, 64))
    by = {r["cap_mib"]: r for r in rows}
    assert by[1]["comm_ms"] > by[16]["comm_ms"]  # 64 latencies vs 4
    assert by[64]["exposed_ms"] > by[4]["exposed_ms"]  # one bucket: everything after backward
    assert cap in (4, 16)


@pytest.mark.parametrize("name,bwd_s", [("resnet50", 0.028), ("resnet152", 0.060)])
def test_resnet_caps_at_8_gpus(name, bwd_s):
    from distributed_learning_amd.models import resnet50, resnet152

    m = {"resnet50": resnet50, "resnet152": resnet152}[name]()
    ready = cm.ready_times_from_flops(m, (3, 224, 224), bwd_s)
    params = list(m.parameters())
    assert len(ready) == len(params) and max(ready.values()) <= bwd_s * 1.0001
    # the classifier is the first gradient, the stem conv the last
    assert ready[id(m.fc.weight)] < ready[id(m.conv1.weight)]
    for model in (cm.builtin_model(8), cm.ring_model(8, 7)):
        cap, rows = cm.choose_bucket_cap(params, ready, bwd_s, model, wire_bytes_per_elem=4)
        by = {r["cap_mib"]: r for r in rows}
        assert by[cap]["cost_ms"] <= by[25]["cost_ms"] + 1e-9  # never worse than the reference's 25 MiB
        assert 2 <= cap <= 64


def test_ring_alpha_defaults_to_the_measured_issue_cost():
    a1, a7 = cm.measured_step_alpha_us(1), cm.measured_step_alpha_us(7)
    assert a1 == cm.VRANK_STEP_ALPHA_US[("ring", 1, "eager")] + cm.RCCL_GROUP_US
    assert a7 == cm.VRANK_STEP_ALPHA_US[("ring", 7, "eager")] + cm.RCCL_GROUP_US
    assert a1 < cm.measured_step_alpha_us(4) < a7
    assert cm.ring_model(8, 7).alpha_s == 14 * a7 * 1e-6
    assert cm.ring_model(8, 7, graph=True).alpha_s < cm.ring_model(8, 7).alpha_s
