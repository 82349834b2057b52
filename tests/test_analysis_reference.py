"""analysis.py on the reference's own raw CSVs (/root/reference/measurements), reproducing the
published numbers exactly (collect_data.py:26-48,78-107).
Skipped where the reference checkout is absent (e.g. on the GPU box)."""
import os

import pytest

from distributed_learning_amd import analysis as A

R = "/root/reference/measurements"
pytestmark = pytest.mark.skipif(not os.path.isdir(R), reason="reference measurements not available")

SINGLE = ["gpu2/results/experiment_single_1_33846316"]
E1 = [f"gpu2/results/{f}" for f in ["experiment1_1_33847002", "experiment1_2_33846550", "experiment1_4_33846297",
                                    "experiment1_8_33846299", "experiment1_16_33846301"]]
E2 = [f"gpu2/results/{f}" for f in ["experiment2_1_33846552", "experiment2_2_33846303", "experiment2_4_33846305",
                                    "experiment2_8_33846308", "experiment2_16_33895822"]]

PUBLISHED = {  # BASELINE.md headline table, img/s at 1 / 2 / 4 / 8 / 16 devices
    "single": [317.5, 634.9, 1269.8, 2539.6, 5079.2],
    "ddp": [298.6, 573.6, 1096.7, 2040.9, 3703.6],
    "onestep_reduce": [254.3, 444.5, 876.1, 1631.8, 3054.0],
    "onestep_central": [254.7, 445.9, 851.8, 1490.5, 2221.4],
    "ourdist": [205.0, 288.7, 334.2, 629.4, 2866.0],
    "seq_merge": [215.7, 312.2, 374.0, 704.0, 2565.8],
    "central_node_reduce": [206.3, 287.4, 333.8, 622.8, 2583.6],
    "overlap": [133.6, 169.1, 184.6, 346.2, 1170.1],
}


def test_throughput_table_reproduces_published_numbers():
    data = A.with_ideal(A.load([os.path.join(R, f) for f in SINGLE + E1 + E2]))
    for exp, vals in PUBLISHED.items():
        for dev, want in zip([1, 2, 4, 8, 16], vals):
            assert round(data[(dev, exp)]["throughput"], 1) == want, (exp, dev)


def test_phase_breakdown_single_and_ddp():
    data = A.load([os.path.join(R, f) for f in SINGLE + E2])
    single = data[(1, "single")]
    want = {"get_data": 129.7, "data2dev": 9.4, "zero_grad": 5.5, "forward": 21.1, "backprop": 14.1, "sync": 0.0,
            "optimizer_step": 69.5, "batch": 403.2}
    for k, v in want.items():
        assert round(single[k], 1) == v, k
    for dev, batch in [(1, 428.6), (8, 501.7), (16, 553.0)]:
        assert round(data[(dev, "ddp")]["batch"], 1) == batch
    for dev, sync in [(1, 200.7), (8, 328.1), (16, 372.7)]:
        assert round(data[(dev, "onestep_reduce")]["sync"], 1) == sync


def test_fusion_sweep_reproduces_figure6():
    rows = A.fusion_sweep(os.path.join(R, "gpu1/results/fusion_experiment_ourdist_16_33723740"))
    got = {kib: (round(b, 1), round(s, 1)) for kib, b, s in rows}
    assert got == {1024: (1771.0, 1260.0), 4096: (1223.5, 738.4), 16384: (1196.4, 706.2), 65536: (1226.7, 914.2)}
