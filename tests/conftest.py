import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_learning_amd.ops import _ext

    _ext.require()  # GPU tests must run the native path, never a silent fallback
    return torch.device("cuda:0")


_STATE = (("distributed_learning_amd.ops.nn", ("_BACKEND", "_NATIVE_CONV", "DUAL_RESIDUAL", "FORK_SUBSAMPLE")),
          ("distributed_learning_amd.ops.conv", ("DUAL_1X1", "DUAL_BN", "DUAL_1X1_MAX_COUT", "WGRAD_DEFER",
                                                 "WGRAD_JOIN", "BN_EPILOGUE", "RESIDUAL_HANDOFF")))


@pytest.fixture(autouse=True)
def _restore_module_switches():
    """Module-level backend switches a test flips (native backend / native convs / kernel choices) are put
    back after it, so a test that forgets its finally cannot change what later tests run (seen: a native
    stem conv leaking into test_gpu_stem's torch-conv comparison)."""
    saved = []
    for mod, names in _STATE:
        m = sys.modules.get(mod)
        if m is not None:
            saved.append((m, {n: getattr(m, n) for n in names if hasattr(m, n)}))
    yield
    for m, vals in saved:
        for n, v in vals.items():
            setattr(m, n, v)
    for mod, names in _STATE:  # modules first imported by this test: back to their defaults
        m = sys.modules.get(mod)
        if m is not None and not any(m is s for s, _ in saved) and mod.endswith(".nn"):
            if getattr(m, "_BACKEND", "torch") != "torch" and hasattr(m, "set_backend"):
                m.set_backend("torch")
            if getattr(m, "_NATIVE_CONV", False) and hasattr(m, "set_native_conv"):
                m.set_native_conv(False)
