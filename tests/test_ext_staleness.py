"""The native extension refuses to load when it was not built from the sources next to it (VERDICT r4
next-round 3): _build.py links a digest of csrc/ into _C.so (``_C.source_hash``) and ops/_ext.py compares it
with the tree it runs from. Here a copy of the package with one kernel source edited after the build must
raise on require(), name both digests, and load again only with DLA_ALLOW_STALE=1."""
import os
import shutil
import subprocess
import sys

import pytest

from distributed_learning_amd import _build
from distributed_learning_amd.ops import _ext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not _ext.available(), reason="native extension not built")


def test_in_tree_binary_matches_its_sources():
    C = _ext.require()
    assert C.source_hash == _build.source_digest()
    assert _ext.stale_reason(C) == ""


def _copy_tree(dst):
    shutil.copytree(os.path.join(ROOT, "distributed_learning_amd"), os.path.join(dst, "distributed_learning_amd"),
                    ignore=shutil.ignore_patterns("__pycache__"))
    shutil.copytree(os.path.join(ROOT, "csrc"), os.path.join(dst, "csrc"))


def _require_in(root, extra_env=None):
    env = {k: v for k, v in os.environ.items() if not k.startswith("DLA_")}
    env.update(extra_env or {})
    code = ("import sys; sys.path.insert(0, sys.argv[1]); from distributed_learning_amd.ops import _ext; "
            "C = _ext.require(); print('loaded', C.source_hash[:16])")
    return subprocess.run([sys.executable, "-c", code, root], capture_output=True, text=True, env=env, timeout=240)


def test_stale_binary_is_refused(tmp_path):
    root = str(tmp_path)
    _copy_tree(root)
    r = _require_in(root)
    assert r.returncode == 0 and "loaded" in r.stdout, r.stderr[-2000:]
    with open(os.path.join(root, "csrc", "kernels", "loss.hip"), "a") as f:
        f.write("\n// edited after the build\n")
    C = _ext.require()
    assert "stale native extension" in _ext.stale_reason(C, root)
    r = _require_in(root)
    assert r.returncode != 0
    assert "stale native extension" in r.stderr and C.source_hash[:16] in r.stderr, r.stderr[-2000:]
    r = _require_in(root, {"DLA_ALLOW_STALE": "1"})
    assert r.returncode == 0 and "loaded" in r.stdout, r.stderr[-2000:]
