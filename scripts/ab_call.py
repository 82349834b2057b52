#!/usr/bin/env python3
"""Run a script after one setter call on the native extension, for same-box A/B runs of settings that
have no environment knob: ``python scripts/ab_call.py "set_tile256_min_k(1024)" bench.py --steps 15``.
The statement is evaluated with the extension module's functions in scope."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_learning_amd.ops import _ext  # noqa: E402

if __name__ == "__main__":
    stmt, script, rest = sys.argv[1], sys.argv[2], sys.argv[3:]
    C = _ext.require()
    exec(stmt, {k: getattr(C, k) for k in dir(C) if not k.startswith("_")})
    sys.argv = [script] + rest
    runpy.run_path(script, run_name="__main__")
