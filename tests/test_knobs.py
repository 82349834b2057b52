"""Every environment switch is in one documented table (distributed_learning_amd/knobs.py).

Checks that each ``DLA_*`` variable read anywhere in the package or the native sources (``getenv`` in
csrc, ``knobs.get`` in Python) is listed, that Python reads none of them behind the table's back, and
that the bench record's ``knobs`` field is empty at defaults and names what was changed.
"""
import os
import re

from distributed_learning_amd import knobs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _files(sub, exts):
    for d, _, fs in os.walk(os.path.join(ROOT, sub)):
        for f in fs:
            if f.endswith(exts):
                yield os.path.join(d, f)


def test_native_getenv_knobs_are_listed():
    rx = re.compile(r'getenv\("DLA_([A-Z0-9_]+)"\)')
    found = set()
    for p in _files("csrc", (".cpp", ".h", ".hip")):
        found |= set(rx.findall(open(p).read()))
    assert found, "no native knob found (pattern broken?)"
    missing = sorted(n for n in found if n not in knobs.TABLE)
    assert not missing, f"native knobs missing from knobs.TABLE: {missing}"


def test_python_reads_knobs_through_the_table():
    rx = re.compile(r'os\.environ(?:\.get)?[\[(]\s*"DLA_([A-Z0-9_]+)"')
    offenders = []
    for p in list(_files("distributed_learning_amd", (".py",))) + [os.path.join(ROOT, "bench.py")]:
        if p.endswith("knobs.py"):
            continue
        for n in rx.findall(open(p).read()):
            offenders.append((os.path.relpath(p, ROOT), n))
    assert not offenders, f"read DLA_* through knobs.get instead: {offenders}"
    rx2 = re.compile(r'knobs\.(?:get|flag|env_name)\("([A-Z0-9_]+)"\)')
    used = set()
    for p in list(_files("distributed_learning_amd", (".py",))) + [os.path.join(ROOT, "bench.py")]:
        used |= set(rx2.findall(open(p).read()))
    assert used and all(n in knobs.TABLE for n in used), sorted(used - set(knobs.TABLE))


def test_non_default_reports_changes_only():
    env = {"DLA_WGRAD_DEFER": "3x3", "DLA_TILE256": "0", "DLA_TYPO": "1", "PATH": "/bin"}
    assert knobs.non_default(env) == {"TILE256": "0", "DLA_TYPO": "1"}
    assert knobs.non_default({}) == {}
    assert "| `WGRAD_DEFER` |" in knobs.table_markdown()
