"""The comm engine's host-side C++ (plan builder, virtual-rank host executor, IPC host protocol) built with
AddressSanitizer + UndefinedBehaviorSanitizer and run as a standalone executable (csrc/tests/host_check.cpp,
``python -m distributed_learning_amd._build --sanitize``): 5.5k schedule / protocol cases must pass with no
sanitizer report. Its first run found a dangling ``const Topology&`` member in VirtualRun (csrc/comm/vexec.h)
when the run is built from a temporary topology; the member is now held by value and host_check constructs
every run that way, so a regression aborts this test."""
import shutil
import subprocess

import pytest

from distributed_learning_amd import _build


def _has_asan() -> bool:
    if shutil.which("g++") is None:
        return False
    r = subprocess.run(["g++", "-fsanitize=address,undefined", "-x", "c++", "-", "-o", "/dev/null"],
                       input="int main(){return 0;}", capture_output=True, text=True)
    return r.returncode == 0


@pytest.mark.skipif(not _has_asan(), reason="no g++ with ASan/UBSan")
def test_host_comm_code_is_sanitizer_clean():
    assert _build.sanitize_check() == 0
