"""In-tree build of the native extension ``distributed_learning_amd._C`` for gfx950.

Every ``csrc/**/*.hip`` kernel file and ``csrc/*.cpp`` binding file is compiled directly with
``hipcc --offload-arch=gfx950`` (no hipify step, no CUDA sources) and linked into
``distributed_learning_amd/_C.so`` next to this file, so the built object travels with the repo
snapshot to the GPU box. Objects are cached under ``build/obj`` keyed by a hash of the source,
the headers and the flags; a no-op rebuild takes well under a second.

Usage: ``python -m distributed_learning_amd._build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = ROOT / "distributed_learning_amd"
OUT = PKG / "_C.so"
OBJ_DIR = ROOT / "build" / "obj"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch  # noqa: F401  (only for paths)
    from torch.utils import cpp_extension

    tdir = Path(torch.__file__).resolve().parent
    incs = [str(tdir / "include"), str(tdir / "include" / "torch" / "csrc" / "api" / "include")]
    del cpp_extension
    pyb = [
        f'-DPYBIND11_{k}="{getattr(torch._C, "_PYBIND11_" + k)}"'
        for k in ("COMPILER_TYPE", "STDLIB", "BUILD_ABI")
        if getattr(torch._C, "_PYBIND11_" + k, None) is not None
    ]
    return tdir, incs + pyb, int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc() -> str:
    p = Path(ROCM) / "bin" / "hipcc"
    return str(p) if p.exists() else "hipcc"


def _sources():
    kern = sorted((CSRC / "kernels").glob("*.hip"))
    binds = sorted(CSRC.glob("*.cpp")) + sorted((CSRC / "comm").glob("*.cpp"))
    return kern, binds


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted((CSRC / "include").glob("*.h")) + sorted((CSRC / "comm").glob("*.h")):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def source_digest(root: Path | None = None) -> str:
    """sha256 over every file the extension is built from (kernels, bindings, comm, headers), in a fixed
    order. Embedded in _C.so at link time; ops/_ext.py compares it with the tree it runs from."""
    csrc = (Path(root) if root is not None else ROOT) / "csrc"
    files = sorted((csrc / "kernels").glob("*.hip")) + sorted(csrc.glob("*.cpp")) + sorted((csrc / "comm").glob("*.cpp"))
    files += sorted((csrc / "include").glob("*.h")) + sorted((csrc / "comm").glob("*.h"))
    h = hashlib.sha256()
    for p in files:
        h.update(str(p.relative_to(csrc)).encode())
        h.update(b"\0")
        h.update(p.read_bytes())
    return h.hexdigest()


def _hash_object(bflags, digest: str, force: bool, verbose: bool) -> Path:
    src = OBJ_DIR / f"source_hash-{digest[:16]}.cpp"
    if not src.exists():
        src.write_text(f'extern "C" const char* dla_source_hash() {{ return "{digest}"; }}\n')
    return _compile_one(src, [f for f in bflags if f.startswith(("-O", "-f", "--offload"))], "", force, verbose)


def _flags(kind: str, tdir: Path, incs, abi: int, defines=()):
    common = [f"-D{d}" for d in defines] + [
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"-I{CSRC / 'include'}",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
    ]
    if kind == "kernel":
        return common + ["-ffp-contract=fast"]
    py_inc = sysconfig.get_paths()["include"]
    return common + [i if i.startswith("-D") else f"-I{i}" for i in incs] + [
        f"-I{py_inc}",
        f"-I{ROCM}/include",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
    ]


def _compile_one(src: Path, flags, hdr_digest: str, force: bool, verbose: bool) -> Path:
    key = hashlib.sha256()
    key.update(src.read_bytes())
    key.update(" ".join(flags).encode())
    key.update(hdr_digest.encode())
    obj = OBJ_DIR / f"{src.stem}-{key.hexdigest()[:16]}.o"
    if obj.exists() and not force:
        return obj
    cmd = [_hipcc(), *flags, "-c", str(src), "-o", str(obj)]
    if src.suffix == ".cpp":
        cmd.insert(1, "-x")
        cmd.insert(2, "hip")
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int | None = None, force: bool = False, verbose: bool = False, defines=(),
          out: Path | None = None) -> Path:
    """Compile and link; ``defines`` (e.g. ``DLA_MFMA_SHAPE=32``) build a variant, linked to ``out``
    (variants are loaded for A/B runs through ``DLA_EXT_SO=<path>``, see ops/_ext.py)."""
    out = Path(out) if out is not None else OUT
    tdir, incs, abi = _torch_paths()
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    kern, binds = _sources()
    hd = _headers_digest()
    jobs = jobs or min(8, (os.cpu_count() or 4))
    kflags = _flags("kernel", tdir, incs, abi, defines)
    bflags = _flags("binding", tdir, incs, abi, defines)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile_one, s, kflags, hd, force, verbose) for s in kern]
        futs += [ex.submit(_compile_one, s, bflags, hd, force, verbose) for s in binds]
        objs = [f.result() for f in futs]
    objs.append(_hash_object(bflags, source_digest(), force, verbose))
    tlib = tdir / "lib"
    link_key = hashlib.sha256(("".join(sorted(o.name for o in objs)) + str(out)).encode()).hexdigest()[:16]
    stamp = OBJ_DIR / f"link-{out.stem}-{link_key}.stamp"
    if out.exists() and stamp.exists() and not force:
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    # Link against torch's own HIP runtime / RCCL first (same SONAMEs as /opt/rocm), so the
    # extension shares one HIP runtime instance with torch at run time.
    cmd = [
        _hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(out), *map(str, objs),
        f"-L{tlib}", f"-Wl,-rpath,{tlib}",
        "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
        "-lamdhip64", "-lrccl",
    ]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    for old in OBJ_DIR.glob(f"link-{out.stem}-*.stamp"):
        old.unlink()
    stamp.touch()
    return out


SANITIZE_DIR = ROOT / "build" / "sanitize"


def sanitize_check(run: bool = True) -> int:
    """CPU AddressSanitizer + UndefinedBehaviorSanitizer build of the comm engine's host C++ (plan builder,
    virtual-rank host executor, IPC host protocol; csrc/tests/host_check.cpp) -- the GPU pool runs no
    sanitizers, so this is where they apply. Returns the check's exit status (0 = clean)."""
    SANITIZE_DIR.mkdir(parents=True, exist_ok=True)
    exe = SANITIZE_DIR / "host_check"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-pthread", str(CSRC / "tests" / "host_check.cpp"), str(CSRC / "comm" / "plan.cpp"),
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"sanitizer build failed:\n{r.stdout}\n{r.stderr}")
    if not run:
        return 0
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    return subprocess.run([str(exe)], env=env).returncode


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-D", "--define", action="append", default=[], help="extra -D for a variant build")
    ap.add_argument("--out", default=None, help="output .so (variant builds)")
    ap.add_argument("--sanitize", action="store_true",
                    help="build and run the ASan/UBSan CPU check of the host-side comm C++ instead")
    a = ap.parse_args(argv)
    if a.sanitize:
        return sanitize_check()
    out = build(a.jobs, a.force, a.verbose, tuple(a.define), a.out)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
