"""Every environment switch of the framework, in one table, read in one place.

Each knob is the environment variable ``DLA_<NAME>``. Python reads it only through :func:`get`
(parsed once, cached); the C++/HIP side reads its own (``std::getenv`` once per process, in the
file named in the table) and the table documents those too, so :func:`non_default` reports every
switch a run was started with. ``bench.py`` records ``non_default()`` as ``"knobs"`` in its JSON
line: ``{}`` means the shipped defaults, the only combination the end-to-end tests and the credited
numbers use. Defaults are the measured-best settings; the alternatives stay for A/B runs
(the profile that decided each default is cited).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, Optional


@dataclass(frozen=True)
class Knob:
    default: str
    where: str
    what: str


PREFIX = "DLA_"

TABLE: Dict[str, Knob] = {
    # ---- run configuration -------------------------------------------------------------------------
    "KERNELS": Knob("native", "bench.py", "native | torch: the model's kernels (bench --kernels default)"),
    "PRECISION": Knob("bf16", "bench.py", "bf16 | autocast | fp32 (bench --precision default)"),
    "CONV": Knob("native", "bench.py", "native | miopen 1x1 convolutions (bench --conv default)"),
    "GRAPH": Knob("off", "bench.py", "on | off: HIP-graph capture of the whole step (bench --graph default)"),
    "SAME_DEVICE": Knob("0", "parallel/context.py", "1: every rank on cuda:0 (gloo + IPC transport)"),
    "TRANSPORT": Knob("", "parallel/context.py", "rccl | ipc gradient transport (default rccl; ipc with SAME_DEVICE)"),
    "COMPUTE_STREAM": Knob("default", "bench.py", "high: the training step runs on a high-priority stream, so its "
                                                  "kernels dispatch ahead of the late weight gradients' side stream"),
    "LAUNCH_GROUPS": Knob("1", "parallel/grad_sync.py", "0: fusion off (bucket cap 0) issues one collective launch per "
                                                        "gradient tensor, the reference's semantics (main.py:168-179); 1: "
                                                        "the per-tensor collectives launch in groups (profiles/r5/g04/)"),
    "DEFER_APPLY": Knob("1", "ops/bn_act.py", "1: a bottleneck block's final BN(+residual)+ReLU output is written by the "
                                              "next block's conv1 GEMM (gemm_apply.hip) instead of its own apply pass"),
    "APPLY_MAX_K": Knob("512", "csrc/kernels/gemm_apply.hip", "largest conv1 input width whose deferred block-final "
                                                               "apply the conv1 GEMM writes (<= 2048)"),
    "WGRAD_W4": Knob("0", "csrc/kernels/conv.hip", "1: 128x256 four-wave tiles for the Cout-128 3x3 weight gradients"),
    "DEFER_MID": Knob("0", "models/resnet.py", "1: a bottleneck's bn2+ReLU output is written by conv3's streaming GEMM "
                                              "(gemm_stream.hip kAp) at the short-K stages instead of its own apply pass; measured slower, profiles/r6/g22/"),
    "APPLY_SUBSAMPLE": Knob("1", "ops/conv.py", "1: at a stage transition the fused conv1 apply also writes the stride-2 "
                                                "subsample of the block output (no subsample2 pass)"),
    "AUTOTUNE_BUDGET_S": Knob("90", "parallel/autotune.py", "wall-clock budget of the all-reduce selection at N > 1"),
    "COMM_TIMEOUT_S": Knob("600", "csrc/comm/engine.cpp", "seconds before a collective / IPC barrier is declared dead"),
    # ---- scheduling of the backward ----------------------------------------------------------------
    "WGRAD_DEFER": Knob("3x3", "ops/conv.py", "3x3 | auto | all | 0: weight gradients on the side stream "
                                              "(profiles/r3/g18_g19_wgrad_defer.md, g47_defer_batch_ab.md; 'all' "
                                              "stalls for seconds at bs1280, profiles/r6/g27/)"),
    "WGRAD_JOIN": Knob("end", "ops/conv.py", "end | conv: where the compute stream joins the side stream"),
    "WGRAD_DEFER_MIN_AI": Knob("200", "ops/conv.py", "WGRAD_DEFER=auto: 1x1 arithmetic-intensity threshold"),
    "BN_EPILOGUE": Knob("0", "ops/conv.py", "1 / stream: BN-backward partials in every / the streaming dgrad "
                                            "GEMM epilogue (profiles/r4/g02/, bn_epilogue_ab_bs512.jsonl)"),
    "STEM_BN": Knob("1", "ops/conv.py", "0: stem BN+ReLU+max-pool backward apply as its own pass, not inside the "
                                        "stem weight gradient (profiles/r5/g11/)"),
    # ---- GoogLeNet Inception fusions ---------------------------------------------------------------
    "BN_GROUPED": Knob("1", "ops/inception.py", "0: one BN launch chain per Inception branch (profiles/r3p/)"),
    "FANIN_CAT": Knob("1", "ops/inception.py", "0: three separate fan-in 1x1 GEMMs (profiles/r3y/)"),
    # ---- kernel selection (C++) --------------------------------------------------------------------
    "STEM_STREAM": Knob("0", "csrc/kernels/gemm_stream.hip", "1: the stem forward (with BN statistics) on the persistent "
                                                             "streaming GEMM instead of the 128x64 tile kernel"),
    "GEMM256_DIRECT": Knob("0", "csrc/kernels/gemm.hip", "1: the 256x256 statistics forwards store their tile and "
                                                          "statistics from registers (dla_mfma.h epilogue_direct)"),
    "TILE256": Knob("1", "csrc/kernels/gemm.hip", "0: no 256x256 tiles for fwd / dgrad (profiles/r5a/)"),
    "TILE512": Knob("1", "csrc/kernels/conv.hip", "0: no 512x128 tiles for the Cout-128 3x3 fwd / dgrad (profiles/r5/g54/)"),
    "TILE256_MIN_K_STATS": Knob("256", "csrc/kernels/gemm.hip", "smallest K of the 256x256 tiles for the forward GEMMs "
                                                                  "with BN statistics (profiles/r6/g11/)"),
    "TN256": Knob("1", "csrc/kernels/gemm.hip", "0: no 256x256 weight-gradient tiles (profiles/r5c/, r5d/)"),
    "SPLITK_XCD": Knob("1", "csrc/kernels/gemm.hip", "0: no XCD-aware split-K grids (round-2 README row)"),
    "SPLITK_BLOCKS": Knob("512", "csrc/kernels/gemm.hip", "split-K grid target in blocks"),
    "SPLITK_SG": Knob("1", "csrc/kernels/gemm.hip", "0: no split-group split-K reduce (profiles/r3n/)"),
    "GEMM_SPLITK": Knob("1", "csrc/nn_bindings.cpp", "0: no split-K for the FC heads"),
    "GEMM_DIRECT": Knob("0", "csrc/kernels/gemm_direct.hip", "1: 128x128 1x1 GEMM tiles stored straight from the "
                                                             "registers, not staged through LDS (neutral: profiles/r6/g03/)"),
    "GEMM_PERSIST": Knob("0", "csrc/kernels/gemm_direct.hip", "n > 0: the register-stored 128x128 tiles (GEMM_DIRECT=1) as a "
                                                              "persistent kernel with n blocks per CU"),
    "GEMM_STREAM": Knob("1", "csrc/kernels/gemm_stream.hip", "0: no persistent streaming 1x1 GEMM (profiles/r3/)"),
    "CONV_PIPE": Knob("-1", "csrc/kernels/conv.hip", "3x3 conv main-loop pipeline for K >= 256 (-1: per shape)"),
    "HALO": Knob("2", "csrc/kernels/conv_halo.hip", "0 off, 1 dgrad only, 2 fwd + dgrad halo-tiled 64-ch 3x3 (r5l/)"),
    "HALO_V": Knob("3", "csrc/kernels/conv_halo.hip", "halo kernel version (1 / 2 / 3 = 2 forward + 1 data "
                                                    "gradient, profiles/r6/g32/)"),
    "HALO_FASTDIV": Knob("1", "csrc/kernels/conv_halo.hip", "0: integer divisions for the halo conv's per-strip tap masks "
                                                            "(A/B of the multiply-shift form, profiles/r6/g30/)"),
    "HALO_DIRECT": Knob("1", "csrc/kernels/conv_halo.hip", "1: the variant-1 halo data gradient stores its tile from "
                                                           "registers (transposed product) instead of through LDS "
                                                           "(profiles/r6/g34/)"),
    "HALO_DIRECT_FWD": Knob("0", "csrc/kernels/conv_halo.hip", "1: the variant-2 halo forward stores its tile and "
                                                               "statistics from registers"),
    "HALO_WGRAD": Knob("1", "csrc/kernels/conv_halo_wgrad.hip", "0: implicit-GEMM 64-ch 3x3 weight gradient"),
    "POOL3_SEP": Knob("4", "csrc/kernels/pool.hip", "separable 3x3 stride-1 max-pool variant (4 / 7; other: off; r3w/)"),
    "BN_RED_BLOCKS": Knob("1024", "csrc/kernels/bn_act.hip", "BN reduction-pass block target"),
    # ---- diagnostics -------------------------------------------------------------------------------
    "HOOK_TIMING": Knob("0", "parallel/grad_sync.py", "1: host time inside the gradient hooks"),
    "TRACE": Knob("0", "utils/trace.py", "1: roctx ranges per phase"),
    "VERBOSE": Knob("", "utils/log.py", "log level (default INFO)"),
    "TORCH_PROF": Knob("", "bench.py", "path: torch.profiler table after the timed region"),
    # ---- build / load ------------------------------------------------------------------------------
    "AUTOBUILD": Knob("0", "ops/_ext.py", "1: build the extension on first import"),
    "EXT_SO": Knob("", "ops/_ext.py", "path of a variant _C.so (A/B builds, _build.py --out)"),
    "ALLOW_STALE": Knob("0", "ops/_ext.py", "1: load a _C.so whose embedded source digest differs from csrc/"),
}

_CACHE: Dict[str, str] = {}


def get(name: str) -> str:
    """The knob's value (environment or default), read once per process."""
    if name not in TABLE:
        raise KeyError(f"unknown knob {name!r}; every switch must be listed in knobs.TABLE")
    if name not in _CACHE:
        _CACHE[name] = os.environ.get(PREFIX + name, TABLE[name].default)
    return _CACHE[name]


def flag(name: str) -> bool:
    return get(name) not in ("", "0", "off", "false", "False")


def env_name(name: str) -> str:
    return PREFIX + name


def non_default(environ: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """Every knob set in the environment to something other than its default, plus any unknown
    ``DLA_*`` variable (reported under its full name, so a typo is visible too)."""
    env = os.environ if environ is None else environ
    out: Dict[str, str] = {}
    for k, v in env.items():
        if not k.startswith(PREFIX):
            continue
        name = k[len(PREFIX):]
        knob = TABLE.get(name)
        if knob is None:
            out[k] = v
        elif v != knob.default:
            out[name] = v
    return out


def table_markdown() -> str:
    rows = ["| knob (env `DLA_<NAME>`) | default | read in | what |", "|---|---|---|---|"]
    for n, k in TABLE.items():
        rows.append(f"| `{n}` | `{k.default}` | `{k.where}` | {k.what} |")
    return "\n".join(rows)
