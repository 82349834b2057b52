"""Render scripts/bench_conv.py + bench_gemm.py JSON-line logs as the markdown tables in profiles/."""
import json
import sys


def rows(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.startswith("{")]


def main(conv_log, gemm_log, out_path):
    out = ["# Native MFMA kernels vs MIOpen / hipBLASLt at the ResNet-50 bs256 shapes (MI355X, 1 GPU)", "",
           "Times in ms per call (scripts/bench_conv.py, scripts/bench_gemm.py). p0 = register-staged main loop,",
           "p2 / p3 = 2 / 3-stage LDS-DMA (global_load_lds) main loop. The native forwards include the fused",
           "BatchNorm-statistics epilogue.", "",
           "## 3x3 convolutions (implicit GEMM, csrc/kernels/conv.hip)", "",
           "| Cin | H | Cout | stride | fwd MIOpen | fwd p0 | fwd p2 | fwd p3 | dgrad MIOpen | dgrad p0 | dgrad p2 | "
           "wgrad MIOpen | wgrad p0 | wgrad p2 |",
           "|" + "---:|" * 14]
    for r in rows(conv_log):
        g = lambda k: r.get(k, "-")  # noqa: E731
        out.append(f"| {r['Cin']} | {r['H']} | {r['Cout']} | {r['stride']} | {g('fwd_miopen')} | {g('fwd_p0')} | "
                   f"{g('fwd_p2')} | {g('fwd_p3')} | {g('dgrad_miopen')} | {g('dgrad_p0')} | {g('dgrad_p2')} | "
                   f"{g('wgrad_miopen')} | {g('wgrad_p0')} | {g('wgrad_p2')} |")
    out += ["", "## 1x1 convolutions as GEMMs (csrc/kernels/gemm.hip)", "",
            "| M | Cin | Cout | fwd p0 | fwd p2 | dgrad p0 | dgrad p2 | wgrad p0 | wgrad p2 | torch mm fwd | "
            "MIOpen conv fwd | hipBLASLt wgrad |",
            "|" + "---:|" * 12]
    for r in rows(gemm_log):
        g = lambda k: r.get(k, "-")  # noqa: E731
        out.append(f"| {r['M']} | {r['Cin']} | {r['Cout']} | {g('fwd_p0')} | {g('fwd_p2')} | {g('dgrad_p0')} | "
                   f"{g('dgrad_p2')} | {g('wgrad_p0')} | {g('wgrad_p2')} | {g('fwd_torch_mm_ms')} | "
                   f"{g('fwd_miopen_conv_ms')} | {g('wgrad_torch_mm_ms')} |")
    with open(out_path, "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:4])
