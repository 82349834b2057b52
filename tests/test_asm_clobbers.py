"""Static check of the hand-written inline assembly (CPU): every asm statement whose text contains a scalar
ALU instruction that writes SCC (s_add / s_sub / s_cmp / s_and / s_or / shifts ...) must list "scc" among its
clobbers. hipcc otherwise keeps a branch condition in SCC across the statement: that silently disabled the
tile stores of the streaming GEMM's K = 128 instantiations (round 3), and moved a prologue branch of the
256x128 GEMM tile kernel."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1] / "csrc"
SCC_WRITERS = re.compile(r"\bs_(add|addc|sub|subb|cmp\w*|and|or|xor|andn2|orn2|nand|nor|xnor|lshl|lshr|ashr|"
                         r"bfe|abs|min|max|bitcmp\w*|cselect)\w*\b")


def _asm_statements(text):
    for m in re.finditer(r"asm\s+volatile\s*\(", text):
        depth, i = 1, m.end()
        while depth and i < len(text):
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        yield text[m.start():i]


def test_scc_writing_asm_declares_the_clobber():
    offenders = []
    n = 0
    for p in sorted(list(ROOT.rglob("*.h")) + list(ROOT.rglob("*.hip")) + list(ROOT.rglob("*.cpp"))):
        for stmt in _asm_statements(p.read_text()):
            n += 1
            code = " ".join(re.findall(r'"([^"]*)"', stmt.split(":")[0]))
            if SCC_WRITERS.search(code) and '"scc"' not in stmt:
                offenders.append(f"{p.name}: {code[:80]}")
    assert n > 0
    assert not offenders, offenders
