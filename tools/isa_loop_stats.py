"""Instruction mix of each kernel's innermost pair loop (the basic block that contains
v_exp_f32 and branches back to itself), from a hipcc --save-temps .s file.

    python tools/isa_loop_stats.py build.s [kernel-substring ...]
"""
import re
import sys
from collections import Counter


def kernels(text):
    for m in re.finditer(r"^(_Z\w+):\s*;", text, re.M):
        start = m.end()
        end = text.find(".Lfunc_end", start)
        yield m.group(1), text[start:end]


def loops(body):
    blocks = re.split(r"^(\.LBB\w+):", body, flags=re.M)
    # blocks = [pre, label1, text1, label2, text2, ...]
    for i in range(1, len(blocks) - 1, 2):
        lab, txt = blocks[i], blocks[i + 1]
        if re.search(r"s_cbranch_\w+\s+" + re.escape(lab) + r"\b", txt) and "v_exp_f32" in txt:
            yield lab, txt


def main():
    text = open(sys.argv[1]).read()
    pats = sys.argv[2:]
    for name, body in kernels(text):
        if pats and not any(p in name for p in pats):
            continue
        for lab, txt in loops(body):
            ins = [l.split()[0] for l in txt.split("\n") if l.strip() and not l.strip().startswith((";", "."))]
            c = Counter(ins)
            nexp = c.get("v_exp_f32_e32", 0) + c.get("v_exp_f32_e64", 0)
            valu = sum(v for k, v in c.items() if k.startswith("v_"))
            lds = sum(v for k, v in c.items() if k.startswith("ds_"))
            print(f"{name[:90]} {lab}: exp={nexp} valu={valu} ({valu / max(nexp, 1):.1f}/exp) lds={lds} "
                  f"movs={c.get('v_mov_b32_e32', 0)} pk={sum(v for k, v in c.items() if 'pk' in k)}")


if __name__ == "__main__":
    main()
