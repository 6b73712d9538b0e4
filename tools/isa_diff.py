"""Which kernels' machine code changed between two device-assembly builds (hipcc -S
--cuda-device-only) of the same source file: a kernel is "same" when its instruction stream,
with labels and comments stripped, is identical.  Used to check that a change aimed at some
kernels leaves the tuned ones (the headline VJP and forward) bit-for-bit alone.

    python tools/isa_diff.py old.s new.s [kernel-substring ...]
"""
import re
import sys


def kernels(text):
    out = {}
    for m in re.finditer(r"^(_Z\w+):\s*;", text, re.M):
        start = m.end()
        end = text.find(".Lfunc_end", start)
        body = []
        for l in text[start:end].split("\n"):
            l = l.split(";")[0].strip()
            if not l or l.startswith(".") or l.endswith(":"):
                continue
            body.append(re.sub(r"\.LBB\w+", "L", l))
        out[m.group(1)] = body
    return out


def main():
    a = kernels(open(sys.argv[1]).read())
    b = kernels(open(sys.argv[2]).read())
    pats = sys.argv[3:]
    same = changed = 0
    for k in sorted(set(a) | set(b)):
        if pats and not any(p in k for p in pats):
            continue
        if k not in a or k not in b:
            print(("new     " if k in b else "removed ") + k[:150])
        elif a[k] != b[k]:
            changed += 1
            print(f"changed {k[:150]} ({len(a[k])} -> {len(b[k])} instr.)")
        else:
            same += 1
    print(f"same {same}, changed {changed}")


if __name__ == "__main__":
    main()
