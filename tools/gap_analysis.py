"""Idle gaps of the device timeline of a `rocprofv3 --kernel-trace` csv: histogram and the
largest gaps with the kernels on either side (what the host was doing between them).

    python tools/gap_analysis.py <kernel_trace.csv> [bench_line.json] [--top 15]
(with the bench line: only the timed window, the last steps x ms_per_step of the trace)
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench_line", nargs="?")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(a.trace))), key=lambda t: t[0])
    if a.bench_line:
        import json
        bl = json.load(open(a.bench_line))
        t_end = max(e for _, e, n in rows if "dicp" in n or "lse_" in n)
        t0 = t_end - int(bl["steps"] * bl["ms_per_step"] * 1e6)
        rows = [r for r in rows if r[0] >= t0 and r[1] <= t_end]
    gaps = []
    last_end, last_name = rows[0][1], rows[0][2]
    for s, e, n in rows[1:]:
        if s > last_end:
            gaps.append((s - last_end, last_name, n))
        if e > last_end:
            last_end, last_name = e, n
    hist = collections.Counter()
    tot = collections.Counter()
    for g, _, _ in gaps:
        b = "<10us" if g < 1e4 else "<100us" if g < 1e5 else "<1ms" if g < 1e6 else ">=1ms"
        hist[b] += 1
        tot[b] += g
    print("gaps:", {k: (hist[k], round(tot[k] / 1e6, 2)) for k in ("<10us", "<100us", "<1ms", ">=1ms")},
          "(count, ms)")
    pair = collections.Counter()
    for g, p, n in gaps:
        if g >= 1e4:
            pair[(p[:60], n[:60])] += g
    print("largest total gap time by (before, after) kernel pair:")
    for (p, n), g in pair.most_common(a.top):
        print(f"  {g / 1e6:8.2f} ms  {p}  ->  {n}")


if __name__ == "__main__":
    main()
