"""Device-timeline summary of a `rocprofv3 --kernel-trace` run of bench.py (W warmup iterations,
then K timed ones): busy time, idle gaps and hot-kernel share over the timed window = the
last K x ms_per_step of the trace (ms_per_step from the bench line printed by that run).

    python tools/timeline_summary.py <kernel_trace.csv> <bench_line.json>
"""
import argparse
import csv
import json

HOT = ("sym_bwd_kernel", "sym_bwd_pk_kernel", "rowred_pk_kernel", "lse_finalize", "OpOdeSelf", "lse_rowred", "OpGmm", "sym_merge", "merge_slabs",
       "sym_kernel", "OpOdeExt", "rowred_kernel")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench_line")
    a = ap.parse_args()
    bl = json.load(open(a.bench_line))
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(a.trace))), key=lambda t: t[0])
    hot_rows = [r for r in rows if any(h in r[2] for h in HOT)]
    t_end = max(e for _, e, _ in hot_rows)
    t0 = t_end - int(bl["steps"] * bl["ms_per_step"] * 1e6)
    win = [r for r in rows if r[0] >= t0 and r[1] <= t_end]
    t1 = max(e for _, e, _ in win)
    busy, hot, gaps, last = 0, 0, 0, t0
    for s, e, n in win:
        if s > last:
            gaps += s - last
        busy += max(0, e - max(s, last))
        last = max(last, e)
        if any(h in n for h in HOT):
            hot += e - s
    out = {"window": f"last {bl['steps']} x {bl['ms_per_step']} ms (the timed PSR iterations) of "
                     f"`bench.py --steps {bl['steps']} --warmup {bl['warmup']}` under rocprofv3 --kernel-trace",
           "span_ms": round((t1 - t0) / 1e6, 1), "device_busy_ms": round(busy / 1e6, 1),
           "hot_kernels_ms": round(hot / 1e6, 1), "other_kernels_ms": round((busy - hot) / 1e6, 1),
           "idle_gaps_ms": round(gaps / 1e6, 1), "kernels": len(win)}
    # where the idle time is: gap histogram and the kernel boundaries of the largest gaps
    gl, last, prev = [], t0, "(window start)"
    for s, e, n in win:
        if s > last:
            gl.append((s - last, prev, n))
        if e > last:
            last, prev = e, n
    short = lambda n: n.split("(")[0][-60:]
    edges = [(0, 10e3), (10e3, 50e3), (50e3, 200e3), (200e3, 1e6), (1e6, 1e12)]
    out["gap_histogram_ns"] = {f"{int(a)}-{int(b) if b < 1e12 else 'inf'}": {
        "count": sum(1 for g, _, _ in gl if a <= g < b),
        "ms": round(sum(g for g, _, _ in gl if a <= g < b) / 1e6, 2)} for a, b in edges}
    ctx = {}
    for g, p, n in gl:
        if g >= 50e3:
            k = f"{short(p)} -> {short(n)}"
            c = ctx.setdefault(k, [0, 0.0])
            c[0] += 1
            c[1] += g / 1e6
    out["gaps_over_50us_by_boundary"] = {k: {"count": v[0], "ms": round(v[1], 2)}
                                         for k, v in sorted(ctx.items(), key=lambda kv: -kv[1][1])[:15]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
