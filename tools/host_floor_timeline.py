"""Device timeline of the host-floor run (`tools/host_floor.py --sizes 2000`) under
`rocprofv3 --kernel-trace`: over the last `window_ms` of the trace (the timed PSR iterations),
device busy time, idle gaps, kernel count and the kernels by launch count -- how much of the
2k-point iteration is device work and how much the host's issue and decision latency.

    python tools/host_floor_timeline.py <kernel_trace.csv> <window_ms>
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("window_ms", type=float)
    a = ap.parse_args()
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(a.trace))), key=lambda t: t[0])
    t_end = max(e for _, e, _ in rows)
    t0 = t_end - int(a.window_ms * 1e6)
    win = [r for r in rows if r[0] >= t0]
    busy, gaps, last = 0, 0, t0
    hist = collections.Counter()
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in win:
        if s > last:
            g = s - last
            gaps += g
            hist["<10us" if g < 10_000 else "10-50us" if g < 50_000 else "50-200us" if g < 200_000 else ">200us"] += 1
        busy += max(0, e - max(s, last))
        last = max(last, e)
        k = n.split("(")[0][:90]
        per[k][0] += 1
        per[k][1] += e - s
    top = sorted(per.items(), key=lambda kv: -kv[1][0])[:25]
    print(json.dumps({"window_ms": a.window_ms, "device_busy_ms": round(busy / 1e6, 2),
                      "idle_gaps_ms": round(gaps / 1e6, 2), "kernels": len(win),
                      "gap_counts": dict(hist),
                      "by_count": [{"kernel": k, "n": c, "ms": round(t / 1e6, 3)} for k, (c, t) in top]},
                     indent=1))


if __name__ == "__main__":
    main()
