"""Does a blocking device-to-host read release the GIL?  The main thread queues ~200 ms of
device work (large GEMMs), THEN starts a thread counting pure-Python loop iterations and
reads a scalar back (three ways).  If the read holds the GIL while it waits for the device,
the counter stalls for the wait.

    python tools/probes/gil_probe.py
"""
import json
import threading
import time

import torch


def main():
    dev = torch.device("cuda:0")
    a = torch.rand(8192, 8192, device=dev)
    torch.mm(a, a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        torch.mm(a, a)
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / 5
    n = max(1, int(0.2 / per))
    pinned = torch.empty(1, dtype=torch.float64, pin_memory=True)
    print(json.dumps({"gemm_ms": round(per * 1e3, 2), "n": n}), flush=True)

    def read_tolist(y):
        return y.sum().double().reshape(1).tolist()

    def read_item(y):
        return y.sum().item()

    def read_event(y):
        pinned.copy_(y.sum().double().reshape(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        ev.synchronize()
        return pinned.tolist()

    out = {}
    for name, rd in (("tolist", read_tolist), ("item", read_item), ("event_sync_pinned", read_event)):
        y = None
        for _ in range(n):
            y = torch.mm(a, a)
        stop = threading.Event()
        count = [0]

        def spin():
            c = 0
            while not stop.is_set():
                c += 1
            count[0] = c

        th = threading.Thread(target=spin)
        t1 = time.perf_counter()
        th.start()
        rd(y)
        t2 = time.perf_counter()
        stop.set()
        th.join()
        out[name] = {"read_wait_ms": round((t2 - t1) * 1e3, 1), "spin_iters_M": round(count[0] / 1e6, 3),
                     "spin_rate_M_per_s": round(count[0] / (t2 - t1) / 1e6, 2)}
        print(json.dumps({name: out[name]}), flush=True)
    stop = threading.Event()
    count = [0]

    def spin2():
        c = 0
        while not stop.is_set():
            c += 1
        count[0] = c

    th = threading.Thread(target=spin2)
    th.start()
    time.sleep(0.2)
    stop.set()
    th.join()
    out["idle_spin_rate_M_per_s"] = round(count[0] / 0.2 / 1e6, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
