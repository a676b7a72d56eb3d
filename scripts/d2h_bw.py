#!/usr/bin/env python3
"""Device -> pinned host copy rate on this box (the drop-in download's ceiling): one
copy of S bytes on one stream, and the same bytes split over 2 / 4 streams (one copy
engine each, if the runtime assigns them).  Prints one JSON line."""
import json
import time

import torch


def rate(nbytes: int, nstreams: int, reps: int = 10) -> float:
    n = nbytes // 8
    dev = torch.empty(n, dtype=torch.float64, device="cuda")
    dev.fill_(1.0)
    host = torch.empty(n, dtype=torch.float64, pin_memory=True)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    parts = [(i * n // nstreams, (i + 1) * n // nstreams) for i in range(nstreams)]
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for st, (a, b) in zip(streams, parts):
            with torch.cuda.stream(st):
                host[a:b].copy_(dev[a:b], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return nbytes / best / 1e9


def main():
    out = {}
    for mb in (6, 49, 98):
        for ns in (1, 2, 4):
            out[f"{mb}MB_{ns}streams_GBps"] = round(rate(mb << 20, ns), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
