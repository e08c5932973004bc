"""Probe: does an H2D copy from page-locked memory return before the copy is
done? Host time of the enqueue against enqueue + sync, for 341 KB (one
GNLeNet staging row) and 2.4 MB (all seven), median µs.

    python scripts/probes/probe_h2d_enqueue.py
"""
import json
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    res = {}
    for nbytes in (341_440, 2_389_912, 24_000_000):
        src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        enq, tot = [], []
        for i in range(300):
            st.synchronize()
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            t1 = time.perf_counter()
            st.synchronize()
            t2 = time.perf_counter()
            if i >= 20:
                enq.append(t1 - t0)
                tot.append(t2 - t0)
        enq.sort()
        tot.sort()
        res[f"{nbytes}_enqueue_us"] = round(enq[len(enq) // 2] * 1e6, 1)
        res[f"{nbytes}_total_us"] = round(tot[len(tot) // 2] * 1e6, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
