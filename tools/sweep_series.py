"""Per-sweep GPU time over a run (torch events between sweeps on the context stream): does a
short timed region start below the steady rate?  python tools/sweep_series.py [--prewarm-ms 300]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--prewarm-ms", type=float, default=300.0)
    ap.add_argument("--sweeps", type=int, default=60)
    ap.add_argument("--gap-ms", type=float, default=500.0, help="idle host gap before the series")
    args = ap.parse_args()
    import torch
    import pmc_amd
    from pmc_amd.plan import sweep_plan
    stream = torch.cuda.Stream()
    sim = pmc_amd.PmcContext(128, stream=stream.cuda_stream)
    sim.init_lattice(10_000_000)
    for s in range(5):
        for c in sweep_plan(1234, s, 2.5)[0]:
            sim.phase(c, s)
        sim.shift(s)
    sim.synchronize()
    time.sleep(args.gap_ms / 1e3)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.prewarm_ms:
        sim.energy()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.sweeps + 1)]
    plans = [sweep_plan(1234, 5 + k, 2.5)[0] for k in range(args.sweeps)]
    ev[0].record(stream)
    for k in range(args.sweeps):
        for c in plans[k]:
            sim.phase(c, 5 + k)
        sim.shift(5 + k)
        ev[k + 1].record(stream)
    sim.synchronize()
    ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(args.sweeps)]
    print(json.dumps({"prewarm_ms": args.prewarm_ms, "gap_ms": args.gap_ms,
                      "sweep_ms": [round(m, 4) for m in ms]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
