"""Aggregate kernel-timeline statistics of a slab rehearsal from a rocprofv3 --kernel-trace CSV: over
the last N sweeps (between context-stream shiftCells launches), per hardware queue the kernels, their
busy time and mean duration, and the fraction of the sweep in which no kernel runs at all or only
the exchange queue's kernels run.

  python tools/timeline_stats.py <kernel_trace.csv> [sweeps=10] > profiles/<tag>_timeline.txt
"""
import collections
import csv
import re
import sys


def main() -> int:
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    main_q = min(int(r["Queue_Id"]) for r in rows if "k_shift" in r["Kernel_Name"])
    shifts = [r for r in rows if "k_shift" in r["Kernel_Name"] and int(r["Queue_Id"]) == main_q]
    a, b = int(shifts[-n - 1]["End_Timestamp"]), int(shifts[-1]["End_Timestamp"])
    span = b - a
    per_q = collections.defaultdict(lambda: collections.defaultdict(list))
    iv = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e <= a or s >= b:
            continue
        s, e = max(s, a), min(e, b)
        m = re.search(r"(k_\w+|ncclKernel\w*|\w*[Cc]opy\w*|rccl\w*)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        q = int(r["Queue_Id"])
        per_q[q][name].append(e - s)
        iv.append((s, e, q))
    print(f"{n} sweeps, {span / n / 1e3:.1f} us per sweep (between context-stream shiftCells ends)")
    for q in sorted(per_q):
        busy = sum(sum(v) for v in per_q[q].values())
        print(f"queue {q}: busy {100 * busy / span:5.1f}% of the span")
        for name, v in sorted(per_q[q].items(), key=lambda kv: -sum(kv[1])):
            print(f"    {name:28s} {len(v) / n:6.1f} per sweep, mean {sum(v) / len(v) / 1e3:7.2f} us, "
                  f"{sum(v) / n / 1e3:7.1f} us per sweep")
    # coverage: time with no kernel running, and time with kernels only on the exchange queue
    ev = []
    for s, e, q in iv:
        ev.append((s, 1, q))
        ev.append((e, -1, q))
    ev.sort()
    active = collections.Counter()
    last = a
    idle = only_x = 0
    xq = max(per_q, key=lambda q: sum(len(v) for k, v in per_q[q].items() if "copy" in k.lower() or "spin" in k))
    for t, d, q in ev:
        dt = t - last
        if dt > 0:
            tot = sum(active.values())
            if tot == 0:
                idle += dt
            elif tot == active[xq]:
                only_x += dt
        active[q] += d
        last = t
    print(f"no kernel running: {100 * idle / span:5.1f}% ({idle / n / 1e3:.1f} us per sweep); "
          f"only queue {xq} (the exchange queue) running: {100 * only_x / span:5.1f}% ({only_x / n / 1e3:.1f} us per sweep)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
