"""Summarise A/B bench lines (tools/archive/r04_strong_ab.sh, r04_variants_ab.sh, r04_env_ab.sh outputs:
<variant>[_d<delay>_R<ranks>]_<rep>.json) as one table row per file, grouped by variant.

  python tools/ab_summary.py gpurun_out/r04c_ab [...] > profiles/r04_strong_variants.txt
"""
import collections
import json
import os
import re
import sys


def main() -> int:
    for d in sys.argv[1:]:
        rows = collections.defaultdict(list)
        for f in sorted(os.listdir(d)):
            if not f.endswith(".json"):
                continue
            m = re.match(r"(.+?)(?:_d(\d+)_R(\d+))?_(\d+)\.json$", f)
            if not m:
                continue
            try:
                line = open(os.path.join(d, f)).read().strip().splitlines()[-1]
                r = json.loads(line)
            except (ValueError, IndexError):
                continue
            key = (m.group(1), m.group(2) or "-", m.group(3) or "-")
            rows[key].append((int(m.group(4)), r["ms_per_step"], r["roofline"].get("launch_ms"),
                              r["roofline"].get("shift_ms"), r.get("error_flags")))
        print(f"== {d}")
        print(f"{'variant':<12} {'delay_us':>8} {'ranks':>5}  ms per sweep (rep: value) ... | flags")
        for (v, dl, rk), vals in sorted(rows.items()):
            vals.sort()
            cells = "  ".join(f"{rep}: {ms:.4f}" for rep, ms, *_ in vals)
            flags = sorted({fl for *_, fl in vals})
            print(f"{v:<12} {dl:>8} {rk:>5}  {cells} | {flags}")
        print()
    return 0


if __name__ == "__main__":
    sys.exit(main())
