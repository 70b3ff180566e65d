"""Generate tests/golden/known_answers.json: statistical known answers <E> of the reference's model
from the independent textbook Metropolis code tools/textbook_mc.c (no cells, full minimum image,
truncated LJ subsweep.h:90-103, accept rule subsweep.h:209-216).

  python tools/make_known_answers.py [--jobs 8]

Two models, both beta = 0.3, sigma = 0.5, rc = w = 2.5, L = 10 (4^3 cells of the oracle):
  n64   N = 64   (SURVEY.md section 4's -21.240 +- 0.022, tightened);
  n305  N = 305  (density 0.305, 4.77 particles per cell: the density of BASELINE configs 3-5).
Each model: several independent seeds, each equilibrated and then averaged over batch means; the
known answer pools every seed's block means (mean, standard error of the pooled blocks).  Seeds
are fixed, so the file is reproducible bit for bit on the same compiler.  Test infrastructure only.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "textbook_mc.c")
OUT = os.path.join(REPO, "tests", "golden", "known_answers.json")

MODELS = {
    "n64": dict(N=64, L=10.0, beta=0.3, sigma=0.5, rc=2.5, equil=2000, sweeps=200000, blocks=20,
                seeds=[101, 102, 103, 104, 105, 106, 107, 108]),
    "n305": dict(N=305, L=10.0, beta=0.3, sigma=0.5, rc=2.5, equil=2000, sweeps=40000, blocks=20,
                 seeds=[201, 202, 203, 204, 205, 206, 207, 208]),
}


def build(tmp: str) -> str:
    exe = os.path.join(tmp, "textbook_mc")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-o", exe, SRC, "-lm"], check=True)
    return exe


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--models", nargs="*", default=list(MODELS))
    args = ap.parse_args()
    out = {"generator": "tools/make_known_answers.py", "tool": "tools/textbook_mc.c",
           "tool_sha256": hashlib.sha256(open(SRC, "rb").read()).hexdigest(),
           "compiler": subprocess.run(["gcc", "--version"], capture_output=True, text=True).stdout.splitlines()[0],
           "models": {}}
    if os.path.exists(OUT):
        out["models"] = json.load(open(OUT)).get("models", {})
    with tempfile.TemporaryDirectory() as tmp:
        exe = build(tmp)
        for name in args.models:
            m = MODELS[name]
            cmds = [[exe, str(m["N"]), repr(m["L"]), repr(m["beta"]), repr(m["sigma"]), repr(m["rc"]),
                     str(m["equil"]), str(m["sweeps"]), str(m["blocks"]), str(s)] for s in m["seeds"]]
            runs = []
            for k in range(0, len(cmds), args.jobs):
                procs = [subprocess.Popen(c, stdout=subprocess.PIPE, text=True) for c in cmds[k:k + args.jobs]]
                for p in procs:
                    o, _ = p.communicate()
                    if p.returncode:
                        raise SystemExit(f"textbook_mc failed: {p.returncode}")
                    runs.append(json.loads(o))
            blocks = np.concatenate([np.array(r["block_means"]) for r in runs])
            mean = float(blocks.mean())
            se = float(blocks.std(ddof=1) / np.sqrt(len(blocks)))
            out["models"][name] = {
                "N": m["N"], "L": m["L"], "beta": m["beta"], "sigma": m["sigma"], "rc": m["rc"],
                "cells_per_side_of_the_oracle": int(round(m["L"] / m["rc"])),
                "particles_per_cell": m["N"] / (m["L"] / m["rc"]) ** 3,
                "mean": mean, "se": se, "se_rel": abs(se / mean),
                "acceptance": float(np.mean([r["acceptance"] for r in runs])),
                "sweeps_per_seed": m["sweeps"], "equil_sweeps": m["equil"], "blocks_per_seed": m["blocks"],
                "seeds": m["seeds"], "per_seed": [{"seed": r["seed"], "mean": r["mean"], "se": r["se"]} for r in runs],
                "command": "textbook_mc N L beta sigma rc equil_sweeps sweeps blocks seed",
            }
            print(f"{name}: <E> = {mean:.5f} +- {se:.5f} ({100 * abs(se / mean):.3f}%), "
                  f"acceptance {out['models'][name]['acceptance']:.4f}", flush=True)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
