"""VALU-issue roof of the dominant kernel from a rocprofv3 SQ counter summary (tools/sq_summary.py
output, `<COUNTER> mean per dispatch <value>` lines) -> profiles/pmc_valu.json, which bench.py
attaches to its roofline as `roofline.valu`.

  python tools/valu_roof.py profiles/r04x_sq_counters.txt [--tag r04x] [--out profiles/pmc_valu.json]

Model: a SIMD issues at most one VALU instruction at a time; a wave64 instruction occupies it for
the measured cycles of its class (tools/ubench/alu_rates.hip, 8 waves/SIMD):
full rate 2.5 (f32 add/mul/fma, moves, integer adds, logic), half rate 4.5 (compares, selects,
shifts, mbcnt, integer multiplies, conversions, f64, DPP), quarter rate 8.2 (transcendentals).
The SQ counters split f32 add/mul/fma, f64, conversions and transcendentals out; INT32/INT64 and
the unclassified rest (moves, logic, compares, DPP) mix both rates, so the issue cycles are given
as a range: those at full rate (low) and at half rate (high).  The launch's cycles per SIMD are
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs' GUI-active cycles; MI355X_MICROARCH.md 'DVFS
give-back').  frac = issue cycles per SIMD / launch cycles.
"""
import argparse
import json
import re
import sys

SIMDS = 256 * 4
FULL, HALF, QUARTER = 2.5, 4.5, 8.2


def read_counters(path: str) -> dict:
    c = {}
    for line in open(path):
        m = re.match(r"(\w+)\s+mean per dispatch\s+([0-9.eE+]+)", line)
        if m:
            c[m.group(1)] = float(m.group(2))
    return c


def valu_roof(c: dict) -> dict:
    v = c["SQ_INSTS_VALU"]
    f32 = c.get("SQ_INSTS_VALU_ADD_F32", 0) + c.get("SQ_INSTS_VALU_MUL_F32", 0) + c.get("SQ_INSTS_VALU_FMA_F32", 0)
    half_known = (c.get("SQ_INSTS_VALU_ADD_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) +
                  c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_CVT", 0))
    trans = c.get("SQ_INSTS_VALU_TRANS_F32", 0)
    mixed = v - f32 - half_known - trans            # INT32/INT64 + unclassified: full or half rate
    low = (f32 * FULL + half_known * HALF + trans * QUARTER + mixed * FULL) / SIMDS
    high = (f32 * FULL + half_known * HALF + trans * QUARTER + mixed * HALF) / SIMDS
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    return {"bound": "valu-issue", "valu_instructions_per_launch": v, "valu_instructions_per_simd": v / SIMDS,
            "salu_instructions_per_launch": c.get("SQ_INSTS_SALU"), "lds_instructions_per_launch": c.get("SQ_INSTS_LDS"),
            "mix": {"f32_full_rate": f32, "f64_cvt_half_rate": half_known, "trans_quarter_rate": trans,
                    "int_and_unclassified": mixed},
            "cycles_per_instruction": {"full": FULL, "half": HALF, "quarter": QUARTER},
            "issue_cycles_per_simd": [low, high], "launch_cycles_per_simd": cyc,
            "frac": [low / cyc, high / cyc]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("counters")
    ap.add_argument("--tag", default="")
    ap.add_argument("--out", default="profiles/pmc_valu.json")
    a = ap.parse_args()
    r = valu_roof(read_counters(a.counters))
    r["source"] = f"{a.counters} (rocprofv3 SQ counters, tools/valu_roof.py)"
    r["tag"] = a.tag
    with open(a.out, "w") as f:
        json.dump(r, f, indent=1)
        f.write("\n")
    print(json.dumps({k: r[k] for k in ("valu_instructions_per_simd", "issue_cycles_per_simd",
                                        "launch_cycles_per_simd", "frac")}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
