"""Summarise the SQ counter passes of k_hm_compress (scripts/gpu_hm_pmc.sh: gpurun_out/hpmc_{a,b,c})
into profiles/hm_pmc_<tag>.json: per-CTU instruction mix, the wave-cycle split (issuing / waiting
on dependencies and memory / waiting for an issue slot) and the chip-level issue fractions that
bench.py's roofline reports beside the HBM fraction.

Units (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units"): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles summed over waves; SQ_INSTS_* count wave instructions.
usage: python scripts/hm_pmc_summary.py TAG [clock_ghz]"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 256 * 4


def load(p):
    rows = list(csv.DictReader(open(os.path.join(ROOT, "gpurun_out", f"hpmc_{p}", f"{p}_counter_collection.csv"))))
    d = collections.defaultdict(float)
    dur, grid = None, None
    for r in rows:
        if "k_hm_compress" in r["Kernel_Name"]:
            d[r["Counter_Name"]] += float(r["Counter_Value"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            grid = int(r["Grid_Size"])
    return d, dur, grid


def main():
    tag = sys.argv[1]
    clock = float(sys.argv[2]) if len(sys.argv) > 2 else 2.2  # GHz under load (in-kernel s_memtime clock)
    a, dur_a, grid = load("a")
    b, dur_b, _ = load("b")
    c, _, _ = load("c")
    waves = grid // 64  # one wave per chain, one CTU per chain per launch
    dur = dur_b
    per = lambda v: v / waves
    wave_cyc = b["SQ_WAVE_CYCLES"]
    out = {
        "kernel": "k_hm_compress", "waves": waves, "ctus_per_launch": waves, "launch_s": round(dur, 4),
        "clock_ghz_assumed": clock,
        "per_ctu_wave_instructions": {k.replace("SQ_INSTS_", "").lower(): round(per(v)) for k, v in sorted(a.items())
                                      if k.startswith("SQ_INSTS_")},
        "per_ctu_flat_instructions": round(per(c.get("SQ_INSTS_FLAT", 0))),
        "wave_cycle_split": {
            "issuing": round(b["SQ_ACTIVE_INST_ANY"] / wave_cyc, 4),
            "valu": round(b["SQ_ACTIVE_INST_VALU"] / wave_cyc, 4),
            "salu": round(b["SQ_ACTIVE_INST_SCA"] / wave_cyc, 4),
            "lds": round(b["SQ_ACTIVE_INST_LDS"] / wave_cyc, 4),
            "waiting_dependency_or_memory": round(b["SQ_WAIT_ANY"] / wave_cyc, 4),
            "waiting_issue_slot": round(b["SQ_WAIT_INST_ANY"] / wave_cyc, 4),
        },
        # chip-level: issue cycles of all waves / (SIMDs x cycles of the launch)
        "simd_issue_frac": round(4 * b["SQ_ACTIVE_INST_ANY"] / (SIMDS * clock * 1e9 * dur), 4),
        "valu_frac": round(4 * a["SQ_INSTS_VALU"] / (SIMDS * clock * 1e9 * dur), 4),
        "lds_bank_conflict_per_ctu": round(per(c.get("SQ_LDS_BANK_CONFLICT", 0))),
        "raw": {**{k: v for k, v in a.items()}, **{k: v for k, v in b.items()}, **{k: v for k, v in c.items()}},
    }
    path = os.path.join(ROOT, "profiles", f"hm_pmc_{tag}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "raw"}, indent=1))


if __name__ == "__main__":
    main()
