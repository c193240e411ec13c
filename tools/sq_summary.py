"""Per-kernel SQ counter summary of tools/gpu_run.sh sq=<script>'s two rocprofv3 --pmc
passes (mean over each kernel's launches, counters summed over the pass'
rows of one dispatch), with the derived fractions used in DESIGN §3:

  mfma_busy_frac  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
  lds_bank_conflict_over_lds_active, wait_any_over_wave_cycles,
  valu_per_mfma   = SQ_INSTS_VALU / SQ_INSTS_MFMA

python tools/sq_summary.py <dir with sq_a/ and sq_b/> <out.json>
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        yield from csv.DictReader(open(f))


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0]


def main():
    base, out = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ("sq_a", "sq_b"):
        disp = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in rows(os.path.join(base, sub)):
            if "k_" not in r["Kernel_Name"]:
                continue
            key = (sub, r["Dispatch_Id"])
            names[key] = short(r["Kernel_Name"])
            disp[key][r["Counter_Name"]] += float(r["Counter_Value"])
        for key, cs in disp.items():
            for c, v in cs.items():
                per[names[key]][c].append(v)
    res = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        g = m.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            m["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_bank_conflict_over_lds_active"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("SQ_WAVE_CYCLES"):
            m["wait_any_over_wave_cycles"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        if m.get("SQ_INSTS_MFMA"):
            m["valu_per_mfma"] = m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"]
        res[k] = m
    json.dump(dict(source="tools/gpu_run.sh sq= (rocprofv3 --pmc, two passes) over "
                          "tools/ab_teacher_conv.py --K 500; tools/sq_summary.py",
                   kernels=res), open(out, "w"), indent=1)
    for k, m in res.items():
        print(k, {a: round(b, 3) for a, b in m.items() if "frac" in a or "over" in a or "per" in a})


if __name__ == "__main__":
    main()
