"""Per-launch averages of PMC counters for one kernel from a rocprofv3 --pmc output directory (any
path), as one JSON line: the counters of summarize_profile.counters without its gpurun_out layout.

    python tools/pmc_quick.py DIR [KERNEL_SUBSTRING] [LABEL]"""
import collections
import csv
import glob
import json
import sys


def main(d, match="rmr_jit_trace", label=""):
    p = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(p)) if match in r["Kernel_Name"]]
    big = max(int(r["Grid_Size"]) for r in rows)
    agg = collections.defaultdict(list)
    for r in rows:
        if int(r["Grid_Size"]) == big:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: sum(v) / len(v) for k, v in agg.items()}
    out["launches"] = max(len(v) for v in agg.values())
    if "SQ_LDS_BANK_CONFLICT" in out and "SQ_INSTS_LDS" in out:
        out["bank_conflict_cycles_per_lds_inst"] = out["SQ_LDS_BANK_CONFLICT"] / max(1.0, out["SQ_INSTS_LDS"])
    print(json.dumps({"label": label, "dir": d, "kernel": match, "per_launch": out}))


if __name__ == "__main__":
    main(*sys.argv[1:])
