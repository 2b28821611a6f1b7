"""Summarise a tools/profile_round.sh run (gpurun_out/{prof,pmcf,pmcw,pmcs,pmcv}_<tag>) into profiles/.

    python tools/summarize_profile.py r01 [CONFIG]     (CONFIG: bench.py --config, default c2)

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats of the bench command, verbatim),
profiles/<tag>_pmc.json (per-launch PMC values of the dominant kernel and derived ratios) and
profiles/traffic_<config>.json (HBM bytes per k_trace launch, read by bench.py for roofline.traffic).

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads, so it is
doubled. k_trace reads are scratch (spill) reloads + scene-table s_loads, not 16-B streaming loads, so
the doubled figure is an upper bound; WRITE_SIZE is exact for the 16-B sample-plane stores.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def counters(d, match):
    """Per-launch counter averages over the dominant kernel's production launches (its largest grid:
    a bench may also launch the kernel on a tile or two, e.g. C5's first live-primitive build)."""
    agg = collections.defaultdict(list)
    p = os.path.join(GO, d, "run_counter_collection.csv")
    meta = {}
    rows = [r for r in csv.DictReader(open(p)) if match in r["Kernel_Name"]]
    big = max(int(r["Grid_Size"]) for r in rows)
    for r in rows:
        if int(r["Grid_Size"]) == big:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                     "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
    return {k: sum(v) / len(v) for k, v in agg.items()}, meta


def main(tag, config="c2"):
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(GO, "prof_%s" % tag, "run_kernel_stats.csv"),
                os.path.join(PROF, "%s_kernel_stats.csv" % tag))
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(PROF, "%s_kernel_stats.csv" % tag)))}
    # the dominant kernel: the hipRTC-specialised trace kernel when the bench used it
    match = "rmr_jit_trace" if any("rmr_jit_trace" in n for n in stats) else "k_trace"
    trace = [r for n, r in stats.items() if match in n][0]
    out = {"tag": tag, "kernel_name": trace["Name"],
           "command": "python3 bench.py --config %s --no-cpu-baseline --no-psnr --no-count-pass "
                      "(tools/profile_round.sh)" % config,
           "k_trace_avg_ns": float(trace["AverageNs"]), "k_trace_calls": int(trace["Calls"])}
    # the production launches alone (largest grid), from the kernel trace of the same run
    kt = [r for r in csv.DictReader(open(os.path.join(GO, "prof_%s" % tag, "run_kernel_trace.csv")))
          if match in r["Kernel_Name"]]
    gs = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    big = max(gs(r) for r in kt)
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt if gs(r) == big]
    # the first production launch is the bench's warm-up step, which its own timing leaves out too
    warm = 1 if len(durs) > 1 else 0
    out["k_trace_avg_ns_all_launches"] = out["k_trace_avg_ns"]
    out["k_trace_avg_ns"] = sum(durs[warm:]) / len(durs[warm:])
    out["k_trace_calls"] = len(durs) - warm
    out["k_trace_note"] = ("production launches (grid %d) after the warm-up one; %d smaller launch(es) excluded"
                           % (big, len(kt) - len(durs)))
    c = {}
    meta = {}
    for d in ("pmcf", "pmcw", "pmcs", "pmcv"):
        v, m = counters("%s_%s" % (d, tag), match)
        c.update(v)
        meta = m or meta
    out["kernel"] = meta
    out["counters_per_launch"] = c
    fetch = c["FETCH_SIZE"] * 1024.0
    write = c["WRITE_SIZE"] * 1024.0
    hbm = 2.0 * fetch + write
    secs = out["k_trace_avg_ns"] * 1e-9
    simd_quads = c["SQ_WAVE_CYCLES"]
    out["derived"] = {
        "fetch_bytes_raw": fetch, "fetch_bytes_x2": 2 * fetch, "write_bytes": write, "hbm_bytes": hbm,
        "hbm_GBps": hbm / secs / 1e9,
        "valu_insts": c["SQ_INSTS_VALU"], "salu_insts": c["SQ_INSTS_SALU"], "smem_insts": c["SQ_INSTS_SMEM"],
        # per-wave time split (quad-cycles, disjoint buckets per the guide's SQ table)
        "frac_active_inst": c["SQ_ACTIVE_INST_ANY"] / simd_quads,
        "frac_wait_inst_any": c["SQ_WAIT_INST_ANY"] / simd_quads,
        "frac_wait_any": c["SQ_WAIT_ANY"] / simd_quads,
        # active lanes per VALU cycle / 64
        "valu_lane_util": c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]),
        # VALU issue: one wave64 VALU instruction per SIMD per 2 cycles; 1024 SIMDs; 2.4 GHz
        "valu_issue_util_at_2p4GHz": c["SQ_INSTS_VALU"] / (secs * 2.4e9 * 1024 / 2.0),
    }
    with open(os.path.join(PROF, "%s_pmc.json" % tag), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    with open(os.path.join(PROF, "traffic_%s.json" % config), "w") as f:
        json.dump({"tag": tag, "hbm_bytes_per_launch": round(hbm), "fetch_bytes_x2": round(2 * fetch),
                   "write_bytes": round(write),
                   "note": "FETCH_SIZE x2 + WRITE_SIZE (KiB->B) per k_trace launch; see %s_pmc.json" % tag},
                  f, indent=1)
    print(json.dumps(out["derived"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01", sys.argv[2] if len(sys.argv) > 2 else "c2")
