"""The round's measurement table for DESIGN.md §6, from the round's profiles:
profiles/<TAG>_bench_<cfg>.json (bench.py lines, tools/gpu_benchall.sh) and profiles/<TAG>_<cfg>_pmc.json
(tools/round_profiles.sh + summarize_profile.py).

    python tools/round_table.py r05z [PMC_TAG ...]
(a config without a PMC profile under TAG takes the first of the PMC_TAGs that has one, marked with *)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
ROWS = [("c1", "C1 sphere 256² 1 spp"), ("c2", "**C2 Cornell-5 1080p 64 spp**"), ("c3", "C3 Mandelbulb 1080p 128 spp"),
        ("c4", "C4 256-prim union 4K 256 spp"), ("c5", "C5 animated Cornell-5 1080p 512 spp"),
        ("rm3", "RM3 as wired 1080p 4 spp 16 bounces"), ("rm2", "RM2 simple.scene 1080p 4 spp 16 bounces")]


def load(name):
    p = os.path.join(P, name)
    return json.load(open(p)) if os.path.exists(p) else None


def main(tag, fallbacks=()):
    print("| config | Msamples/s | ms per step | kernel ms per launch: bench / rocprof | roofline frac (executed flops) "
          "| HBM per launch (PMC) | VALU lane util | wait on memory | CPU leg: Msamples/s (threads), per core | PSNR vs reference |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for cfg, name in ROWS:
        b = load("%s_bench_%s.json" % (tag, cfg))
        m = load("%s_%s_pmc.json" % (tag, cfg))
        star = ""
        for fb in fallbacks:
            if m is not None:
                break
            m, star = load("%s_%s_pmc.json" % (fb, cfg)), "*"
        if b is None:
            continue
        r, c, ps = b["roofline"], b.get("cpu_baseline") or {}, b.get("psnr_vs_reference") or {}
        d = (m or {}).get("derived", {})
        rp = ("%.3f" % ((m or {}).get("k_trace_avg_ns", 0) / 1e6) + star) if m else "—"
        hbm = d.get("hbm_bytes")
        hbm_s = ("%.2f GB" % (hbm / 1e9)) if hbm and hbm >= 1e8 else (("%.1f MB" % (hbm / 1e6)) if hbm else "—")
        cpu = ("%.3g (%d), %.3g" % (c["value"], c["cores"], c.get("per_core", c["value"] / c["cores"]))) if c else "—"
        print("| %s | %.0f | %.3f | %.3f / %s | %.4f | %s | %s | %s | %s | %s |" % (
            name, b["value"], b["ms_per_step"], r.get("avg_launch_ms", 0.0), rp, r["frac"], hbm_s,
            ("%.2f" % d["valu_lane_util"]) if "valu_lane_util" in d else "—",
            ("%.2f" % d["frac_wait_any"]) if "frac_wait_any" in d else "—", cpu,
            ("%.1f dB" % ps["psnr_db"]) if "psnr_db" in ps else "—"))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r05z", sys.argv[2:])
