"""Summarise tools/pmc_attr.sh TAG: where the trace kernel's waves wait, per launch.

    python tools/pmc_attr.py TAG [OUT.json]

SQ counters count quad-cycles (MI355X_MICROARCH.md, s_memtime row), per wave summed over waves; the
LEVEL counters accumulate the number of in-flight instructions of a kind every (quad-)cycle, so
LEVEL / INSTS is the kind's average latency and LEVEL / WAVE_CYCLES its average number in flight per
wave. SQ_WAIT_ANY is a wave parked on s_waitcnt: vmcnt covers the vector memory loads and stores
(grid cells, candidate lists, sample-plane stores, global primitive table), lgkmcnt the scalar
loads (scene tables) and LDS (chunk rays, primitive table copy, cold-state stash, cert table)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from summarize_profile import counters  # noqa: E402


def main(tag, out=None):
    c, meta = {}, {}
    for i in range(1, 7):
        try:
            v, m = counters("%s_a%d" % (tag, i), "rmr_jit_trace")
        except (FileNotFoundError, ValueError):
            continue
        c.update({k.replace("_sum", ""): x for k, x in v.items()})
        meta = m or meta
    W = c["SQ_WAVE_CYCLES"]
    d = {
        "wave_split": {"wait_any (s_waitcnt)": c["SQ_WAIT_ANY"] / W, "wait_inst_any (issue stall)": c["SQ_WAIT_INST_ANY"] / W,
                       "active_inst_any": c["SQ_ACTIVE_INST_ANY"] / W},
        "instructions_per_launch": {k: c.get(k) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                                                           "SQ_INSTS_VMEM_WR", "SQ_INSTS_FLAT")},
        "avg_latency_quadcycles": {k: (c["SQ_INST_LEVEL_" + k] / max(1.0, c[n]) if "SQ_INST_LEVEL_" + k in c and n in c else None)
                                   for k, n in (("VMEM", "SQ_INSTS_VMEM"), ("SMEM", "SQ_INSTS_SMEM"), ("LDS", "SQ_INSTS_LDS"))},
        "in_flight_per_wave": {k: c.get("SQ_INST_LEVEL_" + k, 0.0) / W for k in ("VMEM", "SMEM", "LDS")},
        "lds": {"wait_inst_lds / wave": c.get("SQ_WAIT_INST_LDS", 0.0) / W, "bank_conflict_cycles": c.get("SQ_LDS_BANK_CONFLICT"),
                "active_inst_lds / wave": c.get("SQ_ACTIVE_INST_LDS", 0.0) / W},
        "issue_cycles_per_wave": {k: c.get(k, 0.0) / W for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM",
                                                                    "SQ_ACTIVE_INST_MISC", "SQ_INST_CYCLES_SMEM",
                                                                    "SQ_INST_CYCLES_VMEM_RD", "SQ_INST_CYCLES_VMEM_WR")},
    }
    if "TCC_HIT" in c:
        d["l2"] = {"hit_rate": c["TCC_HIT"] / max(1.0, c["TCC_HIT"] + c["TCC_MISS"]), "hits": c["TCC_HIT"], "misses": c["TCC_MISS"],
                   "ea_rdreq": c.get("TCC_EA0_RDREQ"), "ea_rdreq_dram": c.get("TCC_EA0_RDREQ_DRAM")}
    if "TCP_TOTAL_CACHE_ACCESSES" in c:
        d["l1"] = {"accesses": c["TCP_TOTAL_CACHE_ACCESSES"], "tcc_read_req": c["TCP_TCC_READ_REQ"],
                   "tcc_write_req": c["TCP_TCC_WRITE_REQ"],
                   "read_req_per_access": c["TCP_TCC_READ_REQ"] / max(1.0, c["TCP_TOTAL_CACHE_ACCESSES"]),
                   "pending_stall_cycles": c.get("TCP_PENDING_STALL_CYCLES"), "td_tc_stall": c.get("TD_TC_STALL"),
                   "td_busy": c.get("TD_TD_BUSY"), "ta_addr_stalled_by_tc": c.get("TA_ADDR_STALLED_BY_TC_CYCLES"),
                   "ta_data_stalled_by_tc": c.get("TA_DATA_STALLED_BY_TC_CYCLES")}
    if "TCC_EA0_WRREQ" in c:
        d["writes"] = {"ea_wrreq": c["TCC_EA0_WRREQ"], "ea_wrreq_64b": c.get("TCC_EA0_WRREQ_64B"),
                       "tcc_writeback": c.get("TCC_WRITEBACK"), "tcc_normal_evict": c.get("TCC_NORMAL_EVICT"),
                       "bytes_upper (64B x wrreq)": 64.0 * c["TCC_EA0_WRREQ"]}
    res = {"tag": tag, "kernel": meta, "counters_per_launch": c, "derived": d}
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
