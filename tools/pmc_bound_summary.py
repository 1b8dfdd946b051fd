#!/usr/bin/env python3
"""What bounds each kernel, from the five rocprofv3 --pmc passes of tools/gpu_pmc_bound.sh.

Per kernel (averages per dispatch; SQ_*CYCLES counters count quad-cycles, MI355X_MICROARCH.md
"s_memtime tick vs SQ PMC units"; clk = GRBM_GUI_ACTIVE / 8 XCDs):
* occupancy: mean resident waves per CU = 4 SQ_WAVE_CYCLES / (clk x 256 CUs);
* wave-time split (fractions of SQ_WAVE_CYCLES, disjoint): wait (s_waitcnt / barrier parked:
  SQ_WAIT_ANY), issue stall (SQ_WAIT_INST_ANY), active (SQ_ACTIVE_INST_ANY); of it VALU
  (SQ_ACTIVE_INST_VALU), LDS (SQ_ACTIVE_INST_LDS), VMEM (SQ_ACTIVE_INST_VMEM);
* mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (duration x 2.4 GHz x 1024 SIMDs);
* LDS bank-conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / all);
* write path: TCP stall fractions (TCR->TCP stall, write tag conflict, pending) per TCP-cycle,
  mean L1->L2 write / read latency (TCP_TCC_*_REQ_LATENCY / TCP_TCC_*_REQ, cycles);
* fabric: L2 -> memory-side requests (TCC_EA0_RDREQ / WRREQ, 64 B nominal), their mean
  latency in cycles (TCC_EA0_*REQ_LEVEL / *REQ: outstanding-request level accumulated per
  cycle over requests), the share destined for DRAM (TCC_EA0_RDREQ_DRAM / RDREQ) and the EA
  write-stall cycles (TCC_EA0_WRREQ_STALL).  The memory-side Infinity Cache has no counter of
  its own on gfx950: the EA read latency is the separating signal — ~545 cycles an
  Infinity-Cache hit, ~900 an HBM miss on an idle chip (MI355X_MICROARCH.md cycle constants),
  both higher under load; k_gather's random replay rows (a 3 GB ring) are the in-run HBM-miss
  control.

usage: pmc_bound_summary.py <pass dir> <out.json> [bench args]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import counters, csrc_digest  # noqa: E402

CLK = 2.4e9


def per(p, k, c):
    v = p.get(k, {})
    for name in (c, c + "_sum"):
        if name in v and v[name][1]:
            return v[name][0] / v[name][1]
    return None


def ratio(a, b):
    return a / b if a is not None and b else None


def main(root, out, args=""):
    p = [counters(os.path.join(root, f"p{i}")) for i in range(1, 6)]
    kernels = sorted(set().union(*p))
    rows = {}
    for k in kernels:
        g = lambda i, c: per(p[i], k, c)
        dur = g(0, "duration_ns")
        if dur is None:
            continue
        clk = (g(0, "GRBM_GUI_ACTIVE") or 0) / 8
        wc = g(0, "SQ_WAVE_CYCLES")
        r = {"launches": p[0][k]["duration_ns"][1], "duration_us": dur / 1e3, "gui_cycles": clk,
             "waves": g(0, "SQ_WAVES"),
             "waves_per_cu": ratio(4 * wc if wc else None, clk * 256),
             "wait_frac": ratio(g(0, "SQ_WAIT_ANY"), wc),
             "issue_stall_frac": ratio(g(0, "SQ_WAIT_INST_ANY"), wc),
             "active_frac": ratio(g(0, "SQ_ACTIVE_INST_ANY"), wc),
             "valu_frac": ratio(g(0, "SQ_ACTIVE_INST_VALU"), wc),
             "lds_frac": ratio(g(2, "SQ_ACTIVE_INST_LDS"), wc),
             "mean_waves_level": ratio(g(2, "SQ_LEVEL_WAVES"), clk * 256),
             "vmem_frac": ratio(g(2, "SQ_ACTIVE_INST_VMEM"), wc),
             "vmem_wr_issue_frac": ratio(g(2, "SQ_INST_CYCLES_VMEM_WR"), wc),
             "mfma_busy": ratio(g(0, "SQ_VALU_MFMA_BUSY_CYCLES"), dur * 1e-9 * CLK * 1024),
             "lds_conflict_share": ratio(g(1, "SQ_LDS_BANK_CONFLICT"), g(1, "SQ_LDS_IDX_ACTIVE")),
             "lds_issue_stall_frac": ratio(g(1, "SQ_WAIT_INST_LDS"), wc),
             "insts": {c: g(1, c) for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS",
                                            "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")},
             "tcp_tcr_stall_frac": ratio(g(2, "TCP_TCR_TCP_STALL_CYCLES"), clk * 256),
             "tcp_write_tagconflict_frac": ratio(g(2, "TCP_WRITE_TAGCONFLICT_STALL_CYCLES"), clk * 256),
             "tcp_pending_stall_frac": ratio(g(2, "TCP_PENDING_STALL_CYCLES"), clk * 256),
             "l1_l2_write_latency": ratio(g(2, "TCP_TCC_WRITE_REQ_LATENCY"), g(3, "TCP_TCC_WRITE_REQ")),
             "l1_l2_read_latency": ratio(g(3, "TCP_TCC_READ_REQ_LATENCY"), g(3, "TCP_TCC_READ_REQ")),
             "ea_rd_bytes": (g(3, "TCC_EA0_RDREQ") or 0) * 64, "ea_wr_bytes": (g(3, "TCC_EA0_WRREQ") or 0) * 64,
             "ea_rd_latency": ratio(g(3, "TCC_EA0_RDREQ_LEVEL"), g(3, "TCC_EA0_RDREQ")),
             "ea_wr_latency": ratio(g(3, "TCC_EA0_WRREQ_LEVEL"), g(3, "TCC_EA0_WRREQ")),
             "ea_rd_dram_share": ratio(g(4, "TCC_EA0_RDREQ_DRAM"), g(3, "TCC_EA0_RDREQ")),
             "ea_wr_dram_share": ratio(g(4, "TCC_EA0_WRREQ_DRAM"), g(3, "TCC_EA0_WRREQ")),
             "ea_wr_stall_frac": ratio(g(4, "TCC_EA0_WRREQ_STALL"), clk * 16 * 8),
             "tcc_tag_stall_frac": ratio(g(4, "TCC_TAG_STALL"), clk * 16 * 8)}
        r["ea_rate_tbs"] = (r["ea_rd_bytes"] + r["ea_wr_bytes"]) / (dur * 1e-9) / 1e12
        rows[k] = r
    res = {"bench_args": args, "csrc_digest": csrc_digest(), "kernels": rows,
           "notes": __doc__.split("usage:")[0].strip()}
    json.dump(res, open(out, "w"), indent=1)
    top = sorted(rows, key=lambda k: -rows[k]["duration_us"] * rows[k]["launches"])[:16]
    f = lambda x, n=2: "-" if x is None else f"{x:.{n}f}"
    print(f"{'kernel':58s} {'us':>7s} {'w/CU':>5s} {'wait':>5s} {'istl':>5s} {'actv':>5s} {'valu':>5s} "
          f"{'mfma':>5s} {'ldsC':>5s} {'tcrS':>5s} {'wrTg':>5s} {'L1L2w':>6s} {'eaRdL':>6s} {'eaWrL':>6s} "
          f"{'dram':>5s} {'eaTB/s':>6s}")
    for k in top:
        r = rows[k]
        print(f"{k[:58]:58s} {r['duration_us']:7.1f} {f(r['waves_per_cu'], 1):>5s} {f(r['wait_frac']):>5s} "
              f"{f(r['issue_stall_frac']):>5s} {f(r['active_frac']):>5s} {f(r['valu_frac']):>5s} "
              f"{f(r['mfma_busy']):>5s} {f(r['lds_conflict_share']):>5s} {f(r['tcp_tcr_stall_frac']):>5s} "
              f"{f(r['tcp_write_tagconflict_frac']):>5s} {f(r['l1_l2_write_latency'], 0):>6s} "
              f"{f(r['ea_rd_latency'], 0):>6s} {f(r['ea_wr_latency'], 0):>6s} {f(r['ea_rd_dram_share']):>5s} "
              f"{r['ea_rate_tbs']:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
