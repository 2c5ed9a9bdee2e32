"""profiles/<tag>_counters.json (tools/rocpd_summary.py) -> profiles/traffic.json,
the per-launch HBM traffic and VALU busy figures bench.py reports for its
dominant kernel.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts half the
bytes of coalesced streaming reads (MI355X_MICROARCH.md, HBM / rocprofv3
section), so it is doubled; WRITE_SIZE is taken as is.  GRBM_GUI_ACTIVE is
summed over the 8 XCDs; VALU busy = SQ_ACTIVE_INST_VALU * 4 / 1024 SIMDs /
(GRBM_GUI_ACTIVE / 8).

    python tools/make_traffic.py profiles/r01_v6_counters.json k_score_sorted [cand/launch]

The raw SQ_ACTIVE_INST_VALU / GRBM_GUI_ACTIVE figures and the candidates per
launch are kept for bench.py's VALU-issue roofline (bench.valu_issue).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, kernel, cand=None):
    c = json.load(open(src))[kernel]
    fetch = 2.0 * c["FETCH_SIZE"] * 1024.0
    write = c.get("WRITE_SIZE", 0.0) * 1024.0  # not collected -> 0 (noted in "correction")
    out = {"kernel": kernel, "bytes_per_launch": fetch + write, "fetch_bytes": fetch,
           "write_bytes": write, "source": os.path.relpath(src, HERE),
           "correction": "FETCH_SIZE x2 (gfx950 half-count), KiB -> B"
                         + ("" if "WRITE_SIZE" in c else "; WRITE_SIZE not collected")}
    if "SQ_ACTIVE_INST_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        out["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4.0 / 1024.0 / (c["GRBM_GUI_ACTIVE"] / 8.0)
    if "SQ_INSTS_VALU" in c:
        out["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
    if "SQ_ACTIVE_INST_VALU" in c:
        out["active_inst_valu"] = c["SQ_ACTIVE_INST_VALU"]
    if "GRBM_GUI_ACTIVE" in c:
        out["grbm_gui_active"] = c["GRBM_GUI_ACTIVE"]
    if cand:
        out["candidates_per_launch"] = int(cand)
    json.dump(out, open(os.path.join(HERE, "profiles", "traffic.json"), "w"), indent=1)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:4])
