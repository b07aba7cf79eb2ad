"""Per-kernel-family sums of rocprofv3 --pmc counters over one or more output directories.
usage: python scripts/pmc_kernels.py REGEX DIR [DIR ...]   (REGEX selects kernel names; the
family is the matched text).  Prints per family: dispatches, each counter's total, and the
derived ratios the codec / prefill analysis uses: MFMA util = MFMA busy / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8), wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES, LDS conflict share =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, HBM bytes = FETCH_SIZE x 2 (KB, gfx950) + WRITE_SIZE (KB)."""
import csv
import glob
import json
import os
import re
import sys

rx = re.compile(sys.argv[1])
per = {}
for d in sys.argv[2:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = rx.search(r.get("Kernel_Name", ""))
            if not m:
                continue
            fam = per.setdefault(m.group(0), {})
            disp = fam.setdefault((d, r.get("Dispatch_Id", r.get("Correlation_Id"))), {})
            disp[r["Counter_Name"]] = disp.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
out = {}
for fam, disps in per.items():
    tot = {}
    for v in disps.values():
        for k, x in v.items():
            tot[k] = tot.get(k, 0.0) + x
    res = dict(dispatches=len(disps), totals=tot)
    g = tot.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in tot:
        res["mfma_util"] = round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8), 4)
    if tot.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in tot:
                res[k.lower() + "_share"] = round(tot[k] / tot["SQ_WAVE_CYCLES"], 4)
    if tot.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in tot:
        res["lds_conflict_share"] = round(tot["SQ_LDS_BANK_CONFLICT"] / tot["SQ_LDS_IDX_ACTIVE"], 4)
    if "FETCH_SIZE" in tot:
        res["hbm_read_bytes_per_dispatch"] = tot["FETCH_SIZE"] * 2 * 1024 / len(disps)
    if "WRITE_SIZE" in tot:
        res["hbm_write_bytes_per_dispatch"] = tot["WRITE_SIZE"] * 1024 / len(disps)
    out[fam] = res
print(json.dumps(out, indent=1))
