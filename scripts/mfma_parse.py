"""MFMA-pipe utilisation per kernel family from rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES +
GRBM_GUI_ACTIVE passes: util = sum(MFMA busy cycles) / (SIMDs x sum(GRBM_GUI_ACTIVE / 8)),
SIMDs = 256 CUs x 4.  (SQ_VALU_MFMA_BUSY_CYCLES counts cycles; GRBM_GUI_ACTIVE is summed
over the 8 XCDs, MI355X_MICROARCH.md.)"""
import csv
import glob
import json
import os
import re
import sys

SIMDS = 256 * 4
res = {}
for d in sys.argv[1:]:
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            m = re.search(r"(gemm_bx3_kernel|gemm_f32_kernel|pgemm_kernel|wgemm_kernel|codec_attn_kernel)(<[^>(]*>)?", name)
            if not m:
                continue
            key = m.group(1) + (m.group(2) or "")
            disp = per.setdefault(key, {}).setdefault(r.get("Dispatch_Id", r.get("Correlation_Id")), {})
            disp[r["Counter_Name"]] = disp.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for key, disps in per.items():
        busy = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in disps.values())
        act = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in disps.values()) / 8.0
        if act > 0:
            res[key] = dict(dispatches=len(disps), mfma_busy_cycles=busy, active_cycles=act,
                            mfma_util=round(busy / (SIMDS * act), 4))
print(json.dumps(res, indent=1))
