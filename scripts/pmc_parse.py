"""Parse the two rocprofv3 --pmc passes of scripts/pmc_traffic.sh: per-dispatch FETCH_SIZE /
WRITE_SIZE (KB) of the probed kernel's launches -> bytes per launch (FETCH doubled: gfx950
correction, MI355X_MICROARCH.md HBM section)."""
import csv
import glob
import json
import os
import re
import sys

out, kern, rows = sys.argv[1], sys.argv[2], int(sys.argv[3])
res = {"kernel": kern, "rows": rows}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob(os.path.join(out, f"{kern}_{rows}_{c}", "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != c:
                continue
            name = r.get("Kernel_Name", "")
            vals.setdefault(name, []).append(float(r["Counter_Value"]))
    # the probed kernel = the wgemm/attention instantiation with the most dispatches
    probed = {k: v for k, v in vals.items() if re.search(r"wgemm_kernel|attn_decode|attn_kernel|head_screen_kernel", k)}
    name, v = max(probed.items(), key=lambda kv: len(kv[1]))
    v = v[1:] if len(v) > 2 else v  # drop the warm-up launch
    kb = sum(v) / len(v)
    res[c] = dict(kernel_name=name, dispatches=len(v), kb_per_launch=kb)
fetch = res["FETCH_SIZE"]["kb_per_launch"] * 1024 * 2  # x2: gfx950 FETCH_SIZE tallies half
write = res["WRITE_SIZE"]["kb_per_launch"] * 1024
res["hbm_bytes_per_launch"] = fetch + write
res["note"] = "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE; KB = 1024 B"
json.dump(res, open(os.path.join(out, f"{kern}_{rows}.json"), "w"), indent=1)
print(json.dumps(res))
