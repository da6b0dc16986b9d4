"""Turn a FETCH_SIZE / WRITE_SIZE rocprofv3 pass into per-launch HBM bytes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half of
the bytes of a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE KiB;
WRITE_SIZE reads exactly for 16-B streaming stores (our stores are a few bytes
per segment, negligible).  Writes/updates profiles/pmc_traffic.json.

usage: python scripts/pmc_traffic.py <pmc dir> <key> <containers_per_rank> [kernel substring]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, key, containers = sys.argv[1], sys.argv[2], int(sys.argv[3])
ksub = sys.argv[4] if len(sys.argv) > 4 else "k_simple"
vals = defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if ksub in row.get("Kernel_Name", ""):
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
fetch = sum(vals["FETCH_SIZE"]) / max(len(vals["FETCH_SIZE"]), 1)
write = sum(vals["WRITE_SIZE"]) / max(len(vals["WRITE_SIZE"]), 1)
rec = {
    "containers_per_rank": containers,
    "fetch_size_kib_per_launch": fetch,
    "write_size_kib_per_launch": write,
    "hbm_bytes_per_launch": int(2 * fetch * 1024 + write * 1024),
    "correction": "read bytes = 2 x FETCH_SIZE KiB (gfx950 wide-read halving); + WRITE_SIZE KiB",
    "source": os.path.relpath(root),
}
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
doc = {}
if os.path.exists(path):
    with open(path) as fh:
        doc = json.load(fh)
doc[key] = rec
with open(path, "w") as fh:
    json.dump(doc, fh, indent=1, sort_keys=True)
print(key, rec)
