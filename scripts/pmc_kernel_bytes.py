"""HBM bytes of one kernel from separate rocprofv3 FETCH_SIZE and WRITE_SIZE passes (MI355X_MICROARCH.md § HBM):
FETCH_SIZE is doubled (gfx950 tallies 128-B wide requests at 64 B), WRITE_SIZE read as is; both in KiB.

    python scripts/pmc_kernel_bytes.py <fetch counter_collection.csv> <write counter_collection.csv> <kernel substring>
Reports the LAST dispatch of the kernel in each pass (the passes run the same command; earlier dispatches are
warm-ups), with every dispatch's values beside it."""
import csv
import json
import sys


def per_dispatch(path, counter, kname):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and kname in r["Kernel_Name"]:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


f = per_dispatch(sys.argv[1], "FETCH_SIZE", sys.argv[3])
w = per_dispatch(sys.argv[2], "WRITE_SIZE", sys.argv[3])
rd = 2 * 1024 * f[-1] if f else 0.0
wr = 1024 * w[-1] if w else 0.0
print(json.dumps({"kernel": sys.argv[3], "dispatches": [len(f), len(w)], "hbm_read_bytes": rd, "hbm_write_bytes": wr,
                  "hbm_bytes": rd + wr, "fetch_doubled": True, "last_dispatch": True, "per_dispatch_fetch_kib": f[-4:],
                  "per_dispatch_write_kib": w[-4:]}))
