"""Per-kernel SQ counter table for the XCD-local decoder launches (dec_xcd_fwd / dec_xcd_bwd) from rocprofv3 --pmc
passes (one dispatch per launch, counters summed over the dispatch's instances):
python tools/pmc_dec.py <dir with pmc1_<config>/ pmc2_<config>/ ...>  ->  CSV on stdout."""
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1]
    rows = {}
    for sub in sorted(glob.glob(os.path.join(d, "pmc*_*"))):
        cfg = os.path.basename(sub).split("_", 1)[1]
        for f in glob.glob(os.path.join(sub, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                m = re.search(r"(dec_xcd_(fwd|bwd))<([^>]*)>", k)
                if not m:
                    continue
                key = (cfg, m.group(1))
                disp = rows.setdefault(key, {}).setdefault(r["Counter_Name"], {})
                did = r.get("Dispatch_Id")
                disp[did] = disp.get(did, 0.0) + float(r["Counter_Value"])
    ctrs = sorted({c for v in rows.values() for c in v})
    w = csv.writer(sys.stdout)
    w.writerow(["config", "kernel"] + ctrs)
    for (cfg, kern), v in sorted(rows.items()):
        w.writerow([cfg, kern] + [round(sum(v[c].values()) / len(v[c])) if c in v else "" for c in ctrs])


if __name__ == "__main__":
    main()
