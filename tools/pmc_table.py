"""Per-kernel HBM traffic table from the two rocprofv3 PMC passes written by tools/profile_round.sh
(python tools/pmc_table.py <dir with pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/>).  Bytes per dispatch =
(2 * FETCH_SIZE + WRITE_SIZE) KiB: on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane
reads (MI355X_MICROARCH.md, HBM / rocprofv3)."""
import csv
import glob
import os
import re
import sys


def per_kernel(d, ctr):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != ctr:
                continue
            name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("s2s::(anonymous namespace)::", "")).replace("void ", "")
            a = acc.setdefault(name, [0.0, 0])
            a[0] += float(r["Counter_Value"])
            a[1] += 1
    return acc


def main():
    d = sys.argv[1]
    f = per_kernel(os.path.join(d, "pmc_FETCH_SIZE"), "FETCH_SIZE")
    w = per_kernel(os.path.join(d, "pmc_WRITE_SIZE"), "WRITE_SIZE")
    rows = []
    for k in f:
        if k not in w:
            continue
        fk, wk = f[k][0] / f[k][1], w[k][0] / w[k][1]
        rows.append((k, f[k][1], fk, wk, (2 * fk + wk) * 1024))
    rows.sort(key=lambda r: -r[4])
    out = csv.writer(sys.stdout)
    out.writerow(["kernel", "dispatches", "FETCH_SIZE_KB_per_dispatch", "WRITE_SIZE_KB_per_dispatch",
                  "hbm_bytes_per_dispatch_(2F+W)KiB"])
    for k, n, fk, wk, b in rows:
        out.writerow([k, n, round(fk, 1), round(wk, 1), round(b)])


if __name__ == "__main__":
    main()
