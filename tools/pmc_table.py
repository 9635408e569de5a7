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


def mfma_table(d):
    """MFMA pass: per kernel F32 MFMA ops (x512 = flops), MFMA-busy cycles and the busy fraction of the
    1024 SIMDs over the dispatch (GRBM_GUI_ACTIVE / 8 cycles: rocprofv3 sums it over the 8 XCDs)."""
    p = os.path.join(d, "pmc_MFMA")
    mops = per_kernel(p, "SQ_INSTS_VALU_MFMA_MOPS_F32")
    busy = per_kernel(p, "SQ_VALU_MFMA_BUSY_CYCLES")
    grbm = per_kernel(p, "GRBM_GUI_ACTIVE")
    out = csv.writer(sys.stdout)
    out.writerow(["kernel", "dispatches", "mfma_f32_flops_per_dispatch", "mfma_busy_cycles_per_dispatch",
                  "grbm_gui_active_per_dispatch", "mfma_busy_frac"])
    rows = []
    for k in mops:
        n = mops[k][1]
        m = mops[k][0] / n
        b = busy.get(k, [0.0, 1])[0] / busy.get(k, [0.0, 1])[1]
        g = grbm.get(k, [0.0, 1])[0] / grbm.get(k, [0.0, 1])[1]
        rows.append((k, n, 512 * m, b, g, b / (g / 8 * 1024) if g else 0.0))
    rows.sort(key=lambda r: -r[2])
    for k, n, f, b, g, u in rows:
        out.writerow([k, n, round(f), round(b), round(g), round(u, 4)])


def all_counters(d):
    """Every counter of one pass directory, averaged per dispatch, one row per kernel."""
    names = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            names.add(r.get("Counter_Name"))
    tabs = {c: per_kernel(d, c) for c in sorted(n for n in names if n)}
    kernels = sorted({k for t in tabs.values() for k in t})
    out = csv.writer(sys.stdout)
    out.writerow(["kernel", "dispatches"] + list(tabs))
    for k in kernels:
        n = max(t.get(k, [0, 0])[1] for t in tabs.values())
        out.writerow([k, n] + [round(tabs[c][k][0] / tabs[c][k][1]) if k in tabs[c] else "" for c in tabs])


def main():
    if sys.argv[1] == "--mfma":
        return mfma_table(sys.argv[2])
    if sys.argv[1] == "--all":
        return all_counters(sys.argv[2])
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
