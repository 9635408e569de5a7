"""Print the kernels of one replayed step from a rocprofv3 kernel trace (csv), grouped by queue, with start offsets
and durations: python tools/trace_one_step.py <kernel_trace.csv> [marker-kernel substring] [which: -2 = 2nd last]"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "multi_tensor_apply"
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
    r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
    st = [i for i, x in enumerate(r) if marker in x["Kernel_Name"]]
    s0 = st[which]
    s1 = st[which + 1] if which + 1 < 0 or which + 1 < len(st) else len(r)
    t0 = int(r[s0]["Start_Timestamp"])
    end = 0
    for x in r[s0:s1]:
        n = re.sub(r"s2s::\(anonymous namespace\)::", "", x["Kernel_Name"]).replace("void ", "")[:58]
        a, b = int(x["Start_Timestamp"]) - t0, int(x["End_Timestamp"]) - t0
        end = max(end, b)
        print(f"{a / 1000:8.1f} {(b - a) / 1000:7.1f} q{x['Queue_Id']:>2} {n}")
    print(f"step span {end / 1000:.1f} us")


if __name__ == "__main__":
    main()
