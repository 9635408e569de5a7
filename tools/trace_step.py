"""Diagnostic: one training step's kernel timeline from a rocprofv3 --kernel-trace csv
(python tools/trace_step.py gpurun_out/tr/tr_kernel_trace.csv): kernels of the last step in
start order with queue, start offset, duration, and the idle gaps of the main queue."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows]
ks.sort()
# a step starts at its head: step_head_kernel (pad + pack + first sync prep in one launch), or pad_cols_kernel
# (the layer-1 input padding) when the head runs as separate launches (S2S_HEAD_FUSED=0)
starts = [i for i, k in enumerate(ks) if "step_head_kernel" in k[3]] or \
    [i for i, k in enumerate(ks) if "pad_cols_kernel" in k[3]]
a, b = starts[-2], starts[-1]
step = ks[a:b]
t0 = step[0][0]
t_end = max(e for _, e, _, _ in step)
print(f"step span {(t_end - t0) / 1000:.1f} us, {len(step)} kernels")
agg = {}
for s, e, q, n in step:
    short = re.sub(r"\(.*", "", n.replace("s2s::(anonymous namespace)::", "")).replace("void ", "")
    print(f"q{q:>2} {(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  {short[:70]}")
    agg.setdefault(short[:40], [0, 0.0])
    agg[short[:40]][0] += 1
    agg[short[:40]][1] += (e - s) / 1000
print("---- per kernel family")
for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{us:9.1f} us  x{c:3d}  {k}")
