"""Which HIP API calls launch the runtime's blit kernels (__amd_rocclr_copyBuffer / fillBuffer) in a rocprofv3
trace: kernel-trace rows joined to hip-api-trace rows by correlation id, counted per API function and per queue.
    python tools/copy_origin.py <run_kernel_trace.csv> <run_hip_api_trace.csv>"""
import csv
import sys
from collections import Counter

api = {r["Correlation_Id"]: r["Function"] for r in csv.DictReader(open(sys.argv[2]))}
by = Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "rocclr" in r["Kernel_Name"]:
        by[(r["Kernel_Name"][:40], api.get(r["Correlation_Id"], "?"), r["Queue_Id"])] += 1
for (k, f, q), n in by.most_common():
    print(f"{n:6d}  {k:40s} {f:32s} queue {q}")
