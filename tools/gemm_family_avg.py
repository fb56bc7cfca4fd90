"""Average duration of the bench's roofline family (the MFMA GEMM / implicit-GEMM conv kernels, as
pmc_mfma.py groups them) in a rocprofv3 --kernel-trace --stats summary, to set beside the bench
line's roofline.avg_launch_ms.  usage: python tools/gemm_family_avg.py <run_kernel_stats.csv>"""
import csv
import sys

FAM = ("gemm_glds_kernel", "gemm_kernel", "gemm_pp256_kernel", "gemm_sk_kernel", "k_conv3x3_c32",
       "gemm_sk2_kernel", "gemm_stk_kernel")
n = t = 0
for r in csv.DictReader(open(sys.argv[1])):
    if any(p in r["Name"] for p in FAM):
        n += int(r["Calls"])
        t += float(r["TotalDurationNs"])
print(f"GEMM family in the trace: {n} calls, average {t / max(n, 1) / 1e3:.1f} us per launch")
