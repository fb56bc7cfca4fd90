"""Live rocprofv3 PMC passes for bench.py's roofline line (imported by bench.py, rank 0, N=1).

Three passes of ONE child process each (`rocprofv3 --pmc <counters> -- python bench.py
--pmc-child ...`): FETCH_SIZE, WRITE_SIZE (TCC: 3 + 2 of its 4 slots, so one per pass) and
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE.  The child runs two eager forwards of the bench's
workload; every dispatch of the MFMA GEMM family is averaged.  Corrections as
MI355X_MICROARCH.md ("HBM [CDNA4]") prescribes and tools/pmc_traffic.py applies: FETCH_SIZE is
KiB and reports half the bytes of a wide streaming read on gfx950 (x 2 x 1024); WRITE_SIZE is
KiB, exact for 16-B-per-lane stores.  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8
XCDs x 1024 SIMDs) over the family's dispatches (tools/pmc_mfma.py).

The passes run BEFORE the parent process touches the GPU (children only), each under its own
SIGKILL timeout; any failure returns None and bench.py falls back to the committed record.
"""
from __future__ import annotations

import csv
import glob
import os
import shutil
import subprocess
import sys
from collections import defaultdict

GEMM = ("gemm_glds_kernel", "gemm_kernel", "gemm_pp256_kernel", "gemm_sk_kernel", "gemm_skr_kernel", "k_conv3x3_c32")
PASSES = {"fetch": ("FETCH_SIZE",), "write": ("WRITE_SIZE",), "mfma": ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")}


def _rows(d):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        return None
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(files[0])):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    return [(names[k], cs) for k, cs in per.items()]


def _gemm(rows):
    return [cs for n, cs in rows if any(p in n for p in GEMM)]


def collect(child_argv, out_dir, timeout=240):
    rocprof = shutil.which("rocprofv3")
    if rocprof is None:
        return None
    env = dict(os.environ, TMPDIR="/tmp")
    res = {}
    for name, ctrs in PASSES.items():
        d = os.path.join(out_dir, name)
        shutil.rmtree(d, ignore_errors=True)
        cmd = [rocprof, "--pmc", *ctrs, "-d", d, "-o", "run", "--output-format", "csv", "--", sys.executable,
               *child_argv]
        try:
            r = subprocess.run(cmd, env=env, cwd="/tmp", timeout=timeout, stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE)
        except subprocess.TimeoutExpired:
            return None
        if r.returncode != 0:
            sys.stderr.write(f"pmc pass {name} failed rc={r.returncode}: {r.stderr.decode()[-400:]}\n")
            return None
        rows = _rows(d)
        if not rows:
            return None
        res[name] = _gemm(rows)
    f, w, m = res["fetch"], res["write"], res["mfma"]
    if not f or not w or not m:
        return None
    read_b = sum(cs.get("FETCH_SIZE", 0.0) for cs in f) * 2.0 * 1024.0 / len(f)
    write_b = sum(cs.get("WRITE_SIZE", 0.0) for cs in w) * 1024.0 / len(w)
    cyc = sum(cs.get("GRBM_GUI_ACTIVE", 0.0) for cs in m) / 8.0
    busy = sum(cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for cs in m) / (cyc * 1024.0) if cyc else None
    return {"bytes_per_launch": read_b + write_b, "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
            "launches_per_pass": len(f), "mfma_busy": busy}
