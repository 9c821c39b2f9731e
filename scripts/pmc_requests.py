"""What FETCH_SIZE is made of, per kernel (profiles/r05/README.md): the L2's
memory-side read requests (TCC_EA0_RDREQ, of which TCC_EA0_RDREQ_32B are
32-byte and TCC_BUBBLE 128-byte ones; FETCH_SIZE = 128 x BUBBLE + 64 x (the
rest) + 32 x 32B), the scalar cache's read requests to the L2
(SQC_TC_DATA_READ_REQ) and the L2's hits and misses -- for the calibration
classes of scripts/pmc_calib.hip (streaming read; k_segments_pk's descriptor
pattern: scalar span loads, vector loads, both) and for the headline kernel
k_segments_pk itself (bench.py --pmc-child --config mtu).  One counter set
per rocprofv3 pass, every pass under its own time limit.

  python scripts/pmc_requests.py OUTDIR > OUTDIR/pmc_requests.txt
"""
import csv
import glob
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_BUBBLE_sum"],
          ["SQC_TC_DATA_READ_REQ"],
          ["TCC_HIT_sum", "TCC_MISS_sum"]]
PROGRAMS = {
    "calib": [os.path.join(ROOT, "scripts", "build", "pmc_calib")],
    "mtu": [sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child", "--config", "mtu", "--steps", "3",
            "--warmup", "1"],
}
KERNELS = ("k_stream<true>", "k_pkdesc<0>", "k_pkdesc<1>", "k_pkdesc<2>", "k_desc<24>", "k_segments_pk")


def run_pass(cmd, counters, keep):
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    d = tempfile.mkdtemp(prefix="pmcreq_")
    args = ["timeout", "-s", "KILL", "120", prof, "--pmc"] + counters + ["--output-format", "csv", "-d", d, "-o",
                                                                           "pmc", "--"] + cmd
    r = subprocess.run(args, capture_output=True, text=True, env=dict(os.environ, TMPDIR=d))
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        shutil.copy(f, os.path.join(keep, f"pmcreq_{'_'.join(c.lower() for c in counters)}_{os.path.basename(f)}"))
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                for k in KERNELS:
                    if name.startswith(k) or (k == "k_segments_pk" and "k_segments_pk" in name):
                        per.setdefault((k, row["Counter_Name"]), []).append(float(row["Counter_Value"]))
    shutil.rmtree(d, ignore_errors=True)
    return r.returncode, {k: sorted(v)[len(v) // 2] for k, v in per.items()}


def main():
    keep = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcreq"
    os.makedirs(keep, exist_ok=True)
    for prog, cmd in PROGRAMS.items():
        vals = {}
        for counters in PASSES:
            rc, v = run_pass(cmd, counters, keep)
            print(f"# {prog}: pass {counters} rc {rc}", flush=True)
            vals.update(v)
        for k in KERNELS:
            row = {c: vals.get((k, c)) for p in PASSES for c in p}
            if all(x is None for x in row.values()):
                continue
            rq, r32, b128 = (row.get("TCC_EA0_RDREQ_sum") or 0, row.get("TCC_EA0_RDREQ_32B_sum") or 0,
                             row.get("TCC_BUBBLE_sum") or 0)
            fetch = 128 * b128 + 64 * (rq - b128 - r32) + 32 * r32
            print(f"{prog:6s} {k:16s} " + "  ".join(f"{c}={v:.0f}" for c, v in row.items() if v is not None)
                  + f"  -> FETCH_SIZE bytes {fetch:.0f}", flush=True)


if __name__ == "__main__":
    main()
