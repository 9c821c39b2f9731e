"""Calibrate FETCH_SIZE / WRITE_SIZE per access class (profiles/history/DESIGN_rounds1-5.md §6).

Runs scripts/build/pmc_calib (scripts/pmc_calib.hip) under rocprofv3 twice,
one counter per pass (FETCH_SIZE, then WRITE_SIZE: they cannot share a pass),
pairs each class kernel's per-dispatch counter (median of 3) with the bytes
the class moves, and prints one JSON object: for every class, the counter
bytes per algorithmic byte.  bench.py's pmc_traffic divides each kernel's
counters by the sum of its classes' expected counter bytes.

  python scripts/pmc_calib.py OUT.json
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "scripts", "build", "pmc_calib")


def build():
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(EXE.replace("build/", "") + ".hip"):
        os.makedirs(os.path.dirname(EXE), exist_ok=True)
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-o", EXE,
                        os.path.join(ROOT, "scripts", "pmc_calib.hip")], check=True)


def rows(counter):
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    d = tempfile.mkdtemp(prefix=f"calib_{counter}_")
    r = subprocess.run([prof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--", EXE],
                       check=True, timeout=300, capture_output=True, text=True, env=dict(os.environ, TMPDIR=d))
    classes = json.loads(r.stdout[r.stdout.index("["):])
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name", counter) == counter:
                    out.append((int(row.get("Dispatch_Id", 0)), row["Kernel_Name"], float(row["Counter_Value"])))
    shutil.rmtree(d, ignore_errors=True)
    out.sort()
    return classes, out


def main():
    build()
    res = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        classes, rs = rows(counter)
        per = {}
        for _, name, v in rs:
            base = name.split("(")[0].replace("void ", "").strip()
            per.setdefault(base, []).append(v)
        # k_sparse16 runs twice per rep: stride 1500, then 4532
        if "k_sparse16" in per:
            s = per.pop("k_sparse16")
            per["k_sparse16@1500"], per["k_sparse16@4532"] = s[0::2], s[1::2]
        for c in classes:
            if c["write"] != (counter == "WRITE_SIZE"):
                continue
            vals = per.get(c["kernel"])
            if not vals:
                res[c["kernel"]] = dict(c, counter=counter, error="no rows")
                continue
            med = sorted(vals)[len(vals) // 2] * 1024.0  # KiB -> bytes
            res[c["kernel"]] = dict(c, counter=counter, counter_bytes=med, dispatches=len(vals),
                                    counter_per_byte=round(med / c["bytes"], 4))
    text = json.dumps(res, indent=1)
    print(text)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
