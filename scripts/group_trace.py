"""Group a rocprofv3 kernel_trace.csv by (kernel, grid): calls and duration
statistics per launch shape, so the headline kernel's full-size launches can
be compared with bench.py's ms_per_step (the same kernel name also serves the
small e2e chunks and the synchronous drop-in calls).

  python scripts/group_trace.py KERNEL_TRACE.csv [TITLE] > by_launch.txt
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name.split("(")[0] if "(" in name else name


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    groups = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            wg = int(r["Workgroup_Size_X"]) or 1
            blocks = int(r["Grid_Size_X"]) // wg
            groups[(short(r["Kernel_Name"]), blocks)].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(title)
    print(f"{'kernel':44s} {'workgroups':>10s} {'calls':>6s} {'mean_us':>9s} {'median_us':>9s} "
          f"{'min_us':>8s} {'max_us':>8s}")
    for (k, blocks), ds in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[:44]:44s} {blocks:10d} {len(ds):6d} {statistics.mean(ds):9.1f} "
              f"{statistics.median(ds):9.1f} {min(ds):8.1f} {max(ds):8.1f}")


if __name__ == "__main__":
    main()
