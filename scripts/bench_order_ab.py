"""Why does configs[3]'s `mixed` line read lower inside the default bench
line than alone (0.897 in the line, 0.928 alone)?

Runs `bench.py` several ways on ONE box, one process each, in interleaved
rounds, and prints every secondary config's roofline frac per variant:

  default     the line as the driver runs it (secondaries tso, mixed, ...,
              the CPU-baseline legs after tso and mixed)
  no_cpu      the same without the CPU-baseline legs
  mixed_first the secondaries with mixed before tso (no CPU legs)
  alone       `--config mixed` alone (its own line)
With --arenas instead: free (the default's arena handling), keep (no
secondary arena freed), prealloc (all allocated before the first is timed),
gap2s (2 s idle between the secondary configs).  With --children: the
headline after its PMC / trace children with and without bench.py's pause
after them, and with no children at all.

  python scripts/bench_order_ab.py [ROUNDS] > out.txt
The host-memory legs (e2e, PMC and trace children) are off in every variant.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--no-pmc", "--no-trace", "--no-e2e"]
SEC = "tso,mixed,mixed_aligned,mixed_rx"
VARIANTS = {
    "default": ["--secondary", SEC],
    "no_cpu": ["--secondary", SEC, "--no-cpu"],
    "mixed_first": ["--secondary", "mixed,tso,mixed_aligned,mixed_rx", "--no-cpu"],
    "alone": ["--config", "mixed", "--secondary", "", "--no-cpu"],
}
if "--children" in sys.argv:  # the headline after the PMC / trace children, with and without the pause
    BASE = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--no-e2e", "--no-cpu", "--secondary", ""]
    VARIANTS = {
        "children_gap2s": [],
        "children_nogap": ["--child-gap-ms", "0"],
        "no_children": ["--no-pmc", "--no-trace"],
    }
elif "--arenas" in sys.argv:  # round 5's second pass: what about running after TSO slows the next config
    VARIANTS = {
        "free": ["--secondary", SEC, "--no-cpu"],
        "keep": ["--secondary", SEC, "--no-cpu", "--arena-policy", "keep"],
        "prealloc": ["--secondary", SEC, "--no-cpu", "--arena-policy", "prealloc"],
        "gap2s": ["--secondary", SEC, "--no-cpu", "--gap-ms", "2000"],
    }


def run(args):
    r = subprocess.run(BASE + args, capture_output=True, text=True, timeout=600, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"rc {r.returncode}: {r.stderr[-400:]}"}
    line = json.loads(lines[-1])
    head = args[args.index("--config") + 1] if "--config" in args else "mtu"
    fr = {head: line["roofline"]["frac"]}
    for k, v in line.get("configs", {}).items():
        fr[k] = v["roofline"]["frac"]
    return fr


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 2
    names = list(VARIANTS)
    res = {k: [] for k in names}
    for r in range(rounds):
        for i in range(len(names)):
            name = names[(r + i) % len(names)]
            out = run(VARIANTS[name])
            res[name].append(out)
            print(f"round {r} {name:12s} {json.dumps(out)}", flush=True)
    print("# roofline frac per config (each round)")
    for name in names:
        cfgs = {}
        for o in res[name]:
            for k, v in o.items():
                if k != "error":
                    cfgs.setdefault(k, []).append(v)
        print(f"{name:12s} " + "  ".join(f"{k}={','.join(f'{x:.4f}' for x in v)}" for k, v in sorted(cfgs.items())),
              flush=True)


if __name__ == "__main__":
    main()
